// cpu_plugins.cpp — the CPU reference plugins of cpu_plugins.hpp (upstream citations there).  Each
// Filter / Score call evaluates one (pod, node) pair from the k8s objects; the framework runtime
// (framework.cpp) runs them over the nodes with its Parallelizer.
#include "cpu_plugins.hpp"

#include <algorithm>
#include <cmath>

#include "intern.hpp"

namespace qsfw {
namespace {

constexpr int64_t kMaxNodeScore = MaxNodeScore;

const PodResources &resources_of(CycleState &s, const Pod &pod, const Handle *h, PodResources *tmp) {
    if (auto *pr = s.Read<PodResourcesState>(kPodResourcesKey)) return pr->res;
    *tmp = ComputePodResources(pod, h->ExtendedResourceNames());
    return *tmp;
}

const NodeInfo *node_of(const Handle *h, const std::string &name) {
    const int i = h->NodeIndex(name);
    return i < 0 ? nullptr : &h->NodeInfos()[(size_t)i];
}

// UP noderesources/least_allocated.go#leastRequestedScore
int64_t least_requested_score(int64_t requested, int64_t capacity) {
    if (capacity == 0) return 0;
    if (requested > capacity) return 0;
    return ((capacity - requested) * kMaxNodeScore) / capacity;
}

// UP helper/normalize_score.go#DefaultNormalizeScore
void default_normalize(NodeScoreList &scores, bool reverse) {
    int64_t mx = 0;
    for (const auto &s : scores) mx = std::max(mx, s.score);
    if (mx == 0) {
        if (reverse)
            for (auto &s : scores) s.score = kMaxNodeScore;
        return;
    }
    for (auto &s : scores) {
        int64_t v = kMaxNodeScore * s.score / mx;
        s.score = reverse ? kMaxNodeScore - v : v;
    }
}

bool hard_effect(const std::string &e) { return e == kNoSchedule || e == kNoExecute; }

// NodeResourcesFitArgs.ScoringStrategy.Resources / NodeResourcesBalancedAllocationArgs.Resources as
// (qs_resource, weight) in list order; the defaults [cpu: fit_weight_cpu, memory: fit_weight_mem] and
// [cpu, memory] (UP apis/config/v1/defaults.go)
using ResList = std::vector<std::pair<int32_t, int64_t>>;
ResList fit_list(const qs_config &c) {
    if (c.n_fit_resources == 0) return {{QS_RES_CPU, c.fit_weight_cpu}, {QS_RES_MEMORY, c.fit_weight_mem}};
    ResList r;
    for (int i = 0; i < c.n_fit_resources; ++i) r.push_back({c.fit_resources[i].resource, c.fit_resources[i].weight});
    return r;
}
ResList balanced_list(const qs_config &c) {
    if (c.n_balanced_resources == 0) return {{QS_RES_CPU, 1}, {QS_RES_MEMORY, 1}};
    ResList r;
    for (int i = 0; i < c.n_balanced_resources; ++i) r.push_back({c.balanced_resources[i], 1});
    return r;
}

int64_t lookup(const std::map<std::string, int64_t> &m, const std::string &k) {
    auto it = m.find(k);
    return it == m.end() ? 0 : it->second;
}

// UP noderesources/resource_allocation.go#calculateResourceAllocatableRequest: (allocatable,
// requested + the pod's request) of one scoring resource; cpu / memory from NonZeroRequested and the
// pod's non-zero requests (useRequested = false, LeastAllocated) or Requested and the plain requests
// (true, BalancedAllocation); an extended (scalar) resource the pod does not request is (0, 0), and
// so is one the node does not have (Allocatable.ScalarResources lookup).
std::pair<int64_t, int64_t> alloc_request(const NodeInfo &ni, const PodResources &r, int32_t res,
                                          bool use_requested, const std::vector<std::string> &ext_names) {
    switch (res) {
        case QS_RES_CPU:
            return {ni.allocatable.milli_cpu,
                    use_requested ? ni.requested.milli_cpu + r.cpu : ni.non_zero_requested.milli_cpu + r.nz_cpu};
        case QS_RES_MEMORY:
            return {ni.allocatable.memory,
                    use_requested ? ni.requested.memory + r.mem : ni.non_zero_requested.memory + r.nz_mem};
        default: {
            const size_t k = (size_t)(res - QS_RES_EXT0);
            if (k >= ext_names.size()) return {0, 0};
            const std::string &name = ext_names[k];
            const int64_t q = lookup(r.scalar, name);
            if (q == 0 || !ni.allocatable.scalar.count(name)) return {0, 0};
            return {ni.allocatable.scalar.at(name), lookup(ni.requested.scalar, name) + q};
        }
    }
}

// ---- NodeResourcesFit ------------------------------------------------------------------------
class NodeResourcesFit final : public PreFilterPlugin, public FilterPlugin, public ScorePlugin {
   public:
    NodeResourcesFit(const qs_config &cfg, Handle *h) : res_(fit_list(cfg)), h_(h) {}
    std::string Name() const override { return kNodeResourcesFit; }

    // UP fit.go#PreFilter computes the pod's requests once per cycle (preFilterState)
    std::pair<PreFilterResult, Status> PreFilter(CycleState &s, const Pod &pod) override {
        if (!s.Read<PodResourcesState>(kPodResourcesKey))
            s.Write(kPodResourcesKey, std::make_shared<PodResourcesState>(ComputePodResources(pod, h_->ExtendedResourceNames())));
        return {PreFilterResult{}, Status::OK()};
    }

    // UP fit.go#fitsRequest: every insufficient resource is a reason
    Status Filter(CycleState &s, const Pod &pod, const NodeInfo &ni) override {
        PodResources tmp;
        const PodResources &r = resources_of(s, pod, h_, &tmp);
        std::vector<std::string> why;
        if (ni.pods + 1 > ni.allocatable.allowed_pod_number) why.push_back("Too many pods");
        bool any_scalar = false;
        for (const auto &kv : r.scalar) any_scalar |= kv.second != 0;
        if (r.cpu == 0 && r.mem == 0 && !any_scalar) {
            return why.empty() ? Status::OK() : Status(Code::Unschedulable, why);
        }
        if (r.cpu > 0 && r.cpu > ni.allocatable.milli_cpu - ni.requested.milli_cpu) why.push_back("Insufficient cpu");
        if (r.mem > 0 && r.mem > ni.allocatable.memory - ni.requested.memory) why.push_back("Insufficient memory");
        for (const auto &kv : r.scalar) {
            if (kv.second == 0) continue;
            auto a = ni.allocatable.scalar.find(kv.first);
            auto u = ni.requested.scalar.find(kv.first);
            const int64_t alloc = a == ni.allocatable.scalar.end() ? 0 : a->second;
            const int64_t used = u == ni.requested.scalar.end() ? 0 : u->second;
            if (kv.second > alloc - used) why.push_back("Insufficient " + kv.first);
        }
        return why.empty() ? Status::OK() : Status(Code::Unschedulable, why);
    }

    // LeastAllocated strategy over the scoring resources (UP least_allocated.go#leastResourceScorer,
    // resource_allocation.go#score): requested = NonZeroRequested + the pod's non-zero requests for
    // cpu / memory, Requested + the request for extended resources; resources with allocatable 0 are
    // skipped (their weight not counted)
    std::pair<int64_t, Status> Score(CycleState &s, const Pod &pod, const std::string &node) override {
        const NodeInfo *ni = node_of(h_, node);
        if (!ni) return {0, Status::AsError("node " + node + " not found")};
        PodResources tmp;
        const PodResources &r = resources_of(s, pod, h_, &tmp);
        int64_t score = 0, wsum = 0;
        for (const auto &rw : res_) {
            const auto ar = alloc_request(*ni, r, rw.first, false, h_->ExtendedResourceNames());
            if (ar.first == 0) continue;
            score += least_requested_score(ar.second, ar.first) * rw.second;
            wsum += rw.second;
        }
        return {wsum == 0 ? 0 : score / wsum, Status::OK()};
    }

   private:
    ResList res_;
    Handle *h_;
};

// ---- NodeResourcesBalancedAllocation ---------------------------------------------------------
class BalancedAllocation final : public ScorePlugin {
   public:
    BalancedAllocation(const qs_config &cfg, Handle *h)
        : res_(balanced_list(cfg)), skip_be_(cfg.balanced_skip_besteffort != 0), h_(h) {}
    std::string Name() const override { return kNodeResourcesBalancedAllocation; }

    // UP balanced_allocation.go#balancedResourceScorer over the configured resources, float64:
    // fractions of Requested + the pod's requests (capped at 1) in list order, std = |f0 - f1| / 2 for
    // two, the population standard deviation (mean, sum of squared deviations, sqrt) for more,
    // int64((1 - std) * MaxNodeScore)
    std::pair<int64_t, Status> Score(CycleState &s, const Pod &pod, const std::string &node) override {
        const NodeInfo *ni = node_of(h_, node);
        if (!ni) return {0, Status::AsError("node " + node + " not found")};
        PodResources tmp;
        const PodResources &r = resources_of(s, pod, h_, &tmp);
        if (skip_be_ && r.qos == QS_QOS_BESTEFFORT) return {0, Status::OK()};
        double fr[QS_MAX_SCORE_RES], total = 0.0;
        int cnt = 0;
        for (const auto &rw : res_) {
            const auto ar = alloc_request(*ni, r, rw.first, true, h_->ExtendedResourceNames());
            if (ar.first == 0) continue;
            const double f = (double)ar.second / (double)ar.first;
            fr[cnt] = f > 1 ? 1 : f;
            total += fr[cnt++];
        }
        double sd = 0.0;
        if (cnt == 2) {
            sd = std::fabs((fr[0] - fr[1]) / 2);
        } else if (cnt > 2) {
            const double mean = total / (double)cnt;
            double sum = 0.0;
            for (int i = 0; i < cnt; ++i) sum = sum + (fr[i] - mean) * (fr[i] - mean);
            sd = std::sqrt(sum / (double)cnt);
        }
        const double scaled = (1 - sd) * (double)kMaxNodeScore;
        return {(int64_t)scaled, Status::OK()};
    }

   private:
    ResList res_;
    bool skip_be_;
    Handle *h_;
};

// ---- TaintToleration -------------------------------------------------------------------------
class TaintToleration final : public FilterPlugin, public ScorePlugin {
   public:
    explicit TaintToleration(Handle *h) : h_(h) {}
    std::string Name() const override { return kTaintToleration; }

    // UP taint_toleration.go#Filter: an untolerated NoSchedule / NoExecute taint rejects the node
    Status Filter(CycleState &, const Pod &pod, const NodeInfo &ni) override {
        for (const auto &t : ni.node.taints) {
            if (!hard_effect(t.effect)) continue;
            bool tol = false;
            for (const auto &x : pod.tolerations) tol = tol || tolerates(x, t);
            if (!tol)
                return Status(Code::UnschedulableAndUnresolvable,
                              {"node(s) had untolerated taint {" + t.key + ": " + t.value + "}"});
        }
        return Status::OK();
    }
    // UP taint_toleration.go#Score: intolerable PreferNoSchedule taints, counted against the
    // tolerations with effect "" or PreferNoSchedule (getAllTolerationPreferNoSchedule)
    std::pair<int64_t, Status> Score(CycleState &, const Pod &pod, const std::string &node) override {
        const NodeInfo *ni = node_of(h_, node);
        if (!ni) return {0, Status::AsError("node " + node + " not found")};
        int64_t n = 0;
        for (const auto &t : ni->node.taints) {
            if (t.effect != kPreferNoSchedule) continue;
            bool tol = false;
            for (const auto &x : pod.tolerations)
                tol = tol || ((x.effect.empty() || x.effect == kPreferNoSchedule) && tolerates(x, t));
            n += tol ? 0 : 1;
        }
        return {n, Status::OK()};
    }
    bool HasScoreExtensions() const override { return true; }
    Status NormalizeScore(CycleState &, const Pod &, NodeScoreList &scores) override {
        default_normalize(scores, /*reverse=*/true);
        return Status::OK();
    }

   private:
    Handle *h_;
};

// ---- NodeAffinity ----------------------------------------------------------------------------
bool term_matches(const NodeSelectorTerm &t, const std::map<std::string, std::string> &labels) {
    if (t.match_expressions.empty()) return false;  // UP nodeaffinity#NewNodeSelector: matches nothing
    for (const auto &r : t.match_expressions)
        if (!requirement_matches(r, labels)) return false;
    return true;
}

class NodeAffinity final : public FilterPlugin, public ScorePlugin {
   public:
    explicit NodeAffinity(Handle *h) : h_(h) {}
    std::string Name() const override { return kNodeAffinity; }

    // UP node_affinity.go#Filter: nodeSelector, then the required terms (OR of ANDs)
    Status Filter(CycleState &, const Pod &pod, const NodeInfo &ni) override {
        bool ok = true;
        for (const auto &kv : pod.node_selector) {
            auto it = ni.node.labels.find(kv.first);
            ok = ok && it != ni.node.labels.end() && it->second == kv.second;
        }
        if (ok && !pod.required_terms.empty()) {
            bool any = false;
            for (const auto &t : pod.required_terms) any = any || term_matches(t, ni.node.labels);
            ok = any;
        }
        return ok ? Status::OK()
                  : Status(Code::UnschedulableAndUnresolvable, {"node(s) didn't match Pod's node affinity/selector"});
    }
    // UP node_affinity.go#Score: sum of the weights of the matching preferred terms (weight 0 skipped)
    std::pair<int64_t, Status> Score(CycleState &, const Pod &pod, const std::string &node) override {
        const NodeInfo *ni = node_of(h_, node);
        if (!ni) return {0, Status::AsError("node " + node + " not found")};
        int64_t s = 0;
        for (const auto &pt : pod.preferred_terms)
            if (pt.weight > 0 && term_matches(pt.preference, ni->node.labels)) s += pt.weight;
        return {s, Status::OK()};
    }
    bool HasScoreExtensions() const override { return true; }
    Status NormalizeScore(CycleState &, const Pod &, NodeScoreList &scores) override {
        default_normalize(scores, /*reverse=*/false);
        return Status::OK();
    }

   private:
    Handle *h_;
};

// spec S8 (shape of UP queuesort/priority_sort.go#Less): QoS class, then priority, then FIFO
class QoSSort final : public QueueSortPlugin {
   public:
    std::string Name() const override { return kCPUQoSSort; }
    bool Less(const QueuedPodInfo &a, const QueuedPodInfo &b) const override {
        if (a.res.qos != b.res.qos) return a.res.qos > b.res.qos;
        if (a.pod.priority != b.pod.priority) return a.pod.priority > b.pod.priority;
        return a.arrival < b.arrival;
    }
};

const char *kProfileName[3] = {"besteffort", "burstable", "guaranteed"};

}  // namespace

Registry CPURegistry(const qs_config &cfg) {
    Registry r;
    r[kNodeResourcesFit] = [cfg](Handle *h) { return std::make_shared<NodeResourcesFit>(cfg, h); };
    r[kNodeResourcesBalancedAllocation] = [cfg](Handle *h) { return std::make_shared<BalancedAllocation>(cfg, h); };
    r[kTaintToleration] = [](Handle *h) { return std::make_shared<TaintToleration>(h); };
    r[kNodeAffinity] = [](Handle *h) { return std::make_shared<NodeAffinity>(h); };
    r[kCPUQoSSort] = [](Handle *) { return std::make_shared<QoSSort>(); };
    return r;
}

std::vector<Profile> CPUProfiles(const qs_config &cfg) {
    std::vector<Profile> out;
    for (int q = 0; q < 3; ++q) {
        Profile p;
        p.scheduler_name = kProfileName[q];
        p.queue_sort = kCPUQoSSort;
        p.pre_filter = {{kNodeResourcesFit}};
        // upstream's default filter order: TaintToleration, NodeAffinity, ..., NodeResourcesFit
        if (cfg.enable_taint) p.filter.push_back({kTaintToleration});
        if (cfg.enable_affinity) p.filter.push_back({kNodeAffinity});
        p.filter.push_back({kNodeResourcesFit});
        auto add = [&](const char *n, int32_t w) { if (w > 0) p.score.push_back({n, w}); };
        add(kNodeResourcesFit, cfg.w_fit[q]);
        add(kNodeResourcesBalancedAllocation, cfg.w_bal[q]);
        if (cfg.enable_taint) add(kTaintToleration, cfg.w_taint);
        if (cfg.enable_affinity) add(kNodeAffinity, cfg.w_affinity);
        out.push_back(p);
    }
    return out;
}

std::string CPUProfileOf(const Pod &, const PodResources &r) { return kProfileName[std::clamp(r.qos, 0, 2)]; }

}  // namespace qsfw
