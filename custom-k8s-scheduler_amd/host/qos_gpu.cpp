// qos_gpu.cpp — QoSGPU / score-component / QoSSort plugins over libqsched (see qos_gpu.hpp).
#include "qos_gpu.hpp"

#include <algorithm>
#include <stdexcept>

namespace qsfw {

// ---- backend -------------------------------------------------------------------------------
GpuBackend::GpuBackend(const qs_config &cfg, int device) : cfg_(cfg) {
    const qs_status st = qs_open(&cfg_, device, &ctx_);
    if (st != QS_OK)
        throw std::runtime_error("QoSGPU: qs_open failed (status " + std::to_string((int)st) +
                                 "): libqsched needs an MI355X device; there is no CPU fallback");
}

GpuBackend::~GpuBackend() {
    if (ctx_) qs_close(ctx_);
}

std::string GpuBackend::err(const char *what) const {
    return std::string("QoSGPU: ") + what + ": " + qs_last_error(ctx_);
}

void GpuBackend::node_row(const Handle &h, const NodeInfo &ni, qs_node_row *r) {
    *r = qs_node_row{};
    r->alloc_cpu = ni.allocatable.milli_cpu;
    r->alloc_mem = ni.allocatable.memory;
    r->max_pods = ni.allocatable.allowed_pod_number;
    r->req_cpu = ni.requested.milli_cpu;
    r->req_mem = ni.requested.memory;
    r->nz_cpu = ni.non_zero_requested.milli_cpu;
    r->nz_mem = ni.non_zero_requested.memory;
    r->pods = ni.pods;
    const auto &ext = h.ExtendedResourceNames();
    for (size_t k = 0; k < ext.size() && k < QS_MAX_EXT; ++k) {
        auto a = ni.allocatable.scalar.find(ext[k]);
        auto q = ni.requested.scalar.find(ext[k]);
        r->alloc_ext[k] = a == ni.allocatable.scalar.end() ? 0 : a->second;
        r->req_ext[k] = q == ni.requested.scalar.end() ? 0 : q->second;
    }
    intern_.node_masks(ni.node, &r->taint_hard, &r->taint_soft, r->label_bits);
}

Status GpuBackend::load_all(const Handle &h) {
    const auto &nodes = h.NodeInfos();
    const size_t n = nodes.size();
    std::vector<int64_t> ac(n), am(n), mp(n), rc(n), rm(n), zc(n), zm(n), np(n);
    std::vector<int64_t> ae(n * QS_MAX_EXT), re(n * QS_MAX_EXT);
    std::vector<uint64_t> th(n), ts(n), lb(2 * n);
    for (size_t i = 0; i < n; ++i) {
        qs_node_row r;
        node_row(h, nodes[i], &r);
        ac[i] = r.alloc_cpu; am[i] = r.alloc_mem; mp[i] = r.max_pods;
        rc[i] = r.req_cpu; rm[i] = r.req_mem; zc[i] = r.nz_cpu; zm[i] = r.nz_mem; np[i] = r.pods;
        for (int k = 0; k < QS_MAX_EXT; ++k) { ae[i * QS_MAX_EXT + k] = r.alloc_ext[k]; re[i * QS_MAX_EXT + k] = r.req_ext[k]; }
        th[i] = r.taint_hard; ts[i] = r.taint_soft; lb[2 * i] = r.label_bits[0]; lb[2 * i + 1] = r.label_bits[1];
    }
    qs_node_soa soa{ac.data(), am.data(), ae.data(), mp.data(), rc.data(), rm.data(), re.data(),
                    zc.data(), zm.data(), np.data(), th.data(), ts.data(), lb.data(), nullptr};
    if (qs_nodes_load(ctx_, &soa, (uint32_t)n) != QS_OK) return Status::AsError(err("qs_nodes_load"));
    gen_.resize(n);
    for (size_t i = 0; i < n; ++i) gen_[i] = nodes[i].generation;
    label_gen_ = intern_.requirement_generation();
    ++full_loads_;
    return Status::OK();
}

Status GpuBackend::sync(const Handle &h) {
    const auto &nodes = h.NodeInfos();
    if (nodes.size() != gen_.size() || label_gen_ != intern_.requirement_generation()) return load_all(h);
    for (size_t i = 0; i < nodes.size(); ++i) {
        if (gen_[i] == nodes[i].generation) continue;
        qs_node_row r;
        node_row(h, nodes[i], &r);
        if (qs_node_upsert(ctx_, (uint32_t)i, &r, (uint64_t)nodes[i].generation) != QS_OK)
            return Status::AsError(err("qs_node_upsert"));
        gen_[i] = nodes[i].generation;
        ++row_upserts_;
    }
    return Status::OK();
}

Status GpuBackend::Evaluate(const Handle &h, const Pod &pod, const PodResources &res, QoSGPUCycle *out) {
    std::lock_guard<std::mutex> lk(mu_);
    try {
        const auto &ext = h.ExtendedResourceNames();
        qs_pod &rec = out->rec;
        rec = qs_pod{};
        rec.req_cpu = res.cpu;
        rec.req_mem = res.mem;
        rec.nz_cpu = res.nz_cpu;
        rec.nz_mem = res.nz_mem;
        rec.qos = res.qos;
        rec.priority = pod.priority;
        for (const auto &kv : res.scalar) {
            auto it = std::find(ext.begin(), ext.end(), kv.first);
            if (it == ext.end()) {
                if (kv.second > 0)  // no node advertises it: NodeResourcesFit rejects every node
                    return Status(Code::Unschedulable, {"Insufficient " + kv.first});
                continue;
            }
            rec.req_ext[it - ext.begin()] = kv.second;
        }
        intern_.pod_masks(pod, &rec);  // may intern new requirements -> label bits reloaded below
        Status st = sync(h);
        if (!st.IsSuccess()) return st;
        intern_.pod_masks(pod, &rec);  // tolerations over every taint interned by the sync
        const size_t n = h.NodeInfos().size();
        const uint32_t *pk = nullptr;
        if (qs_score_pod_packed(ctx_, &rec, &pk, &out->best) != QS_OK) return Status::AsError(err("qs_score_pod_packed"));
        out->packed.assign(pk, pk + (pk ? n : 0));
        out->packed.resize(n, 0xFFFFFFFFu);
        return Status::OK();
    } catch (const std::exception &e) {
        return Status::AsError(std::string("QoSGPU: ") + e.what());
    }
}

Status GpuBackend::Reserve(const Handle &h, int row, const qs_pod &rec) {
    std::lock_guard<std::mutex> lk(mu_);
    if (qs_reserve(ctx_, (uint32_t)row, &rec) != QS_OK) return Status::AsError(err("qs_reserve"));
    gen_[row] = h.NodeInfos()[row].generation;  // the runner assumed the pod before Reserve
    return Status::OK();
}

Status GpuBackend::Unreserve(const Handle &h, int row, const qs_pod &rec) {
    std::lock_guard<std::mutex> lk(mu_);
    if (qs_unreserve(ctx_, (uint32_t)row, &rec) != QS_OK) return Status::AsError(err("qs_unreserve"));
    (void)h;
    return Status::OK();
}

// ---- plugins ---------------------------------------------------------------------------------
namespace {

QoSGPUCycle *cycle_of(CycleState &s) { return s.Read<QoSGPUCycle>(kQoSGPU); }

class QoSGPUPlugin final : public PreFilterPlugin, public FilterPlugin, public ReservePlugin {
   public:
    QoSGPUPlugin(std::shared_ptr<GpuBackend> b, Handle *h) : b_(std::move(b)), h_(h) {}
    std::string Name() const override { return kQoSGPU; }

    std::pair<PreFilterResult, Status> PreFilter(CycleState &s, const Pod &pod) override {
        auto *pr = s.Read<PodResourcesState>(kPodResourcesKey);
        const PodResources res = pr ? pr->res : ComputePodResources(pod, h_->ExtendedResourceNames());
        auto c = std::make_shared<QoSGPUCycle>();
        Status st = b_->Evaluate(*h_, pod, res, c.get());
        if (!st.IsSuccess()) return {PreFilterResult{}, st};
        s.Write(kQoSGPU, c);
        return {PreFilterResult{}, Status::OK()};
    }

    // The device decided; on rejection the reasons are derived on the host for this node only,
    // in upstream's default filter order (TaintToleration, NodeAffinity, NodeResourcesFit).
    Status Filter(CycleState &s, const Pod &pod, const NodeInfo &ni) override {
        auto *c = cycle_of(s);
        if (!c) return Status::AsError("QoSGPU: PreFilter did not run");
        const int i = h_->NodeIndex(ni.node.name);
        if (i < 0 || (size_t)i >= c->packed.size()) return Status::AsError("QoSGPU: unknown node " + ni.node.name);
        if (c->feasible((size_t)i)) return Status::OK();
        return reasons(s, pod, ni);
    }

    Status Reserve(CycleState &s, const Pod &, const std::string &node) override {
        auto *c = cycle_of(s);
        if (!c) return Status::AsError("QoSGPU: PreFilter did not run");
        return b_->Reserve(*h_, h_->NodeIndex(node), c->rec);
    }
    void Unreserve(CycleState &s, const Pod &, const std::string &node) override {
        if (auto *c = cycle_of(s)) (void)b_->Unreserve(*h_, h_->NodeIndex(node), c->rec);
    }

   private:
    Status reasons(CycleState &s, const Pod &pod, const NodeInfo &ni) {
        const qs_config &cfg = b_->config();
        if (cfg.enable_taint) {
            for (const auto &t : ni.node.taints) {
                if (t.effect != kNoSchedule && t.effect != kNoExecute) continue;
                bool tol = false;
                for (const auto &x : pod.tolerations) tol |= tolerates(x, t);
                if (!tol)
                    return Status(Code::UnschedulableAndUnresolvable,
                                  {"node(s) had untolerated taint {" + t.key + ": " + t.value + "}"});
            }
        }
        if (cfg.enable_affinity) {
            bool ok = true;
            for (const auto &kv : pod.node_selector) ok &= requirement_matches({kv.first, "In", {kv.second}}, ni.node.labels);
            if (ok && !pod.required_terms.empty()) {
                bool any = false;
                for (const auto &t : pod.required_terms) {
                    bool all = !t.match_expressions.empty();
                    for (const auto &r : t.match_expressions) all &= requirement_matches(r, ni.node.labels);
                    any |= all;
                }
                ok = any;
            }
            if (!ok) return Status(Code::UnschedulableAndUnresolvable, {"node(s) didn't match Pod's node affinity/selector"});
        }
        auto *pr = s.Read<PodResourcesState>(kPodResourcesKey);
        const PodResources res = pr ? pr->res : ComputePodResources(pod, h_->ExtendedResourceNames());
        std::vector<std::string> why;  // UP noderesources/fit.go#fitsRequest insufficient resources
        if (ni.pods + 1 > ni.allocatable.allowed_pod_number) why.push_back("Too many pods");
        if (res.cpu > 0 && res.cpu > ni.allocatable.milli_cpu - ni.requested.milli_cpu) why.push_back("Insufficient cpu");
        if (res.mem > 0 && res.mem > ni.allocatable.memory - ni.requested.memory) why.push_back("Insufficient memory");
        for (const auto &kv : res.scalar) {
            if (kv.second == 0) continue;
            auto a = ni.allocatable.scalar.find(kv.first);
            auto q = ni.requested.scalar.find(kv.first);
            const int64_t alloc = a == ni.allocatable.scalar.end() ? 0 : a->second;
            const int64_t used = q == ni.requested.scalar.end() ? 0 : q->second;
            if (kv.second > alloc - used) why.push_back("Insufficient " + kv.first);
        }
        if (why.empty()) why.push_back("node(s) didn't satisfy plugin QoSGPU");
        return Status(Code::Unschedulable, why);
    }

    std::shared_ptr<GpuBackend> b_;
    Handle *h_;
};

// One normalized component of the device evaluation as a Score plugin.
class QoSGPUComponent final : public ScorePlugin {
   public:
    QoSGPUComponent(std::string name, int k, Handle *h) : name_(std::move(name)), k_(k), h_(h) {}
    std::string Name() const override { return name_; }
    std::pair<int64_t, Status> Score(CycleState &s, const Pod &, const std::string &node) override {
        auto *c = cycle_of(s);
        if (!c) return {0, Status::AsError(name_ + ": QoSGPU PreFilter did not run")};
        const int i = h_->NodeIndex(node);
        if (i < 0 || (size_t)i >= c->packed.size()) return {0, Status::AsError(name_ + ": unknown node " + node)};
        return {c->score((size_t)i, k_), Status::OK()};
    }

   private:
    std::string name_;
    int k_;
    Handle *h_;
};

class QoSSortPlugin final : public QueueSortPlugin {
   public:
    std::string Name() const override { return kQoSSort; }
    // spec S8 (shape of UP queuesort/priority_sort.go#Less): QoS class, then priority, then FIFO
    bool Less(const QueuedPodInfo &a, const QueuedPodInfo &b) const override {
        if (a.res.qos != b.res.qos) return a.res.qos > b.res.qos;
        if (a.pod.priority != b.pod.priority) return a.pod.priority > b.pod.priority;
        return a.arrival < b.arrival;
    }
};

}  // namespace

Registry QoSRegistry(std::shared_ptr<GpuBackend> backend) {
    Registry r;
    r[kQoSGPU] = [backend](Handle *h) { return std::make_shared<QoSGPUPlugin>(backend, h); };
    const char *names[4] = {kQoSGPULeastAllocated, kQoSGPUBalancedAllocation, kQoSGPUTaintToleration, kQoSGPUNodeAffinity};
    for (int k = 0; k < 4; ++k) {
        const std::string n = names[k];
        r[n] = [n, k](Handle *h) { return std::make_shared<QoSGPUComponent>(n, k, h); };
    }
    r[kQoSSort] = [](Handle *) { return std::make_shared<QoSSortPlugin>(); };
    return r;
}

static const char *kQoSProfile[3] = {"besteffort", "burstable", "guaranteed"};

std::vector<Profile> QoSProfiles(const qs_config &cfg) {
    std::vector<Profile> out;
    for (int q = 0; q < 3; ++q) {
        Profile p;
        p.scheduler_name = kQoSProfile[q];
        p.queue_sort = kQoSSort;
        p.pre_filter = {{kQoSGPU}};
        p.filter = {{kQoSGPU}};
        p.reserve = {{kQoSGPU}};
        auto add = [&](const char *n, int32_t w) { if (w > 0) p.score.push_back({n, w}); };
        add(kQoSGPULeastAllocated, cfg.w_fit[q]);
        add(kQoSGPUBalancedAllocation, cfg.w_bal[q]);
        if (cfg.enable_taint) add(kQoSGPUTaintToleration, cfg.w_taint);
        if (cfg.enable_affinity) add(kQoSGPUNodeAffinity, cfg.w_affinity);
        out.push_back(p);
    }
    return out;
}

std::string QoSProfileOf(const Pod &, const PodResources &r) { return kQoSProfile[std::clamp(r.qos, 0, 2)]; }

}  // namespace qsfw
