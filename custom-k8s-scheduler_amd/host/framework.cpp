// framework.cpp — the framework runtime and scheduling loop of framework.hpp (upstream citations
// there).  Host logic only: the Filter/Score decisions come from the plugins — the device-backed
// QoS plugins (qos_gpu.cpp) or the CPU reference plugins (cpu_plugins.cpp) — and this file orders,
// weights and combines them the way upstream's runtime does, with upstream's node Parallelizer.
#include "framework.hpp"

#include <algorithm>
#include <exception>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "../../include/qsched.h"

namespace qsfw {

std::string Status::Message() const {
    std::string m;
    for (size_t i = 0; i < reasons_.size(); ++i) m += (i ? ", " : "") + reasons_[i];
    return m;
}

// ---- pod requests (spec S2/S3 through the C ABI helper) -----------------------------------
namespace {
void fill_container(const Container &c, int kind, const std::vector<std::string> &ext, qs_container *o) {
    *o = qs_container{};
    o->kind = kind;
    auto rq = c.requests.find(kCPU), rm = c.requests.find(kMemory);
    auto lc = c.limits.find(kCPU), lm = c.limits.find(kMemory);
    if (rq != c.requests.end()) { o->has_req_cpu = 1; o->req_cpu = milli_value(rq->second); }
    if (rm != c.requests.end()) { o->has_req_mem = 1; o->req_mem = value(rm->second); }
    if (lc != c.limits.end()) { o->has_lim_cpu = 1; o->lim_cpu = milli_value(lc->second); }
    if (lm != c.limits.end()) { o->has_lim_mem = 1; o->lim_mem = value(lm->second); }
    for (size_t k = 0; k < ext.size() && k < QS_MAX_EXT; ++k) {
        auto e = c.requests.find(ext[k]);
        if (e != c.requests.end()) o->req_ext[k] = value(e->second);
    }
}
}  // namespace

PodResources ComputePodResources(const Pod &p, const std::vector<std::string> &ext_names) {
    std::vector<qs_container> cs;
    for (const auto &c : p.containers) { cs.emplace_back(); fill_container(c, 0, ext_names, &cs.back()); }
    for (const auto &c : p.init_containers) { cs.emplace_back(); fill_container(c, c.restartable ? 2 : 1, ext_names, &cs.back()); }
    int64_t ov[2] = {0, 0};
    const bool has_ov = !p.overhead.empty();
    if (has_ov) {
        auto oc = p.overhead.find(kCPU), om = p.overhead.find(kMemory);
        if (oc != p.overhead.end()) ov[0] = milli_value(oc->second);
        if (om != p.overhead.end()) ov[1] = value(om->second);
    }
    qs_pod rec{};
    if (qs_pod_from_containers(cs.data(), (uint32_t)cs.size(), has_ov ? ov : nullptr, &rec) != QS_OK)
        throw std::invalid_argument("pod " + p.name + ": invalid container resources");
    PodResources r;
    r.cpu = rec.req_cpu;
    r.mem = rec.req_mem;
    r.nz_cpu = rec.nz_cpu;
    r.nz_mem = rec.nz_mem;
    r.qos = rec.qos;
    for (size_t k = 0; k < ext_names.size() && k < QS_MAX_EXT; ++k)
        if (rec.req_ext[k]) r.scalar[ext_names[k]] = rec.req_ext[k];
    // requests of extended resources no node advertises: kept so Filter can reject them
    for (const auto *list : {&p.containers, &p.init_containers})
        for (const auto &c : *list)
            for (const auto &kv : c.requests)
                if (kv.first != kCPU && kv.first != kMemory &&
                    std::find(ext_names.begin(), ext_names.end(), kv.first) == ext_names.end())
                    r.scalar[kv.first] += value(kv.second);
    return r;
}

PodResources ComputePodResources(const Pod &p) { return ComputePodResources(p, {}); }

NodeInfo NewNodeInfo(const Node &n) {
    NodeInfo ni;
    ni.node = n;
    for (const auto &kv : n.allocatable) {
        if (kv.first == kCPU) ni.allocatable.milli_cpu = milli_value(kv.second);
        else if (kv.first == kMemory) ni.allocatable.memory = value(kv.second);
        else if (kv.first == kPods) ni.allocatable.allowed_pod_number = value(kv.second);
        else ni.allocatable.scalar[kv.first] = value(kv.second);
    }
    if (!n.allocatable.count(kPods)) ni.allocatable.allowed_pod_number = 110;  // kubelet default
    ni.generation = 1;
    return ni;
}

void NodeInfo::AddPod(const Pod &p, const PodResources &r) {
    requested.milli_cpu += r.cpu;
    requested.memory += r.mem;
    for (const auto &kv : r.scalar) requested.scalar[kv.first] += kv.second;
    non_zero_requested.milli_cpu += r.nz_cpu;
    non_zero_requested.memory += r.nz_mem;
    ++pods;
    pod_names.push_back(p.ns + "/" + p.name);
    ++generation;
}

void NodeInfo::RemovePod(const Pod &p, const PodResources &r) {
    requested.milli_cpu -= r.cpu;
    requested.memory -= r.mem;
    for (const auto &kv : r.scalar) requested.scalar[kv.first] -= kv.second;
    non_zero_requested.milli_cpu -= r.nz_cpu;
    non_zero_requested.memory -= r.nz_mem;
    --pods;
    auto it = std::find(pod_names.begin(), pod_names.end(), p.ns + "/" + p.name);
    if (it != pod_names.end()) pod_names.erase(it);
    ++generation;
}

// ---- Parallelizer (UP framework/parallelize/parallelism.go) -----------------------------------
struct Parallelizer::Impl {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, done;
    std::atomic<uint64_t> gen{0};
    bool stop = false;
    const std::function<void(int)> *fn = nullptr;
    int n = 0, chunk = 1;
    std::atomic<int> next{0}, active{0};
    std::exception_ptr err;  // the first exception a piece of work threw (rethrown by Until)
    void chunks() {
        try {
            for (;;) {
                const int b = next.fetch_add(chunk, std::memory_order_relaxed);
                if (b >= n) return;
                const int e = std::min(n, b + chunk);
                for (int i = b; i < e; ++i) (*fn)(i);
            }
        } catch (...) {
            // keep the first exception, stop handing out pieces; Until still waits for every
            // worker to leave fn (it points at the caller's stack) before rethrowing it
            std::lock_guard<std::mutex> g(mu);
            if (!err) err = std::current_exception();
            next.store(n, std::memory_order_relaxed);
        }
    }
    void worker() {
        uint64_t seen = 0;
        for (;;) {
            // spin a little for the next section (~20 us), then sleep on the condition variable
            for (int k = 0; k < 2000 && gen.load(std::memory_order_acquire) == seen; ++k) std::this_thread::yield();
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || gen.load(std::memory_order_acquire) != seen; });
                if (stop) return;
                seen = gen.load(std::memory_order_acquire);
            }
            chunks();
            if (active.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> g(mu);
                done.notify_one();
            }
        }
    }
};

Parallelizer::Parallelizer(int workers) : workers_(std::max(1, workers)), m_(new Impl) {
    for (int w = 1; w < workers_; ++w) m_->th.emplace_back([this] { m_->worker(); });
}

Parallelizer::~Parallelizer() {
    {
        std::lock_guard<std::mutex> g(m_->mu);
        m_->stop = true;
    }
    m_->cv.notify_all();
    for (auto &t : m_->th) t.join();
}

void Parallelizer::Until(int n, const std::function<void(int)> &fn) {
    if (n <= 0) return;
    if (workers_ <= 1 || n == 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    // UP parallelize#chunkSizeFor
    int chunk = (int)std::sqrt((double)n);
    chunk = std::min(chunk, n / workers_ + 1);
    chunk = std::max(chunk, 1);
    {
        std::lock_guard<std::mutex> g(m_->mu);
        m_->fn = &fn;
        m_->n = n;
        m_->chunk = chunk;
        m_->err = nullptr;
        m_->next.store(0, std::memory_order_relaxed);
        m_->active.store(workers_ - 1, std::memory_order_relaxed);
        m_->gen.fetch_add(1, std::memory_order_release);
    }
    m_->cv.notify_all();
    m_->chunks();
    if (m_->active.load(std::memory_order_acquire) != 0) {
        std::unique_lock<std::mutex> lk(m_->mu);
        m_->done.wait(lk, [&] { return m_->active.load(std::memory_order_acquire) == 0; });
    }
    std::exception_ptr e;
    {
        std::lock_guard<std::mutex> g(m_->mu);
        e = m_->err;
        m_->err = nullptr;
        m_->fn = nullptr;
    }
    if (e) std::rethrow_exception(e);  // as upstream's sequential loop would have surfaced it
}

// ---- Framework (UP framework/runtime/framework.go) -----------------------------------------
Framework::Framework(const Profile &p, const Registry &r, Handle *h) : name_(p.scheduler_name) {
    std::map<std::string, std::shared_ptr<Plugin>> inst;  // one instance per plugin per profile
    auto get = [&](const std::string &n) {
        auto it = inst.find(n);
        if (it != inst.end()) return it->second;
        auto f = r.find(n);
        if (f == r.end()) throw std::invalid_argument("profile " + name_ + ": plugin " + n + " not registered");
        return inst[n] = f->second(h);
    };
    auto as = [&](const std::string &n, auto *tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        auto q = std::dynamic_pointer_cast<T>(get(n));
        if (!q) throw std::invalid_argument("plugin " + n + " does not implement the requested extension point");
        return q;
    };
    if (!p.queue_sort.empty()) queue_sort_ = as(p.queue_sort, (QueueSortPlugin *)nullptr);
    for (const auto &x : p.pre_filter) pre_filter_.push_back(as(x.name, (PreFilterPlugin *)nullptr));
    for (const auto &x : p.filter) filter_.push_back(as(x.name, (FilterPlugin *)nullptr));
    for (const auto &x : p.score) score_.emplace_back(as(x.name, (ScorePlugin *)nullptr), x.weight);
    for (const auto &x : p.reserve) reserve_.push_back(as(x.name, (ReservePlugin *)nullptr));
}

std::pair<PreFilterResult, Status> Framework::RunPreFilterPlugins(CycleState &s, const Pod &p) {
    PreFilterResult merged;
    for (auto &pl : pre_filter_) {
        auto [r, st] = pl->PreFilter(s, p);
        if (st.IsSkip()) continue;
        if (!st.IsSuccess()) return {merged, st.WithPlugin(pl->Name())};
        if (!r.all_nodes) {  // intersect (UP PreFilterResult.Merge)
            if (merged.all_nodes) {
                merged = r;
            } else {
                std::set<std::string> in;
                for (const auto &n : r.node_names)
                    if (merged.node_names.count(n)) in.insert(n);
                merged.node_names = in;
            }
        }
    }
    return {merged, Status::OK()};
}

Status Framework::RunFilterPlugins(CycleState &s, const Pod &p, const NodeInfo &n) {
    for (auto &pl : filter_) {
        Status st = pl->Filter(s, p, n);
        if (!st.IsSuccess()) return st.WithPlugin(pl->Name());
    }
    return Status::OK();
}

std::pair<std::vector<int64_t>, Status> Framework::RunScorePlugins(
    CycleState &s, const Pod &p, const std::vector<const NodeInfo *> &nodes, Parallelizer *par) {
    const size_t nn = nodes.size(), np = score_.size();
    std::vector<int64_t> total(nn, 0);
    lists_.resize(np);
    for (auto &l : lists_) l.resize(nn);
    // every score plugin per node, the nodes in parallel (UP prioritizeNodes -> RunScorePlugins);
    // the first failing (plugin, node) in node order is reported
    std::vector<Status> bad(nn);
    std::atomic<bool> any_bad{false};
    auto one = [&](int i) {
        for (size_t k = 0; k < np; ++k) {
            auto [v, st] = score_[k].first->Score(s, p, nodes[i]->node.name);
            if (!st.IsSuccess()) {
                bad[i] = st.WithPlugin(score_[k].first->Name());
                any_bad.store(true, std::memory_order_relaxed);
                return;
            }
            lists_[k][i] = {nodes[i]->node.name, v};
        }
    };
    if (par) par->Until((int)nn, one);
    else for (size_t i = 0; i < nn; ++i) one((int)i);
    if (any_bad.load())
        for (size_t i = 0; i < nn; ++i)
            if (!bad[i].IsSuccess()) return {total, bad[i]};
    for (size_t k = 0; k < np; ++k) {
        auto &[pl, w] = score_[k];
        NodeScoreList &list = lists_[k];
        if (pl->HasScoreExtensions()) {
            Status st = pl->NormalizeScore(s, p, list);
            if (!st.IsSuccess()) return {total, st.WithPlugin(pl->Name())};
        }
        for (size_t i = 0; i < nn; ++i) {
            if (list[i].score > MaxNodeScore || list[i].score < MinNodeScore)
                return {total, Status::AsError("plugin " + pl->Name() + " returns an invalid score " +
                                               std::to_string(list[i].score) + ", it should in the range of [0, 100] after normalizing")};
            total[i] += list[i].score * w;
        }
    }
    return {total, Status::OK()};
}

Status Framework::RunReservePluginsReserve(CycleState &s, const Pod &p, const std::string &node) {
    for (auto &pl : reserve_) {
        Status st = pl->Reserve(s, p, node);
        if (!st.IsSuccess()) return st.WithPlugin(pl->Name());
    }
    return Status::OK();
}

void Framework::RunReservePluginsUnreserve(CycleState &s, const Pod &p, const std::string &node) {
    for (auto it = reserve_.rbegin(); it != reserve_.rend(); ++it) (*it)->Unreserve(s, p, node);  // reverse order
}

// ---- Scheduler (UP schedule_one.go) ----------------------------------------------------------
Scheduler::Scheduler(const Registry &registry, const std::vector<Profile> &profiles,
                     std::function<std::string(const Pod &, const PodResources &)> profile_of, int parallelism)
    : registry_(registry), profile_of_(std::move(profile_of)) {
    if (parallelism > 1) par_ = std::make_unique<Parallelizer>(parallelism);
    if (profiles.empty()) throw std::invalid_argument("at least one profile");
    for (const auto &p : profiles) fw_[p.scheduler_name] = std::make_unique<Framework>(p, registry_, this);
    if (!profile_of_) {
        const std::string first = profiles.front().scheduler_name;
        profile_of_ = [first](const Pod &, const PodResources &) { return first; };
    }
}

void Scheduler::AddNode(const Node &n) {
    if (index_.count(n.name)) throw std::invalid_argument("node " + n.name + " already exists");
    index_[n.name] = (int)nodes_.size();
    nodes_.push_back(NewNodeInfo(n));
    for (const auto &kv : nodes_.back().allocatable.scalar)
        if (std::find(ext_names_.begin(), ext_names_.end(), kv.first) == ext_names_.end()) {
            if (ext_names_.size() >= QS_MAX_EXT)
                throw std::invalid_argument("more than 2 extended resource names in the cluster");
            ext_names_.push_back(kv.first);
        }
}

void Scheduler::UpdateNode(const Node &n) {
    const int i = NodeIndex(n.name);
    if (i < 0) throw std::invalid_argument("node " + n.name + " not found");
    NodeInfo ni = NewNodeInfo(n);
    ni.requested = nodes_[i].requested;
    ni.non_zero_requested = nodes_[i].non_zero_requested;
    ni.pods = nodes_[i].pods;
    ni.pod_names = nodes_[i].pod_names;
    ni.generation = nodes_[i].generation + 1;
    nodes_[i] = ni;
}

int Scheduler::NodeIndex(const std::string &name) const {
    auto it = index_.find(name);
    return it == index_.end() ? -1 : it->second;
}

void Scheduler::AddPod(const Pod &p) {
    QueuedPodInfo q;
    q.pod = p;
    q.res = ComputePodResources(p, ext_names_);
    q.arrival = arrivals_++;
    queue_.push_back(std::move(q));
}

std::vector<ScheduleResult> Scheduler::Run() {
    const QueueSortPlugin *qs = fw_.begin()->second->QueueSort();
    std::vector<QueuedPodInfo> q;
    q.swap(queue_);
    if (qs) std::stable_sort(q.begin(), q.end(), [qs](const QueuedPodInfo &a, const QueuedPodInfo &b) { return qs->Less(a, b); });
    std::vector<ScheduleResult> out;
    out.reserve(q.size());
    for (auto &p : q) out.push_back(ScheduleOne(p));
    return out;
}

ScheduleResult Scheduler::ScheduleOne(const QueuedPodInfo &qp) {
    ScheduleResult res;
    res.pod = qp.pod.ns + "/" + qp.pod.name;
    res.arrival = qp.arrival;
    res.profile = profile_of_(qp.pod, qp.res);
    auto fit = fw_.find(res.profile);
    if (fit == fw_.end()) {
        res.status = Status::AsError("profile " + res.profile + " not found");
        return res;
    }
    Framework &fw = *fit->second;
    CycleState state;
    state.Write(kPodResourcesKey, std::make_shared<PodResourcesState>(qp.res));
    // findNodesThatFitPod
    auto [pfr, st] = fw.RunPreFilterPlugins(state, qp.pod);
    if (!st.IsSuccess()) {
        res.status = st;
        return res;
    }
    std::vector<const NodeInfo *> feasible;
    std::vector<int> feasible_ix;
    std::map<std::string, int> reasons;
    // findNodesThatPassFilters: the Filter plugins of every node, the nodes in parallel; the
    // results are then taken in node order (feasible list, reason counts, first error)
    const int nn = (int)nodes_.size();
    fstat_.assign(nn, Status::OK());
    std::vector<uint8_t> skip(nn, 0);
    for (int i = 0; i < nn; ++i)
        skip[i] = !pfr.all_nodes && !pfr.node_names.count(nodes_[i].node.name);
    auto filter_one = [&](int i) {
        if (!skip[i]) fstat_[i] = fw.RunFilterPlugins(state, qp.pod, nodes_[i]);
    };
    if (par_) par_->Until(nn, filter_one);
    else for (int i = 0; i < nn; ++i) filter_one(i);
    for (size_t i = 0; i < nodes_.size(); ++i) {
        if (skip[i]) {
            ++reasons["node(s) didn't satisfy plugin(s) [" + st.Plugin() + "]"];
            continue;
        }
        ++res.evaluated_nodes;
        const Status &fs = fstat_[i];
        if (fs.IsSuccess()) {
            feasible.push_back(&nodes_[i]);
            feasible_ix.push_back((int)i);
        } else if (fs.IsRejected()) {
            for (const auto &r : fs.Reasons()) ++reasons[r];
        } else {
            res.status = fs;
            return res;
        }
    }
    res.feasible_nodes = (int)feasible.size();
    if (feasible.empty()) {
        res.status = Status(Code::Unschedulable, {FitErrorMessage((int)nodes_.size(), reasons)});
        return res;
    }
    int pick = 0;
    if (feasible.size() > 1) {  // prioritizeNodes + deterministic selectHost (spec S7)
        auto [total, sst] = fw.RunScorePlugins(state, qp.pod, feasible, par_.get());
        if (!sst.IsSuccess()) {
            res.status = sst;
            return res;
        }
        for (size_t i = 1; i < total.size(); ++i)
            if (total[i] > total[pick]) pick = (int)i;  // ties keep the lower node index
    }
    const int ix = feasible_ix[pick];
    // assume, then Reserve (Unreserve + forget on failure)
    nodes_[ix].AddPod(qp.pod, qp.res);
    Status rs = fw.RunReservePluginsReserve(state, qp.pod, nodes_[ix].node.name);
    if (!rs.IsSuccess()) {
        fw.RunReservePluginsUnreserve(state, qp.pod, nodes_[ix].node.name);
        nodes_[ix].RemovePod(qp.pod, qp.res);
        res.status = rs;
        return res;
    }
    res.node_index = ix;
    res.suggested_host = nodes_[ix].node.name;
    return res;
}

std::string FitErrorMessage(int num_nodes, const std::map<std::string, int> &reason_counts) {
    std::vector<std::string> rs;
    for (const auto &kv : reason_counts) rs.push_back(std::to_string(kv.second) + " " + kv.first);
    std::sort(rs.begin(), rs.end());
    std::string m = "0/" + std::to_string(num_nodes) + " nodes are available:";
    if (!rs.empty()) {
        m += " ";
        for (size_t i = 0; i < rs.size(); ++i) m += (i ? ", " : "") + rs[i];
        m += ".";
    }
    return m;
}

}  // namespace qsfw
