// framework.hpp — the kube-scheduler framework surface the QoS scheduling path sits behind,
// mirrored in C++ with upstream's names and argument meaning (the north_star's Go plugin cannot be
// built here: no Go toolchain).  Sources (upstream v1.32, `UP <path>#<symbol>`):
//   UP pkg/scheduler/framework/interface.go#{Code, Status, PreFilterPlugin, FilterPlugin,
//     ScorePlugin, ScoreExtensions, ReservePlugin, QueueSortPlugin, PreFilterResult, NodeScore}
//   UP pkg/scheduler/framework/cycle_state.go#CycleState
//   UP pkg/scheduler/framework/types.go#{NodeInfo, Resource, QueuedPodInfo, FitError}
//   UP pkg/scheduler/framework/runtime/framework.go#{RunPreFilterPlugins, RunFilterPlugins,
//     RunScorePlugins, RunReservePluginsReserve, RunReservePluginsUnreserve}
//   UP pkg/scheduler/schedule_one.go#{ScheduleOne, schedulePod, findNodesThatFitPod,
//     prioritizeNodes, selectHost, assume}
//   UP cmd/kube-scheduler/app/server.go#WithPlugin, UP framework/runtime/registry.go#Registry
// selectHost is the deterministic one of spec/semantics.md S7 (highest total, ties -> lowest node
// index) instead of upstream's reservoir sampling, so a run is reproducible and bit-exact.
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "k8s.hpp"

namespace qsfw {

// ---- Status (UP framework/interface.go#Code: Success 0 ... Pending 6) ------------------------
enum class Code : int {
    Success = 0,
    Error = 1,
    Unschedulable = 2,
    UnschedulableAndUnresolvable = 3,
    Wait = 4,
    Skip = 5,
    Pending = 6
};

class Status {
   public:
    Status() = default;
    Status(Code c, std::vector<std::string> reasons = {}) : code_(c), reasons_(std::move(reasons)) {}
    static Status OK() { return Status(); }
    static Status AsError(const std::string &msg) { return Status(Code::Error, {msg}); }
    Code code() const { return code_; }
    bool IsSuccess() const { return code_ == Code::Success; }
    bool IsSkip() const { return code_ == Code::Skip; }
    bool IsRejected() const {
        return code_ == Code::Unschedulable || code_ == Code::UnschedulableAndUnresolvable || code_ == Code::Pending;
    }
    const std::vector<std::string> &Reasons() const { return reasons_; }
    std::string Message() const;
    const std::string &Plugin() const { return plugin_; }
    Status &WithPlugin(const std::string &p) { plugin_ = p; return *this; }

   private:
    Code code_ = Code::Success;
    std::vector<std::string> reasons_;
    std::string plugin_;
};

// ---- CycleState (UP framework/cycle_state.go) --------------------------------------------------
struct StateData {
    virtual ~StateData() = default;
};
class CycleState {
   public:
    void Write(const std::string &key, std::shared_ptr<StateData> v) { m_[key] = std::move(v); }
    template <class T>
    T *Read(const std::string &key) const {
        auto it = m_.find(key);
        return it == m_.end() ? nullptr : dynamic_cast<T *>(it->second.get());
    }

   private:
    std::map<std::string, std::shared_ptr<StateData>> m_;
};

// ---- NodeInfo / Resource (UP framework/types.go) ----------------------------------------------
struct Resource {
    int64_t milli_cpu = 0, memory = 0, allowed_pod_number = 0;
    std::map<std::string, int64_t> scalar;  // extended resources (e.g. amd.com/gpu)
};

// A pod's effective requests (spec S2, through qs_pod_from_containers) and QoS class (S3).
struct PodResources {
    int64_t cpu = 0, mem = 0, nz_cpu = 0, nz_mem = 0;
    std::map<std::string, int64_t> scalar;
    int qos = 0;  // qs_qos
};
PodResources ComputePodResources(const Pod &p);
// ext_names: the cluster's extended resource names in table-slot order (<= QS_MAX_EXT)
PodResources ComputePodResources(const Pod &p, const std::vector<std::string> &ext_names);
// The runner computes a pod's resources once and hands them to the plugins in the CycleState
// (the role of NodeResourcesFit's preFilterState upstream).
struct PodResourcesState : StateData {
    explicit PodResourcesState(PodResources r) : res(std::move(r)) {}
    PodResources res;
};
inline const char *kPodResourcesKey = "PodResources";

struct NodeInfo {
    Node node;
    Resource allocatable, requested, non_zero_requested;
    int64_t pods = 0;
    int64_t generation = 0;  // bumped on every change (UP NodeInfo.Generation)
    std::vector<std::string> pod_names;
    void AddPod(const Pod &p, const PodResources &r);
    void RemovePod(const Pod &p, const PodResources &r);
};
NodeInfo NewNodeInfo(const Node &n);

// ---- Parallelizer (UP framework/parallelize/parallelism.go) -----------------------------------
// Until(n, fn) runs fn(i) for i in [0, n) on `workers` threads (the caller is one of them) in chunks
// of chunkSizeFor(n) = min(floor(sqrt(n)), n / workers + 1) indices, as upstream's workqueue-based
// Parallelizer does (DefaultParallelism = 16).  Workers spin briefly for the next section before
// sleeping (a scheduling cycle runs two sections per pod back to back).  workers <= 1: inline.
class Parallelizer {
   public:
    explicit Parallelizer(int workers = 16);
    ~Parallelizer();
    Parallelizer(const Parallelizer &) = delete;
    Parallelizer &operator=(const Parallelizer &) = delete;
    int Workers() const { return workers_; }
    void Until(int n, const std::function<void(int)> &fn);

   private:
    struct Impl;
    int workers_;
    std::unique_ptr<Impl> m_;
};

// ---- plugins (UP framework/interface.go) -------------------------------------------------------
struct PreFilterResult {
    bool all_nodes = true;            // nil NodeNames upstream
    std::set<std::string> node_names;
};
struct NodeScore {
    std::string name;
    int64_t score = 0;
};
using NodeScoreList = std::vector<NodeScore>;
constexpr int64_t MaxNodeScore = 100, MinNodeScore = 0;

struct QueuedPodInfo {
    Pod pod;
    PodResources res;
    int64_t arrival = 0;  // queue insertion order
};

class Handle;

class Plugin {
   public:
    virtual ~Plugin() = default;
    virtual std::string Name() const = 0;
};
class QueueSortPlugin : public virtual Plugin {
   public:
    virtual bool Less(const QueuedPodInfo &a, const QueuedPodInfo &b) const = 0;
};
class PreFilterPlugin : public virtual Plugin {
   public:
    virtual std::pair<PreFilterResult, Status> PreFilter(CycleState &state, const Pod &pod) = 0;
};
class FilterPlugin : public virtual Plugin {
   public:
    virtual Status Filter(CycleState &state, const Pod &pod, const NodeInfo &node) = 0;
};
class ScorePlugin : public virtual Plugin {
   public:
    virtual std::pair<int64_t, Status> Score(CycleState &state, const Pod &pod, const std::string &node) = 0;
    // ScoreExtensions().NormalizeScore; plugins without extensions keep the default (no-op)
    virtual bool HasScoreExtensions() const { return false; }
    virtual Status NormalizeScore(CycleState &, const Pod &, NodeScoreList &) { return Status::OK(); }
};
class ReservePlugin : public virtual Plugin {
   public:
    virtual Status Reserve(CycleState &state, const Pod &pod, const std::string &node) = 0;
    virtual void Unreserve(CycleState &state, const Pod &pod, const std::string &node) = 0;
};

// The snapshot the plugins see (UP framework.Handle#SnapshotSharedLister): NodeInfos in table
// order (index = row of the device node table).
class Handle {
   public:
    virtual ~Handle() = default;
    virtual const std::vector<NodeInfo> &NodeInfos() const = 0;
    virtual int NodeIndex(const std::string &name) const = 0;  // -1 if unknown
    // extended resource names advertised by the nodes, in device-table slot order (<= 2)
    virtual const std::vector<std::string> &ExtendedResourceNames() const = 0;
};

// ---- registry / profile (UP framework/runtime/registry.go, apis/config#KubeSchedulerProfile) --
using PluginFactory = std::function<std::shared_ptr<Plugin>(Handle *)>;
using Registry = std::map<std::string, PluginFactory>;

struct PluginRef {
    std::string name;
    int32_t weight = 1;  // Score plugins only
};
struct Profile {
    std::string scheduler_name;
    std::string queue_sort;
    std::vector<PluginRef> pre_filter, filter, score, reserve;
};

class Framework {
   public:
    Framework(const Profile &p, const Registry &r, Handle *h);
    const std::string &ProfileName() const { return name_; }
    const QueueSortPlugin *QueueSort() const { return queue_sort_.get(); }
    std::pair<PreFilterResult, Status> RunPreFilterPlugins(CycleState &s, const Pod &p);
    Status RunFilterPlugins(CycleState &s, const Pod &p, const NodeInfo &n);
    // weighted totals per feasible node (index-aligned with `nodes`); errors if a plugin returns
    // a score outside [0, 100] after normalization (UP RunScorePlugins)
    // (par: the node-parallel Score pass runs every score plugin per node on it, UP prioritizeNodes)
    std::pair<std::vector<int64_t>, Status> RunScorePlugins(CycleState &s, const Pod &p,
                                                            const std::vector<const NodeInfo *> &nodes,
                                                            Parallelizer *par = nullptr);
    Status RunReservePluginsReserve(CycleState &s, const Pod &p, const std::string &node);
    void RunReservePluginsUnreserve(CycleState &s, const Pod &p, const std::string &node);

   private:
    std::string name_;
    std::shared_ptr<QueueSortPlugin> queue_sort_;
    std::vector<std::shared_ptr<PreFilterPlugin>> pre_filter_;
    std::vector<std::shared_ptr<FilterPlugin>> filter_;
    std::vector<std::pair<std::shared_ptr<ScorePlugin>, int32_t>> score_;
    std::vector<std::shared_ptr<ReservePlugin>> reserve_;
    std::vector<NodeScoreList> lists_;  // per score plugin, reused across cycles
};

// ---- the scheduling loop (UP schedule_one.go) ---------------------------------------------------
struct ScheduleResult {
    std::string pod;             // namespace/name
    int64_t arrival = 0;         // queue insertion order of the pod
    std::string suggested_host;  // empty: unschedulable / error
    int node_index = -1;
    int evaluated_nodes = 0, feasible_nodes = 0;
    Status status;
    std::string profile;
};

class Scheduler : public Handle {
   public:
    // profile_of(pod) picks the profile (upstream: pod.Spec.SchedulerName)
    // parallelism: workers of findNodesThatPassFilters / prioritizeNodes (upstream default 16; 1 runs
    // them inline, as the device-backed QoSGPU plugins want: their Filter / Score are lookups)
    Scheduler(const Registry &registry, const std::vector<Profile> &profiles,
              std::function<std::string(const Pod &, const PodResources &)> profile_of, int parallelism = 1);
    void AddNode(const Node &n);      // appended: its row index is the current node count
    void UpdateNode(const Node &n);   // allocatable / labels / taints changed (Generation bump)
    void AddPod(const Pod &p);        // enqueue
    // Pop every queued pod in QueueSort order (stable) and run ScheduleOne on each.
    std::vector<ScheduleResult> Run();
    ScheduleResult ScheduleOne(const QueuedPodInfo &qp);

    const std::vector<NodeInfo> &NodeInfos() const override { return nodes_; }
    int NodeIndex(const std::string &name) const override;
    const std::vector<std::string> &ExtendedResourceNames() const override { return ext_names_; }

   private:
    Registry registry_;
    std::map<std::string, std::unique_ptr<Framework>> fw_;
    std::function<std::string(const Pod &, const PodResources &)> profile_of_;
    std::vector<NodeInfo> nodes_;
    std::map<std::string, int> index_;
    std::vector<QueuedPodInfo> queue_;
    std::vector<std::string> ext_names_;
    int64_t arrivals_ = 0;
    std::unique_ptr<Parallelizer> par_;
    std::vector<Status> fstat_;  // per-node Filter results of the current cycle
};

// UP framework/types.go#FitError message: "0/N nodes are available: <count> <reason>, ..."
std::string FitErrorMessage(int num_nodes, const std::map<std::string, int> &reason_counts);

}  // namespace qsfw
