// qos_gpu.hpp — the QoS scheduling plugins over libqsched (include/qsched.h): the C++ form of the
// north_star's Go framework plugin (BASELINE.json:5; INTEGRATION.md shows the cgo version).
//
//   QoSGPU            PreFilter: sync the device node table with the snapshot (NodeInfo
//                     Generation diff -> qs_node_upsert; full qs_nodes_load when nodes were added
//                     or the requirement dictionary grew), then ONE qs_score_pod call evaluates
//                     NodeResourcesFit + TaintToleration + NodeAffinity filters and the four
//                     normalized scores for every node.  Filter: a lookup (FitError reasons are
//                     derived on the host only for the nodes the device rejected).
//                     Reserve / Unreserve: qs_reserve / qs_unreserve.
//   QoSGPULeastAllocated, QoSGPUBalancedAllocation, QoSGPUTaintToleration, QoSGPUNodeAffinity
//                     Score plugins returning the device's normalized [0,100] components, so a
//                     profile's plugin weights realise spec S6's weighted total (per-QoS weights
//                     of S9 come from one profile per QoS class).
//   QoSSort           QueueSort: QoS class desc, priority desc, arrival asc (spec S8).
// All plugin instances of all profiles share one GpuBackend (one device node table), the role of
// upstream's shared scheduler cache.
#pragma once
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/qsched.h"
#include "framework.hpp"
#include "intern.hpp"

namespace qsfw {

// Per-cycle device results (CycleState key "QoSGPU").
// One word per node as qs_score_pod_packed returns it (0xFFFFFFFF = infeasible, else the four plugin
// scores as bytes): 4 bytes per node copied out of the library's pinned buffer per cycle, and the
// per-node Filter / Score lookups decode their node's word.
struct QoSGPUCycle : StateData {
    qs_pod rec{};
    std::vector<uint32_t> packed;
    int32_t best = -1;            // spec S7 choice of the library config
    bool feasible(size_t i) const { return packed[i] != 0xFFFFFFFFu; }
    // k: 0 LeastAllocated, 1 Balanced, 2 TaintToleration, 3 NodeAffinity (0 where infeasible)
    int32_t score(size_t i, int k) const { return feasible(i) ? (int32_t)((packed[i] >> (8 * k)) & 255u) : 0; }
};

class GpuBackend {
   public:
    // cfg: taint/affinity plugin switches and weights for the library's own `total`/`best`.
    // Throws std::runtime_error when libqsched cannot open the device (no CPU fallback).
    GpuBackend(const qs_config &cfg, int device = 0);
    ~GpuBackend();
    GpuBackend(const GpuBackend &) = delete;
    GpuBackend &operator=(const GpuBackend &) = delete;

    // PreFilter: pod record (spec S2/S3 + interned masks), table sync, qs_score_pod.
    Status Evaluate(const Handle &h, const Pod &pod, const PodResources &res, QoSGPUCycle *out);
    Status Reserve(const Handle &h, int row, const qs_pod &rec);
    Status Unreserve(const Handle &h, int row, const qs_pod &rec);

    const qs_config &config() const { return cfg_; }
    Interner &interner() { return intern_; }
    qs_ctx *ctx() const { return ctx_; }
    uint64_t full_loads() const { return full_loads_; }
    uint64_t row_upserts() const { return row_upserts_; }

   private:
    Status sync(const Handle &h);
    Status load_all(const Handle &h);
    void node_row(const Handle &h, const NodeInfo &ni, qs_node_row *row);
    std::string err(const char *what) const;

    qs_config cfg_{};
    qs_ctx *ctx_ = nullptr;
    Interner intern_;
    std::vector<int64_t> gen_;       // NodeInfo.Generation mirrored per device row
    uint64_t label_gen_ = ~0ull;     // requirement dictionary generation of the device label bits
    uint64_t full_loads_ = 0, row_upserts_ = 0;
    std::mutex mu_;                  // Unreserve may come from another thread (binding cycle)
};

// Plugin names (registry keys)
inline const char *kQoSGPU = "QoSGPU";
inline const char *kQoSGPULeastAllocated = "QoSGPULeastAllocated";
inline const char *kQoSGPUBalancedAllocation = "QoSGPUBalancedAllocation";
inline const char *kQoSGPUTaintToleration = "QoSGPUTaintToleration";
inline const char *kQoSGPUNodeAffinity = "QoSGPUNodeAffinity";
inline const char *kQoSSort = "QoSSort";

// Registry with the QoS plugins bound to one backend (UP app.WithPlugin(name, factory)).
Registry QoSRegistry(std::shared_ptr<GpuBackend> backend);
// One profile per QoS class ("besteffort", "burstable", "guaranteed") with spec S9's weights taken
// from `cfg` (w_fit[q], w_bal[q], w_taint, w_affinity; taint/affinity plugins only when enabled).
std::vector<Profile> QoSProfiles(const qs_config &cfg);
// profile_of for the Scheduler: the pod's QoS class picks its profile.
std::string QoSProfileOf(const Pod &p, const PodResources &r);

}  // namespace qsfw
