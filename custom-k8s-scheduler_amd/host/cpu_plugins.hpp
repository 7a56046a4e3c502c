// cpu_plugins.hpp — the CPU reference plugin set: the north_star's "CPU reference plugin
// (NodeResourcesFit + LeastAllocated + QoS weight) ... which serves as the baseline"
// (BASELINE.json:5, configs[0] :7).  The north_star names Go; no Go toolchain exists here or on the
// GPU box, so the plugins are C++ over the same framework runtime (framework.hpp:
// Registry, per-QoS profiles, Run*Plugins with upstream's 16-worker node Parallelizer, the
// deterministic selectHost), evaluated on k8s objects (NodeInfo / Pod: resource lists, label maps,
// taint lists), one (pod, node) at a time, as upstream's plugins are:
//   NodeResourcesFit                  PreFilter / Filter (UP noderesources/fit.go#{PreFilter,Filter,
//                                     fitsRequest}) and Score with the LeastAllocated strategy
//                                     (UP noderesources/least_allocated.go#leastResourceScorer over
//                                     NonZeroRequested, resource_allocation.go#score)
//   NodeResourcesBalancedAllocation   Score (UP noderesources/balanced_allocation.go#
//                                     balancedResourceScorer over Requested, float64)
//   TaintToleration                   Filter / Score / NormalizeScore reverse (UP tainttoleration/
//                                     taint_toleration.go)
//   NodeAffinity                      Filter / Score / NormalizeScore (UP nodeaffinity/node_affinity.go)
//   QoSSort                           queue sort of spec S8
// The QoS-class weight is the profile's plugin weights (one profile per QoS class, spec S9), as for
// the device-backed QoSGPU plugins (qos_gpu.hpp).  Placements are spec S7's, bit-exact with the
// oracle and the GPU paths (tests/native/test_framework.cpp --cpu, tools/cpu_framework.cpp).
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "../../include/qsched.h"
#include "framework.hpp"

namespace qsfw {

inline const char *kNodeResourcesFit = "NodeResourcesFit";
inline const char *kNodeResourcesBalancedAllocation = "NodeResourcesBalancedAllocation";
inline const char *kTaintToleration = "TaintToleration";
inline const char *kNodeAffinity = "NodeAffinity";
inline const char *kCPUQoSSort = "QoSSort";

// cfg: the scoring-resource lists (fit_resources / balanced_resources, or fit_weight_cpu / _mem and
// [cpu, memory]; extended resource k = the handle's ExtendedResourceNames()[k]), balanced_skip_besteffort.
Registry CPURegistry(const qs_config &cfg);
// One profile per QoS class ("besteffort", "burstable", "guaranteed"): NodeResourcesFit weight
// w_fit[q], NodeResourcesBalancedAllocation w_bal[q], TaintToleration w_taint / NodeAffinity
// w_affinity when enabled.
std::vector<Profile> CPUProfiles(const qs_config &cfg);
std::string CPUProfileOf(const Pod &, const PodResources &r);

}  // namespace qsfw
