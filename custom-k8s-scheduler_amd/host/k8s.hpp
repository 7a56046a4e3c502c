// k8s.hpp — the slice of core/v1 the scheduling path reads, plus resource.Quantity parsing and
// the test wrappers (MakePod / MakeNode) upstream's plugin tests are written with.
//
// This is the host side above the C ABI (include/qsched.h) for a C++ embedding: the north_star's
// Go plugin cannot be built here (no Go toolchain), so the framework surface it
// would sit behind is mirrored in C++ with upstream's names and argument meaning:
//   UP k8s.io/api/core/v1 {Pod, Container, Node, Taint, Toleration, NodeSelectorRequirement,
//   NodeSelectorTerm, PreferredSchedulingTerm}, UP k8s.io/apimachinery/pkg/api/resource#Quantity,
//   UP pkg/scheduler/testing/wrappers.go#{MakePod, MakeNode}.
#pragma once
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace qsfw {

// resource names (UP core/v1/types.go#ResourceCPU, ResourceMemory, ResourcePods)
inline const char *kCPU = "cpu";
inline const char *kMemory = "memory";
inline const char *kPods = "pods";

// Taint effects / toleration operators / node-selector operators (UP core/v1/types.go)
inline const char *kNoSchedule = "NoSchedule";
inline const char *kPreferNoSchedule = "PreferNoSchedule";
inline const char *kNoExecute = "NoExecute";

struct QuantityError : std::invalid_argument {
    using std::invalid_argument::invalid_argument;
};

// resource.Quantity parsed to an exact integer scaled by 10^-3 ("milli units"): "500m" -> 500,
// "2" -> 2000, "1.5" -> 1500, "2Gi" -> 2*2^30*1000, "1e3" -> 10^6.  Throws QuantityError on
// malformed input or a value not representable in int64 milli units.
int64_t parse_quantity_milli(const std::string &s);
// Quantity.MilliValue() (cpu) and Quantity.Value() (memory, counts: rounds up like upstream).
inline int64_t milli_value(const std::string &s) { return parse_quantity_milli(s); }
int64_t value(const std::string &s);

using ResourceList = std::map<std::string, std::string>;  // name -> Quantity string

struct Container {
    std::string name;
    ResourceList requests, limits;
    bool restartable = false;  // init container with restartPolicy Always (sidecar)
};

struct Toleration {
    std::string key, op = "Equal", value, effect;  // op: "Equal" | "Exists"
};

struct Taint {
    std::string key, value, effect;
};

struct NodeSelectorRequirement {
    std::string key, op;  // In | NotIn | Exists | DoesNotExist | Gt | Lt
    std::vector<std::string> values;
};

struct NodeSelectorTerm {
    std::vector<NodeSelectorRequirement> match_expressions;
};

struct PreferredSchedulingTerm {
    int32_t weight = 0;  // 1..100
    NodeSelectorTerm preference;
};

struct Pod {
    std::string name, ns = "default", uid;
    std::vector<Container> containers, init_containers;
    ResourceList overhead;
    int32_t priority = 0;
    std::vector<Toleration> tolerations;
    std::map<std::string, std::string> node_selector;
    std::vector<NodeSelectorTerm> required_terms;          // requiredDuringScheduling...
    std::vector<PreferredSchedulingTerm> preferred_terms;  // preferredDuringScheduling...
};

struct Node {
    std::string name;
    ResourceList allocatable;
    std::map<std::string, std::string> labels;
    std::vector<Taint> taints;
};

// ---- test wrappers (UP pkg/scheduler/testing/wrappers.go) ----------------------------------
class PodWrapper {
   public:
    explicit PodWrapper(std::string name) { p_.name = std::move(name); p_.uid = p_.name; }
    // one more regular container with these requests (MakePod().Req(...))
    PodWrapper &Req(const ResourceList &r) { p_.containers.push_back({"c" + std::to_string(p_.containers.size()), r, {}, false}); return *this; }
    // requests == limits container (Guaranteed when cpu and memory are both set)
    PodWrapper &ReqLim(const ResourceList &r, const ResourceList &l) { p_.containers.push_back({"c" + std::to_string(p_.containers.size()), r, l, false}); return *this; }
    PodWrapper &InitReq(const ResourceList &r) { p_.init_containers.push_back({"i" + std::to_string(p_.init_containers.size()), r, {}, false}); return *this; }
    PodWrapper &SidecarReq(const ResourceList &r) { p_.init_containers.push_back({"s" + std::to_string(p_.init_containers.size()), r, {}, true}); return *this; }
    PodWrapper &Overhead(const ResourceList &r) { p_.overhead = r; return *this; }
    PodWrapper &Priority(int32_t v) { p_.priority = v; return *this; }
    PodWrapper &Toleration(const std::string &key, const std::string &op, const std::string &value, const std::string &effect) { p_.tolerations.push_back({key, op, value, effect}); return *this; }
    PodWrapper &NodeSelector(const std::map<std::string, std::string> &m) { p_.node_selector = m; return *this; }
    PodWrapper &NodeAffinityIn(const std::string &key, const std::vector<std::string> &vals) { p_.required_terms.push_back({{{key, "In", vals}}}); return *this; }
    PodWrapper &RequiredTerm(const NodeSelectorTerm &t) { p_.required_terms.push_back(t); return *this; }
    PodWrapper &PreferredTerm(int32_t w, const NodeSelectorTerm &t) { p_.preferred_terms.push_back({w, t}); return *this; }
    Pod Obj() const { return p_; }

   private:
    Pod p_;
};
inline PodWrapper MakePod(const std::string &name = "pod") { return PodWrapper(name); }

class NodeWrapper {
   public:
    explicit NodeWrapper(std::string name) { n_.name = std::move(name); }
    NodeWrapper &Capacity(const ResourceList &r) { n_.allocatable = r; return *this; }
    NodeWrapper &Label(const std::string &k, const std::string &v) { n_.labels[k] = v; return *this; }
    NodeWrapper &Taint(const std::string &k, const std::string &v, const std::string &effect) { n_.taints.push_back({k, v, effect}); return *this; }
    Node Obj() const { return n_; }

   private:
    Node n_;
};
inline NodeWrapper MakeNode(const std::string &name = "node") { return NodeWrapper(name); }

}  // namespace qsfw
