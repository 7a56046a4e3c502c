// intern.hpp — host-side interning of taints and node-selector requirements into the bitmasks of
// the device node table (spec/semantics.md S1, S5).
//
// Taints: every distinct (key, value, effect) a node carries gets one of 64 bits.  A node's
// taint_hard holds its NoSchedule / NoExecute taints, taint_soft its PreferNoSchedule taints; a
// pod's tol_hard / tol_soft hold the dictionary taints its tolerations tolerate (UP
// core/v1/toleration.go#ToleratesTaint; the soft set only through tolerations with effect "" or
// PreferNoSchedule, UP tainttoleration/taint_toleration.go#getAllTolerationPreferNoSchedule).
// Requirements: every distinct NodeSelectorRequirement (nodeSelector entries as `key In [v]`)
// gets one of 128 bits, evaluated per node on the host (In, NotIn, Exists, DoesNotExist, Gt, Lt:
// UP component-helpers/scheduling/corev1/nodeaffinity, UP apimachinery labels.Requirement), so
// the device only tests subset relations.  An empty term matches no node upstream; it maps to a
// reserved bit no node carries.
#pragma once
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/qsched.h"
#include "k8s.hpp"

namespace qsfw {

struct DictionaryFull : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// UP core/v1/toleration.go#ToleratesTaint
bool tolerates(const Toleration &t, const Taint &taint);
// UP labels.Requirement.Matches restricted to node-selector operators; invalid requirements
// (e.g. In with no values, Gt with a non-integer) match nothing
bool requirement_matches(const NodeSelectorRequirement &r, const std::map<std::string, std::string> &labels);

class Interner {
   public:
    static constexpr int kMaxTaints = 64;
    static constexpr int kMaxRequirements = 128;
    static constexpr int kNeverBit = 127;  // reserved: carried by no node (empty terms)

    // Bit of a taint / requirement, interned on first sight.  Throws DictionaryFull.
    int taint_bit(const Taint &t);
    int requirement_bit(const NodeSelectorRequirement &r);

    // Node masks against the current dictionaries (interns the node's taints).
    void node_masks(const Node &n, uint64_t *taint_hard, uint64_t *taint_soft, uint64_t label_bits[2]);
    // Label bits only (every interned requirement evaluated on the node's labels).
    void label_bits(const Node &n, uint64_t out[2]) const;
    // Pod masks: tol_hard/tol_soft over the interned taints, nodeSelector / required / preferred
    // terms as requirement bits (interning new requirements).  Throws DictionaryFull, or
    // std::invalid_argument for more than QS_MAX_TERMS terms or a preferred weight outside 0..100.
    void pod_masks(const Pod &p, qs_pod *out);

    // Bumped whenever a requirement is interned: every node's label_bits must be recomputed.
    uint64_t requirement_generation() const { return req_gen_; }
    int n_taints() const { return (int)taints_.size(); }
    int n_requirements() const { return (int)reqs_.size(); }

   private:
    std::map<std::string, int> taint_ix_, req_ix_;
    std::vector<Taint> taints_;
    std::vector<NodeSelectorRequirement> reqs_;
    uint64_t req_gen_ = 0;
    uint64_t term_mask(const NodeSelectorTerm &t, uint64_t out[2]);
};

}  // namespace qsfw
