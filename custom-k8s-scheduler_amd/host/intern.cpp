// intern.cpp — taint / requirement dictionaries and the node / pod bitmasks (see intern.hpp).
#include "intern.hpp"

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>

namespace qsfw {
namespace {

void set_bit(uint64_t m[2], int b) { m[b >> 6] |= 1ULL << (b & 63); }

bool parse_int64(const std::string &s, int64_t *v) {
    if (s.empty()) return false;
    errno = 0;
    char *end = nullptr;
    const long long x = std::strtoll(s.c_str(), &end, 10);
    if (errno != 0 || end != s.c_str() + s.size()) return false;
    *v = (int64_t)x;
    return true;
}

bool is_hard(const std::string &effect) { return effect == kNoSchedule || effect == kNoExecute; }

}  // namespace

bool tolerates(const Toleration &t, const Taint &taint) {
    if (!t.effect.empty() && t.effect != taint.effect) return false;
    if (!t.key.empty() && t.key != taint.key) return false;
    if (t.op.empty() || t.op == "Equal") return t.value == taint.value;
    if (t.op == "Exists") return true;
    return false;
}

bool requirement_matches(const NodeSelectorRequirement &r, const std::map<std::string, std::string> &labels) {
    const auto it = labels.find(r.key);
    const bool has = it != labels.end();
    if (r.op == "In" || r.op == "NotIn") {
        if (r.values.empty()) return false;  // invalid selector
        const bool in = has && std::find(r.values.begin(), r.values.end(), it->second) != r.values.end();
        return r.op == "In" ? in : !in;
    }
    if (r.op == "Exists") return r.values.empty() && has;
    if (r.op == "DoesNotExist") return r.values.empty() && !has;
    if (r.op == "Gt" || r.op == "Lt") {
        int64_t want = 0, got = 0;
        if (r.values.size() != 1 || !parse_int64(r.values[0], &want)) return false;
        if (!has || !parse_int64(it->second, &got)) return false;
        return r.op == "Gt" ? got > want : got < want;
    }
    return false;
}

int Interner::taint_bit(const Taint &t) {
    const std::string k = t.key + '\x1f' + t.value + '\x1f' + t.effect;
    const auto it = taint_ix_.find(k);
    if (it != taint_ix_.end()) return it->second;
    if ((int)taints_.size() >= kMaxTaints)
        throw DictionaryFull("more than 64 distinct taints (key, value, effect) in the cluster");
    const int b = (int)taints_.size();
    taint_ix_[k] = b;
    taints_.push_back(t);
    return b;
}

int Interner::requirement_bit(const NodeSelectorRequirement &r) {
    std::vector<std::string> vals = r.values;
    if (r.op == "In" || r.op == "NotIn") std::sort(vals.begin(), vals.end());  // set semantics
    std::string k = r.key + '\x1f' + r.op;
    for (const auto &v : vals) k += '\x1f' + v;
    const auto it = req_ix_.find(k);
    if (it != req_ix_.end()) return it->second;
    if ((int)reqs_.size() >= kNeverBit)
        throw DictionaryFull("more than 127 distinct node-selector requirements in the pod stream");
    const int b = (int)reqs_.size();
    req_ix_[k] = b;
    reqs_.push_back({r.key, r.op, vals});
    ++req_gen_;
    return b;
}

void Interner::label_bits(const Node &n, uint64_t out[2]) const {
    out[0] = out[1] = 0;
    for (size_t b = 0; b < reqs_.size(); ++b)
        if (requirement_matches(reqs_[b], n.labels)) set_bit(out, (int)b);
}

void Interner::node_masks(const Node &n, uint64_t *th, uint64_t *ts, uint64_t lb[2]) {
    *th = *ts = 0;
    for (const auto &t : n.taints) {
        const int b = taint_bit(t);
        if (is_hard(t.effect)) *th |= 1ULL << b;
        else if (t.effect == kPreferNoSchedule) *ts |= 1ULL << b;
    }
    label_bits(n, lb);
}

uint64_t Interner::term_mask(const NodeSelectorTerm &t, uint64_t out[2]) {
    out[0] = out[1] = 0;
    if (t.match_expressions.empty()) {  // matches no node (UP nodeaffinity#NewNodeSelector)
        set_bit(out, kNeverBit);
        return 1;
    }
    for (const auto &r : t.match_expressions) set_bit(out, requirement_bit(r));
    return 1;
}

void Interner::pod_masks(const Pod &p, qs_pod *out) {
    out->tol_hard = out->tol_soft = 0;
    std::memset(out->req_terms, 0, sizeof out->req_terms);
    std::memset(out->pref_terms, 0, sizeof out->pref_terms);
    std::memset(out->pref_weight, 0, sizeof out->pref_weight);
    for (size_t b = 0; b < taints_.size(); ++b) {
        const Taint &t = taints_[b];
        for (const auto &tol : p.tolerations) {
            if (!tolerates(tol, t)) continue;
            if (is_hard(t.effect)) out->tol_hard |= 1ULL << b;
            if (t.effect == kPreferNoSchedule && (tol.effect.empty() || tol.effect == kPreferNoSchedule))
                out->tol_soft |= 1ULL << b;
        }
    }
    out->sel[0] = out->sel[1] = 0;
    for (const auto &kv : p.node_selector) set_bit(out->sel, requirement_bit({kv.first, "In", {kv.second}}));
    if (p.required_terms.size() > QS_MAX_TERMS || p.preferred_terms.size() > QS_MAX_TERMS)
        throw std::invalid_argument("pod " + p.name + ": more than 4 node-affinity terms");
    out->n_req_terms = (int32_t)p.required_terms.size();
    for (size_t t = 0; t < p.required_terms.size(); ++t) term_mask(p.required_terms[t], out->req_terms[t]);
    int np = 0;
    for (const auto &pt : p.preferred_terms) {
        if (pt.weight < 0 || pt.weight > 100)
            throw std::invalid_argument("pod " + p.name + ": preferred term weight outside 0..100");
        if (pt.weight == 0) continue;  // UP nodeaffinity#NewPreferredSchedulingTerms skips weight 0
        term_mask(pt.preference, out->pref_terms[np]);
        out->pref_weight[np++] = pt.weight;
    }
    out->n_pref_terms = np;
}

}  // namespace qsfw
