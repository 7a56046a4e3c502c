// oracle_cfg.hpp — the CPU oracle's configuration (oracle/qs_oracle.h) of a qs_config: plugin
// weights, profile flags and the scoring-resource lists.  Test / baseline tooling only.
#pragma once
#include "../include/qsched.h"
extern "C" {
#include "../oracle/qs_oracle.h"
}

inline or_config oracle_cfg(const qs_config &c) {
    or_config o{};
    o.wc = c.fit_weight_cpu;
    o.wm = c.fit_weight_mem;
    for (int q = 0; q < 3; ++q) {
        o.w_fit[q] = c.w_fit[q];
        o.w_bal[q] = c.w_bal[q];
    }
    o.w_tt = c.w_taint;
    o.w_na = c.w_affinity;
    o.enable_taint = c.enable_taint;
    o.enable_affinity = c.enable_affinity;
    o.balanced_skip_besteffort = c.balanced_skip_besteffort;
    o.qos_sort = c.qos_sort;
    o.n_fit_res = c.n_fit_resources;
    for (int i = 0; i < c.n_fit_resources; ++i) {
        o.fit_res[i] = c.fit_resources[i].resource;
        o.fit_w[i] = c.fit_resources[i].weight;
    }
    o.n_bal_res = c.n_balanced_resources;
    for (int i = 0; i < c.n_balanced_resources; ++i) o.bal_res[i] = c.balanced_resources[i];
    return o;
}
