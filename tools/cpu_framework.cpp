// cpu_framework.cpp — the north_star's CPU reference-plugin baseline (BASELINE.json:5, configs[0]
// :7) timed on this host: spec/synth.md's cluster as k8s objects (tools/synth_objects.hpp) through
// the framework runtime (framework.hpp: per-QoS profiles, QoSSort, RunFilterPlugins /
// RunScorePlugins over the nodes with upstream's Parallelizer, deterministic selectHost, assume)
// with the CPU plugins of host/cpu_plugins.hpp (NodeResourcesFit + LeastAllocated,
// BalancedAllocation, QoS-class weights; TaintToleration / NodeAffinity for config 4).  Go is
// absent here, so this C++ plugin set is the stand-in.  The placements of the pods scheduled are
// diffed against the CPU oracle on the same pods (oracle/liboracle.so, test infrastructure).
//
//   cpu_framework <config 2|4> <nodes> <pods> <threads>  ->  one JSON line
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../custom-k8s-scheduler_amd/host/cpu_plugins.hpp"
#include "oracle_cfg.hpp"
#include "synth_objects.hpp"
extern "C" {
#include "../oracle/qs_oracle.h"
}

using namespace qsfw;

int main(int argc, char **argv) {
    const int config = argc > 1 ? atoi(argv[1]) : 2;
    const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 5000;
    const uint32_t p = argc > 3 ? (uint32_t)atoi(argv[3]) : 2000;
    const int threads = argc > 4 ? atoi(argv[4]) : 16;
    const uint64_t seed = 0x5EED0000ull + (uint64_t)config;
    std::vector<Node> nodes;
    std::vector<Pod> pods;
    synth_objects(config, seed, n, p, &nodes, &pods);
    qs_config cfg;
    qs_config_default(&cfg);
    cfg.enable_taint = cfg.enable_affinity = config == 4 ? 1 : 0;
    Scheduler sched(CPURegistry(cfg), CPUProfiles(cfg), CPUProfileOf, threads);
    for (const auto &x : nodes) sched.AddNode(x);
    for (const auto &x : pods) sched.AddPod(x);
    const auto t0 = std::chrono::steady_clock::now();
    const auto res = sched.Run();
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<int32_t> loop(p, -2);
    int errors = 0;
    for (const auto &r : res) {
        loop[r.arrival] = r.node_index;
        errors += r.status.code() == Code::Error;
    }

    // the oracle on the generator's arrays of the same cluster and pods (QoS-sorted the same way)
    std::vector<int64_t> o[10];
    for (auto &v : o) v.assign(n, 0);
    std::vector<int64_t> oae(2 * (size_t)n), ore(2 * (size_t)n);
    std::vector<uint64_t> oth(n), ots(n), olb(2 * (size_t)n);
    std::vector<int32_t> ozone(n);
    or_nodes on{n, o[0].data(), o[1].data(), oae.data(), o[2].data(), o[3].data(), o[4].data(), ore.data(),
                o[5].data(), o[6].data(), o[7].data(), oth.data(), ots.data(), olb.data(), ozone.data()};
    std::vector<int64_t> prc(p), prm(p), pre(2 * (size_t)p), pzc(p), pzm(p);
    std::vector<int32_t> pq(p), ppr(p), pnr(p), pnp(p), ppw(4 * (size_t)p), papp(p), paa(p);
    std::vector<uint64_t> pth(p), pts(p), psel(2 * (size_t)p), prt(8 * (size_t)p), ppt(8 * (size_t)p);
    or_pods op{p, prc.data(), prm.data(), pre.data(), pzc.data(), pzm.data(), pq.data(), ppr.data(), pth.data(),
               pts.data(), psel.data(), pnr.data(), pnp.data(), prt.data(), ppt.data(), ppw.data(), papp.data(),
               paa.data()};
    or_generate(config, seed, &on, &op);
    or_config oc = oracle_cfg(cfg);
    oc.qos_sort = 1;
    std::vector<int32_t> ref(p);
    or_schedule(&oc, &on, &op, ref.data(), nullptr, nullptr, 16);
    int diff = 0, unsched = 0;
    for (uint32_t j = 0; j < p; ++j) {
        diff += loop[j] != ref[j];
        unsched += loop[j] < 0;
    }
    std::printf("{\"config\": %d, \"nodes\": %u, \"pods\": %u, \"threads\": %d, \"seconds\": %.3f, "
                "\"pods_per_s\": %.1f, \"evals_per_s\": %.1f, \"unschedulable\": %d, \"errors\": %d, "
                "\"placements_match\": %s}\n",
                config, n, p, threads, secs, p / secs, (double)p * n / secs, unsched, errors, diff == 0 ? "true" : "false");
    return diff == 0 && errors == 0 ? 0 : 1;
}
