// synth_objects.hpp — spec/synth.md's clusters as k8s objects (Node / Pod with resource lists,
// labels, taints, tolerations, affinity terms), for the framework-level tests and the CPU
// reference-plugin baseline (tests/native/test_framework.cpp, tools/cpu_framework.cpp).  Same draws
// as qs_synth_generate / or_generate (G1-G3): configs 1-3 are the node / pod basics, config 4 adds
// amd.com/gpu, taints, zones / pools / disktypes and the pods' tolerations, nodeSelector and
// affinity terms.  Test and bench infrastructure, not part of libqsched.
#pragma once
#include <string>
#include <vector>

#include "../custom-k8s-scheduler_amd/host/k8s.hpp"

namespace qsfw {

inline uint64_t sm_at(uint64_t seed, uint64_t c) {
    uint64_t z = seed + (c + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
inline uint32_t pick(uint64_t seed, uint64_t c, uint32_t k) { return (uint32_t)((sm_at(seed, c) >> 33) % k); }

inline void synth_objects(int config, uint64_t seed, uint32_t n, uint32_t p, std::vector<Node> *nodes,
                          std::vector<Pod> *pods) {
    const bool features = config == 4;
    static const int64_t kNodeCpu[6] = {4000, 8000, 16000, 32000, 64000, 96000}, kMpc[3] = {2, 4, 8};
    static const int64_t kPodCpu[6] = {500, 1000, 1500, 2000, 4000, 8000}, kPodMemMi[7] = {128, 256, 512, 1024, 2048, 4096, 8192};
    static const int64_t kGpu[4] = {1, 2, 4, 8};
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t c = 8ULL * i;
        const int64_t cpu = kNodeCpu[pick(seed, c, 6)], mpc = kMpc[pick(seed, c + 1, 3)];
        auto w = MakeNode("node-" + std::to_string(i));
        ResourceList cap = {{kCPU, std::to_string(cpu) + "m"}, {kMemory, std::to_string(cpu / 1000 * mpc) + "Gi"}, {kPods, "110"}};
        if (!features) {
            nodes->push_back(w.Capacity(cap).Obj());
            continue;
        }
        const bool gpu = pick(seed, c + 2, 10) == 0, maint = pick(seed, c + 3, 20) == 0;
        const int zone = (int)pick(seed, c + 4, 10);
        const char *pool = gpu ? "gpu" : (pick(seed, c + 5, 2) ? "highmem" : "general");
        const bool ssd = pick(seed, c + 6, 2) == 0;
        if (gpu) { cap["amd.com/gpu"] = "8"; w.Taint("gpu", "true", kNoSchedule); }
        if (maint) w.Taint("maint", "true", kPreferNoSchedule);
        w.Capacity(cap).Label("zone", "z" + std::to_string(zone)).Label("pool", pool).Label("disktype", ssd ? "ssd" : "hdd");
        nodes->push_back(w.Obj());
    }
    for (uint32_t j = 0; j < p; ++j) {
        const uint64_t c = 8ULL * n + 16ULL * j;
        const uint32_t qd = pick(seed, c, 10);
        const std::string cpu = std::to_string(kPodCpu[pick(seed, c + 1, 6)]) + "m";
        const int64_t mem_mi = kPodMemMi[pick(seed, c + 2, 7)];
        const std::string mem = std::to_string(mem_mi) + "Mi", mem2 = std::to_string(2 * mem_mi) + "Mi";
        const uint32_t memmode = pick(seed, c + 3, 4), limmode = pick(seed, c + 4, 2);
        const std::string cpu2 = std::to_string(2 * kPodCpu[pick(seed, c + 1, 6)]) + "m";
        ResourceList req, lim;
        if (qd < 2) {
            req = {{kCPU, cpu}, {kMemory, mem}};
            lim = req;
        } else if (qd < 7) {
            req = {{kCPU, cpu}};
            if (memmode != 0) req[kMemory] = mem;
            if (limmode == 1) {
                lim = {{kCPU, cpu2}};
                if (memmode != 0) lim[kMemory] = mem2;
            }
        }
        auto w = MakePod("pod-" + std::to_string(j));
        if (!features) {
            pods->push_back(w.ReqLim(req, lim).Obj());
            continue;
        }
        if (pick(seed, c + 5, 20) == 0) {
            req["amd.com/gpu"] = std::to_string(kGpu[pick(seed, c + 6, 4)]);
            w.Toleration("gpu", "Equal", "true", kNoSchedule).NodeSelector({{"pool", "gpu"}});
        }
        if (pick(seed, c + 7, 5) == 0) {
            const int za = (int)pick(seed, c + 8, 10), zb = (za + 1 + (int)pick(seed, c + 9, 9)) % 10;
            w.NodeAffinityIn("zone", {"z" + std::to_string(za), "z" + std::to_string(zb)});
        }
        if (pick(seed, c + 10, 5) == 0) {
            const uint32_t which = pick(seed, c + 11, 3);
            if (which == 0 || which == 2) w.PreferredTerm(50, {{{"disktype", "In", {"ssd"}}}});
            if (which == 1 || which == 2) w.PreferredTerm(20, {{{"pool", "In", {"highmem"}}}});
        }
        if (pick(seed, c + 12, 10) == 0) w.Toleration("maint", "Equal", "true", kPreferNoSchedule);
        w.ReqLim(req, lim);
        pods->push_back(w.Obj());
    }
}

}  // namespace qsfw
