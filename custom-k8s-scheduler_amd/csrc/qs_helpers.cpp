// qs_helpers.cpp — host-side pod precompute (spec S2/S3) and the spec/synth.md generator.
#include <algorithm>
#include <cstring>

#include "../../include/qsched.h"

namespace {
constexpr int64_t kDefCpu = 100;                  // UP util/pod_resources.go#DefaultMilliCPURequest
constexpr int64_t kDefMem = 200LL * 1024 * 1024;  // UP util/pod_resources.go#DefaultMemoryRequest

struct Res {
    int64_t cpu = 0, mem = 0, ext[QS_MAX_EXT] = {0, 0};
    void add(const Res &o) {
        cpu += o.cpu; mem += o.mem;
        for (int k = 0; k < QS_MAX_EXT; k++) ext[k] += o.ext[k];
    }
    void max_with(const Res &o) {
        cpu = std::max(cpu, o.cpu); mem = std::max(mem, o.mem);
        for (int k = 0; k < QS_MAX_EXT; k++) ext[k] = std::max(ext[k], o.ext[k]);
    }
};

Res container_req(const qs_container &c, bool non_missing) {
    Res r;
    r.cpu = c.has_req_cpu ? c.req_cpu : (non_missing ? kDefCpu : 0);
    r.mem = c.has_req_mem ? c.req_mem : (non_missing ? kDefMem : 0);
    for (int k = 0; k < QS_MAX_EXT; k++) r.ext[k] = c.req_ext[k];
    return r;
}

// UP component-helpers/resource/helpers.go#PodRequests: regular containers summed, restartable
// init containers (sidecars) added to the sum and to the running sidecar total, each init
// container's need = its request + the sidecars started before it, result = max(sum, max init).
Res pod_requests(const qs_container *c, uint32_t nc, bool non_missing) {
    Res reqs, init_max, sidecars;
    for (uint32_t i = 0; i < nc; i++)
        if (c[i].kind == 0) reqs.add(container_req(c[i], non_missing));
    for (uint32_t i = 0; i < nc; i++) {
        if (c[i].kind == 0) continue;
        Res cr = container_req(c[i], non_missing);
        if (c[i].kind == 2) {
            reqs.add(cr);
            sidecars.add(cr);
            cr = sidecars;
        } else {
            cr.add(sidecars);
        }
        init_max.max_with(cr);
    }
    reqs.max_with(init_max);
    return reqs;
}

// spec/synth.md G1 counter-based SplitMix64
inline uint64_t sm_at(uint64_t seed, uint64_t c) {
    uint64_t z = seed + (c + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
inline uint32_t pick(uint64_t seed, uint64_t c, uint32_t k) { return (uint32_t)((sm_at(seed, c) >> 33) % k); }

int zone_pair_bit(int a, int b) {  // a < b: 3 + lexicographic index among the 45 pairs
    int idx = 0;
    for (int x = 0; x < a; x++) idx += 9 - x;
    return 3 + idx + (b - a - 1);
}
void set_bit128(uint64_t *m, int bit) { m[bit >> 6] |= 1ULL << (bit & 63); }
}  // namespace

extern "C" {

// UP pkg/apis/core/v1/helper/qos/qos.go#ComputePodQOS (cpu and memory only, quantities <= 0 ignored)
int32_t qs_compute_qos(const qs_container *c, uint32_t nc) {
    int64_t req_cpu = 0, req_mem = 0, lim_cpu = 0, lim_mem = 0;
    bool has_req_cpu = false, has_req_mem = false, has_lim_cpu = false, has_lim_mem = false;
    bool guaranteed = true;
    for (uint32_t i = 0; i < nc; i++) {
        if (c[i].has_req_cpu && c[i].req_cpu > 0) { req_cpu += c[i].req_cpu; has_req_cpu = true; }
        if (c[i].has_req_mem && c[i].req_mem > 0) { req_mem += c[i].req_mem; has_req_mem = true; }
        bool lc = c[i].has_lim_cpu && c[i].lim_cpu > 0, lm = c[i].has_lim_mem && c[i].lim_mem > 0;
        if (lc) { lim_cpu += c[i].lim_cpu; has_lim_cpu = true; }
        if (lm) { lim_mem += c[i].lim_mem; has_lim_mem = true; }
        if (!(lc && lm)) guaranteed = false;
    }
    const int nreq = (int)has_req_cpu + (int)has_req_mem, nlim = (int)has_lim_cpu + (int)has_lim_mem;
    if (nreq == 0 && nlim == 0) return QS_QOS_BESTEFFORT;
    if (guaranteed) {
        if (has_req_cpu && (!has_lim_cpu || lim_cpu != req_cpu)) guaranteed = false;
        if (has_req_mem && (!has_lim_mem || lim_mem != req_mem)) guaranteed = false;
    }
    if (guaranteed && nreq == nlim) return QS_QOS_GUARANTEED;
    return QS_QOS_BURSTABLE;
}

qs_status qs_pod_from_containers(const qs_container *c, uint32_t nc, const int64_t *overhead,
                                 qs_pod *out) {
    if (!out || (nc && !c)) return QS_EINVAL;
    std::memset(out, 0, sizeof(*out));
    Res r = pod_requests(c, nc, false), z = pod_requests(c, nc, true);
    if (overhead) {  // pod overhead adds to both (UP PodRequests, opts.ExcludeOverhead = false)
        r.cpu += overhead[0]; r.mem += overhead[1];
        z.cpu += overhead[0]; z.mem += overhead[1];
    }
    out->req_cpu = r.cpu;
    out->req_mem = r.mem;
    for (int k = 0; k < QS_MAX_EXT; k++) out->req_ext[k] = r.ext[k];
    out->nz_cpu = z.cpu;
    out->nz_mem = z.mem;
    out->qos = qs_compute_qos(c, nc);
    return QS_OK;
}

// spec/synth.md generator.  nodes arrays: n entries (ext [n][2], label_bits [n][2]); pods: p.
qs_status qs_synth_generate(int config, uint64_t seed, uint32_t n, uint32_t p,
                            const qs_node_soa_out *nd, qs_pod *pods) {
    static const int64_t kNodeCpu[6] = {4000, 8000, 16000, 32000, 64000, 96000};
    static const int64_t kMpc[3] = {2, 4, 8};
    static const int64_t kPodCpu[6] = {500, 1000, 1500, 2000, 4000, 8000};
    static const int64_t kPodMemMi[7] = {128, 256, 512, 1024, 2048, 4096, 8192};
    static const int64_t kGpu[4] = {1, 2, 4, 8};
    const int64_t GiB = 1LL << 30, MiB = 1LL << 20;
    const bool c4 = config == 4, c5 = config == 5;
    if (n && (!nd || !nd->alloc_cpu || !nd->alloc_mem)) return QS_EINVAL;
    if (p && !pods) return QS_EINVAL;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t c = 8ULL * i;
        const int64_t cpu = kNodeCpu[pick(seed, c + 0, 6)];
        const int64_t mpc = kMpc[pick(seed, c + 1, 3)];
        nd->alloc_cpu[i] = cpu;
        nd->alloc_mem[i] = (cpu / 1000) * mpc * GiB;
        if (nd->max_pods) nd->max_pods[i] = 110;
        for (int64_t *col : {nd->req_cpu, nd->req_mem, nd->nz_cpu, nd->nz_mem, nd->pods})
            if (col) col[i] = 0;
        for (int k = 0; k < QS_MAX_EXT; k++) {
            if (nd->alloc_ext) nd->alloc_ext[(size_t)i * QS_MAX_EXT + k] = 0;
            if (nd->req_ext) nd->req_ext[(size_t)i * QS_MAX_EXT + k] = 0;
        }
        uint64_t th = 0, ts = 0, lb[2] = {0, 0};
        if (c4) {
            const bool gpu = pick(seed, c + 2, 10) == 0;
            const bool maint = pick(seed, c + 3, 20) == 0;
            const int zone = (int)pick(seed, c + 4, 10);
            const int pool = gpu ? 2 : (int)pick(seed, c + 5, 2);  // 0 general, 1 highmem, 2 gpu
            const bool ssd = pick(seed, c + 6, 2) == 0;
            if (gpu) {
                if (nd->alloc_ext) nd->alloc_ext[(size_t)i * QS_MAX_EXT] = 8;
                th |= 1ULL;  // gpu=true:NoSchedule
            }
            if (maint) ts |= 2ULL;  // maint=true:PreferNoSchedule
            if (pool == 2) set_bit128(lb, 0);
            if (ssd) set_bit128(lb, 1);
            if (pool == 1) set_bit128(lb, 2);
            for (int a = 0; a < 10; a++)
                for (int b = a + 1; b < 10; b++)
                    if (a == zone || b == zone) set_bit128(lb, zone_pair_bit(a, b));
        }
        if (nd->zone) nd->zone[i] = (c4 || c5) ? (int32_t)pick(seed, c + 4, 10) : 0;  // zone z0..z9
        if (nd->taint_hard) nd->taint_hard[i] = th;
        if (nd->taint_soft) nd->taint_soft[i] = ts;
        if (nd->label_bits) { nd->label_bits[2 * (size_t)i] = lb[0]; nd->label_bits[2 * (size_t)i + 1] = lb[1]; }
    }
    for (uint32_t j = 0; j < p; j++) {
        const uint64_t c = 8ULL * n + 16ULL * j;
        const uint32_t qd = pick(seed, c + 0, 10);
        const int64_t cpu = kPodCpu[pick(seed, c + 1, 6)];
        const int64_t mem = kPodMemMi[pick(seed, c + 2, 7)] * MiB;
        const uint32_t memmode = pick(seed, c + 3, 4);
        const uint32_t limmode = pick(seed, c + 4, 2);
        qs_container ct{};
        if (qd < 2) {  // Guaranteed: requests = limits
            ct.has_req_cpu = ct.has_req_mem = ct.has_lim_cpu = ct.has_lim_mem = 1;
            ct.req_cpu = ct.lim_cpu = cpu;
            ct.req_mem = ct.lim_mem = mem;
        } else if (qd < 7) {  // Burstable
            ct.has_req_cpu = 1;
            ct.req_cpu = cpu;
            if (memmode != 0) { ct.has_req_mem = 1; ct.req_mem = mem; }
            if (limmode == 1) {
                ct.has_lim_cpu = 1; ct.lim_cpu = 2 * cpu;
                if (ct.has_req_mem) { ct.has_lim_mem = 1; ct.lim_mem = 2 * mem; }
            }
        }
        qs_pod &pd = pods[j];
        uint64_t tol_hard = 0, tol_soft = 0, sel[2] = {0, 0};
        int32_t nreq = 0, npref = 0;
        uint64_t req_term[2] = {0, 0};
        uint64_t pref_terms[QS_MAX_TERMS][2] = {};
        int32_t pref_w[QS_MAX_TERMS] = {};
        if (c4) {
            if (pick(seed, c + 5, 20) == 0) {
                ct.req_ext[0] = kGpu[pick(seed, c + 6, 4)];
                tol_hard |= 1ULL;
                set_bit128(sel, 0);
            }
            if (pick(seed, c + 7, 5) == 0) {
                const int za = (int)pick(seed, c + 8, 10);
                const int zb = (za + 1 + (int)pick(seed, c + 9, 9)) % 10;
                set_bit128(req_term, zone_pair_bit(std::min(za, zb), std::max(za, zb)));
                nreq = 1;
            }
            if (pick(seed, c + 10, 5) == 0) {
                const uint32_t which = pick(seed, c + 11, 3);
                if (which == 0 || which == 2) { pref_terms[npref][0] = 1ULL << 1; pref_w[npref++] = 50; }
                if (which == 1 || which == 2) { pref_terms[npref][0] = 1ULL << 2; pref_w[npref++] = 20; }
            }
            if (pick(seed, c + 12, 10) == 0) tol_soft |= 2ULL;
        }
        qs_pod_from_containers(&ct, 1, nullptr, &pd);
        if (c5) {  // spec/synth.md G5: app group and its required anti-affinity kind
            pd.app = (int32_t)pick(seed, c + 13, 1000);
            const uint32_t kind = pick(seed, 8ULL * n + 16ULL * p + (uint64_t)pd.app, 10);
            pd.anti_affinity = kind < 5 ? QS_AA_HOSTNAME : (kind == 5 ? QS_AA_ZONE : QS_AA_NONE);
        }
        pd.tol_hard = tol_hard;
        pd.tol_soft = tol_soft;
        pd.sel[0] = sel[0];
        pd.sel[1] = sel[1];
        pd.n_req_terms = nreq;
        pd.req_terms[0][0] = req_term[0];
        pd.req_terms[0][1] = req_term[1];
        pd.n_pref_terms = npref;
        for (int t = 0; t < QS_MAX_TERMS; t++) {
            pd.pref_terms[t][0] = pref_terms[t][0];
            pd.pref_terms[t][1] = pref_terms[t][1];
            pd.pref_weight[t] = pref_w[t];
        }
    }
    return QS_OK;
}

}  // extern "C"
