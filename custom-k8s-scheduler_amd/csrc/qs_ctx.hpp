// qs_ctx.hpp — internal host-side state shared by the libqsched translation units (qs_host.cpp,
// qs_dist.cpp): the context behind the opaque qs_ctx handle, prepared streams, device buffers.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/qsched.h"
#include "qs_device.hpp"
#include "qs_launch.hpp"

namespace qs_host {

constexpr int64_t kLimit = (1LL << 24) - 1;  // 24-bit multiplier range of the kernels (spec S10)
// Wide layout (f64 memory columns in bytes): every memory quantity below 2^46 (64 TiB) keeps
// (alloc - reqd) * 100 and the quotient-correction products exact in f64.
constexpr int64_t kWideMemLimit = (1LL << 46) - 1;
// Largest value a Requested / NonZeroRequested column may reach during a stream: int32 columns
// (compact layout, cpu in both layouts) and f64-exact integers (wide memory).
constexpr int64_t kGrowLimit32 = (1LL << 31) - 1;
constexpr int64_t kGrowLimitF64 = (1LL << 53) - 1;
// Tables at least this large also keep the SoA copy the SCAN engine streams (L2-resident below).
constexpr uint32_t kSoaMinNodes = 1u << 16;
// Tables up to this size also keep the batched-mode anti-affinity state (128 B of app bits per
// node + the (app, zone) counts) inside the table allocation, so save/restore covers it.
constexpr uint32_t kAaMaxNodes = 1u << 20;

struct QsError {
    qs_status st;
    std::string msg;
};

#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess)                                                              \
            throw QsError{QS_EDEVICE, std::string(#x) + ": " + hipGetErrorString(e_)};     \
    } while (0)

[[noreturn]] inline void fail(qs_status st, const std::string &m) { throw QsError{st, m}; }

// Why the calling thread's last qs_open / qs_open_shard failed (there is no context to hold the
// message): qs_last_error(NULL) returns it.
inline thread_local std::string g_open_err;
inline qs_status open_failed(qs_status st, const std::string &m) {
    g_open_err = m;
    return st;
}

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    void ensure(size_t b) {
        if (b <= bytes) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        HIPCHK(hipMalloc(&p, b));
        bytes = b;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    T *as() const { return (T *)p; }
};

// Host mirror of the canonical table.
struct Mirror {
    uint32_t n = 0;
    std::vector<int64_t> ac, am, mp, rc, rm, zc, zm, np;
    std::vector<int64_t> ae, re;  // [n][QS_MAX_EXT]
    std::vector<uint64_t> th, ts, lb;  // lb [n][2]
    std::vector<int32_t> zone;
    std::vector<uint64_t> gen;
    void resize(uint32_t nn) {
        n = nn;
        zone.assign(nn, 0);
        for (auto *v : {&ac, &am, &mp, &rc, &rm, &zc, &zm, &np}) v->assign(nn, 0);
        ae.assign((size_t)nn * QS_MAX_EXT, 0);
        re.assign((size_t)nn * QS_MAX_EXT, 0);
        th.assign(nn, 0);
        ts.assign(nn, 0);
        lb.assign((size_t)nn * 2, 0);
        gen.assign(nn, 0);
    }
};

inline int ctz64(int64_t v) { return v == 0 ? 64 : __builtin_ctzll((uint64_t)v); }

}  // namespace qs_host

struct qs_stream {
    uint32_t p = 0;
    uint32_t feat = 0;  // kFeat* bits of this stream (profile + extended resources in use)
    std::vector<qs_pod> pods;      // canonical, arrival order
    std::vector<uint32_t> order;   // stream position -> arrival index
    qs_host::DevBuf d_pods, d_podx, d_node, d_key, d_stamp;
    bool ran = false;
    int mode_ran = -1;        // qs_mode of the last run
    uint64_t epoch_after = 0;  // the context's table epoch right after the last run (FitError replay)
    int shift = 0;
    bool wide = false;  // pod records are DPodW (the table's wide layout) when set
    // LOOKAHEAD window sequence as an instantiated HIP graph, valid while gkey matches
    hipGraphExec_t gexec = nullptr;
    std::vector<uint8_t> gkey;
    ~qs_stream() {
        if (gexec) (void)hipGraphExecDestroy(gexec);
    }
};

struct qs_ctx {
    std::mutex mu;
    uint64_t table_epoch = 0;  // bumped by every change of the node table (load, upsert, Reserve, restore, run)
    qs_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;   // resolve chain, copies, single-kernel engines
    hipStream_t stream2 = nullptr;  // lookahead select chain (overlapped windows)
    std::string err;
    qs_host::Mirror m;
    int shift = 20;  // memory unit 2^shift bytes on the device (compact layout)
    bool wide = false;  // wide layout: f64 memory columns in bytes (DevTable::wrows)
    bool dev_valid = false;
    qs::DevTable dt{};
    qs::DevCfg dc{};
    qs_host::DevBuf tbl;  // all columns in one allocation
    qs_host::DevBuf soa;  // SoA int32 copy (kSCols x cap) when n >= soa_min_nodes
    bool soa_valid = false;  // SoA copy matches the rows (engines that update rows only clear it)
    qs_host::DevBuf tbl_saved;  // qs_table_save snapshot (whole allocation)
    qs_host::Mirror m_saved;    // ... and the host mirror it corresponds to
    bool saved = false;
    bool saved_wide = false;
    int saved_shift = 20;
    bool mirror_stale = false;  // device table changed since the last mirror sync
    uint64_t device_faults = 0; // QS_EDEVICE results so far (each one drops the device table)
    qs_host::DevBuf diag;
    qs_host::DevBuf scratch, lists, clists, dio, npart, normi, nstat, nfall, nrec, bctrl, one_pod, one_podx;
    qs_host::DevBuf vshard;  // the all-reduce engine's virtual-world node ranges ([V][lo, hi])
    void *pin = nullptr;   // qs_score_pod's packed outputs, written by the kernel (pinned host memory)
    size_t pin_bytes = 0;
    uint64_t score_seq = 0;  // the kernel's done word for the call in flight
    qs_host::DevBuf score_gs;  // the multi-workgroup score launch's {best, arrivals, taint max, affinity max} (zero between calls)
    uint32_t pend = 0xFFFFFFFFu;  // a qs_reserve / qs_unreserve row not yet written to the device:
                                  // the next qs_score_pod writes it, every other call first flushes it
    qs_host::DevBuf hand;  // window hand-off words: {unused, ready, timeout flag} (u64 each)
    bool handoff_off = false;  // a hand-off timed out once: cross-stream events from then on
    qs_host::DevBuf resctl;    // resident stream's hand-off counters
    // Resident-stream timeouts (QS_ETIMEOUT of a resident run): the run right after one uses
    // per-window launches (cooldown), the next is resident again; a second consecutive resident
    // timeout keeps per-window launches for the context's life (qs_dist_mailbox_connect resets both)
    int res_timeouts = 0;
    bool res_cooldown = false;
    uint32_t inject_used = 0;  // QS_INJECT_FAULT test hooks already fired on this context (bit per hook)
    bool last_resident = false;  // the last lookahead run was a resident stream
    int cus = 0;               // compute units of the device (resident stream's selector count)
    uint64_t run_seq = 0;      // lookahead runs of this context (the hand-off's epoch)
    bool last_waits = false;   // the last lookahead run waited on device words (hand-off / mailbox)
    uint32_t cap = 0;
    // sharding (qs_open_shard): RCCL communicator of this rank, nullptr when unsharded
    int rank = 0, world = 1;
    ncclComm_t comm = nullptr;
    // peer-memory mailbox transport (qs_dist_mailbox_*): this rank's mailbox, the
    // device array of every rank's mailbox base (peers mapped with hipIpcOpenMemHandle), on when
    // connected
    qs_host::DevBuf mbox, mbox_peers;
    std::vector<void *> mbox_opened;
    bool mbox_on = false;
    bool mbox_fine = false;  // the mailbox is fine-grained device memory (hipDeviceMallocFinegrained)
    bool mbox_broken = false;  // a mailbox wait timed out: the ranks are out of step until every
                               // rank calls qs_dist_mailbox_connect again
    // QS_MBOX_HOST=1 at qs_dist_mailbox_export: every rank's mailbox is POSIX shared host memory
    // registered with HIP (mapped, the GPU reads and writes it over the host link), so no GPU L2 is
    // shared by the ranks' mailboxes even with every rank on one GPU (the test form of the
    // cross-device protocol).  mbox.p is then the device alias of the own mapping.
    bool mbox_host = false;
    void *mbox_hptr = nullptr;                        // own mapping (host address)
    std::string mbox_shm;                             // own segment name (unlinked at close)
    std::vector<void *> mbox_hmaps;                   // peers' mappings (host addresses)
};
namespace qs_host {
void mbox_host_release(qs_ctx *c);  // qs_dist.cpp: unregister / unmap the host-memory mailboxes
}

namespace qs_host {
// Node shards of the LOOKAHEAD select for this context: W shards in total, this process scores
// shards [v0, v0 + nv).  qs_open_shard: (world, rank, 1); cfg.virtual_shards = V > 1: (V, 0, V).
struct ShardPlan {
    uint32_t W, v0, nv;
};
inline ShardPlan shard_plan(const qs_ctx *c) {
    if (c->world > 1) return {(uint32_t)c->world, (uint32_t)c->rank, 1u};
    if (c->cfg.virtual_shards > 1) return {(uint32_t)c->cfg.virtual_shards, 0u, (uint32_t)c->cfg.virtual_shards};
    return {1u, 0u, 1u};
}
// The per-window exchange of the sharded engine (qs_dist.cpp): all-gather of each rank's
// [K][GLp] list block into [world][K][GLp] (in place), on the context's stream.
void exchange_lists(qs_ctx *c, uint64_t *lists, size_t per_rank_entries, hipStream_t stream);
// The same in-place all-gather for 32-bit words (normalizing profiles' partial maxima).
void exchange_u32(qs_ctx *c, uint32_t *buf, size_t per_rank_words, hipStream_t stream);
// In-place max all-reduces of the per-pod engine QS_ENGINE_ALLREDUCE.
void allreduce_max_u64(qs_ctx *c, uint64_t *buf, size_t count, hipStream_t stream);
void allreduce_max_u32(qs_ctx *c, uint32_t *buf, size_t count, hipStream_t stream);
// {count, nodes[64]} dirty-set hand-off between overlapped lookahead windows (+ pad)
constexpr size_t kDioWords = 68;
// Mailbox layout (bytes from the base): flags [2 phases][16 ranks] u64 | lists [3 slots][16 ranks]
// [64 pods][64] u64 | normalization partials [3 slots][16 ranks][4096] uint4.  Window w uses slot
// w % 3: a rank writes window w+2 into a peer's slot only after seeing that peer's window-w+1
// flags, by which time the peer's resolver of window w-1 (the slot's previous user) has finished.
constexpr size_t kMbRanks = 16, kMbSlots = 3, kMbPartPerRank = 4096;
constexpr size_t kMbFlags = 2 * kMbRanks * 8;
constexpr size_t kMbListSlot = kMbRanks * 64 * 64 * 8;
constexpr size_t kMbPartSlot = kMbRanks * kMbPartPerRank * 16;
// Resident sharded stream, after the per-window regions: hello[16] (each rank's run
// sequence, the in-launch entry barrier), flags[4 slots][32 pods][16 ranks] and shard lists
// [4 slots][32 pods][16 ranks][64] u64 (window w uses slot w % 4), then the normalizing profiles'
// partial-maxima flags and partials of the same shape.
constexpr size_t kMbResSlots = 4, kMbResPods = 32;
constexpr size_t kMbResHello = kMbFlags + kMbSlots * (kMbListSlot + kMbPartSlot);
constexpr size_t kMbResFlags = kMbResHello + 256;
constexpr size_t kMbResLists = kMbResFlags + kMbResSlots * kMbResPods * kMbRanks * 8;
// normalizing profiles: flags[4 slots][32 pods][16 ranks] u64 and partial maxima [4][32][16] uint4
constexpr size_t kMbResNFlags = kMbResLists + kMbResSlots * kMbResPods * kMbRanks * 64 * 8;
constexpr size_t kMbResNorm = kMbResNFlags + kMbResSlots * kMbResPods * kMbRanks * 8;
constexpr size_t kMbBytes = kMbResNorm + kMbResSlots * kMbResPods * kMbRanks * 16;
inline uint64_t *mbox_lists(qs_ctx *c, uint32_t slot) {
    return reinterpret_cast<uint64_t *>(static_cast<char *>(c->mbox.p) + kMbFlags + slot * kMbListSlot);
}
inline uint4 *mbox_npart(qs_ctx *c, uint32_t slot) {
    return reinterpret_cast<uint4 *>(static_cast<char *>(c->mbox.p) + kMbFlags + kMbSlots * kMbListSlot +
                                     slot * kMbPartSlot);
}
// One mailbox exchange on `stream`: copy this rank's block of the slot region (phase 0: partials,
// phase 1: lists; L > 0: lists of `pods` x 64 entries, entries >= L written as 0) into every peer's
// mailbox, raise flag[phase][rank] = seq there, then wait until every rank's flag reaches seq in
// this rank's mailbox (bounded; a timeout sets *werr).
void mbox_exchange(qs_ctx *c, int phase, uint32_t slot, size_t block_bytes, uint32_t pods, uint32_t L,
                   uint64_t seq, uint32_t *werr, hipStream_t stream);
}  // namespace qs_host

