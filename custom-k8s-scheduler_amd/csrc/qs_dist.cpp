// qs_dist.cpp — multi-GPU entry points: one process per GPU, the node table sharded by contiguous
// ranges, one RCCL all-gather of top-L lists per lookahead window over xGMI.
//
// Why an all-gather of lists and not the per-pod key all-reduce of SURVEY.md §3.3: the exact
// lookahead resolves K pods from per-shard top-L lists, so one collective of K*GLp keys per rank
// replaces K latency-bound 8-byte all-reduces (SURVEY.md §7 H4 option 3).  Every rank then runs the
// same resolver over the same gathered lists and its replicated table, so placements and table
// updates are identical on all ranks without a second exchange.
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <string>

#include "qs_ctx.hpp"

using namespace qs_host;

namespace {

const char *nccl_msg(ncclResult_t r) { return ncclGetErrorString(r); }

#define NCCLCHK(x)                                                                          \
    do {                                                                                    \
        ncclResult_t r_ = (x);                                                              \
        if (r_ != ncclSuccess) throw QsError{QS_EDEVICE, std::string(#x) + ": " + nccl_msg(r_)}; \
    } while (0)

}  // namespace

namespace qs_host {

void exchange_lists(qs_ctx *c, uint64_t *lists, size_t per_rank_entries, hipStream_t stream) {
    // in place: rank r's block already sits at lists + r * per_rank_entries
    NCCLCHK(ncclAllGather(lists + (size_t)c->rank * per_rank_entries, lists, per_rank_entries,
                          ncclUint64, c->comm, stream));
}

void exchange_u32(qs_ctx *c, uint32_t *buf, size_t per_rank_words, hipStream_t stream) {
    NCCLCHK(ncclAllGather(buf + (size_t)c->rank * per_rank_words, buf, per_rank_words, ncclUint32,
                          c->comm, stream));
}

// The as-is RCCL baseline: one latency-bound max all-reduce per pod, in place.
void allreduce_max_u64(qs_ctx *c, uint64_t *buf, size_t count, hipStream_t stream) {
    NCCLCHK(ncclAllReduce(buf, buf, count, ncclUint64, ncclMax, c->comm, stream));
}
void allreduce_max_u32(qs_ctx *c, uint32_t *buf, size_t count, hipStream_t stream) {
    NCCLCHK(ncclAllReduce(buf, buf, count, ncclUint32, ncclMax, c->comm, stream));
}

// ---- peer-memory mailbox: one hop per exchange instead of a ring ----------
// Block p writes this rank's block into rank p's mailbox over xGMI (p == rank: only the zero
// padding of its own lists), then publishes flag[phase][rank] = seq there with a system-scope
// release after a system-scope fence, so a peer that observes the flag also observes the block.
__global__ __launch_bounds__(256) void k_mbox_put(char *const *__restrict__ peers, uint32_t rank,
                                                  size_t region, size_t block_bytes, uint32_t pods,
                                                  uint32_t L, uint32_t phase, uint64_t seq) {
    const uint32_t p = blockIdx.x;
    char *dst = peers[p] + region + (size_t)rank * block_bytes;
    const char *src = peers[rank] + region + (size_t)rank * block_bytes;
    if (L > 0) {  // lists: pods x 64 entries, entries >= L are padding
        uint64_t *d = reinterpret_cast<uint64_t *>(dst);
        const uint64_t *q = reinterpret_cast<const uint64_t *>(src);
        for (uint32_t i = threadIdx.x; i < pods * 64u; i += blockDim.x) {
            const uint32_t e = i & 63u;
            if (e >= L) d[i] = 0ull;
            else if (p != rank) d[i] = q[i];
        }
    } else if (p != rank) {
        uint4 *d = reinterpret_cast<uint4 *>(dst);
        const uint4 *q = reinterpret_cast<const uint4 *>(src);
        for (size_t i = threadIdx.x; i < block_bytes / 16; i += blockDim.x) d[i] = q[i];
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<uint64_t *>(peers[p]) + phase * kMbRanks + rank, seq,
                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Waits until every rank's flag[phase] in this rank's mailbox reaches seq (0.5 s bound: *werr = 1).
// Once a wait of the run has timed out, later waits return at once: the run is void anyway, and
// a dead peer would otherwise cost the bound once per remaining window.
// The bound is 0.5 s per window, and 5 s for a run's first window, whose peers may still be in
// their host-side preparation.
__global__ void k_mbox_wait(const uint64_t *__restrict__ flags, uint32_t world, uint32_t phase, uint64_t seq,
                            uint32_t *__restrict__ werr, uint64_t bound) {
    if (threadIdx.x != 0) return;
    if (__hip_atomic_load(werr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t r = 0; r < world; ++r)
        while (__hip_atomic_load(flags + phase * kMbRanks + r, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > bound) {
                __hip_atomic_store(werr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
        }
}

void mbox_exchange(qs_ctx *c, int phase, uint32_t slot, size_t block_bytes, uint32_t pods, uint32_t L,
                   uint64_t seq, uint32_t *werr, hipStream_t stream) {
    const size_t region = phase == 1 ? kMbFlags + slot * kMbListSlot
                                     : kMbFlags + kMbSlots * kMbListSlot + slot * kMbPartSlot;
    hipLaunchKernelGGL(k_mbox_put, dim3(c->world), dim3(256), 0, stream, c->mbox_peers.as<char *>(),
                       (uint32_t)c->rank, region, block_bytes, pods, L, (uint32_t)phase, seq);
    HIPCHK(hipGetLastError());
    const bool first = (uint32_t)seq == 1u;  // window 0 of the run (seq = run << 32 | w + 1)
    hipLaunchKernelGGL(k_mbox_wait, dim3(1), dim3(64), 0, stream, c->mbox.as<uint64_t>(), (uint32_t)c->world,
                       (uint32_t)phase, seq, werr, first ? 500000000ull : 50000000ull);
    HIPCHK(hipGetLastError());
}

}  // namespace qs_host

extern "C" {

qs_status qs_dist_unique_id(uint8_t out[128]) {
    if (!out) return QS_EINVAL;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return QS_EDEVICE;
    std::memcpy(out, &id, sizeof id);
    return QS_OK;
}

qs_status qs_open_shard(const qs_config *cfg, int device, int rank, int world,
                        const uint8_t nccl_id[128], qs_ctx **out) {
    if (!cfg || !out || world < 1 || world > 16 || rank < 0 || rank >= world)
        return open_failed(QS_EINVAL, "qs_open_shard: need 0 <= rank < world <= 16 and a config");
    qs_status st = qs_open(cfg, device, out);
    if (st != QS_OK) return st;
    qs_ctx *c = *out;
    c->rank = rank;
    c->world = world;
    // no id: the peer-memory mailbox transport, connected with qs_dist_mailbox_export/_connect;
    // world == 1 with an id still builds a (one-rank) communicator: the RCCL path on one GPU
    if (!nccl_id) return QS_OK;
    ncclUniqueId id;
    std::memcpy(&id, nccl_id, sizeof id);
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, world, id, rank);
    if (r != ncclSuccess) {
        const char *last = ncclGetLastError(nullptr);
        qs_close(c);
        *out = nullptr;
        return open_failed(QS_EDEVICE, std::string("ncclCommInitRank(world ") + std::to_string(world) + ", rank " +
                                           std::to_string(rank) + ", device " + std::to_string(device) +
                                           "): " + nccl_msg(r) + (last && *last ? std::string(" — ") + last : ""));
    }
    c->comm = comm;
    return QS_OK;
}

}  // extern "C"

namespace qs_host {

// A kMbBytes POSIX shared-memory segment, mapped and registered with HIP; returns the host address.
static void *mbox_host_map(const char *name, bool create) {
    const int fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0) fail(QS_EDEVICE, std::string("shm_open ") + name + ": " + std::strerror(errno));
    if (create && ftruncate(fd, (off_t)kMbBytes) != 0) {
        ::close(fd);
        fail(QS_EDEVICE, std::string("ftruncate ") + name);
    }
    void *h = mmap(nullptr, kMbBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (h == MAP_FAILED) fail(QS_EDEVICE, std::string("mmap ") + name);
    if (hipHostRegister(h, kMbBytes, hipHostRegisterMapped) != hipSuccess) {
        (void)hipGetLastError();
        munmap(h, kMbBytes);
        fail(QS_EDEVICE, std::string("hipHostRegister ") + name);
    }
    return h;
}
static char *mbox_host_dev(void *h) {
    void *d = nullptr;
    HIPCHK(hipHostGetDevicePointer(&d, h, 0));
    return static_cast<char *>(d);
}
void mbox_host_release(qs_ctx *c) {
    if (!c->mbox_host) return;
    for (void *h : c->mbox_hmaps) {
        (void)hipHostUnregister(h);
        munmap(h, kMbBytes);
    }
    c->mbox_hmaps.clear();
    if (c->mbox_hptr) {
        (void)hipHostUnregister(c->mbox_hptr);
        munmap(c->mbox_hptr, kMbBytes);
        shm_unlink(c->mbox_shm.c_str());
    }
    c->mbox_hptr = nullptr;
    c->mbox.p = nullptr;  // (the device alias of a host mapping: nothing for DevBuf to free)
    c->mbox.bytes = 0;
    c->mbox_host = false;
}

}  // namespace qs_host

extern "C" {

qs_status qs_dist_mailbox_export(qs_ctx *c, uint8_t handle[64]) {
    if (!c || !handle) return QS_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    try {
        HIPCHK(hipSetDevice(c->device));
        const char *hm = getenv("QS_MBOX_HOST");
        if (!c->mbox.p && hm && hm[0] == '1') {
            // host-memory mailbox: the handle is 'H' + the segment's name
            static int seq = 0;
            c->mbox_shm = "/qsched_mb_" + std::to_string((long)getpid()) + "_" + std::to_string(seq++);
            c->mbox_hptr = mbox_host_map(c->mbox_shm.c_str(), true);
            c->mbox_host = true;
            c->mbox.p = mbox_host_dev(c->mbox_hptr);
            c->mbox.bytes = kMbBytes;
            std::memset(c->mbox_hptr, 0, kMbBytes);
            __sync_synchronize();
        }
        if (c->mbox_host) {
            std::memset(handle, 0, 64);
            handle[0] = 'H';
            std::memcpy(handle + 1, c->mbox_shm.c_str(), std::min<size_t>(62, c->mbox_shm.size()));
            return QS_OK;
        }
        if (!c->mbox.p) {
            // Fine-grained device memory: peers write it over xGMI while this GPU polls
            // its flags and reads its slots, so it must stay coherent with remote writers without
            // relying on the coarse-grained L2's write-back/invalidate points.  If this pool
            // cannot export a fine-grained allocation, fall back to hipMalloc (the sc1 / system-scope
            // accesses of the kernels remain); c->mbox_fine records which one is in use.
            void *p = nullptr;
            hipIpcMemHandle_t probe;
            if (hipExtMallocWithFlags(&p, kMbBytes, hipDeviceMallocFinegrained) == hipSuccess &&
                hipIpcGetMemHandle(&probe, p) == hipSuccess) {
                c->mbox.p = p;
                c->mbox.bytes = kMbBytes;
                c->mbox_fine = true;
            } else {
                if (p) (void)hipFree(p);
                (void)hipGetLastError();
                c->mbox.ensure(kMbBytes);
                c->mbox_fine = false;
            }
            HIPCHK(hipMemset(c->mbox.p, 0, kMbBytes));
            HIPCHK(hipDeviceSynchronize());
        }
        hipIpcMemHandle_t h;
        static_assert(sizeof(h) == 64, "hipIpcMemHandle_t is 64 bytes");
        HIPCHK(hipIpcGetMemHandle(&h, c->mbox.p));
        std::memcpy(handle, &h, sizeof h);
        return QS_OK;
    } catch (const QsError &e) {
        c->err = e.msg;
        return e.st;
    }
}

qs_status qs_dist_mailbox_connect(qs_ctx *c, const uint8_t *handles) {
    if (!c || !handles) return QS_EINVAL;
    std::lock_guard<std::mutex> lk(c->mu);
    try {
        if (!c->mbox.p) fail(QS_ESTATE, "qs_dist_mailbox_export first");
        if (c->comm) fail(QS_ESTATE, "this context already uses RCCL");
        HIPCHK(hipSetDevice(c->device));
        // (re)connect: a second call after a mailbox timeout brings the ranks back in step — every
        // rank's runs have returned (no write is in flight), the caller barriers before and after
        // this call on every rank, and each rank restarts from an empty mailbox and sequence 0
        for (void *p : c->mbox_opened) (void)hipIpcCloseMemHandle(p);
        c->mbox_opened.clear();
        for (void *h : c->mbox_hmaps) {
            (void)hipHostUnregister(h);
            munmap(h, kMbBytes);
        }
        c->mbox_hmaps.clear();
        c->mbox_on = false;
        if (c->mbox_host) {
            std::memset(c->mbox_hptr, 0, kMbBytes);
            __sync_synchronize();
        } else {
            HIPCHK(hipMemset(c->mbox.p, 0, kMbBytes));
        }
        HIPCHK(hipDeviceSynchronize());
        c->run_seq = 0;
        c->mbox_broken = false;
        // every rank starts the new connection from the same resident / per-window choice
        c->res_timeouts = 0;
        c->res_cooldown = false;
        std::vector<char *> bases((size_t)c->world);
        for (int r = 0; r < c->world; ++r) {
            if (r == c->rank) {
                bases[(size_t)r] = static_cast<char *>(c->mbox.p);
                continue;
            }
            const uint8_t *hr = handles + 64 * (size_t)r;
            if ((hr[0] == 'H') != c->mbox_host) fail(QS_EINVAL, "mailbox handles of mixed kinds (QS_MBOX_HOST on some ranks only)");
            if (c->mbox_host) {
                char name[64] = {0};
                std::memcpy(name, hr + 1, 62);
                void *h = mbox_host_map(name, false);
                c->mbox_hmaps.push_back(h);
                bases[(size_t)r] = mbox_host_dev(h);
                continue;
            }
            hipIpcMemHandle_t h;
            std::memcpy(&h, hr, sizeof h);
            void *p = nullptr;
            HIPCHK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
            c->mbox_opened.push_back(p);
            bases[(size_t)r] = static_cast<char *>(p);
        }
        c->mbox_peers.ensure(sizeof(char *) * bases.size());
        HIPCHK(hipMemcpy(c->mbox_peers.p, bases.data(), sizeof(char *) * bases.size(), hipMemcpyHostToDevice));
        c->mbox_on = true;
        return QS_OK;
    } catch (const QsError &e) {
        c->err = e.msg;
        return e.st;
    }
}

}  // extern "C"
