// qs_dist.cpp — multi-GPU entry points: one process per GPU, the node table sharded by contiguous
// ranges, one RCCL all-gather of top-L lists per lookahead window over xGMI.
//
// Why an all-gather of lists and not the per-pod key all-reduce of SURVEY.md §3.3: the exact
// lookahead resolves K pods from per-shard top-L lists, so one collective of K*GLp keys per rank
// replaces K latency-bound 8-byte all-reduces (SURVEY.md §7 H4 option 3).  Every rank then runs the
// same resolver over the same gathered lists and its replicated table, so placements and table
// updates are identical on all ranks without a second exchange.
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
    if (!cfg || !out || world < 1 || world > 16 || rank < 0 || rank >= world) return QS_EINVAL;
    if (world > 1 && !nccl_id) return QS_EINVAL;
    qs_status st = qs_open(cfg, device, out);
    // world == 1 with an id still builds a (one-rank) communicator: the RCCL path on one GPU
    if (st != QS_OK || !nccl_id) return st;
    qs_ctx *c = *out;
    c->rank = rank;
    c->world = world;
    ncclUniqueId id;
    std::memcpy(&id, nccl_id, sizeof id);
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, world, id, rank);
    if (r != ncclSuccess) {
        qs_close(c);
        *out = nullptr;
        return QS_EDEVICE;
    }
    c->comm = comm;
    return QS_OK;
}

}  // extern "C"
