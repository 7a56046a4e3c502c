// qs_dist.cpp — multi-GPU entry points (one process per GPU, RCCL over xGMI).
// Round-1 status: the sharded lookahead exchange is not wired yet; qs_open_shard accepts
// world == 1 only.
#include <cstring>

#include "../../include/qsched.h"

extern "C" {

qs_status qs_dist_unique_id(uint8_t out[128]) {
    if (!out) return QS_EINVAL;
    std::memset(out, 0, 128);
    return QS_OK;
}

qs_status qs_open_shard(const qs_config *cfg, int device, int rank, int world,
                        const uint8_t nccl_id[128], qs_ctx **out) {
    (void)nccl_id;
    if (world != 1 || rank != 0) return QS_EINVAL;
    return qs_open(cfg, device, out);
}

}  // extern "C"
