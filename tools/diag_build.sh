#!/bin/bash
# Builds the diagnostic variant of libqsched (resident resolver busy-cycle stamps,
# -DQS_RES_DIAG_BLOCK) as custom-k8s-scheduler_amd/libqsched_diag.so without touching the in-tree
# library; select it at run time with QSCHED_LIB=<path> and QS_RES_DIAG=1.
# DEF=-DQS_CLAIM_DIAG OUT=libqsched_cdiag.so: the batched claim's phase clocks instead.
set -e
cd "$(dirname "$0")/../custom-k8s-scheduler_amd"
B=build_${OUT:-diag}
mkdir -p $B
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -ffp-contract=off -I../include -mllvm -amdgpu-atomic-optimizer-strategy=None ${DEF:--DQS_RES_DIAG_BLOCK}"
for f in qs_kernels qs_kernels_wide qs_kernels_res qs_kernels_res_wide; do /opt/rocm/bin/hipcc $F -c csrc/$f.hip -o $B/$f.o & done
for f in qs_host qs_helpers qs_dist; do /opt/rocm/bin/hipcc $F -x hip -c csrc/$f.cpp -o $B/$f.o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ${OUT:-libqsched_diag.so} $B/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
