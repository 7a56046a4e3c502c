#!/bin/bash
# Builds an experimental variant of libqsched with extra defines into
# custom-k8s-scheduler_amd/libqsched_<tag>.so (run time: QSCHED_LIB=<path>).
# Usage: tools/var_build.sh <tag> "-DFOO -DBAR"
set -e
cd "$(dirname "$0")/../custom-k8s-scheduler_amd"
tag=$1; defs=$2
B=build_$tag
mkdir -p $B
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -ffp-contract=off -mllvm -amdgpu-atomic-optimizer-strategy=None $defs"
for f in qs_kernels qs_kernels_wide; do /opt/rocm/bin/hipcc $F -c csrc/$f.hip -o $B/$f.o & done
for f in qs_host qs_helpers qs_dist; do /opt/rocm/bin/hipcc $F -x hip -c csrc/$f.cpp -o $B/$f.o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libqsched_$tag.so $B/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
