#!/bin/bash
# Timing variant whose compact-kernel header is a given file (e.g. an earlier commit's), linked with
# the product's other objects: tools/variant_from.sh NAME <qs_kernels.hpp path>  -> libqsched_NAME.so
set -e
cd "$(dirname "$0")/../custom-k8s-scheduler_amd"
d=build/var_$1; rm -rf $d; cp -r csrc $d; cp "$2" $d/qs_kernels.hpp
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -ffp-contract=off -Wno-unused-function -mllvm -amdgpu-atomic-optimizer-strategy=None -I../include"
/opt/rocm/bin/hipcc $F -c $d/qs_kernels.hip -o $d/qs_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libqsched_$1.so $d/qs_kernels.o build/qs_kernels_wide.o \
    build/qs_kernels_res.o build/qs_kernels_res_wide.o build/qs_host.o build/qs_helpers.o build/qs_dist.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo libqsched_$1.so
