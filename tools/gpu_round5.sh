#!/bin/bash
# Round-5 evidence in one GPU call: -m gpu suite + smoke + bench line (gpu_full.sh), rocprofv3
# kernel stats and PMC passes (profile_fetch.sh), framework-path latency (tools/fw_latency).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-r05}
export TMPDIR=/tmp
bash tools/gpu_full.sh $TAG || exit $?
( for a in "5000 5000 1" "5000 5000 2" "50000 3000 1" "50000 3000 2"; do
    timeout -k 10 120 custom-k8s-scheduler_amd/fw_latency $a || exit 7
  done ) > gpurun_out/fw_latency_$TAG.json || exit 7
cat gpurun_out/fw_latency_$TAG.json | cut -c1-200
bash tools/profile_fetch.sh $TAG || exit 8
ls gpurun_out/profiles_new | head -30
echo ROUNDDONE
