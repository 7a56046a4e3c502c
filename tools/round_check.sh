#!/bin/bash
# One GPU call for a candidate tree: resident timing (+ busy-cycle split from the diag build),
# lookahead parity, then the rocprofv3 evidence for profiles/ and the bench line.
# Usage (repo root, through gpurun): bash tools/round_check.sh <tag>
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-r02}
if [ -f custom-k8s-scheduler_amd/libqsched_diag.so ]; then
  QSCHED_LIB=$PWD/custom-k8s-scheduler_amd/libqsched_diag.so QS_RES_DIAG=1 RUNS=lookahead:32 P=32000 \
    timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/rdb.log 2>&1 || exit 1
fi
NOWIN=1 bash tools/res_check.sh || exit 1
grep -q "tests rc=0" gpurun_out/rc_tests.log || exit 1
[ -n "$NOPROF" ] || bash tools/profile_fetch.sh $TAG || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
