#!/bin/bash
# Round 5: selector finish-time distribution (QS_RES_DIAG=2) and unpack-pool sizing of the framework path.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/custom-k8s-scheduler_amd/libqsched.so
QSCHED_LIB=$L QS_RES_DIAG=2 RUNS=1 timeout -k 10 200 python -u tools/p99_probe.py > gpurun_out/p99d_r5d.log 2>&1 || { echo "probe failed"; tail -3 gpurun_out/p99d_r5d.log; exit 6; }
grep -E "QS_RES_DIAG" gpurun_out/p99d_r5d.log
for t in 3 5 7; do
  echo "== unpack helpers $t"
  QS_UNPACK_THREADS=$t timeout -k 10 120 custom-k8s-scheduler_amd/fw_latency 50000 3000 1 || exit 7
  QS_UNPACK_THREADS=$t timeout -k 10 120 custom-k8s-scheduler_amd/fw_latency 5000 5000 1 || exit 7
done
echo ALLDONE
