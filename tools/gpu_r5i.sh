#!/bin/bash
# Round 5: resolver busy-cycle split (diagnostic build) on config 2 and config 4.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
D=$PWD/custom-k8s-scheduler_amd/libqsched_diag.so
for leg in config2 config4; do
  QSCHED_LIB=$D QS_RES_DIAG=1 timeout -k 10 300 python -u bench.py --leg $leg --no-cpu > gpurun_out/diag_$leg.json 2> gpurun_out/diag_$leg.err || exit 9
  echo "== $leg"; grep QS_RES_DIAG gpurun_out/diag_$leg.err | sort | uniq -c | sort -rn | head -12 | cut -c1-250
done
echo ALLDONE
