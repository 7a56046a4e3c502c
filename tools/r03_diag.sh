#!/bin/bash
# Per-role busy cycles of the resident resolver (diagnostic build, tools/diag_build.sh) for
# configs 2 and 4, the selector phase split of config 3, and the plain library's stream times.
# Usage (repo root, through gpurun): bash tools/r03_diag.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DLIB=$PWD/custom-k8s-scheduler_amd/libqsched_diag.so
run() {  # tag, then env assignments for la_sweep
  local tag=$1; shift
  env "$@" RUNS=lookahead:32 timeout -k 10 ${TMO:-150} python -u tools/la_sweep.py > gpurun_out/diag_$tag.log 2>&1
  local rc=$?
  echo "== $tag rc=$rc"; grep -v "^\s*$" gpurun_out/diag_$tag.log | tail -6
  return $rc
}
run c2 QS_RES_DIAG=1 && \
run c2d QSCHED_LIB=$DLIB QS_RES_DIAG=1 P=32000 && \
run c4 QS_RES_DIAG=1 CFG=4 N=5000 P=150000 && \
run c4d QSCHED_LIB=$DLIB QS_RES_DIAG=1 CFG=4 N=5000 P=30000 && \
run c3 QS_RES_DIAG=1 CFG=3 N=50000 P=200000 && \
echo DIAGDONE
