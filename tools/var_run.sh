#!/bin/bash
# Times config 4 (and 2) with each experimental library named on the command line (diag output).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for tag in "$@"; do
  for cfg in ${CFGS:-4}; do
    QSCHED_LIB=$PWD/custom-k8s-scheduler_amd/libqsched_$tag.so QS_RES_DIAG=1 CFG=$cfg N=5000 P=${P:-30000} RUNS=lookahead:32 \
      timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/var_${tag}_$cfg.log 2>&1
    echo "== $tag c$cfg rc=$?"; grep -E "busy|marks|lookahead|resolver" gpurun_out/var_${tag}_$cfg.log | tail -4
  done
done
