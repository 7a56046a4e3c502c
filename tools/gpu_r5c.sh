#!/bin/bash
# Window-boundary variants: resolver-only diagnostics (QS_RES_DIAG=2), plain p99 probe, parity.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARS:-prod e3 e6 e7}; do
  if [ $v = prod ]; then L=$PWD/custom-k8s-scheduler_amd/libqsched.so; else L=$PWD/custom-k8s-scheduler_amd/libqsched_$v.so; fi
  QSCHED_LIB=$L QS_RES_DIAG=2 RUNS=2 timeout -k 10 200 python -u tools/p99_probe.py > gpurun_out/p99d_r5c_$v.log 2>&1 || { echo "probe $v failed"; tail -3 gpurun_out/p99d_r5c_$v.log; exit 6; }
  QSCHED_LIB=$L RUNS=4 timeout -k 10 200 python -u tools/p99_probe.py > gpurun_out/p99_r5c_$v.log 2>&1 || { echo "probe $v failed"; tail -3 gpurun_out/p99_r5c_$v.log; exit 6; }
  echo "== $v"; grep -E "QS_RES_DIAG (resolver|window|prefetch|selector 0)" gpurun_out/p99d_r5c_$v.log | tail -4; grep -E "^run|boundary|k=1 " gpurun_out/p99_r5c_$v.log
  if [ $v != prod ]; then
    QSCHED_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "resident_stream or config2_full_lookahead or lookahead_windows" --maxfail=3 --timeout 200 --timeout-method thread > gpurun_out/par_r5c_$v.log 2>&1
    prc=$?; echo "parity $v rc=$prc"; tail -1 gpurun_out/par_r5c_$v.log
    if [ $prc -ne 0 ] && [ $prc -ne 1 ]; then exit $prc; fi
  fi
done
echo ALLDONE
