#!/bin/bash
# Quick config-4 check: resident norm parity, stream time, busy split + step marks (diag library),
# config-2 time and busy split.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DLIB=$PWD/custom-k8s-scheduler_amd/libqsched_diag.so
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_resident_stream_norm" "tests/test_gpu_parity.py::test_resident_stream" -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/q_par.log 2>&1
rc=$?; echo "par rc=$rc"; tail -3 gpurun_out/q_par.log; [ $rc -eq 0 ] || exit $rc
for cfg in "4 5000 150000" "2 5000 100000"; do
  set -- $cfg
  QS_RES_DIAG=1 CFG=$1 N=$2 P=$3 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/q_c$1.log 2>&1
  echo "c$1 rc=$?"; grep -E "resolver|lookahead" gpurun_out/q_c$1.log | tail -2
  QSCHED_LIB=$DLIB QS_RES_DIAG=1 CFG=$1 N=$2 P=30000 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/q_c$1d.log 2>&1
  echo "c$1 diag rc=$?"; grep -E "busy|marks" gpurun_out/q_c$1d.log | tail -2
done
echo QDONE
