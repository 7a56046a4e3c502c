#!/bin/bash
# Config-4 resident stream check: the smallest normalizing resident cases first (each test under
# its own bound), then the rest of the norm parity, the r03 tests and the bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_resident_stream_norm" -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/c4_res.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -12 gpurun_out/c4_res.log; [ $rc -eq 0 ] || exit $rc
QS_RES_DIAG=1 CFG=4 N=5000 P=150000 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/c4_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -8 gpurun_out/c4_sweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "config4" -m gpu -x -v --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/c4_par.log 2>&1
rc=$?; echo "c4par rc=$rc"; tail -12 gpurun_out/c4_par.log; [ $rc -eq 0 ] || exit $rc
bash tools/r03_check.sh
