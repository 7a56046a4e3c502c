#!/bin/bash
# Resident-stream check (GPU box): config-2 / config-3 stream times resident (with the QS_RES_DIAG
# time split) and per-window, then the lookahead parity tests and goldens.
# Usage (repo root, through gpurun): bash tools/res_check.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
QS_RES_DIAG=1 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/rc_res.log 2>&1 || exit 1
QS_RES_DIAG=1 CFG=3 N=50000 P=1000000 RUNS=lookahead:32 timeout -k 10 200 python -u tools/la_sweep.py > gpurun_out/rc_res3.log 2>&1 || exit 1
[ -n "$NOWIN" ] || { QS_RESIDENT=0 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/rc_win.log 2>&1 || exit 1; }
[ -n "$NOTEST" ] || { timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_golden.py} -m gpu -q -x --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/rc_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/rc_tests.log; }
