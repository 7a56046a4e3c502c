#!/bin/bash
# Two selector workgroups per CU: resident parity across geometries, config-3 full-size checks,
# config-3 / config-2 stream times with the selector phase split.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest "tests/test_gpu_parity.py::test_resident_stream" "tests/test_gpu_parity.py::test_resident_declines_large_tables" \
    "tests/test_gpu_parity.py::test_resident_stream_norm" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/c3_par.log 2>&1
rc=$?; echo "par rc=$rc"; tail -3 gpurun_out/c3_par.log; [ $rc -eq 0 ] || exit $rc
QS_RES_DIAG=1 CFG=3 N=50000 P=200000 RUNS=lookahead:32 timeout -k 10 200 python -u tools/la_sweep.py > gpurun_out/c3_sweep.log 2>&1
rc=$?; echo "c3 rc=$rc"; grep -E "resolver|selector|lookahead" gpurun_out/c3_sweep.log | tail -3; [ $rc -eq 0 ] || exit $rc
QS_RES_DIAG=1 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/c2_sweep.log 2>&1
rc=$?; echo "c2 rc=$rc"; grep -E "resolver|lookahead" gpurun_out/c2_sweep.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/c3_scale.log 2>&1
rc=$?; echo "scale rc=$rc"; tail -3 gpurun_out/c3_scale.log
