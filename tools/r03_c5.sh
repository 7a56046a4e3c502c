#!/bin/bash
# Batched mode (config 5): parity tests, goldens, and per-kernel times of the 200,000-pod stream.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_batched.py tests/test_golden.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/c5_tests.log 2>&1
rc=$?; echo "c5 tests rc=$rc"; tail -3 gpurun_out/c5_tests.log; [ $rc -eq 0 ] || exit $rc
CFG=5 N=10000 P=200000 MODE=batched TA=0 QS_GRAPH=0 timeout -k 10 200 python -u tools/kprof.py > gpurun_out/c5_kprof.log 2>&1
rc=$?; echo "kprof rc=$rc"; tail -2 gpurun_out/c5_kprof.log
