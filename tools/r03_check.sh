#!/bin/bash
# Round-3 GPU check: the new tests first, then (ALL=1) the whole -m gpu suite, smoke and the bench.
# Usage (repo root, through gpurun): bash tools/r03_check.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_scale.py tests/test_gpu_recovery.py tests/test_gpu_mailbox.py"}
timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r03_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/r03_tests.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$SMOKE" ]; then
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 500 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_r03.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r03.log; exit 4; }
  tail -c 6000 gpurun_out/bench_r03.log
fi
echo ALLDONE
