#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.  Stops at the first
# crash/timeout (exit codes other than 0/1 from pytest).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
(command -v go && go version) > gpurun_out/probe.log 2>&1; nproc >> gpurun_out/probe.log; lscpu | head -20 >> gpurun_out/probe.log
rocm-smi --showproductname >> gpurun_out/probe.log 2>&1
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log | tail -20; exit 3; }
cat gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
if [ -n "$BENCH2" ]; then timeout -k 10 300 python -u bench.py $BENCH2 > gpurun_out/bench2.log 2>&1 || { echo "bench2 failed"; tail -20 gpurun_out/bench2.log; exit 4; }; cat gpurun_out/bench2.log; fi
cat gpurun_out/bench.log
if [ -n "$PROFILE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 5; }
  find gpurun_out/prof -name '*stats*' | head
fi
echo ALLDONE
