#!/bin/bash
# One GPU session of round-5 iteration: named pytest selection, then optional probes / bench.
# Usage (repo root, through gpurun): TESTS="..." PROBE=1 BENCH="--no-cpu" bash tools/gpu_step.sh tag
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-step}
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -v --maxfail=${MAXFAIL:-5} --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_$TAG.log | tail -3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$PROBE" ]; then
  timeout -k 10 300 python -u tools/p99_probe.py > gpurun_out/p99_$TAG.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/p99_$TAG.log; exit 3; }
  head -12 gpurun_out/p99_$TAG.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.err; exit 4; }
  cut -c1-600 gpurun_out/bench_$TAG.json
fi
echo ALLDONE
