#!/bin/bash
# Round-end GPU check: the whole -m gpu suite, smoke(), then the default bench line.
# Usage (repo root, through gpurun): bash tools/gpu_full.sh <tag>
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-r04}
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" gpurun_out/gputest_$TAG.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || exit 5
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 6
cut -c1-400 gpurun_out/bench_$TAG.json
echo ALLDONE
