#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes (never combined with tracing domains).  Usage: tools/profile_round.sh r01
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
rm -rf $OUT; mkdir -p $OUT profiles
ARGS="--steps 2 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) profiles/${TAG}_kernel_stats.csv
cp $(find $OUT/fetch -name '*counter_collection.csv' | head -1) profiles/${TAG}_pmc_fetch.csv
cp $(find $OUT/write -name '*counter_collection.csv' | head -1) profiles/${TAG}_pmc_write.csv
tail -1 $OUT/trace.log > profiles/${TAG}_bench_under_rocprof.json || true
ls -la profiles
