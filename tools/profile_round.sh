#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes (never combined with tracing domains), condensed by tools/summarize_pmc.py.
# Usage (on the GPU box): tools/profile_round.sh r01
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
rm -rf $OUT; mkdir -p $OUT profiles
ARGS="--steps 2 --warmup 1 --no-cpu"  # config 3 included: its k_la_stream_res row
PMC_ARGS="--steps 1 --warmup 1 --no-cpu --no-extra"  # the scan leg too; configs 3, 4, 4-gpu-scoring and 5
# heartbeat for the GPU pool's silence watchdog (counter passes print nothing for minutes)
( while sleep 45; do date >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
# (QS_GRAPH=0: rocprofv3 7.2's kernel trace crashed (SIGSEGV in the HIP runtime) on the batched
# leg's graph launch in round 5; the resident streams are single launches either way)
QS_GRAPH=0 QS_SYNC_EVERY=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
echo "trace done"
# counter passes: cross-stream events (QS_HANDOFF=0: counter collection serialises dispatches, so a
# resolver waiting in-kernel for the other stream's lists would time out), individual launches
# (QS_GRAPH=0) and a host sync every 64
# windows (QS_SYNC_EVERY): rocprofv3's counter collection crashed (SIGSEGV) with thousands of
# dispatches in flight
QS_HANDOFF=0 QS_GRAPH=0 QS_SYNC_EVERY=64 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/fetch.log 2>&1
echo "fetch done"
QS_HANDOFF=0 QS_GRAPH=0 QS_SYNC_EVERY=64 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/write.log 2>&1
echo "write done"
# configs 4 (normalizing lookahead) and 5 (batched): kernel-trace stats of their own streams
for cfg in "4 5000 150000 exact 1" "5 10000 200000 batched 0"; do
    set -- $cfg
    CFG=$1 N=$2 P=$3 MODE=$4 TA=$5 QS_GRAPH=0 QS_SYNC_EVERY=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        -d $OUT/cfg$1 -o run --output-format csv -- python3 tools/kprof.py > $OUT/cfg$1.log 2>&1
    echo "config $1 trace done"
done
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) profiles/${TAG}_kernel_stats.csv
python3 tools/summarize_pmc.py $(find $OUT/fetch -name '*counter_collection.csv' | head -1) \
    $(find $OUT/write -name '*counter_collection.csv' | head -1) profiles/${TAG}_pmc_summary.csv
grep '^{' $OUT/trace.log | tail -1 > profiles/${TAG}_bench_under_rocprof.json || true
# keep gpurun_out small: drop the raw traces (the summaries are what is committed)
find $OUT -name '*.csv' -size +20M -delete
ls -la profiles
