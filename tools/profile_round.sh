#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes (never combined with tracing domains), condensed by tools/summarize_pmc.py.
# Usage (on the GPU box): tools/profile_round.sh r01
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
rm -rf $OUT; mkdir -p $OUT profiles
ARGS="--steps 2 --warmup 1 --no-cpu"  # config 3 included: its k_la_stream_res row
PMC_ARGS="--steps 1 --warmup 1 --no-cpu --no-extra"  # the scan leg too
# heartbeat for the GPU pool's silence watchdog (counter passes print nothing for minutes)
( while sleep 45; do date >> $OUT/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
# (QS_GRAPH=0: rocprofv3 7.2's kernel trace crashed (SIGSEGV in the HIP runtime) on the batched
# leg's graph launch in round 5; the resident streams are single launches either way)
QS_GRAPH=0 QS_SYNC_EVERY=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
echo "trace done rc=$?"
# counter passes: cross-stream events (QS_HANDOFF=0: counter collection serialises dispatches, so a
# resolver waiting in-kernel for the other stream's lists would time out), individual launches
# (QS_GRAPH=0) and a host sync every 64
# windows (QS_SYNC_EVERY): rocprofv3's counter collection crashed (SIGSEGV) with thousands of
# dispatches in flight
# One FETCH_SIZE and one WRITE_SIZE pass per leg, each its own process: the headline run (config 2 +
# the scan leg), then configs 3, 4 and 4-gpu-scoring through --leg (round 6: one combined run
# crashed inside the counter collection with SIGSEGV, so a failing leg no longer takes the others)
PMC_SETS=""
for leg in main config3 config4 config4_gpu_scoring; do
    if [ $leg = main ]; then A="$PMC_ARGS --no-config3"; else A="--leg $leg --no-cpu"; fi
    for ctr in FETCH_SIZE WRITE_SIZE; do
        QS_HANDOFF=0 QS_GRAPH=0 QS_SYNC_EVERY=64 timeout -s KILL 240 rocprofv3 --pmc $ctr -d $OUT/${leg}_$ctr -o run --output-format csv -- python3 bench.py $A > $OUT/${leg}_$ctr.log 2>&1
        echo "$leg $ctr rc=$?"
        grep -a -v '^    @ ' $OUT/${leg}_$ctr.log | grep -a -i -B3 -A3 'sigsegv\|signal\|abort\|error' | head -30 > $OUT/${leg}_$ctr.err
    done
    f=$(find $OUT/${leg}_FETCH_SIZE -name '*counter_collection.csv' 2>/dev/null | head -1)
    w=$(find $OUT/${leg}_WRITE_SIZE -name '*counter_collection.csv' 2>/dev/null | head -1)
    [ -n "$f" ] && [ -n "$w" ] && PMC_SETS="$PMC_SETS $leg $f $w"
done
# configs 4 (normalizing lookahead) and 5 (batched): kernel-trace stats of their own streams
for cfg in "4 5000 150000 exact 1" "5 10000 200000 batched 0"; do
    set -- $cfg
    CFG=$1 N=$2 P=$3 MODE=$4 TA=$5 QS_GRAPH=0 QS_SYNC_EVERY=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        -d $OUT/cfg$1 -o run --output-format csv -- python3 tools/kprof.py > $OUT/cfg$1.log 2>&1
    echo "config $1 trace done rc=$?"
done
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) profiles/${TAG}_kernel_stats.csv
[ -n "$PMC_SETS" ] && python3 tools/summarize_pmc.py profiles/${TAG}_pmc_summary.csv $PMC_SETS
grep '^{' $OUT/trace.log | tail -1 > profiles/${TAG}_bench_under_rocprof.json || true
# keep gpurun_out small: drop the raw traces (the summaries are what is committed)
find $OUT -name '*.csv' -size +20M -delete
ls -la profiles
