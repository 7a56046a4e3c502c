set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/prof_r01; mkdir -p $OUT
for cfg in "4 5000 150000 exact 1" "5 10000 200000 batched 0"; do
    set -- $cfg
    CFG=$1 N=$2 P=$3 MODE=$4 TA=$5 QS_GRAPH=0 QS_SYNC_EVERY=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        -d $OUT/cfg$1 -o run --output-format csv -- python3 tools/kprof.py > $OUT/cfg$1.log 2>&1
    echo "config $1 trace done"
done
