cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pmcprobe; export TMPDIR=/tmp
run() { echo "== $1"; shift; timeout -s KILL 200 "$@" > gpurun_out/pmcprobe/last.log 2>&1; rc=$?; grep -v "^    @" gpurun_out/pmcprobe/last.log | grep -E "metric|workload|SIGSEGV|Abort|rror" | cut -c1-300 | head -5; echo "rc=$rc"; return $rc; }
QS_GRAPH=0 QS_SYNC_EVERY=64 run bench-noscan-sync rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcprobe/a -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-config3 --no-scan || exit 1
echo ALLOK
