set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
timeout -k 10 120 python tools/kprof.py 2>&1
CFG=3 N=50000 P=200000 timeout -k 10 120 python tools/kprof.py 2>&1
QS_DIAG=1 timeout -k 10 120 python tools/kprof.py 2>&1 | grep -v "^cfg" | head -1
