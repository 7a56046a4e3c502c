set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batched.py -x -q --timeout 300 --timeout-method thread 2>&1 | grep -v "claim diag" | tail -3
MODE=batched CFG=5 N=10000 P=200000 timeout -k 10 120 python tools/kprof.py 2>&1
