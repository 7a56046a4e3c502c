set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread -k "config4" 2>&1 | tail -3
CFG=4 TA=1 P=150000 timeout -k 10 120 python tools/kprof.py 2>&1
