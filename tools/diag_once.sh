set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -x -q --timeout 120 --timeout-method thread -k "config4" > gpurun_out/t4.log 2>&1 || { tail -30 gpurun_out/t4.log; exit 1; }
tail -2 gpurun_out/t4.log
CFG=4 N=5000 P=150000 TA=1 timeout -k 10 120 python tools/kprof.py 2>&1 | head -1
