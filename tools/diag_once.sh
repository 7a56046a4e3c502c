set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
QS_FUSED=0 QS_RESOLVER_WAVES=8 timeout -k 10 120 python tools/kprof.py 2>&1
