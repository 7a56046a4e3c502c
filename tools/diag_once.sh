set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
QS_DIAG=1 timeout -k 10 120 python tools/kprof.py 2>&1 | tail -4
