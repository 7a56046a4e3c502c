set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 ./tests/native/test_framework --gpu 2>&1 | tail -20
