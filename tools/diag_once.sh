set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python tools/scan_probe.py 2>&1 | tail -1
QS_SCAN_BLOCKS=2048 timeout -k 10 200 python tools/scan_probe.py 2>&1 | tail -1
QS_SCAN_BLOCKS=1024 timeout -k 10 200 python tools/scan_probe.py 2>&1 | tail -1
timeout -k 10 400 python -u -m pytest tests/test_gpu_framework.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
