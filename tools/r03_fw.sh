#!/bin/bash
# Framework-path latency + config-4 timing + the tests touching qs_score_pod / qs_reserve.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 custom-k8s-scheduler_amd/fw_latency 5000 2000 1 > gpurun_out/fw.log 2>&1; echo "fw rc=$?"; cat gpurun_out/fw.log
timeout -k 10 60 custom-k8s-scheduler_amd/fw_latency 5000 2000 0 >> gpurun_out/fw.log 2>&1; echo "fw0 rc=$?"; tail -1 gpurun_out/fw.log
QS_RES_DIAG=1 CFG=4 N=5000 P=150000 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/c4_sweep.log 2>&1
echo "sweep rc=$?"; tail -2 gpurun_out/c4_sweep.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_framework.py tests/test_framework_native.py tests/test_gpu_recovery.py \
    tests/test_gpu_adversarial.py tests/test_gpu_wide.py "tests/test_gpu_parity.py" -k "not full_persistent" -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fwt.log 2>&1
echo "tests rc=$?"; tail -4 gpurun_out/fwt.log
