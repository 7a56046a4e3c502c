#!/bin/bash
# Config-4 resident stream (slot statics) check: the normalizing resident parity cases, the
# config-4 stream time (+ busy split with the diagnostic library if built), then every config-4 /
# normalizing parity test.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_resident_stream_norm" -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/c4_res.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -12 gpurun_out/c4_res.log; [ $rc -eq 0 ] || exit $rc
QS_RES_DIAG=1 CFG=4 N=5000 P=150000 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/c4_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -4 gpurun_out/c4_sweep.log; [ $rc -eq 0 ] || exit $rc
if [ -f custom-k8s-scheduler_amd/libqsched_diag.so ]; then
  QSCHED_LIB=$PWD/custom-k8s-scheduler_amd/libqsched_diag.so QS_RES_DIAG=1 CFG=4 N=5000 P=30000 RUNS=lookahead:32 \
    timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/c4_diag.log 2>&1
  echo "diag rc=$?"; tail -4 gpurun_out/c4_diag.log
fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -k "config4 or norm or normalizing" -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/c4_par.log 2>&1
rc=$?; echo "c4par rc=$rc"; tail -8 gpurun_out/c4_par.log; [ $rc -eq 0 ] || exit $rc
echo C4DONE
