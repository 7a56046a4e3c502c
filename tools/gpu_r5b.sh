#!/bin/bash
# Round-5 iteration: FitError + framework tests, framework-path latency, boundary-variant p99 probes.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fiterror.py tests/test_gpu_framework.py tests/test_gpu_parity.py::test_resident_stream -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/pytest_r5b.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_r5b.log | tail -2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
FW=custom-k8s-scheduler_amd/fw_latency
for args in "5000 5000 1" "50000 3000 1" "50000 3000 2"; do
  timeout -k 10 120 $FW $args > gpurun_out/fw_one.json || exit 5; tail -1 gpurun_out/fw_one.json
done > gpurun_out/fw_r5b.jsonl
QS_UNPACK_PAR_MIN=100000000 timeout -k 10 120 $FW 50000 3000 1 > gpurun_out/fw_one.json || exit 5; tail -1 gpurun_out/fw_one.json >> gpurun_out/fw_r5b.jsonl
cat gpurun_out/fw_r5b.jsonl
for v in prod e1 e2 e3 e4 e5; do
  if [ $v = prod ]; then L=$PWD/custom-k8s-scheduler_amd/libqsched.so; else L=$PWD/custom-k8s-scheduler_amd/libqsched_$v.so; fi
  QSCHED_LIB=$L RUNS=4 timeout -k 10 200 python -u tools/p99_probe.py > gpurun_out/p99_r5b_$v.log 2>&1 || { echo "probe $v failed"; tail -3 gpurun_out/p99_r5b_$v.log; exit 6; }
  echo "== $v"; grep -E "^run|boundary|k=1 " gpurun_out/p99_r5b_$v.log
  if [ $v = e3 ] || [ $v = e4 ] || [ $v = e5 ]; then
    QSCHED_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "resident_stream or config2_full_lookahead or lookahead_windows" --maxfail=3 --timeout 200 --timeout-method thread > gpurun_out/par_r5b_$v.log 2>&1
    prc=$?; echo "parity $v rc=$prc"; tail -1 gpurun_out/par_r5b_$v.log
    if [ $prc -ne 0 ] && [ $prc -ne 1 ]; then exit $prc; fi
  fi
done
echo ALLDONE
