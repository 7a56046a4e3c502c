#!/bin/bash
# Iteration probe (round 4): the GPU tests named in $TESTS, then the probes named in $PROBES.
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t1.log | tail -40
  [ $rc -le 1 ] || exit $rc
fi
for p in $PROBES; do
  case $p in
    fw50) for m in 1 0 2; do timeout -k 10 120 custom-k8s-scheduler_amd/fw_latency 50000 3000 $m || exit 7; done ;;
    fw5) for m in 1 2; do timeout -k 10 120 custom-k8s-scheduler_amd/fw_latency 5000 5000 $m || exit 7; done ;;
    fwprof) timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/fwprof -o run --output-format csv -- custom-k8s-scheduler_amd/fw_latency 50000 3000 2 > gpurun_out/fwprof.log 2>&1 || exit 8
            find gpurun_out/fwprof -name '*kernel_stats*' -exec cat {} \; | cut -c1-200 ;;
    diag2) QSCHED_LIB=custom-k8s-scheduler_amd/libqsched_diag.so QS_RES_DIAG=1 timeout -k 10 200 python -u bench.py --leg config2 --no-cpu > gpurun_out/diag2.json 2> gpurun_out/diag2.err || exit 9
           grep QS_RES_DIAG gpurun_out/diag2.err | sort | uniq -c | head -20; cat gpurun_out/diag2.json ;;
    wide) timeout -k 10 200 python -u bench.py --leg wide > gpurun_out/leg_wide.json 2>gpurun_out/leg_wide.err || exit 9; cat gpurun_out/leg_wide.json ;;
    c2|c3|c4|c5) leg=config${p#c}; timeout -k 10 300 python -u bench.py --leg $leg > gpurun_out/leg_$p.json 2>gpurun_out/leg_$p.err || exit 9; cat gpurun_out/leg_$p.json ;;
  esac
done
echo ALLDONE
