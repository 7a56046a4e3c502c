#!/bin/bash
# Round 5: parallel-round batched claim (parity, kernel time, config 5 leg) for 16 / 8 / 4 waves.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/custom-k8s-scheduler_amd
for v in ${VS:-libqsched.so}; do
  echo "== $v"
  QSCHED_LIB=$P/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_batched.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bat_r5g_$v.log 2>&1; rc=$?; tail -1 gpurun_out/bat_r5g_$v.log; [ $rc -eq 0 ] || exit 3
  QSCHED_LIB=$P/$v CFG=5 N=10000 P=200000 MODE=batched TA=0 QS_GRAPH=0 timeout -k 10 300 python -u tools/kprof.py > gpurun_out/kprof_c5_r5g_$v.log 2>&1 || exit 8
  cut -c1-300 gpurun_out/kprof_c5_r5g_$v.log | tail -1
  QSCHED_LIB=$P/$v timeout -k 10 300 python -u bench.py --leg config5 > gpurun_out/leg_c5_r5g_$v.json 2> gpurun_out/leg_c5_r5g_$v.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/leg_c5_r5g_$v.json'));print('config5', d['value'], d['check']['placements_match'], d['check']['keys_match'])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_adversarial.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/adv_r5g.log 2>&1; rc=$?; tail -1 gpurun_out/adv_r5g.log; [ $rc -eq 0 ] || exit 4
if [ -f $P/libqsched_cdiag.so ]; then
  QSCHED_LIB=$P/libqsched_cdiag.so CFG=5 N=10000 P=200000 MODE=batched TA=0 QS_GRAPH=0 timeout -k 10 300 python -u tools/kprof.py > gpurun_out/cdiag_r5g.log 2>&1 || exit 10
  grep "claim diag" gpurun_out/cdiag_r5g.log | tail -1
fi
echo ALLDONE
