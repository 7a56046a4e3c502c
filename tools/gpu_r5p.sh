#!/bin/bash
# Round 5: batched claim staging with unconditional gathers (A/B against the previous tree's claim).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/custom-k8s-scheduler_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_batched.py tests/test_gpu_adversarial.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bat_r5p.log 2>&1; rc=$?; tail -1 gpurun_out/bat_r5p.log; [ $rc -eq 0 ] || exit 3
for v in libqsched.so libqsched_old.so libqsched.so libqsched_old.so; do
  QSCHED_LIB=$P/$v CFG=5 N=10000 P=200000 MODE=batched TA=0 QS_GRAPH=0 timeout -k 10 300 python -u tools/kprof.py > gpurun_out/kprof_r5p_$v.log 2>&1 || exit 8
  echo "$v $(tail -1 gpurun_out/kprof_r5p_$v.log | grep -o 'resolve: .*')"
  QSCHED_LIB=$P/$v timeout -k 10 300 python -u bench.py --leg config5 > gpurun_out/leg_r5p_$v.json 2> gpurun_out/leg_r5p_$v.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/leg_r5p_$v.json'));print('$v config5', d['value'], d['check']['placements_match'])"
done
echo ALLDONE
