#!/bin/bash
# Round 5: batched select with the merge inside the launch (A/B against QS_BATCH_FUSED_MERGE=0).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batched.py tests/test_gpu_adversarial.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bat_r5h.log 2>&1; rc=$?; tail -1 gpurun_out/bat_r5h.log; [ $rc -eq 0 ] || exit 3
for fm in 1 0 1; do
  QS_BATCH_FUSED_MERGE=$fm CFG=5 N=10000 P=200000 MODE=batched TA=0 QS_GRAPH=0 timeout -k 10 300 python -u tools/kprof.py > gpurun_out/kprof_c5_r5h_$fm.log 2>&1 || exit 8
  echo "fused=$fm $(tail -1 gpurun_out/kprof_c5_r5h_$fm.log | cut -c1-300)"
  QS_BATCH_FUSED_MERGE=$fm timeout -k 10 300 python -u bench.py --leg config5 > gpurun_out/leg_c5_r5h_$fm.json 2> gpurun_out/leg_c5_r5h_$fm.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/leg_c5_r5h_$fm.json'));print('config5 fused=$fm', d['value'], d['check']['placements_match'], d['check']['keys_match'], d['check']['table_match'])"
done
echo ALLDONE
