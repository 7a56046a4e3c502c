#!/bin/bash
# Round 5: slot keys split over waves A/B + 5/6 (parity, then config 2 A/B against the one-wave form).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/custom-k8s-scheduler_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_resources.py tests/test_gpu_mailbox.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/par_r5l.log 2>&1; rc=$?; tail -2 gpurun_out/par_r5l.log; [ $rc -eq 0 ] || exit 3
for v in ${VS:-libqsched.so}; do
  QSCHED_LIB=$P/$v timeout -k 10 300 python -u bench.py --leg config2 --no-cpu > gpurun_out/leg_r5l_$v.json 2> gpurun_out/leg_r5l_$v.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/leg_r5l_$v.json'));print('$v', d['value'], d.get('ms_per_step'), d.get('check', d).get('placements_match'))"
done
RUNS=3 timeout -k 10 200 python -u tools/p99_probe.py > gpurun_out/p99_r5l.log 2>&1 || exit 6
grep -E "^run|boundary" gpurun_out/p99_r5l.log
for leg in wide config3; do
  timeout -k 10 300 python -u bench.py --leg $leg --no-cpu > gpurun_out/leg_${leg}_r5l.json 2>gpurun_out/leg_${leg}_r5l.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/leg_${leg}_r5l.json'));print('$leg', d['value'], d.get('ms_per_step'), d.get('check', d).get('placements_match'))"
done
echo ALLDONE
