#!/bin/bash
# Round 5: config-4 resolver variants (A/B in one call; each leg checks placements vs the oracle).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/custom-k8s-scheduler_amd
for v in ${VS:-libqsched.so}; do
  QSCHED_LIB=$P/$v timeout -k 10 300 python -u bench.py --leg ${LEG:-config4} --no-cpu > gpurun_out/leg_r5j_$v.json 2> gpurun_out/leg_r5j_$v.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/leg_r5j_$v.json'));print('$v', d['value'], d.get('ms_per_step'), d.get('check', d).get('placements_match'))"
done
echo ALLDONE
