#!/bin/bash
# A/B of library variants in one GPU call (DESIGN.md's "measured in one call" numbers): every
# library in $VS (built by tools/exp_variant.py next to libqsched.so) runs the bench leg $LEG
# (config2 default; each leg checks its placements against the oracle).
# Usage (through gpurun): VS="libqsched.so libqsched_x.so" LEG=config4 bash tools/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/custom-k8s-scheduler_amd
for v in ${VS:-libqsched.so}; do
  QSCHED_LIB=$P/$v timeout -k 10 300 python -u bench.py --leg ${LEG:-config2} --no-cpu > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', d['value'], d.get('ms_per_step'), d.get('check', d).get('placements_match'))"
done
echo ALLDONE
