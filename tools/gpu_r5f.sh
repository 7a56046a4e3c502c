#!/bin/bash
# Round 5: window boundary after the pod-record spill fix; selector chunking (QS_RES_G); legs.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/custom-k8s-scheduler_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "resident_stream or config2_full_lookahead or lookahead_windows" --timeout 200 --timeout-method thread > gpurun_out/par_r5f.log 2>&1; rc=$?; tail -1 gpurun_out/par_r5f.log; [ $rc -le 1 ] || exit $rc
for g in ${GS:-0 4}; do
  echo "== G=$g"
  QS_RES_G=$g QS_RES_DIAG=2 RUNS=1 timeout -k 10 200 python -u tools/p99_probe.py > gpurun_out/p99d_r5f_$g.log 2>&1 || exit 6
  grep -E "QS_RES_DIAG (last|prefetch|window)" gpurun_out/p99d_r5f_$g.log
  QS_RES_G=$g RUNS=3 timeout -k 10 200 python -u tools/p99_probe.py > gpurun_out/p99_r5f_$g.log 2>&1 || exit 6
  grep -E "^run|boundary|k=1 " gpurun_out/p99_r5f_$g.log
  QS_RES_G=$g timeout -k 10 200 python -u bench.py --leg config2 --no-cpu > gpurun_out/leg_c2_r5f_$g.json 2>gpurun_out/leg_c2_r5f_$g.err || exit 9
  cut -c1-250 gpurun_out/leg_c2_r5f_$g.json
done
for leg in ${LEGS:-config4 wide config3}; do
  timeout -k 10 300 python -u bench.py --leg $leg --no-cpu > gpurun_out/leg_${leg}_r5f.json 2>gpurun_out/leg_${leg}_r5f.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/leg_${leg}_r5f.json'));print('$leg', d['value'], d.get('ms_per_step'), d.get('check', d).get('placements_match'))"
done
QS_RES_G=4 timeout -k 10 300 python -u bench.py --leg config4 --no-cpu > gpurun_out/leg_config4g4_r5f.json 2>gpurun_out/leg_config4g4_r5f.err || exit 9
python -c "import json;d=json.load(open('gpurun_out/leg_config4g4_r5f.json'));print('config4 G=4', d['value'], d.get('ms_per_step'), d['check'].get('placements_match'))"
echo ALLDONE
