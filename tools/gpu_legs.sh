#!/bin/bash
# Bench legs in one GPU call (each leg checks its placements against the oracle):
#   LEGS="config4 config4_gpu_scoring" TESTS="tests/test_gpu_parity.py" bash tools/gpu_legs.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/legs_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/legs_pytest.log
  if [ $rc -ne 0 ]; then grep -a "^E \|FAILED\|Error" gpurun_out/legs_pytest.log | head -20; exit $rc; fi
fi
for l in ${LEGS:-config2}; do
  timeout -k 10 300 python -u bench.py --leg $l --no-cpu > gpurun_out/leg_$l.json 2> gpurun_out/leg_$l.err || { tail -5 gpurun_out/leg_$l.err; exit 9; }
  python -c "import json;d=json.load(open('gpurun_out/leg_$l.json'));c=d.get('check',{});print('$l', d['value'], d.get('ms_per_step'), c.get('placements_match'), c.get('keys_match'), c.get('table_match'), (d.get('roofline') or {}).get('frac'))"
done
echo ALLDONE
