#!/bin/bash
# Round 5: selector chunking (QS_RES_G) x prefetch variant on config 2; batched claim walk.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=$PWD/custom-k8s-scheduler_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_batched.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bat_r5e.log 2>&1; rc=$?; tail -2 gpurun_out/bat_r5e.log; [ $rc -le 1 ] || exit $rc
for lib in libqsched_old.so libqsched.so; do
  echo "== config5 $lib"
  QSCHED_LIB=$P/$lib CFG=5 N=10000 P=200000 MODE=batched TA=0 QS_GRAPH=0 timeout -k 10 300 python -u tools/kprof.py > gpurun_out/kprof_c5_$lib.log 2>&1 || exit 8
  cut -c1-400 gpurun_out/kprof_c5_$lib.log
  QSCHED_LIB=$P/$lib timeout -k 10 300 python -u bench.py --leg config5 > gpurun_out/leg_c5_$lib.json 2> gpurun_out/leg_c5_$lib.err || exit 9
  python -c "import json;d=json.load(open('gpurun_out/leg_c5_$lib.json'));print('config5', d['value'], d['check']['placements_match'])"
done
for v in "prod 0" "prod 4" "e11 4"; do
  set -- $v
  if [ $1 = prod ]; then L=$P/libqsched.so; else L=$P/libqsched_$1.so; fi
  echo "== $1 G=$2"
  QSCHED_LIB=$L QS_RES_G=$2 QS_RES_DIAG=2 RUNS=1 timeout -k 10 200 python -u tools/p99_probe.py > gpurun_out/p99d_r5e_$1_$2.log 2>&1 || exit 6
  grep -E "QS_RES_DIAG (last|prefetch|window)" gpurun_out/p99d_r5e_$1_$2.log
  QSCHED_LIB=$L QS_RES_G=$2 RUNS=3 timeout -k 10 200 python -u tools/p99_probe.py > gpurun_out/p99_r5e_$1_$2.log 2>&1 || exit 6
  grep -E "^run|boundary|k=1 " gpurun_out/p99_r5e_$1_$2.log
  QSCHED_LIB=$L QS_RES_G=$2 timeout -k 10 200 python -u bench.py --leg config2 --no-cpu > gpurun_out/leg_c2_r5e_$1_$2.json 2>gpurun_out/leg_c2_r5e_$1_$2.err || exit 9
  cut -c1-300 gpurun_out/leg_c2_r5e_$1_$2.json
done
echo ALLDONE
