#!/bin/bash
# Round-6 evidence after tools/gpu_full.sh: framework-path latency (tools/fw_latency, with the slow
# calls' launch / wait split, QS_SCORE_DIAG=1), rocprofv3 kernel stats and PMC passes
# (profile_fetch.sh).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-r06}
export TMPDIR=/tmp
( for a in "5000 5000 1" "5000 5000 0" "5000 5000 2" "5000 5000 2" "50000 3000 2" "50000 3000 1"; do
    QS_SCORE_DIAG=1 timeout -k 10 120 custom-k8s-scheduler_amd/fw_latency $a 2>> gpurun_out/fw_diag_$TAG.txt || exit 7
  done ) > gpurun_out/fw_latency_$TAG.json || exit 7
cut -c1-260 gpurun_out/fw_latency_$TAG.json
cat gpurun_out/fw_diag_$TAG.txt | head -20
# the diagnostic build's busy cycles and step marks
if [ -f custom-k8s-scheduler_amd/libqsched_diag.so ]; then
  for l in config2 config4; do
    QSCHED_LIB=$PWD/custom-k8s-scheduler_amd/libqsched_diag.so QS_RES_DIAG=1 timeout -k 10 200 python -u bench.py --leg $l --no-cpu > gpurun_out/diag_$l.json 2> gpurun_out/diag_$l.err || exit 9
    grep -a "busy cycles\|step marks" gpurun_out/diag_$l.err | sort | uniq > gpurun_out/diag_${TAG}_$l.txt
    cat gpurun_out/diag_${TAG}_$l.txt
  done
fi
bash tools/profile_fetch.sh $TAG || exit 8
ls gpurun_out/profiles_new | head -40
echo ROUNDDONE
