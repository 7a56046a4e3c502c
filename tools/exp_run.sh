#!/bin/bash
# Timing experiments: bench.py --leg $LEG against each library named in $LIBS (custom-k8s-scheduler_amd/
# libqsched_<v>.so; "prod" = the product library).  Stops at the first fault or time limit.
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $LIBS; do
  lib=custom-k8s-scheduler_amd/libqsched_$v.so; [ "$v" = prod ] && lib=custom-k8s-scheduler_amd/libqsched.so
  QSCHED_LIB=$lib timeout -k 10 200 python -u bench.py --leg ${LEG:-config2} --no-cpu > gpurun_out/exp_$v.json 2> gpurun_out/exp_$v.err; rc=$?
  echo "$v rc=$rc $(cut -c1-60 gpurun_out/exp_$v.json | head -1) $(grep -o '"value": [0-9.]*' gpurun_out/exp_$v.json | head -1) $(grep -o '"placements_match": [a-z]*' gpurun_out/exp_$v.json | head -1)"
  case $rc in 124|134|137|139) exit $rc ;; esac
done
echo ALLDONE
