#!/bin/bash
# QS_RES_DIAG=1 runs of bench.py --leg config2 against each library in $LIBS (busy cycles per role).
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $LIBS; do
  QSCHED_LIB=custom-k8s-scheduler_amd/libqsched_$v.so QS_RES_DIAG=1 timeout -k 10 200 python -u bench.py --leg ${LEG:-config2} --no-cpu > gpurun_out/expd_${v}_${LEG:-config2}.json 2> gpurun_out/expd_${v}_${LEG:-config2}.err; rc=$?
  echo "$v rc=$rc"; grep "busy\|marks\|per window\|selector task" gpurun_out/expd_${v}_${LEG:-config2}.err | sort | uniq | head -4
  case $rc in 124|134|137|139) exit $rc ;; esac
done
echo ALLDONE
