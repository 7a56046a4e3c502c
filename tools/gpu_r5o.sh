#!/bin/bash
# Round 5: scan grid size and quads in flight with the non-temporal column loads.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
P=$PWD/custom-k8s-scheduler_amd
for b in 0 512 1024 2048; do
  if [ $b = 0 ]; then unset QS_SCAN_BLOCKS; else export QS_SCAN_BLOCKS=$b; fi
  echo "blocks=$b"; RUNS=2 timeout -k 10 200 python -u tools/scan_probe.py 2>&1 | tail -n 2 || exit 6
done
unset QS_SCAN_BLOCKS
QSCHED_LIB=$P/libqsched_sq1.so RUNS=2 timeout -k 10 200 python -u tools/scan_probe.py 2>&1 | tail -n 2 || exit 6
echo ALLDONE
