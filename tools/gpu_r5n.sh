#!/bin/bash
# Round 5: HBM-resident scoring scan variants (k_scan_soa, 2^24 nodes): nt loads, 4 quads in flight.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
P=$PWD/custom-k8s-scheduler_amd
for v in ${VS:-libqsched.so}; do
  QSCHED_LIB=$P/$v RUNS=2 timeout -k 10 200 python -u tools/scan_probe.py 2>&1 | tail -n 2 || exit 6
done
echo ALLDONE
