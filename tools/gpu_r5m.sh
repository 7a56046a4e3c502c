#!/bin/bash
# Round 5: framework-path widening threshold at 5,000 nodes (every output), three runs each.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for m in 16384 2048; do
    echo "par_min=$m $(QS_UNPACK_PAR_MIN=$m timeout -k 10 120 custom-k8s-scheduler_amd/fw_latency 5000 5000 1 | cut -c1-160)" || exit 7
  done
done
echo ALLDONE
