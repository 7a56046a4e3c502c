#!/bin/bash
# Framework path at 5,000 nodes, every output copied out, three runs of 5,000 calls with the slow
# calls' phase split (QS_SCORE_DIAG=1: prep / launch / done-word wait / unpack, calls > 500 us).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in 1 2 3; do
  QS_SCORE_DIAG=1 timeout -k 10 120 custom-k8s-scheduler_amd/fw_latency 5000 5000 1 > gpurun_out/fwu.json 2> gpurun_out/fwu_diag_$r.txt || exit 7
  echo "run $r $(cut -c1-220 gpurun_out/fwu.json)"
  grep -v "call 1:" gpurun_out/fwu_diag_$r.txt | head -5
done
