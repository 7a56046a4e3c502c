#!/bin/bash
# Final evidence of the tree: the whole -m gpu suite, smoke, the bench line, then the rocprofv3
# kernel stats / PMC passes / config-4 and config-5 stats (tools/profile_fetch.sh) and the C++
# framework-path latency.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=tests SMOKE=1 TEST_TIMEOUT=1000 bash tools/r03_check.sh || exit 1
bash tools/profile_fetch.sh ${TAG:-r03} || exit 2
for o in 1 0; do timeout -k 10 60 custom-k8s-scheduler_amd/fw_latency 5000 5000 $o >> gpurun_out/fw_final.log 2>&1 || exit 3; done
cat gpurun_out/fw_final.log
echo FINALDONE
