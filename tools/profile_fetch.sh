#!/bin/bash
# Runs tools/profile_round.sh on the GPU box and brings its summaries back through gpurun_out/
# (only gpurun_out/ is merged back, at most 64 MiB): profiles/ and the config-4/5 stats go to
# gpurun_out/profiles_new/, the raw traces are dropped.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
bash tools/profile_round.sh $TAG > gpurun_out/profile_round.log 2>&1
rc=$?
mkdir -p gpurun_out/profiles_new
cp profiles/* gpurun_out/profiles_new/
for c in 4 5; do
    f=$(find gpurun_out/prof_$TAG/cfg$c -name '*kernel_stats.csv' | head -1)
    [ -n "$f" ] && cp "$f" gpurun_out/profiles_new/${TAG}_config${c}_kernel_stats.csv
    tail -3 gpurun_out/prof_$TAG/cfg$c.log > gpurun_out/profiles_new/cfg$c.tail 2>/dev/null
done
tail -3 gpurun_out/prof_$TAG/trace.log > gpurun_out/profiles_new/trace.tail 2>/dev/null
cat gpurun_out/prof_$TAG/*.err > gpurun_out/profiles_new/pmc_errors.txt 2>/dev/null
rm -rf gpurun_out/prof_$TAG
exit $rc
