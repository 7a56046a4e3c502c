#!/bin/bash
# Per-window cost breakdown of the config-2 lookahead stream (GPU box): resolver QS_DIAG stamps
# (prologue / epilogue per window), host enqueue time, and a kernel-trace timeline.
# Usage (from the repo root, through gpurun): bash tools/window_probe.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
QS_DIAG=1 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/wp_diag.log 2>&1 || exit 1
QS_HOSTTIME=1 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/wp_host.log 2>&1 || exit 1
${EXTRA:-true} || exit 1
P=32000 RUNS=lookahead:32 timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/wp_prof -o run --output-format csv \
    -- python3 tools/la_sweep.py > gpurun_out/wp_prof.log 2>&1 || exit 1
f=$(find gpurun_out/wp_prof -name '*kernel_trace.csv' | head -1)
python3 tools/gap_stats.py "$f" > gpurun_out/wp_gap.txt
rm -f "$f"
