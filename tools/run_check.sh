#!/bin/bash
# Resolver iteration check (GPU box): lookahead parity + goldens, QS_DIAG stamps, short bench.
# Usage (from the repo root, through gpurun): bash tools/run_check.sh
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
rm -f gpurun_out/t3.log gpurun_out/d4.log gpurun_out/b_run.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -q -x --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/t3.log 2>&1 || { echo "rc=$?" >> gpurun_out/t3.log; exit 1; }
QS_DIAG=1 RUNS=lookahead:32 timeout -k 10 120 python -u tools/la_sweep.py > gpurun_out/d4.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --no-extra --no-cpu --no-scan --no-config3 --steps 10 > gpurun_out/b_run.json \
    2> gpurun_out/b_run.err
