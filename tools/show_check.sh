#!/bin/bash
# Prints what tools/run_check.sh left in gpurun_out/.
cd "$(dirname "$0")/.."
tail -2 gpurun_out/call5.out 2>/dev/null
tail -3 gpurun_out/t3.log 2>/dev/null
head -2 gpurun_out/d4.log 2>/dev/null; tail -1 gpurun_out/d4.log 2>/dev/null
python3 -c "
import json
d=json.loads(open('gpurun_out/b_run.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('kernels_us_per_step'))
" 2>/dev/null
