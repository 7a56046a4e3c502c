#!/bin/bash
# LDS counters of the resident streams, config 2 against config 4 (the normalizing
# kernel's slow step-start LDS reads): one --pmc pass per leg, SQ counters only, summed per kernel.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ldsprobe
export TMPDIR=/tmp
CTR="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES"
for leg in config2 config4; do
  QS_HANDOFF=0 QS_GRAPH=0 timeout -s KILL 200 rocprofv3 --pmc $CTR -d gpurun_out/ldsprobe/$leg -o run --output-format csv -- python3 bench.py --leg $leg --no-cpu > gpurun_out/ldsprobe/$leg.log 2>&1 || { echo "$leg rc=$?"; tail -3 gpurun_out/ldsprobe/$leg.log; exit 1; }
  f=$(find gpurun_out/ldsprobe/$leg -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$leg" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(float); n = defaultdict(int)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_la_stream_res" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[2], {k: round(v / max(1, n[k])) for k, v in sorted(acc.items())}, "dispatches", max(n.values()) if n else 0)
PY
  find gpurun_out/ldsprobe/$leg -name '*.csv' -size +5M -delete
done
