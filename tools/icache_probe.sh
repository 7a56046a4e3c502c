#!/bin/bash
# Instruction-cache counters of the resident stream, config 2 vs config 4 (one --pmc pass each,
# kernel-trace-free; three SQC counters, the program itself after --).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 2 4; do
  if [ $c = 2 ]; then export CFG=2 N=5000 P=100000 TA=0; else export CFG=4 N=5000 P=150000 TA=1; fi
  timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES -d gpurun_out/icache$c -o run --output-format csv -- python3 tools/kprof.py > gpurun_out/icache$c.log 2>&1 || { echo "pass $c failed"; tail -3 gpurun_out/icache$c.log; exit 5; }
  f=$(find gpurun_out/icache$c -name '*counter_collection.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
    if "k_la_stream_res" not in k: continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print({k: (v, n[k]) for k, v in agg.items()})
PY
  find gpurun_out/icache$c -name '*.csv' -size +5M -delete
done
echo ALLDONE
