"""Duration distribution of one kernel from a rocprofv3 --kernel-trace CSV (per dispatch), e.g. the
config-4 resume kernel: which windows carry its time.  usage: python tools/resume_hist.py TRACE.csv
[kernel-substring]"""
import csv
import sys

import numpy as np

path, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "k_la_resolve_norm")
d = []
for r in csv.DictReader(open(path)):
    if sub in r["Kernel_Name"]:
        d.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
d = np.sort(np.array(d, dtype=np.int64)) / 1e3  # us
tot = d.sum()
print(f"{sub}: {len(d)} dispatches, total {tot / 1e3:.2f} ms, mean {d.mean():.2f} us")
for q in (50, 90, 94, 95, 97, 99, 99.9):
    print(f"  p{q}: {np.percentile(d, q):.2f} us")
for lo, hi in ((0, 5), (5, 20), (20, 100), (100, 500), (500, 1e9)):
    m = (d >= lo) & (d < hi)
    print(f"  [{lo}, {hi}) us: {int(m.sum())} dispatches, {d[m].sum() / 1e3:.2f} ms ({d[m].sum() / tot:.1%})")
