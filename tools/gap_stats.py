"""Kernel-trace timeline of the lookahead window sequence: per kernel family the mean duration, and
for the resolver the gap between one window's resolve end and the next one's start (dispatch and
cross-stream dependency cost).  usage: python tools/gap_stats.py <rocprofv3 kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    fam = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        short = name.split("(")[0].split("<")[0].replace("void ", "").replace("qs::", "")
        fam[short].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for k, v in sorted(fam.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        d = [e - s for s, e in v]
        print(f"{k:28s} n={len(v):7d} mean {sum(d) / len(d) / 1e3:8.2f} us  total {sum(d) / 1e6:9.2f} ms")
    for k in ("k_la_resolve4", "k_la_resolve_run", "k_la_resolve_norm"):
        v = sorted(fam.get(k, []))
        if len(v) < 2:
            continue
        gaps = [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
        gaps = [g for g in gaps if g < 1_000_000]  # drop gaps between streams (> 1 ms)
        gaps.sort()
        print(f"{k}: launch-to-launch gap mean {sum(gaps) / len(gaps) / 1e3:.2f} us, p50 "
              f"{gaps[len(gaps) // 2] / 1e3:.2f} us, p90 {gaps[int(len(gaps) * 0.9)] / 1e3:.2f} us "
              f"(window period {(v[-1][1] - v[0][0]) / len(v) / 1e3:.2f} us over {len(v)} windows)")


if __name__ == "__main__":
    main(sys.argv[1])
