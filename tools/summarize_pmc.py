"""Condense rocprofv3 --pmc counter_collection CSVs (one pass per counter) into a per-kernel
summary for profiles/: dispatches, mean FETCH_SIZE / WRITE_SIZE (KiB), and HBM bytes per launch
= 2 x FETCH_SIZE (gfx950 correction, MI355X_MICROARCH.md:298) + WRITE_SIZE, in bytes, with the
bench leg each row was collected under (one pair of passes per leg; bench.pmc_traffic takes the
first row that matches, so the headline leg goes first).
usage: python tools/summarize_pmc.py OUT.csv LEG FETCH.csv WRITE.csv [LEG FETCH.csv WRITE.csv ...]"""
import csv
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def load(path, counter):
    acc = defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter:
            acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return acc


def main(out, *legs):
    assert legs and len(legs) % 3 == 0, "LEG FETCH.csv WRITE.csv triples"
    with open(out, "w", newline="") as fh:
        wr = csv.writer(fh)
        wr.writerow(["kernel", "dispatches", "fetch_size_kib_mean", "write_size_kib_mean",
                     "hbm_bytes_per_launch", "leg"])
        for leg, fetch, write in zip(legs[0::3], legs[1::3], legs[2::3]):
            f, w = load(fetch, "FETCH_SIZE"), load(write, "WRITE_SIZE")
            for k in sorted(set(f) | set(w)):
                fm = sum(f[k]) / len(f[k]) if f.get(k) else 0.0
                wm = sum(w[k]) / len(w[k]) if w.get(k) else 0.0
                wr.writerow([k, max(len(f.get(k, [])), len(w.get(k, []))), round(fm, 3), round(wm, 3),
                             round((2 * fm + wm) * 1024), leg])


if __name__ == "__main__":
    main(*sys.argv[1:])
