"""Condense rocprofv3 --pmc counter_collection CSVs (one pass per counter) into a per-kernel
summary for profiles/: dispatches, mean FETCH_SIZE / WRITE_SIZE (KiB), and HBM bytes per launch
= 2 x FETCH_SIZE (gfx950 correction, MI355X_MICROARCH.md:298) + WRITE_SIZE, in bytes.
usage: python tools/summarize_pmc.py FETCH.csv WRITE.csv OUT.csv"""
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


def main(fetch, write, out):
    f, w = load(fetch, "FETCH_SIZE"), load(write, "WRITE_SIZE")
    with open(out, "w", newline="") as fh:
        wr = csv.writer(fh)
        wr.writerow(["kernel", "dispatches", "fetch_size_kib_mean", "write_size_kib_mean",
                     "hbm_bytes_per_launch"])
        for k in sorted(set(f) | set(w)):
            fm = sum(f[k]) / len(f[k]) if f.get(k) else 0.0
            wm = sum(w[k]) / len(w[k]) if w.get(k) else 0.0
            wr.writerow([k, max(len(f.get(k, [])), len(w.get(k, []))), round(fm, 3), round(wm, 3),
                         round((2 * fm + wm) * 1024)])


if __name__ == "__main__":
    main(*sys.argv[1:4])
