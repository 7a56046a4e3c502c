"""Writes tests/golden/fuzz_cases.json: the committed seeds of the adversarial device-parity fuzz
(tests/test_gpu_adversarial.py; SURVEY.md §4 "oracle <-> device" row).

Each case is a seed plus the shape knobs drawn from it; tests/adversarial.py rebuilds the cluster
from the seed alone (numpy PCG64, so the same case on every box).  Memory grids:
  binary  - GiB / MiB multiples (the compact int32 device layout applies);
  ki      - kubelet-style odd-Ki allocatable (1-16 GiB and 64-768 GiB) and odd-Ki pod requests;
  decimal - decimal quantities (100M, 512M, 16G, arbitrary M) on nodes and pods.
The ki / decimal grids cannot be stored in 2^u-byte units below 2^24 and run on the wide (f64
memory column) device layout.

Usage: python tests/golden/make_fuzz_cases.py  (deterministic; rewrite only to add cases)
"""
import json
import os

import numpy as np

N_CASES = 360
GRIDS = ["binary", "ki", "decimal"]


def main():
    rng = np.random.default_rng(0xADF0_2024)
    cases = []
    for i in range(N_CASES):
        grid = GRIDS[i % 3]
        n = int(rng.choice([1, 2, 3, 7, 24, 64, 65, 130, 300]))
        p = int(rng.choice([0, 1, 5, 60, 300, 1000, 3000]))
        cases.append({
            "seed": int(rng.integers(0, 2**63 - 1)),
            "n": n, "p": p, "grid": grid,
            "features": bool(rng.random() < 0.4),
            "qos_sort": int(rng.random() < 0.8),
            "weights": int(rng.integers(0, 3)),     # 0 default, 1 custom, 2 single-resource LA
            "init_usage": bool(rng.random() < 0.5),
            "K": int(rng.choice([1, 3, 8, 16, 32, 64])),
            "vshards": int(rng.choice([2, 3, 4, 8])),
        })
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fuzz_cases.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/make_fuzz_cases.py", "cases": cases}, f, indent=0)
    print(f"wrote {len(cases)} cases to {out}")


if __name__ == "__main__":
    main()
