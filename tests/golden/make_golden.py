"""Regenerate the golden fixtures (committed data) from the CPU oracle.

Each fixture: generator parameters (spec/synth.md), a SHA-256 of the generated inputs, and the
oracle's expected outputs (placement, best key, processing order, final dynamic node columns).
Both oracle restatements must agree before a fixture is written.  The reference itself has no
fixtures (parity unpinned), so these are the repo's own golden vectors.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

CASES = [
    # name, config, nodes, pods, profile
    ("config1", 1, 100, 1000, {}),
    ("config2_small", 2, 500, 6000, {}),
    ("config4_small", 4, 300, 3000, {"enable_taint": 1, "enable_affinity": 1}),
    ("config4_fitonly", 4, 300, 3000, {}),
    ("arrival_order", 2, 200, 2500, {"qos_sort": 0}),
    ("config2_tight", 2, 150, 5000, {}),
    # batched mode (spec S11): 64-pod batches with hostname/zone anti-affinity (config 5 draws)
    ("config5_batched", 5, 400, 8000, {"mode": "batched", "batch": 64}),
]
DYN = ["req_cpu", "req_mem", "req_ext", "nz_cpu", "nz_mem", "pods"]


V1_SKIP = ("zone", "app", "anti_affinity")  # ABI-v2 columns, added after the first fixtures


def input_digest(nodes, pods, full=False):
    """SHA-256 over the generated columns; full=False skips the ABI-v2 columns (the digest the
    first fixtures recorded), full=True covers every column."""
    h = hashlib.sha256()
    for d in (nodes, pods):
        for k in sorted(d):
            if not full and k in V1_SKIP:
                continue
            h.update(k.encode())
            h.update(np.ascontiguousarray(d[k]).tobytes())
    return h.hexdigest()


def build(name, config, n, p, profile, check_python=True):
    nodes, pods = O.generate(config, n, p)
    prof = {k: v for k, v in profile.items() if k not in ("mode", "batch")}
    cfg = dict(O.DEFAULT_CONFIG, **prof)
    digest = input_digest(nodes, pods)
    nc, _ = O.copy_cluster(nodes, pods)
    if profile.get("mode") == "batched":
        pl, best, nb = O.schedule_batched(nc, pods, batch=profile["batch"], cfg=cfg)
        order = np.arange(p, dtype=np.uint32)  # batched mode keeps queue order per batch (S11)
        check_python = False  # the pure-Python restatement covers the exact mode only
    if profile.get("mode") != "batched":
        pl, best, order = O.schedule(nc, pods, cfg)
    if check_python:
        npy, _ = O.copy_cluster(nodes, pods)
        pl2, best2 = O.py_schedule(npy, pods, cfg)
        assert pl.tolist() == pl2 and [int(x) for x in best] == best2, name
    out = dict(placement=pl, best_key=best, order=order)
    for k in DYN:
        out["final_" + k] = nc[k]
    meta = dict(name=name, config=config, nodes=n, pods=p, profile=profile, seed=0x5EED0000 + config,
                input_sha256=digest, input_sha256_full=input_digest(nodes, pods, full=True),
                placed=int((pl >= 0).sum()))
    if profile.get("mode") == "batched":
        meta["batches"] = nb
    return out, meta


def main():
    index = []
    for name, config, n, p, profile in CASES:
        out, meta = build(name, config, n, p, profile, check_python=(n * p <= 3_000_000))
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        index.append(meta)
        print(name, meta["placed"], "/", p)
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
