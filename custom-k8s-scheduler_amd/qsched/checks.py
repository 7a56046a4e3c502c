"""Size-independent invariants of an exact stream's result (spec/semantics.md S4/S7), checkable at any
size without re-running the decision sequence:

* conservation — the final table is the initial table plus the Reserve delta (spec S7) of every
  placed pod, column by column;
* capacity — Fit (spec S4) admitted every placement, so a node's Requested cpu / memory / extended
  resources end at or below Allocatable unless they started above it, and its pod count at or
  below max_pods;
* monotone unschedulability (Fit + Balanced profiles: feasibility only shrinks as Reserve adds
  requests) — a pod that found no feasible node at its turn fits no node of the final table.

Batched mode (spec S11) adds:

* anti-affinity — no two placed pods of an app with hostname anti-affinity share a node, and no two
  of an app with zone anti-affinity share a zone.

Used by tests/test_gpu_scale.py, tests/test_gpu_batched.py and bench.py's config-3 / config-4 /
config-5 legs beside the oracle diffs.
"""
from __future__ import annotations

import numpy as np

COLS = ("req_cpu", "req_mem", "nz_cpu", "nz_mem")


def stream_invariants(nodes0: dict, pods, placement: np.ndarray, final: dict, fit_only: bool = True) -> dict:
    """Returns {"conservation": bool, "capacity": bool, "unschedulable_infeasible": bool|None,
    "placed": int}.  `pods` is the POD_DTYPE array (arrival order), `placement` by arrival index."""
    n = len(nodes0["alloc_cpu"])
    pl = np.asarray(placement)
    ok_range = bool(((pl >= -1) & (pl < n)).all())
    placed = pl >= 0
    idx = pl[placed]
    cons = ok_range
    for c in COLS:
        exp = nodes0[c].astype(np.int64).copy()
        np.add.at(exp, idx, pods[c][placed].astype(np.int64))
        cons &= bool(np.array_equal(exp, final[c]))
    expp = nodes0["pods"].astype(np.int64).copy()
    np.add.at(expp, idx, 1)
    cons &= bool(np.array_equal(expp, final["pods"]))
    for k in range(nodes0["req_ext"].shape[1]):
        exp = nodes0["req_ext"][:, k].astype(np.int64).copy()
        np.add.at(exp, idx, pods["req_ext"][placed, k].astype(np.int64))
        cons &= bool(np.array_equal(exp, final["req_ext"][:, k]))
    cap = bool((final["pods"] <= np.maximum(final["max_pods"], nodes0["pods"])).all())
    cap &= bool((final["req_cpu"] <= np.maximum(final["alloc_cpu"], nodes0["req_cpu"])).all())
    cap &= bool((final["req_mem"] <= np.maximum(final["alloc_mem"], nodes0["req_mem"])).all())
    cap &= bool((final["req_ext"] <= np.maximum(final["alloc_ext"], nodes0["req_ext"])).all())
    unsched = None
    if fit_only:
        unsched = True
        free_c = final["alloc_cpu"] - final["req_cpu"]
        free_m = final["alloc_mem"] - final["req_mem"]
        free_e = final["alloc_ext"] - final["req_ext"]
        room = final["pods"] < final["max_pods"]
        bad = np.nonzero(~placed)[0]
        if bad.size:
            keys = np.stack([pods["req_cpu"][bad], pods["req_mem"][bad], pods["req_ext"][bad, 0],
                             pods["req_ext"][bad, 1]], axis=1)
            for rc, rm, e0, e1 in np.unique(keys, axis=0):
                fits = room.copy()
                if rc > 0:
                    fits &= rc <= free_c
                if rm > 0:
                    fits &= rm <= free_m
                if e0 > 0:
                    fits &= e0 <= free_e[:, 0]
                if e1 > 0:
                    fits &= e1 <= free_e[:, 1]
                if fits.any():
                    unsched = False
                    break
    return {"conservation": bool(cons), "capacity": cap, "unschedulable_infeasible": unsched,
            "placed": int(placed.sum())}


def batched_invariants(nodes0: dict, pods, placement: np.ndarray, final: dict) -> dict:
    """stream_invariants (conservation, capacity) plus spec S11's required anti-affinity."""
    out = stream_invariants(nodes0, pods, placement, final, fit_only=False)
    pl = np.asarray(placement)
    placed = pl >= 0
    app, aa = pods["app"].astype(np.int64), pods["anti_affinity"]
    host = placed & (aa == 1)
    hk = app[host] * (1 << 32) + pl[host]
    zon = placed & (aa == 2)
    zk = app[zon] * 64 + nodes0["zone"][pl[zon]].astype(np.int64)
    out["anti_affinity"] = bool(np.unique(hk).size == hk.size and np.unique(zk).size == zk.size)
    out.pop("unschedulable_infeasible", None)
    return out
