"""CPU ORACLE for the qsched hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module; the product (``custom-k8s-scheduler_amd/``) never does.

Parity status: **PARITY UNPINNED by the reference.**  ``/root/reference/README.md:1`` is a single
title line with no code, tests or fixtures, so nothing in the reference pins results.  The oracle
restates ``spec/semantics.md`` (= SURVEY.md Appendix A = upstream kube-scheduler v1.32 plugin
semantics, cited per function) twice, independently:

* ``liboracle.so`` (``oracle/qs_oracle.c``): straight-line C, int64 + IEEE binary64;
* the pure-Python functions below (``py_*``): straight-line Python ints/floats, small cases only;

and both are pinned by the hand-computed known-answer tests of ``spec/kat.md``.

Data layout shared with the product's Python binding: a *cluster* is two dicts of numpy arrays
(``nodes``, ``pods``) with the field names of ``include/qsched.h`` (``qs_node_soa`` / ``qs_pod``).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MAX_EXT = 2
MAX_TERMS = 4
MIB = 1 << 20
GIB = 1 << 30
DEF_CPU = 100          # UP pkg/scheduler/util/pod_resources.go#DefaultMilliCPURequest
DEF_MEM = 200 * MIB    # UP pkg/scheduler/util/pod_resources.go#DefaultMemoryRequest
MAX_NODE_SCORE = 100   # UP framework/interface.go#MaxNodeScore

NODE_FIELDS_I64 = ["alloc_cpu", "alloc_mem", "max_pods", "req_cpu", "req_mem",
                   "nz_cpu", "nz_mem", "pods"]
POD_FIELDS_I64 = ["req_cpu", "req_mem", "nz_cpu", "nz_mem"]

# spec S9 default profile weights, indexed by QoS class [BestEffort, Burstable, Guaranteed]
DEFAULT_CONFIG = dict(wc=1, wm=1, w_fit=(1, 2, 3), w_bal=(1, 1, 1), w_tt=3, w_na=2,
                      enable_taint=0, enable_affinity=0, balanced_skip_besteffort=0, qos_sort=1,
                      fit_resources=None, balanced_resources=None)

# Scoring-resource names of the configurable lists (NodeResourcesFitArgs.ScoringStrategy.Resources =
# fit_resources [(name, weight), ...]; NodeResourcesBalancedAllocationArgs.Resources =
# balanced_resources [name, ...]); None = upstream's defaults [cpu:1, memory:1] / [cpu, memory].
# "ext0" / "ext1" are the table's two extended-resource columns (e.g. amd.com/gpu).
RES_IDS = {"cpu": 1, "memory": 2, "ext0": 3, "ext1": 4}
MAX_SCORE_RES = 4


def res_id(name) -> int:
    return name if isinstance(name, int) else RES_IDS[name]


def empty_cluster(n: int, p: int):
    nodes = {f: np.zeros(n, np.int64) for f in NODE_FIELDS_I64}
    nodes["alloc_ext"] = np.zeros((n, MAX_EXT), np.int64)
    nodes["req_ext"] = np.zeros((n, MAX_EXT), np.int64)
    nodes["taint_hard"] = np.zeros(n, np.uint64)
    nodes["taint_soft"] = np.zeros(n, np.uint64)
    nodes["label_bits"] = np.zeros((n, 2), np.uint64)
    nodes["zone"] = np.zeros(n, np.int32)
    pods = {f: np.zeros(p, np.int64) for f in POD_FIELDS_I64}
    pods["req_ext"] = np.zeros((p, MAX_EXT), np.int64)
    pods["qos"] = np.zeros(p, np.int32)
    pods["priority"] = np.zeros(p, np.int32)
    pods["tol_hard"] = np.zeros(p, np.uint64)
    pods["tol_soft"] = np.zeros(p, np.uint64)
    pods["sel"] = np.zeros((p, 2), np.uint64)
    pods["n_req_terms"] = np.zeros(p, np.int32)
    pods["n_pref_terms"] = np.zeros(p, np.int32)
    pods["req_terms"] = np.zeros((p, MAX_TERMS, 2), np.uint64)
    pods["pref_terms"] = np.zeros((p, MAX_TERMS, 2), np.uint64)
    pods["pref_weight"] = np.zeros((p, MAX_TERMS), np.int32)
    pods["app"] = np.zeros(p, np.int32)
    pods["anti_affinity"] = np.zeros(p, np.int32)
    return nodes, pods


def copy_cluster(nodes, pods):
    return ({k: v.copy() for k, v in nodes.items()}, {k: v.copy() for k, v in pods.items()})


# --------------------------------------------------------------------------------------------
# C oracle via ctypes
# --------------------------------------------------------------------------------------------
class _Nodes(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32)] + [(f, ctypes.c_void_p) for f in
               ["alloc_cpu", "alloc_mem", "alloc_ext", "max_pods", "req_cpu", "req_mem", "req_ext",
                "nz_cpu", "nz_mem", "pods", "taint_hard", "taint_soft", "label_bits", "zone"]]


class _Pods(ctypes.Structure):
    _fields_ = [("p", ctypes.c_uint32)] + [(f, ctypes.c_void_p) for f in
               ["req_cpu", "req_mem", "req_ext", "nz_cpu", "nz_mem", "qos", "priority", "tol_hard",
                "tol_soft", "sel", "n_req_terms", "n_pref_terms", "req_terms", "pref_terms",
                "pref_weight", "app", "anti_affinity"]]


class _Config(ctypes.Structure):
    _fields_ = [("wc", ctypes.c_int64), ("wm", ctypes.c_int64), ("w_fit", ctypes.c_int32 * 3),
                ("w_bal", ctypes.c_int32 * 3), ("w_tt", ctypes.c_int32), ("w_na", ctypes.c_int32),
                ("enable_taint", ctypes.c_int32), ("enable_affinity", ctypes.c_int32),
                ("balanced_skip_besteffort", ctypes.c_int32), ("qos_sort", ctypes.c_int32),
                ("n_fit_res", ctypes.c_int32), ("fit_res", ctypes.c_int32 * 4), ("fit_w", ctypes.c_int32 * 4),
                ("n_bal_res", ctypes.c_int32), ("bal_res", ctypes.c_int32 * 4)]


_LIB = None


def build_oracle() -> str:
    """Compile oracle/liboracle.so (building the checker is not using it)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return os.path.join(HERE, "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build_oracle()
        L = ctypes.CDLL(path)
        L.or_least_allocated.restype = ctypes.c_int64
        L.or_least_allocated.argtypes = [ctypes.c_int64] * 6
        L.or_balanced.restype = ctypes.c_int64
        L.or_balanced.argtypes = [ctypes.c_int64] * 4
        L.or_least_allocated_v.restype = ctypes.c_int64
        L.or_least_allocated_v.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_int64)] * 3
        L.or_balanced_v.restype = ctypes.c_int64
        L.or_balanced_v.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_int64)] * 2
        L.or_schedule.restype = None
        L.or_schedule.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_int]
        L.or_schedule_incremental.restype = ctypes.c_int
        L.or_schedule_incremental.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_int, ctypes.c_uint64]
        L.or_score_pod.restype = None
        L.or_score_pod.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32] + [ctypes.c_void_p] * 2
        L.or_reserve.restype = None
        L.or_reserve.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint32] * 2 + [ctypes.c_int]
        L.or_schedule_batched.restype = ctypes.c_uint32
        L.or_schedule_batched.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32] + [ctypes.c_void_p] * 2 + [ctypes.c_int]
        L.or_schedule_batched_incremental.restype = ctypes.c_uint32
        L.or_schedule_batched_incremental.argtypes = L.or_schedule_batched.argtypes
        L.or_generate.restype = None
        L.or_generate.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        _LIB = L
    return _LIB


def _ptr(a):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def _mk_nodes(nodes):
    s = _Nodes()
    s.n = len(nodes["alloc_cpu"])
    for f, _ in _Nodes._fields_[1:]:
        setattr(s, f, _ptr(nodes[f]))
    return s


def _mk_pods(pods):
    s = _Pods()
    s.p = len(pods["req_cpu"])
    for f, _ in _Pods._fields_[1:]:
        setattr(s, f, _ptr(pods[f]))
    return s


def _mk_cfg(cfg):
    c = dict(DEFAULT_CONFIG)
    c.update(cfg or {})
    s = _Config()
    s.wc, s.wm = c["wc"], c["wm"]
    for i in range(3):
        s.w_fit[i] = c["w_fit"][i]
        s.w_bal[i] = c["w_bal"][i]
    s.w_tt, s.w_na = c["w_tt"], c["w_na"]
    s.enable_taint, s.enable_affinity = c["enable_taint"], c["enable_affinity"]
    s.balanced_skip_besteffort, s.qos_sort = c["balanced_skip_besteffort"], c["qos_sort"]
    fr = c.get("fit_resources") or []
    s.n_fit_res = len(fr)
    for i, (name, w) in enumerate(fr):
        s.fit_res[i], s.fit_w[i] = res_id(name), w
    br = c.get("balanced_resources") or []
    s.n_bal_res = len(br)
    for i, name in enumerate(br):
        s.bal_res[i] = res_id(name)
    return s


def generate(config: int, n: int, p: int, seed: int | None = None):
    """spec/synth.md cluster via the C restatement (seed defaults to 0x5EED0000 + config)."""
    nodes, pods = empty_cluster(n, p)
    sn, sp = _mk_nodes(nodes), _mk_pods(pods)
    lib().or_generate(config, 0x5EED0000 + config if seed is None else seed,
                      ctypes.byref(sn), ctypes.byref(sp))
    return nodes, pods


def schedule(nodes, pods, cfg=None, nthreads=1):
    """Exact sequential stream (spec S7/S8).  Mutates ``nodes`` (Reserve applied).
    Returns (placement[p] int32, best_key[p] uint64, order[p] uint32)."""
    p = len(pods["req_cpu"])
    placement = np.empty(p, np.int32)
    best = np.empty(p, np.uint64)
    order = np.empty(p, np.uint32)
    sn, sp, sc = _mk_nodes(nodes), _mk_pods(pods), _mk_cfg(cfg)
    lib().or_schedule(ctypes.byref(sc), ctypes.byref(sn), ctypes.byref(sp), _ptr(placement),
                      _ptr(best), _ptr(order), ctypes.c_int(nthreads))
    return placement, best, order


def schedule_incremental(nodes, pods, cfg=None, nthreads=1, max_bytes=8 << 30):
    """or_schedule_incremental: the exact stream with a per-pod-type incremental argmax (same
    results as ``schedule``; Fit + Balanced (+ ext) profiles).  Mutates ``nodes``.  Raises
    ValueError when the profile normalizes or the trees exceed ``max_bytes``."""
    p = len(pods["req_cpu"])
    placement = np.empty(p, np.int32)
    best = np.empty(p, np.uint64)
    order = np.empty(p, np.uint32)
    sn, sp, sc = _mk_nodes(nodes), _mk_pods(pods), _mk_cfg(cfg)
    rc = lib().or_schedule_incremental(ctypes.byref(sc), ctypes.byref(sn), ctypes.byref(sp), _ptr(placement),
                                       _ptr(best), _ptr(order), ctypes.c_int(nthreads),
                                       ctypes.c_uint64(max_bytes))
    if rc != 0:
        raise ValueError("or_schedule_incremental: normalizing profile or tree memory bound exceeded")
    return placement, best, order


def schedule_batched(nodes, pods, batch=64, cfg=None, nthreads=1):
    """Batched mode (spec S11).  Mutates ``nodes``.  Returns (placement[p], key[p], batches)."""
    p = len(pods["req_cpu"])
    placement = np.full(p, -3, np.int32)
    best = np.zeros(p, np.uint64)
    sn, sp, sc = _mk_nodes(nodes), _mk_pods(pods), _mk_cfg(cfg)
    nb = lib().or_schedule_batched(ctypes.byref(sc), ctypes.byref(sn), ctypes.byref(sp),
                                   ctypes.c_uint32(batch), _ptr(placement), _ptr(best),
                                   ctypes.c_int(nthreads))
    return placement, best, int(nb)


def schedule_batched_incremental(nodes, pods, batch=64, cfg=None, nthreads=1):
    """schedule_batched with incremental lists (per pod type and zone a max tree over the nodes'
    keys, only the claimed nodes re-scored per batch): identical results for Fit + Balanced (+ ext)
    profiles.  Mutates ``nodes``.  Returns (placement[p], key[p], batches)."""
    p = len(pods["req_cpu"])
    placement = np.full(p, -3, np.int32)
    best = np.zeros(p, np.uint64)
    sn, sp, sc = _mk_nodes(nodes), _mk_pods(pods), _mk_cfg(cfg)
    nb = lib().or_schedule_batched_incremental(ctypes.byref(sc), ctypes.byref(sn), ctypes.byref(sp),
                                               ctypes.c_uint32(batch), _ptr(placement), _ptr(best),
                                               ctypes.c_int(nthreads))
    if nb == 0xFFFFFFFF:
        raise ValueError("or_schedule_batched_incremental: normalizing profile or zone id >= 64")
    return placement, best, int(nb)


def score_pod(nodes, pods, j, cfg=None):
    """Keys and per-plugin scores of pod j on every node (no state change)."""
    n = len(nodes["alloc_cpu"])
    keys = np.empty(n, np.uint64)
    scores = np.empty((n, 4), np.int64)
    sn, sp, sc = _mk_nodes(nodes), _mk_pods(pods), _mk_cfg(cfg)
    lib().or_score_pod(ctypes.byref(sc), ctypes.byref(sn), ctypes.byref(sp), ctypes.c_uint32(j),
                       _ptr(keys), _ptr(scores))
    return keys, scores


# --------------------------------------------------------------------------------------------
# Independent pure-Python restatement (small cases; Python int + float == Go int64 + float64 here)
# --------------------------------------------------------------------------------------------
def py_least_requested_score(requested, capacity):
    """UP noderesources/least_allocated.go#leastRequestedScore"""
    if capacity == 0 or requested > capacity:
        return 0
    return ((capacity - requested) * MAX_NODE_SCORE) // capacity


def py_least_allocated(alloc, reqd, weights=(1, 1)):
    """UP noderesources/least_allocated.go#leastResourceScorer"""
    node_score = weight_sum = 0
    for a, r, w in zip(alloc, reqd, weights):
        if a == 0:
            continue
        node_score += py_least_requested_score(r, a) * w
        weight_sum += w
    return 0 if weight_sum == 0 else node_score // weight_sum


def py_balanced(alloc, reqd):
    """UP noderesources/balanced_allocation.go#balancedResourceScorer (float64 semantics)"""
    fr = []
    for a, r in zip(alloc, reqd):
        if a == 0:
            continue
        f = float(r) / float(a)
        fr.append(1.0 if f > 1 else f)
    std = 0.0
    if len(fr) == 2:
        std = abs((fr[0] - fr[1]) / 2)
    elif len(fr) > 2:
        mean = sum(fr) / len(fr)
        s = 0.0
        for f in fr:
            s = s + (f - mean) * (f - mean)
        std = math.sqrt(s / len(fr))
    return int((1 - std) * float(MAX_NODE_SCORE))


def _subset(m, bits):
    return (int(m[0]) & int(bits[0])) == int(m[0]) and (int(m[1]) & int(bits[1])) == int(m[1])


def py_feasible(nodes, pods, n, j, cfg):
    """UP fit.go#fitsRequest + taint_toleration.go#Filter + node_affinity.go#Filter"""
    if nodes["pods"][n] + 1 > nodes["max_pods"][n]:
        return False
    rc, rm = int(pods["req_cpu"][j]), int(pods["req_mem"][j])
    ext = [int(x) for x in pods["req_ext"][j]]
    if not (rc == 0 and rm == 0 and not any(ext)):
        if rc > 0 and rc > nodes["alloc_cpu"][n] - nodes["req_cpu"][n]:
            return False
        if rm > 0 and rm > nodes["alloc_mem"][n] - nodes["req_mem"][n]:
            return False
        for k, q in enumerate(ext):
            if q != 0 and q > nodes["alloc_ext"][n][k] - nodes["req_ext"][n][k]:
                return False
    if cfg["enable_taint"] and int(nodes["taint_hard"][n]) & ~int(pods["tol_hard"][j]):
        return False
    if cfg["enable_affinity"]:
        lb = nodes["label_bits"][n]
        if not _subset(pods["sel"][j], lb):
            return False
        nt = int(pods["n_req_terms"][j])
        if nt and not any(_subset(pods["req_terms"][j][t], lb) for t in range(nt)):
            return False
    return True


def py_taint_raw(nodes, pods, n, j):
    return bin(int(nodes["taint_soft"][n]) & ~int(pods["tol_soft"][j]) & (2**64 - 1)).count("1")


def py_affinity_raw(nodes, pods, n, j):
    lb = nodes["label_bits"][n]
    return sum(int(pods["pref_weight"][j][t]) for t in range(int(pods["n_pref_terms"][j]))
               if _subset(pods["pref_terms"][j][t], lb))


def py_normalize(raw, mx, reverse):
    """UP plugins/helper/normalize_score.go#DefaultNormalizeScore"""
    if mx == 0:
        return MAX_NODE_SCORE if reverse else raw
    s = MAX_NODE_SCORE * raw // mx
    return MAX_NODE_SCORE - s if reverse else s


def py_alloc_request(nodes, pods, n, j, res, use_requested):
    """UP noderesources/resource_allocation.go#calculateResourceAllocatableRequest: (allocatable,
    requested + pod request) of one scoring resource; cpu / memory from NonZeroRequested and the
    pod's non-zero request (LeastAllocated) or Requested and the plain request (Balanced); an
    extended resource the pod does not request is (0, 0): skipped."""
    rid = res_id(res)
    if rid == 1:
        k = ("req_cpu", "req_cpu") if use_requested else ("nz_cpu", "nz_cpu")
        return int(nodes["alloc_cpu"][n]), int(nodes[k[0]][n]) + int(pods[k[1]][j])
    if rid == 2:
        k = ("req_mem", "req_mem") if use_requested else ("nz_mem", "nz_mem")
        return int(nodes["alloc_mem"][n]), int(nodes[k[0]][n]) + int(pods[k[1]][j])
    e = rid - 3
    q = int(pods["req_ext"][j][e])
    if q == 0:
        return 0, 0
    return int(nodes["alloc_ext"][n][e]), int(nodes["req_ext"][n][e]) + q


def py_keys(nodes, pods, j, cfg):
    n_nodes = len(nodes["alloc_cpu"])
    feas = [py_feasible(nodes, pods, n, j, cfg) for n in range(n_nodes)]
    mt = max([py_taint_raw(nodes, pods, n, j) for n in range(n_nodes) if feas[n]] or [0]) \
        if cfg["enable_taint"] else 0
    ma = max([py_affinity_raw(nodes, pods, n, j) for n in range(n_nodes) if feas[n]] or [0]) \
        if cfg["enable_affinity"] else 0
    q = int(pods["qos"][j])
    keys = []
    for n in range(n_nodes):
        if not feas[n]:
            keys.append(0)
            continue
        fit = cfg.get("fit_resources") or [("cpu", cfg["wc"]), ("memory", cfg["wm"])]
        la_ar = [py_alloc_request(nodes, pods, n, j, r, False) for r, _ in fit]
        la = py_least_allocated([a for a, _ in la_ar], [r for _, r in la_ar], [w for _, w in fit])
        bal = cfg.get("balanced_resources") or ["cpu", "memory"]
        ba_ar = [py_alloc_request(nodes, pods, n, j, r, True) for r in bal]
        ba = py_balanced([a for a, _ in ba_ar], [r for _, r in ba_ar])
        if cfg["balanced_skip_besteffort"] and q == 0:
            ba = 0
        total = cfg["w_fit"][q] * la + cfg["w_bal"][q] * ba
        if cfg["enable_taint"]:
            total += cfg["w_tt"] * py_normalize(py_taint_raw(nodes, pods, n, j), mt, True)
        if cfg["enable_affinity"]:
            total += cfg["w_na"] * py_normalize(py_affinity_raw(nodes, pods, n, j), ma, False)
        keys.append(((total + 1) << 32) | (0xFFFFFFFF - n))
    return keys


def py_order(pods, cfg):
    """spec S8 QoSSort: stable by (qos desc, priority desc)."""
    p = len(pods["qos"])
    if not cfg["qos_sort"]:
        return list(range(p))
    return sorted(range(p), key=lambda j: (-int(pods["qos"][j]), -int(pods["priority"][j]), j))


def py_schedule(nodes, pods, cfg=None):
    """Pure-Python exact stream; mutates nodes.  Returns (placement list, best-key list)."""
    c = dict(DEFAULT_CONFIG)
    c.update(cfg or {})
    p = len(pods["qos"])
    placement = [-1] * p
    best_keys = [0] * p
    for j in py_order(pods, c):
        keys = py_keys(nodes, pods, j, c)
        best = max(keys) if keys else 0
        best_keys[j] = best
        if best == 0:
            continue
        n = 0xFFFFFFFF - (best & 0xFFFFFFFF)
        placement[j] = n
        nodes["req_cpu"][n] += pods["req_cpu"][j]
        nodes["req_mem"][n] += pods["req_mem"][j]
        nodes["req_ext"][n] += pods["req_ext"][j]
        nodes["nz_cpu"][n] += pods["nz_cpu"][j]
        nodes["nz_mem"][n] += pods["nz_mem"][j]
        nodes["pods"][n] += 1
    return placement, best_keys


# --------------------------------------------------------------------------------------------
# Independent numpy restatement of the spec/synth.md generator (checks the product's generator)
# --------------------------------------------------------------------------------------------
_G = np.uint64(0x9E3779B97F4A7C15)


def _sm_at(seed, c):
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.asarray(c, np.uint64) + np.uint64(1)) * _G
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _pick(seed, c, k):
    return ((_sm_at(seed, c) >> np.uint64(33)) % np.uint64(k)).astype(np.int64)


def py_generate(config: int, n: int, p: int, seed: int | None = None):
    """spec/synth.md generator, vectorised numpy restatement (independent of qs_oracle.c)."""
    seed = 0x5EED0000 + config if seed is None else seed
    nodes, pods = empty_cluster(n, p)
    i = np.arange(n, dtype=np.uint64) * np.uint64(8)
    cpu = np.array([4000, 8000, 16000, 32000, 64000, 96000], np.int64)[_pick(seed, i + np.uint64(0), 6)]
    mpc = np.array([2, 4, 8], np.int64)[_pick(seed, i + np.uint64(1), 3)]
    nodes["alloc_cpu"][:] = cpu
    nodes["alloc_mem"][:] = (cpu // 1000) * mpc * GIB
    nodes["max_pods"][:] = 110
    c4, c5 = config == 4, config == 5
    if c4 or c5:
        nodes["zone"][:] = _pick(seed, i + np.uint64(4), 10).astype(np.int32)
    if c4:
        gpu = _pick(seed, i + np.uint64(2), 10) == 0
        maint = _pick(seed, i + np.uint64(3), 20) == 0
        zone = _pick(seed, i + np.uint64(4), 10)
        pool = np.where(gpu, 2, _pick(seed, i + np.uint64(5), 2))
        ssd = _pick(seed, i + np.uint64(6), 2) == 0
        nodes["alloc_ext"][:, 0] = np.where(gpu, 8, 0)
        nodes["taint_hard"][:] = np.where(gpu, 1, 0).astype(np.uint64)
        nodes["taint_soft"][:] = np.where(maint, 2, 0).astype(np.uint64)
        pairs = [(a, b) for a in range(10) for b in range(a + 1, 10)]
        for k in range(n):
            bits = (1 << 0 if pool[k] == 2 else 0) | (1 << 1 if ssd[k] else 0) | (1 << 2 if pool[k] == 1 else 0)
            for pi, (a, b) in enumerate(pairs):
                if zone[k] in (a, b):
                    bits |= 1 << (3 + pi)
            nodes["label_bits"][k, 0] = bits & (2**64 - 1)
            nodes["label_bits"][k, 1] = bits >> 64
    j = np.uint64(8 * n) + np.arange(p, dtype=np.uint64) * np.uint64(16)
    qd = _pick(seed, j, 10)
    cpu = np.array([500, 1000, 1500, 2000, 4000, 8000], np.int64)[_pick(seed, j + np.uint64(1), 6)]
    mem = np.array([128, 256, 512, 1024, 2048, 4096, 8192], np.int64)[_pick(seed, j + np.uint64(2), 7)] * MIB
    memmode = _pick(seed, j + np.uint64(3), 4)
    q = np.where(qd < 2, 2, np.where(qd < 7, 1, 0))
    pods["qos"][:] = q
    pods["req_cpu"][:] = np.where(q > 0, cpu, 0)
    pods["nz_cpu"][:] = np.where(q > 0, cpu, DEF_CPU)
    has_mem = (q == 2) | ((q == 1) & (memmode != 0))
    pods["req_mem"][:] = np.where(has_mem, mem, 0)
    pods["nz_mem"][:] = np.where(has_mem, mem, DEF_MEM)
    if c5:  # spec/synth.md G5
        app = _pick(seed, j + np.uint64(13), 1000)
        kind = _pick(seed, np.uint64(8 * n + 16 * p) + app.astype(np.uint64), 10)
        pods["app"][:] = app.astype(np.int32)
        pods["anti_affinity"][:] = np.where(kind < 5, 1, np.where(kind == 5, 2, 0)).astype(np.int32)
    if c4:
        pairs = [(a, b) for a in range(10) for b in range(a + 1, 10)]
        gpu = _pick(seed, j + np.uint64(5), 20) == 0
        gcnt = np.array([1, 2, 4, 8], np.int64)[_pick(seed, j + np.uint64(6), 4)]
        pods["req_ext"][:, 0] = np.where(gpu, gcnt, 0)
        pods["tol_hard"][:] = np.where(gpu, 1, 0).astype(np.uint64)
        pods["sel"][:, 0] = np.where(gpu, 1, 0).astype(np.uint64)
        zreq = _pick(seed, j + np.uint64(7), 5) == 0
        za = _pick(seed, j + np.uint64(8), 10)
        zb = (za + 1 + _pick(seed, j + np.uint64(9), 9)) % 10
        pref = _pick(seed, j + np.uint64(10), 5) == 0
        which = _pick(seed, j + np.uint64(11), 3)
        tolm = _pick(seed, j + np.uint64(12), 10) == 0
        pods["tol_soft"][:] = np.where(tolm, 2, 0).astype(np.uint64)
        for k in range(p):
            if zreq[k]:
                a, b = sorted((int(za[k]), int(zb[k])))
                bit = 3 + pairs.index((a, b))
                pods["req_terms"][k, 0, bit // 64] = np.uint64(1 << (bit % 64))
                pods["n_req_terms"][k] = 1
            if pref[k]:
                t = 0
                if which[k] in (0, 2):
                    pods["pref_terms"][k, t, 0] = 2
                    pods["pref_weight"][k, t] = 50
                    t += 1
                if which[k] in (1, 2):
                    pods["pref_terms"][k, t, 0] = 4
                    pods["pref_weight"][k, t] = 20
                    t += 1
                pods["n_pref_terms"][k] = t
    return nodes, pods
