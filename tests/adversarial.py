"""Adversarial cluster builder shared by the device-parity fuzz (tests/test_gpu_adversarial.py) and
its CPU pin (tests/test_adversarial_cpu.py).  Test infrastructure only.

A case (tests/golden/fuzz_cases.json) is a seed plus shape knobs; ``build(case)`` rebuilds the
same nodes / pods / configs from it on any box.  What it stresses (SURVEY.md §4 fuzz row):
  * capacity edges: max_pods in {1, 2, 5, 110}, pre-used nodes, requests near the free capacity;
  * allocatable 0 on either resource (single-resource LeastAllocated / Balanced, spec S4/S5);
  * missing vs explicit-zero requests (non-zero defaults 100m / 200Mi, spec S2);
  * arbitrary cpu denominators and — on the ki / decimal grids — memory quantities that are odd
    multiples of 1 Ki or decimal (10^6) multiples, which only the wide device layout can hold;
  * ties: many identical nodes (the lowest index must win, spec S7);
  * config-4 masks (taints, tolerations, selectors, required / preferred terms, amd.com/gpu);
  * batched-mode anti-affinity groups (hostname / zone) when the profile allows batched mode.
"""
import json
import os

import numpy as np

from oracle import oracle as O

MIB, GIB, KI = 1 << 20, 1 << 30, 1 << 10
HERE = os.path.dirname(os.path.abspath(__file__))
CASES_PATH = os.path.join(HERE, "golden", "fuzz_cases.json")

WEIGHTS = {
    0: ({}, {}),
    1: (dict(w_fit=(10, 20, 30), w_bal=(5, 7, 9), fit_weight_cpu=2, fit_weight_mem=3),
        dict(wc=2, wm=3, w_fit=(10, 20, 30), w_bal=(5, 7, 9))),
    2: (dict(fit_weight_cpu=0, fit_weight_mem=1), dict(wc=0, wm=1)),
}
FEATURES = dict(enable_taint=1, enable_affinity=1)


def load_cases():
    with open(CASES_PATH) as f:
        return json.load(f)["cases"]


def _round_to(v, unit):
    return (v // unit) * unit


def _node_memory(rng, n, grid):
    zero = rng.random(n) < 0.05
    if grid == "binary":
        m = rng.choice([1, 2, 4, 8, 16], n) * GIB
    elif grid == "ki":
        small = (rng.integers(1 << 20, 16 << 20, n) | 1) * KI   # 1-16 GiB, odd Ki
        big = (rng.integers(64 << 20, 768 << 20, n) | 1) * KI   # 64-768 GiB, odd Ki
        m = np.where(rng.random(n) < 0.5, small, big)
    else:
        dec = rng.choice([10**9, 2 * 10**9, 4 * 10**9, 8 * 10**9, 16 * 10**9, 100 * 10**9,
                          500 * 10**9], n)
        arb = rng.integers(500, 800_000, n) * 10**6
        m = np.where(rng.random(n) < 0.5, dec, arb)
    return np.where(zero, 0, m).astype(np.int64)


def _pod_memory(rng, p, grid):
    base = rng.choice([0, 64, 128, 512, 1024, 4096], p) * MIB
    if grid == "binary":
        m = base
    elif grid == "ki":
        m = np.where(rng.random(p) < 0.5, base, (rng.integers(1, 4 << 20, p) | 1) * KI)
    else:
        m = rng.choice([0, 100 * 10**6, 512 * 10**6, 10**9, 2_500_000_000, 128 * MIB,
                        3 * 10**9 + 1], p)
    return m.astype(np.int64)


def _usage_unit(grid):
    return {"binary": MIB, "ki": KI, "decimal": 10**6}[grid]


def build(case):
    """(nodes, pods, gpu_cfg, oracle_cfg) of one fuzz case."""
    rng = np.random.default_rng(case["seed"])
    n, p, grid = case["n"], case["p"], case["grid"]
    nodes, pods = O.empty_cluster(n, p)
    if grid == "binary":
        cpu = rng.choice([1000, 2000, 4000, 6000, 8000], n)
    else:
        cpu = rng.integers(1, 96_001, n)
    nodes["alloc_cpu"][:] = np.where(rng.random(n) < 0.05, 0, cpu)
    nodes["alloc_mem"][:] = _node_memory(rng, n, grid)
    nodes["max_pods"][:] = rng.choice([1, 2, 5, 110], n)
    # ties: a block of identical nodes (equal totals; the lowest index must win)
    if n >= 8:
        a = int(rng.integers(0, n - 4))
        nodes["alloc_cpu"][a:a + 4] = nodes["alloc_cpu"][a]
        nodes["alloc_mem"][a:a + 4] = nodes["alloc_mem"][a]
        nodes["max_pods"][a:a + 4] = nodes["max_pods"][a]
    if case["init_usage"]:
        u = _usage_unit(grid)
        fc, fm = rng.random(n) * 0.95, rng.random(n) * 0.95
        nodes["req_cpu"][:] = (nodes["alloc_cpu"] * fc).astype(np.int64)
        nodes["req_mem"][:] = _round_to((nodes["alloc_mem"] * fm).astype(np.int64), u)
        nodes["nz_cpu"][:] = nodes["req_cpu"] + 100 * rng.integers(0, 3, n)
        nodes["nz_mem"][:] = nodes["req_mem"] + 200 * MIB * rng.integers(0, 3, n)
        nodes["pods"][:] = rng.integers(0, nodes["max_pods"] + 1)
    # pods
    pods["qos"][:] = rng.integers(0, 3, p)
    if grid == "binary":
        cpu = rng.choice([0, 100, 250, 500, 1000, 2000, 4000], p)
    else:
        cpu = np.where(rng.random(p) < 0.5, rng.choice([0, 100, 250, 500, 1000, 2000, 4000], p),
                       rng.integers(1, 8001, p))
    mem = _pod_memory(rng, p, grid)
    cpu_missing = rng.random(p) < 0.3
    mem_missing = rng.random(p) < 0.15
    pods["req_cpu"][:] = np.where(cpu_missing, 0, cpu)
    pods["nz_cpu"][:] = np.where(cpu_missing, O.DEF_CPU, cpu)      # an explicit 0 stays 0
    pods["req_mem"][:] = np.where(mem_missing, 0, mem)
    pods["nz_mem"][:] = np.where(mem_missing, O.DEF_MEM, mem)
    gcfg, ocfg = (dict(x) for x in WEIGHTS[case["weights"]])
    gcfg["qos_sort"] = ocfg["qos_sort"] = case["qos_sort"]
    if case["features"]:
        nodes["alloc_ext"][:, 0] = rng.choice([0, 0, 4, 8], n)
        nodes["alloc_ext"][:, 1] = rng.choice([0, 1, 2], n)
        nodes["taint_hard"][:] = rng.choice([0, 0, 1, 2], n).astype(np.uint64)
        nodes["taint_soft"][:] = rng.choice([0, 4, 8, 12], n).astype(np.uint64)
        nodes["label_bits"][:, 0] = rng.integers(0, 16, n).astype(np.uint64)
        nodes["label_bits"][:, 1] = rng.integers(0, 4, n).astype(np.uint64) << np.uint64(62)
        pods["req_ext"][:, 0] = rng.choice([0, 0, 0, 1, 2, 8], p)
        pods["req_ext"][:, 1] = rng.choice([0, 0, 0, 1], p)
        pods["tol_hard"][:] = rng.choice([0, 1, 3], p).astype(np.uint64)
        pods["tol_soft"][:] = rng.choice([0, 4], p).astype(np.uint64)
        pods["sel"][:, 0] = rng.choice([0, 0, 1], p).astype(np.uint64)
        pods["sel"][:, 1] = rng.choice([0, 0, 0, 1 << 62], p).astype(np.uint64)
        pods["n_req_terms"][:] = rng.integers(0, 3, p)
        pods["req_terms"][:, :, 0] = rng.integers(0, 16, (p, 4)).astype(np.uint64)
        pods["n_pref_terms"][:] = rng.integers(0, 4, p)
        pods["pref_terms"][:, :, 0] = rng.integers(1, 16, (p, 4)).astype(np.uint64)
        pods["pref_weight"][:] = rng.integers(1, 101, (p, 4))
        gcfg.update(FEATURES)
        ocfg.update(FEATURES)
    else:
        nodes["zone"][:] = rng.integers(0, 4, n)
        pods["app"][:] = rng.integers(0, 8, p)
        pods["anti_affinity"][:] = rng.choice([0, 0, 1, 2], p)
    return nodes, pods, gcfg, ocfg


def memory_is_compact(nodes, pods):
    """True when every memory quantity fits the compact int32 layout (spec S10: 2^u-byte units,
    u = the largest power of two dividing every quantity, capped at 20, values < 2^24)."""
    vals = [nodes[k] for k in ("alloc_mem", "req_mem", "nz_mem")] + \
           [pods[k] for k in ("req_mem", "nz_mem")]
    allv = np.concatenate([np.asarray(v, np.int64).ravel() for v in vals])
    nz = allv[allv != 0]
    u = 20 if nz.size == 0 else min(20, int(np.min([(int(x) & -int(x)).bit_length() - 1 for x in nz])))
    return bool((allv >> u).max(initial=0) < (1 << 24))
