"""Known-answer tests pinning the CPU oracle (spec/kat.md = SURVEY.md A.10).

The reference has no tests (parity unpinned); these hand-computed cases are what pins both oracle
restatements (C: oracle/qs_oracle.c, Python: oracle/oracle.py py_*).
"""
import ctypes
import math

import numpy as np
import pytest

from oracle import oracle as O

MIB, GIB = 1 << 20, 1 << 30


def la_c(ac, zc, am, zm, w=(1, 1)):
    return O.lib().or_least_allocated(ac, zc, am, zm, w[0], w[1])


def ba_c(ac, rc, am, rm):
    return O.lib().or_balanced(ac, rc, am, rm)


KAT_SCORES = [
    # name, alloc (cpu, mem), NonZeroRequested after pod (cpu, mem), Requested after pod, LA, BA
    ("K1", (4000, 10000), (3000, 5000), (3000, 5000), 37, 87),
    ("K2", (6000, 10000), (3000, 5000), (3000, 5000), 50, 100),
    ("K3", (4000, 8 * GIB), (100, 200 * MIB), (0, 0), 97, 100),
    ("K4", (4000, 10000), (5000, 1000), (5000, 1000), 45, 55),
    ("K7", (4000, 25 * GIB), (2000, 17 * GIB), (2000, 17 * GIB), 41, 90),
]


@pytest.mark.parametrize("name,alloc,nz,req,la,ba", KAT_SCORES)
def test_kat_scores(name, alloc, nz, req, la, ba):
    assert la_c(alloc[0], nz[0], alloc[1], nz[1]) == la
    assert O.py_least_allocated(alloc, nz) == la
    assert ba_c(alloc[0], req[0], alloc[1], req[1]) == ba
    assert O.py_balanced(alloc, req) == ba


def test_float64_sentinels():
    # spec/kat.md: IEEE binary64 (Go float64) truncation sentinels
    assert (1 - 0.45) * 100.0 == 55.00000000000001
    f0, f1 = 2000 / 4000, (17 * GIB) / (25 * GIB)  # K7: f1 = 0.68 -> std = 0.09000000000000002
    assert abs((f0 - f1) / 2) == 0.09000000000000002
    assert (1 - abs((f0 - f1) / 2)) * 100.0 == 90.99999999999999
    assert O.py_balanced((4000, 25 * GIB), (2000, 17 * GIB)) == 90  # exact rational math: 91
    # (f0, f1) = (1, 41/50) and (1/2, 34/50)
    for (a0, r0), (a1, r1) in [((50, 60), (50, 41)), ((2, 1), (50, 34))]:
        c = ba_c(a0, r0, a1, r1)
        assert c == O.py_balanced((a0, a1), (r0, r1))


def test_kat_single_resource_and_zero_alloc():
    # K8: cpu alloc 0 -> cpu skipped in both scorers; one fraction -> std 0 -> Balanced 100
    assert la_c(0, 100, 10000, 209) == (10000 - 209) * 100 // 10000
    assert ba_c(0, 0, 10000, 5000) == 100
    assert la_c(0, 0, 0, 0) == 0  # weight sum 0


def _one_node(alloc_cpu, alloc_mem, pods=0, max_pods=110, req_cpu=0, req_mem=0):
    nodes, _ = O.empty_cluster(1, 0)
    nodes["alloc_cpu"][0], nodes["alloc_mem"][0] = alloc_cpu, alloc_mem
    nodes["pods"][0], nodes["max_pods"][0] = pods, max_pods
    nodes["req_cpu"][0], nodes["req_mem"][0] = req_cpu, req_mem
    nodes["nz_cpu"][0], nodes["nz_mem"][0] = req_cpu, req_mem
    return nodes


def _one_pod(cpu, mem, qos=1):
    _, pods = O.empty_cluster(0, 1)
    pods["req_cpu"][0] = pods["nz_cpu"][0] = cpu
    pods["req_mem"][0] = pods["nz_mem"][0] = mem
    pods["qos"][0] = qos
    return pods


def test_kat_k5_too_many_pods():
    nodes = _one_node(4000, 8 * GIB, pods=110, max_pods=110)
    keys, _ = O.score_pod(nodes, _one_pod(100, MIB), 0)
    assert keys[0] == 0
    assert O.py_keys(nodes, _one_pod(100, MIB), 0, O.DEFAULT_CONFIG)[0] == 0


def test_kat_k6_lowest_index_wins_ties():
    nodes, _ = O.empty_cluster(10, 0)
    nodes["alloc_cpu"][:] = 1000
    nodes["alloc_mem"][:] = GIB
    nodes["max_pods"][:] = 110
    nodes["alloc_cpu"][[3, 7]] = 8000  # nodes 3 and 7 tie with the best score
    nodes["alloc_mem"][[3, 7]] = 8 * GIB
    pods = _one_pod(500, 256 * MIB)
    pl, best, _ = O.schedule(nodes, pods)
    assert pl[0] == 3
    assert (int(best[0]) & 0xFFFFFFFF) == 0xFFFFFFFF - 3


def test_kat_k9_fit_is_not_strict_at_equality():
    nodes = _one_node(4000, 8 * GIB, req_cpu=3000, req_mem=7 * GIB)
    keys, _ = O.score_pod(nodes, _one_pod(1000, GIB), 0)
    assert keys[0] != 0
    keys, _ = O.score_pod(nodes, _one_pod(1001, GIB), 0)
    assert keys[0] == 0


def test_qos_weights_change_the_winner():
    # node 0: cpu-heavy free capacity (high LeastAllocated), node 1: balanced (high Balanced).
    nodes, _ = O.empty_cluster(2, 0)
    nodes["alloc_cpu"][:] = [16000, 4000]
    nodes["alloc_mem"][:] = [4 * GIB, 4 * GIB]
    nodes["max_pods"][:] = 110
    res = {}
    for q in (0, 1, 2):
        pods = _one_pod(2000, GIB, qos=q)
        keys, sc = O.score_pod(nodes, pods, 0)
        res[q] = (sc[:, 0].tolist(), sc[:, 1].tolist(), (keys >> np.uint64(32)).tolist())
        w = O.DEFAULT_CONFIG["w_fit"][q]
        for n in range(2):
            assert int(keys[n] >> np.uint64(32)) == w * sc[n, 0] + sc[n, 1] + 1
    assert res[0][0] == res[2][0]  # plugin scores do not depend on the class; the weights do


def test_spec_defaults_match_upstream_profile():
    assert O.DEFAULT_CONFIG["w_tt"] == 3 and O.DEFAULT_CONFIG["w_na"] == 2
    assert O.DEF_CPU == 100 and O.DEF_MEM == 209715200


# ---- configurable scoring resources (spec/kat.md K10-K15, spec S5 "Scoring resources") ----------
def _v(vals):
    return (ctypes.c_int64 * len(vals))(*vals)


def la_v(alloc, reqd, w):
    return O.lib().or_least_allocated_v(len(alloc), _v(alloc), _v(reqd), _v(w))


def ba_v(alloc, reqd):
    return O.lib().or_balanced_v(len(alloc), _v(alloc), _v(reqd))


KAT_RES = [
    # name, alloc, reqd (after the pod), weights (None: Balanced only), LA, BA
    ("K10", (8000, 32 * GIB, 8), (4000, 16 * GIB, 6), (1, 1, 5), 32, 88),
    ("K10b", (8000, 32 * GIB, 0), (4000, 16 * GIB, 0), (1, 1, 5), 50, 100),
    ("K12", (4000, 10 * GIB, 5), (3200, 8 * GIB, 4), (1, 1, 1), 20, 99),
    ("K15", (4000, 10, 8, 4), (2000, 5, 9, 4), (1, 1, 1, 1), 25, 75),
]


@pytest.mark.parametrize("name,alloc,reqd,w,la,ba", KAT_RES)
def test_kat_resource_lists(name, alloc, reqd, w, la, ba):
    assert la_v(alloc, reqd, w) == la
    assert O.py_least_allocated(alloc, reqd, w) == la
    assert ba_v(alloc, reqd) == ba
    assert O.py_balanced(alloc, reqd) == ba


def test_three_resource_float64_sentinel():
    # K12: three equal fractions 4/5; the float64 mean is not 0.8, so std > 0 and the score is 99
    f = [3200 / 4000, (8 * GIB) / (10 * GIB), 4 / 5]
    mean = (f[0] + f[1] + f[2]) / 3
    assert mean == 0.8000000000000002
    s = 0.0
    for x in f:
        s = s + (x - mean) * (x - mean)
    assert (1 - math.sqrt(s / 3)) * 100.0 == 99.99999999999999
    assert ba_v((4000, 10 * GIB, 5), (3200, 8 * GIB, 4)) == 99  # exact arithmetic: 100


def _k10_cluster(gpu_req=4):
    nodes, pods = O.empty_cluster(1, 1)
    nodes["alloc_cpu"][0], nodes["alloc_mem"][0], nodes["alloc_ext"][0, 0] = 8000, 32 * GIB, 8
    nodes["max_pods"][0] = 110
    nodes["req_cpu"][0] = nodes["nz_cpu"][0] = 2000
    nodes["req_mem"][0] = nodes["nz_mem"][0] = 8 * GIB
    nodes["req_ext"][0, 0] = 2
    nodes["pods"][0] = 1
    pods["req_cpu"][0] = pods["nz_cpu"][0] = 2000
    pods["req_mem"][0] = pods["nz_mem"][0] = 8 * GIB
    pods["req_ext"][0, 0] = gpu_req
    pods["qos"][0] = 2
    return nodes, pods


@pytest.mark.parametrize("gpu_req,la,ba", [(4, 32, 88), (0, 50, 100)])
def test_kat_k10_k11_through_score_pod(gpu_req, la, ba):
    """K10 / K10b / K11 through the whole per-node evaluation of both oracles."""
    nodes, pods = _k10_cluster(gpu_req)
    cfg = dict(fit_resources=[("cpu", 1), ("memory", 1), ("ext0", 5)],
               balanced_resources=["cpu", "memory", "ext0"])
    keys, scores = O.score_pod(nodes, pods, 0, cfg)
    assert list(scores[0][:2]) == [la, ba]
    c = dict(O.DEFAULT_CONFIG, **cfg)
    assert O.py_keys(nodes, pods, 0, c) == [int(keys[0])]
    assert int(keys[0]) >> 32 == 3 * la + ba + 1  # Guaranteed: w_fit 3, w_bal 1


def test_kat_k13_k14_lists():
    # K13: gpu in the Balanced list but not requested -> the two-resource (K7) path
    nodes, pods = _k10_cluster(0)
    nodes["alloc_cpu"][0], nodes["alloc_mem"][0] = 4000, 25 * GIB
    for f in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pods"):
        nodes[f][0] = 0
    pods["req_cpu"][0] = pods["nz_cpu"][0] = 2000
    pods["req_mem"][0] = pods["nz_mem"][0] = 17 * GIB
    _, sc = O.score_pod(nodes, pods, 0, dict(balanced_resources=["cpu", "memory", "ext0"]))
    assert sc[0][1] == 90
    # K14: LeastAllocated over memory only; BestEffort pod (non-zero defaults)
    nodes["alloc_cpu"][0], nodes["alloc_mem"][0] = 4000, 10 * GIB
    nodes["nz_mem"][0] = 5 * GIB
    pods["req_cpu"][0] = pods["req_mem"][0] = 0
    pods["nz_cpu"][0], pods["nz_mem"][0], pods["qos"][0] = 100, 200 * MIB, 0
    _, sc = O.score_pod(nodes, pods, 0, dict(fit_resources=[("memory", 1)], balanced_resources=["cpu"]))
    assert sc[0][0] == 48 and sc[0][1] == 100  # one Balanced fraction -> std 0
