"""Device-side known-answer tests and adversarial fuzz parity through the C ABI (SURVEY.md §4:
the A.10 KATs "also a device KAT kernel on the GPU box", and fuzzed clusters with ties, capacity
edges, missing requests and alloc = 0).

* KATs (spec/kat.md K1-K9 + the extra float64 sentinels): hand-computed LeastAllocated /
  Balanced values, checked through qs_score_pod (row and column layouts) and as a one-pod stream
  on every engine (persistent, scan, scan over the SoA copy, lookahead overlapped / serial,
  virtual shards, batched).
* Fuzz: the 360 committed cases of tests/golden/fuzz_cases.json (tests/adversarial.py builds
  them: binary / odd-Ki / decimal memory grids, arbitrary cpu denominators, alloc 0, max_pods
  1-5, missing and zero requests, pre-used nodes, tie blocks, config-4 masks, custom weights)
  through every engine and qs_score_pod, bit-exact against the C oracle: placements, best keys,
  final node table.  Batched mode is checked against the oracle's or_schedule_batched on the
  cases whose profile it supports (no taint / affinity plugins).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from qsched import Scheduler, pods_from_struct, pods_to_struct  # noqa: E402

import adversarial as A  # noqa: E402
from oracle import oracle as O  # noqa: E402

MIB, GIB = 1 << 20, 1 << 30

ENGINES = {
    "persistent": dict(engine="persistent"),
    "scan": dict(engine="scan"),
    "scan_soa": dict(engine="scan", scan_soa_min_nodes=1),
    "lookahead": dict(engine="lookahead"),
    "lookahead_serial": dict(engine="lookahead", lookahead_serial=1),
    "vshards": dict(engine="lookahead"),
}
LAYOUTS = {"rows": {"scan_soa_min_nodes": -1}, "soa": {"scan_soa_min_nodes": 1}}


def gpu_stream(nodes, pods, cfg, mode="exact"):
    with Scheduler(cfg) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods)
        stats = st.run(mode=mode)
        pl, keys = st.results()
        st.free()
        final = s.read_nodes()
    return pl, keys, final, stats


def check_same(tag, got, want_pl, want_keys, want_nodes):
    pl, keys, final = got[:3]
    bad = np.nonzero(pl != want_pl)[0]
    assert bad.size == 0, (f"{tag}: {bad.size} placements differ; first pod {bad[0]}: "
                           f"gpu {pl[bad[0]]} oracle {want_pl[bad[0]]}")
    kb = np.nonzero(keys != want_keys)[0]
    assert kb.size == 0, f"{tag}: key differs at pod {kb[0]}: {int(keys[kb[0]]):#x} vs {int(want_keys[kb[0]]):#x}"
    for k in want_nodes:
        assert np.array_equal(final[k], want_nodes[k]), f"{tag}: final table column {k}"


# ---------------------------------------------------------------------------------------------
# Known-answer tests (spec/kat.md)
# ---------------------------------------------------------------------------------------------
def kat_case(alloc, node_req=(0, 0), node_nz=None, pod_req=(None, None), qos=1, max_pods=110,
             pods_on_node=0):
    """One node, one pod.  pod_req entries None = missing (non-zero defaults apply)."""
    nodes, pods = O.empty_cluster(1, 1)
    nodes["alloc_cpu"][0], nodes["alloc_mem"][0] = alloc
    nodes["req_cpu"][0], nodes["req_mem"][0] = node_req
    nz = node_nz if node_nz is not None else node_req
    nodes["nz_cpu"][0], nodes["nz_mem"][0] = nz
    nodes["max_pods"][0], nodes["pods"][0] = max_pods, pods_on_node
    c, m = pod_req
    pods["req_cpu"][0] = 0 if c is None else c
    pods["nz_cpu"][0] = O.DEF_CPU if c is None else c
    pods["req_mem"][0] = 0 if m is None else m
    pods["nz_mem"][0] = O.DEF_MEM if m is None else m
    pods["qos"][0] = qos
    return nodes, pods


# name -> (case kwargs, LeastAllocated, Balanced); None = infeasible
KATS = {
    "K1": (dict(alloc=(4000, 10000), pod_req=(3000, 5000)), 37, 87),
    "K2": (dict(alloc=(6000, 10000), pod_req=(3000, 5000)), 50, 100),
    "K3": (dict(alloc=(4000, 8 * GIB), pod_req=(None, None), qos=0), 97, 100),
    # K4: cpu over-committed through pre-existing usage (node Requested 5000 > allocatable 4000,
    # pod cpu request missing so Fit skips cpu): LeastAllocated cpu 0, Balanced cpu capped at 1
    "K4": (dict(alloc=(4000, 10000), node_req=(5000, 0), node_nz=(4900, 0), pod_req=(None, 1000)), 45, 55),
    "K5": (dict(alloc=(4000, 8 * GIB), pod_req=(100, MIB), max_pods=110, pods_on_node=110), None, None),
    "K7": (dict(alloc=(4000, 25 * GIB), pod_req=(2000, 17 * GIB)), 41, 90),
    # K7b / K7c: the other float64 truncation sentinels (f0, f1) = (1, 41/50) and (1/2, 34/50)
    "K7b": (dict(alloc=(50, 50), node_req=(60, 0), node_nz=(60, 0), pod_req=(None, 41)), None, None),
    "K7c": (dict(alloc=(2, 50), pod_req=(1, 34)), None, None),
    # K8: allocatable 0 on one resource -> that resource is skipped by both scorers
    "K8": (dict(alloc=(0, 10000), pod_req=(None, 5000)), 50, 100),
    "K8b": (dict(alloc=(4000, 0), pod_req=(1000, None)), 75, 100),
    "K8c": (dict(alloc=(0, 0), pod_req=(None, None), qos=0), 0, 100),
    # K9: Fit is not strict at equality
    "K9": (dict(alloc=(4000, 8 * GIB), node_req=(3000, 7 * GIB), pod_req=(1000, GIB)), 0, 100),
    "K9x": (dict(alloc=(4000, 8 * GIB), node_req=(3000, 7 * GIB), pod_req=(1001, GIB)), None, None),
}


def kat_expect(name):
    kw, la, ba = KATS[name]
    nodes, pods = kat_case(**kw)
    if name in ("K7b", "K7c"):  # sentinels: the independent pure-Python restatement
        alloc = (int(nodes["alloc_cpu"][0]), int(nodes["alloc_mem"][0]))
        la = O.py_least_allocated(alloc, (int(nodes["nz_cpu"][0] + pods["nz_cpu"][0]),
                                          int(nodes["nz_mem"][0] + pods["nz_mem"][0])))
        ba = O.py_balanced(alloc, (int(nodes["req_cpu"][0] + pods["req_cpu"][0]),
                                   int(nodes["req_mem"][0] + pods["req_mem"][0])))
    infeasible = name in ("K5", "K9x")
    return nodes, pods, (None if infeasible else la), (None if infeasible else ba)


def test_kat_expectations_are_the_oracles():
    """The hand-computed values agree with the oracle (which tests/test_oracle_kat.py pins)."""
    for name in KATS:
        nodes, pods, la, ba = kat_expect(name)
        keys, sc = O.score_pod(nodes, pods, 0)
        if la is None:
            assert keys[0] == 0, name
        else:
            assert (int(sc[0, 0]), int(sc[0, 1])) == (la, ba), name
    assert kat_expect("K7b")[3] == 90 and kat_expect("K7c")[3] == 90  # truncation: exact math gives 91


def kat_key(la, ba, qos, idx=0):
    if la is None:
        return 0
    w_fit, w_bal = O.DEFAULT_CONFIG["w_fit"][qos], O.DEFAULT_CONFIG["w_bal"][qos]
    return ((w_fit * la + w_bal * ba + 1) << 32) | (0xFFFFFFFF - idx)


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("name", list(KATS))
def test_kat_score_pod(name, layout):
    nodes, pods, la, ba = kat_expect(name)
    with Scheduler(LAYOUTS[layout]) as s:
        s.load_nodes(nodes)
        got = s.score_pod(pods_to_struct(pods)[0])
    if la is None:
        assert not got["feasible"][0] and got["best"] == -1 and got["total"][0] == -1
    else:
        assert got["feasible"][0] and got["best"] == 0
        assert (int(got["scores"][0, 0]), int(got["scores"][0, 1])) == (la, ba)
        q = int(pods["qos"][0])
        assert int(got["total"][0]) == O.DEFAULT_CONFIG["w_fit"][q] * la + O.DEFAULT_CONFIG["w_bal"][q] * ba


@pytest.mark.parametrize("engine", list(ENGINES) + ["batched"])
def test_kat_every_engine(engine):
    """Each KAT as a one-pod stream on every engine: the best key carries the expected total."""
    for name in KATS:
        nodes, pods, la, ba = kat_expect(name)
        cfg = dict(ENGINES.get(engine, {}))
        if engine == "vshards":
            cfg["virtual_shards"] = 2
        pl, keys, final, _ = gpu_stream(nodes, pods_to_struct(pods), cfg,
                                        mode="batched" if engine == "batched" else "exact")
        want = kat_key(la, ba, int(pods["qos"][0]))
        assert int(keys[0]) == want, f"{engine} {name}: key {int(keys[0]):#x} want {want:#x}"
        assert pl[0] == (-1 if la is None else 0), f"{engine} {name}"
        if la is not None:  # Reserve applied once
            assert int(final["pods"][0]) == int(nodes["pods"][0]) + 1
            assert int(final["nz_mem"][0]) == int(nodes["nz_mem"][0] + pods["nz_mem"][0])


@pytest.mark.parametrize("engine", list(ENGINES) + ["batched"])
def test_kat_k6_ties_lowest_index(engine):
    nodes, _ = O.empty_cluster(10, 0)
    nodes["alloc_cpu"][:] = 1000
    nodes["alloc_mem"][:] = GIB
    nodes["max_pods"][:] = 110
    nodes["alloc_cpu"][[3, 7]] = 8000
    nodes["alloc_mem"][[3, 7]] = 8 * GIB
    _, pods = kat_case((0, 0), pod_req=(500, 256 * MIB))
    cfg = dict(ENGINES.get(engine, {}))
    if engine == "vshards":
        cfg["virtual_shards"] = 3  # nodes 3 and 7 in different shards
    pl, keys, _, _ = gpu_stream(nodes, pods_to_struct(pods), cfg,
                                mode="batched" if engine == "batched" else "exact")
    assert pl[0] == 3 and (int(keys[0]) & 0xFFFFFFFF) == 0xFFFFFFFF - 3


def test_empty_table_and_empty_stream():
    nodes, pods = O.empty_cluster(0, 5)
    pods["req_cpu"][:] = pods["nz_cpu"][:] = 100
    pods["nz_mem"][:] = O.DEF_MEM
    pl, keys, _, _ = gpu_stream(nodes, pods_to_struct(pods), {})
    assert (pl == -1).all() and (keys == 0).all()
    nodes, pods = O.empty_cluster(10, 0)
    nodes["alloc_cpu"][:] = 1000
    nodes["alloc_mem"][:] = GIB
    nodes["max_pods"][:] = 110
    pl, keys, final, _ = gpu_stream(nodes, pods_to_struct(pods), {})
    assert pl.size == 0 and np.array_equal(final["pods"], nodes["pods"])


# ---------------------------------------------------------------------------------------------
# Fuzz (tests/golden/fuzz_cases.json)
# ---------------------------------------------------------------------------------------------
CASES = A.load_cases()
CHUNK = 40
GRIDS = ["binary", "ki", "decimal"]
GRID_CASES = {g: [c for c in CASES if c["grid"] == g] for g in GRIDS}
CHUNKS = [(g, i) for g in GRIDS for i in range((len(GRID_CASES[g]) + CHUNK - 1) // CHUNK)]
_ORACLE = {}


def oracle_exact(case):
    key = case["seed"]
    if key not in _ORACLE:
        nodes, pods, _, ocfg = A.build(case)
        on = {k: v.copy() for k, v in nodes.items()}
        pl, keys, _ = O.schedule(on, pods, ocfg, nthreads=8)
        _ORACLE[key] = (pl, keys, on)
    return _ORACLE[key]


def engine_cfg(engine, case, gcfg):
    cfg = dict(gcfg, **ENGINES[engine])
    if engine.startswith("lookahead") or engine == "vshards":
        cfg["lookahead"] = case["K"]
    if engine == "vshards":
        cfg["virtual_shards"] = case["vshards"]
        cfg["lookahead"] = min(case["K"], 32)
    return cfg


@pytest.mark.parametrize("grid,chunk", CHUNKS, ids=[f"{g}{i}" for g, i in CHUNKS])
@pytest.mark.parametrize("engine", list(ENGINES))
def test_fuzz_stream(engine, grid, chunk):
    for case in GRID_CASES[grid][chunk * CHUNK:(chunk + 1) * CHUNK]:
        nodes, pods, gcfg, _ = A.build(case)
        got = gpu_stream(nodes, pods_to_struct(pods), engine_cfg(engine, case, gcfg))
        pl, keys, on = oracle_exact(case)
        check_same(f"{engine} case {case['seed']}", got, pl, keys, on)


@pytest.mark.parametrize("grid,chunk", CHUNKS, ids=[f"{g}{i}" for g, i in CHUNKS])
def test_fuzz_batched(grid, chunk):
    ran = 0
    for case in GRID_CASES[grid][chunk * CHUNK:(chunk + 1) * CHUNK]:
        if case["features"]:
            continue  # batched mode supports the Fit + Balanced (+ extended resources) profile
        nodes, pods, gcfg, ocfg = A.build(case)
        got = gpu_stream(nodes, pods_to_struct(pods), gcfg, mode="batched")
        on = {k: v.copy() for k, v in nodes.items()}
        pl, keys, _ = O.schedule_batched(on, pods, batch=64, cfg=ocfg, nthreads=8)
        check_same(f"batched case {case['seed']}", got,
                   pl, keys, {k: on[k] for k in ("req_cpu", "req_mem", "req_ext", "nz_cpu", "nz_mem", "pods")})
        ran += 1
    assert ran > 0


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("grid,chunk", CHUNKS, ids=[f"{g}{i}" for g, i in CHUNKS])
def test_fuzz_score_pod(layout, grid, chunk):
    for case in GRID_CASES[grid][chunk * CHUNK:(chunk + 1) * CHUNK]:
        nodes, pods, gcfg, ocfg = A.build(case)
        if case["p"] == 0:
            continue
        arr = pods_to_struct(pods)
        with Scheduler(dict(gcfg, **LAYOUTS[layout])) as s:
            s.load_nodes(nodes)
            for j in range(min(3, case["p"])):
                got = s.score_pod(arr[j])
                keys, sc = O.score_pod(nodes, pods, j, ocfg)
                feas = keys != 0
                total = np.where(feas, (keys >> np.uint64(32)).astype(np.int64) - 1, -1)
                best = int(0xFFFFFFFF - (int(keys.max()) & 0xFFFFFFFF)) if keys.max() else -1
                tag = f"case {case['seed']} pod {j}"
                assert np.array_equal(got["feasible"], feas), tag
                assert np.array_equal(got["total"], total), tag
                assert got["best"] == best, tag
                np.testing.assert_array_equal(got["scores"][feas], sc[feas], err_msg=tag)
