"""GPU parity of configurable scoring resources (spec/semantics.md S5 "Scoring
resources"): NodeResourcesFitArgs.ScoringStrategy.Resources with extended
resources (e.g. {cpu:1, memory:1, amd.com/gpu:5}) and NodeResourcesBalancedAllocationArgs.Resources
with three or four entries (the mean / sqrt standard deviation of balanced_allocation.go).

Every engine (resident and per-window lookahead, scan, persistent, batched, sharded lists, the
framework path's qs_score_pod) against the oracle bit for bit: placements, per-pod keys and the
final table.  The oracle's restatement is pinned by spec/kat.md K10-K15.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from qsched import Scheduler, pods_from_struct, synth_generate  # noqa: E402

from rescfg import GPU_CFG, NAMED, add_ext1, random_resource_cfg  # noqa: E402
from test_gpu_framework import oracle_scores  # noqa: E402
from test_gpu_parity import CFG4, assert_same, run_gpu, run_oracle  # noqa: E402
from test_gpu_wide import ki_cluster  # noqa: E402


def cluster(n, p, seed=11):
    """Config-4 shaped cluster (amd.com/gpu = ext0 on 10 % of the nodes) plus a second extended
    resource (ext1) on some nodes and pods, and some gpu already in use."""
    nodes, pods = synth_generate(4, n, p, seed=seed)
    rng = np.random.default_rng(seed)
    op = pods_from_struct(pods)
    add_ext1(rng, nodes, op)
    pods["req_ext"] = op["req_ext"]
    nodes["req_ext"][:, 0] = np.minimum(nodes["alloc_ext"][:, 0], rng.integers(0, 3, n))
    return nodes, pods


ENGINES = [("lookahead", "1"), ("lookahead", "0"), ("scan", "1"), ("persistent", "1")]


@pytest.mark.parametrize("prof", [{}, CFG4], ids=["fit-balanced", "norm"])
@pytest.mark.parametrize("engine,resident", ENGINES, ids=["resident", "per-window", "scan", "persistent"])
@pytest.mark.parametrize("name", list(NAMED))
def test_resource_lists_engines(oracle, monkeypatch, name, engine, resident, prof):
    monkeypatch.setenv("QS_RESIDENT", resident)
    cfg = dict(NAMED[name], **prof)
    nodes, pods = cluster(1800, 4000)
    g = run_gpu(nodes, pods, cfg, engine)
    o = run_oracle(oracle, nodes, pods, cfg)
    assert_same(g[:2], o[:2], g[2], o[2])
    if engine == "lookahead":
        assert g[3]["resident"] == int(resident)


@pytest.mark.parametrize("serial", [0, 1])
def test_config4_full_gpu_scoring(oracle, serial):
    """BASELINE.json configs[3] at full size (5,000 nodes x 150,000 pods, TaintToleration +
    NodeAffinity + amd.com/gpu) with LeastAllocated {cpu:1, memory:1, amd.com/gpu:5} and
    BalancedAllocation over [cpu, memory, amd.com/gpu]: every placement, key and the final table."""
    cfg = dict(CFG4, **GPU_CFG, lookahead_serial=serial)
    nodes, pods = synth_generate(4, 5000, 150000)
    g = run_gpu(nodes, pods, cfg, "lookahead")
    o = run_oracle(oracle, nodes, pods, cfg)
    assert_same(g[:2], o[:2], g[2], o[2])
    assert g[3]["resident"] == (1 if serial == 0 else 0)


@pytest.mark.parametrize("seed", range(8))
def test_random_resource_lists(oracle, seed):
    """Random lists (1-4 distinct resources, random order, weights 1..100) on small clusters with
    zero allocatables and both extended columns, resident lookahead and scan."""
    rng = np.random.default_rng(1000 + seed)
    rc = random_resource_cfg(rng)
    cfg = dict(rc, **(CFG4 if seed % 2 else {}))
    nodes, pods = cluster(int(rng.integers(200, 3000)), 3000, seed=seed)
    nodes["alloc_cpu"][rng.random(len(nodes["alloc_cpu"])) < 0.03] = 0
    o = run_oracle(oracle, nodes, pods, cfg)
    for engine in ("lookahead", "scan"):
        g = run_gpu(nodes, pods, cfg, engine)
        assert_same(g[:2], o[:2], g[2], o[2])


def test_wide_layout_gpu_scoring(oracle):
    """The wide row layout (odd-Ki memory, decimal requests) with the GPU scoring lists."""
    nodes, pods = ki_cluster(3000, 8000, features=True)
    cfg = dict(CFG4, **GPU_CFG)
    g = run_gpu(nodes, pods, cfg, "lookahead")
    assert g[3]["table_layout"] == "wide"
    o = run_oracle(oracle, nodes, pods, cfg)
    assert_same(g[:2], o[:2], g[2], o[2])
    s = run_gpu(nodes, pods, dict(GPU_CFG), "scan")
    o2 = run_oracle(oracle, nodes, pods, dict(GPU_CFG))
    assert_same(s[:2], o2[:2], s[2], o2[2])


@pytest.mark.parametrize("shards", [2, 4])
def test_virtual_shards_gpu_scoring(oracle, shards):
    """The sharded lookahead layout (virtual shards in one process) with the GPU scoring lists."""
    cfg = dict(GPU_CFG, virtual_shards=shards)
    nodes, pods = cluster(6000, 5000)
    g = run_gpu(nodes, pods, cfg, "lookahead")
    o = run_oracle(oracle, nodes, pods, dict(GPU_CFG))
    assert_same(g[:2], o[:2], g[2], o[2])


def test_batched_gpu_scoring(oracle):
    """Batched mode (spec S11) scores its lists with the configured resources too."""
    nodes, pods = synth_generate(5, 3000, 12000)
    op = pods_from_struct(pods)
    rng = np.random.default_rng(5)
    nodes["alloc_ext"][:, 0] = np.where(rng.random(3000) < 0.2, 8, 0)
    op["req_ext"][:, 0] = np.where(rng.random(12000) < 0.05, 1, 0)
    pods["req_ext"] = op["req_ext"]
    with Scheduler(dict(GPU_CFG)) as s:
        s.load_nodes(nodes)
        pl = s.schedule(pods, mode="batched")
    on = {k: v.copy() for k, v in nodes.items()}
    o_pl, _, _ = oracle.schedule_batched(on, pods_from_struct(pods), batch=64, cfg=dict(GPU_CFG), nthreads=16)
    assert np.array_equal(pl, o_pl)


@pytest.mark.parametrize("layout", [{}, {"scan_soa_min_nodes": 1}], ids=["rows", "soa"])
def test_score_pod_resource_lists(oracle, layout):
    """The framework path (qs_score_pod: Filter + the four plugin scores of every node) with the GPU
    scoring lists, across Reserves."""
    nodes, pods = cluster(2500, 60)
    cfg = dict(CFG4, **GPU_CFG)
    on = {k: v.copy() for k, v in nodes.items()}
    op = pods_from_struct(pods)
    with Scheduler(dict(cfg, **layout)) as s:
        s.load_nodes(nodes)
        for j in range(0, 60, 3):
            got = s.score_pod(pods[j])
            feas, sc, total, best = oracle_scores(on, pods, j, cfg)
            assert np.array_equal(got["feasible"], feas)
            assert np.array_equal(got["total"], total)
            np.testing.assert_array_equal(got["scores"][feas], sc[feas])
            assert got["best"] == best
            if best >= 0:
                s.reserve(best, pods[j])
                for f, g in (("req_cpu", "req_cpu"), ("req_mem", "req_mem"), ("nz_cpu", "nz_cpu"),
                             ("nz_mem", "nz_mem")):
                    on[f][best] += op[g][j]
                on["req_ext"][best] += op["req_ext"][j]
                on["pods"][best] += 1
