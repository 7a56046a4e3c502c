"""The incremental-argmax oracle (or_schedule_incremental) against the brute-force oracle
(or_schedule), bit for bit: placements, per-pod best keys and the final node table; likewise the
incremental batched oracle (or_schedule_batched_incremental) against or_schedule_batched.

or_schedule_incremental keeps, per pod type (requests, non-zero requests, extended requests, QoS
class), a max tree over the nodes' packed keys and re-scores only the reserved node per pod; it
evaluates the same node_key() as or_schedule, so it must agree exactly.  It is the checker that
makes the full config-3 stream (50,000 nodes x 1,000,000 pods) diffable in seconds
(tests/test_gpu_scale.py, bench.py's config3 leg).  CPU only.
"""
import numpy as np
import pytest

from qsched import pods_from_struct, synth_generate


def both(oracle, nodes, pods, cfg=None, nthreads=4):
    a = {k: v.copy() for k, v in nodes.items()}
    b = {k: v.copy() for k, v in nodes.items()}
    sub = pods_from_struct(pods)
    p1, k1, o1 = oracle.schedule(a, sub, cfg, nthreads=nthreads)
    p2, k2, o2 = oracle.schedule_incremental(b, sub, cfg, nthreads=nthreads)
    return (p1, k1, o1, a), (p2, k2, o2, b)


def assert_equal(x, y):
    assert np.array_equal(x[0], y[0]), np.nonzero(x[0] != y[0])[0][:5]
    assert np.array_equal(x[1], y[1])
    assert np.array_equal(x[2], y[2])
    for k in x[3]:
        assert np.array_equal(x[3][k], y[3][k]), k


@pytest.mark.parametrize("config,n,p", [(1, 100, 1000), (2, 700, 9000), (2, 1500, 6000), (3, 2000, 12000),
                                        (4, 1800, 5000), (5, 900, 4000)])
def test_incremental_matches_brute_force(oracle, config, n, p):
    x, y = both(oracle, *synth_generate(config, n, p))
    assert_equal(x, y)


@pytest.mark.parametrize("cfg", [dict(qos_sort=0), dict(balanced_skip_besteffort=1),
                                 dict(wc=2, wm=3, w_fit=(10, 20, 30), w_bal=(5, 7, 9)),
                                 dict(wc=0, wm=1), dict(w_fit=(0, 0, 0), w_bal=(1, 1, 1))])
def test_incremental_profiles(oracle, cfg):
    x, y = both(oracle, *synth_generate(2, 600, 5000), cfg)
    assert_equal(x, y)


def test_incremental_tight_and_ragged(oracle):
    """Nodes that fill up (pod limits 1-3, zero allocatable) and pods with missing requests: many
    infeasible and unschedulable decisions, many ties."""
    nodes, pods = synth_generate(2, 257, 3000, seed=11)
    rng = np.random.default_rng(5)
    nodes["max_pods"][:] = rng.integers(1, 4, 257)
    nodes["alloc_cpu"][::7] = 0
    nodes["alloc_mem"][::11] = 0
    pods["req_cpu"][::5] = 0
    x, y = both(oracle, nodes, pods)
    assert_equal(x, y)
    assert (x[0] < 0).mean() > 0.3


def test_incremental_empty_inputs(oracle):
    nodes, pods = synth_generate(2, 50, 0)
    x, y = both(oracle, nodes, pods)
    assert x[0].size == y[0].size == 0


def test_incremental_rejects_normalizing_profiles(oracle):
    nodes, pods = synth_generate(4, 100, 100)
    with pytest.raises(ValueError):
        oracle.schedule_incremental({k: v.copy() for k, v in nodes.items()}, pods_from_struct(pods),
                                    dict(enable_taint=1, enable_affinity=1))


def both_batched(oracle, nodes, pods, batch=64, cfg=None, nthreads=4):
    a = {k: v.copy() for k, v in nodes.items()}
    b = {k: v.copy() for k, v in nodes.items()}
    sub = pods_from_struct(pods)
    p1, k1, n1 = oracle.schedule_batched(a, sub, batch=batch, cfg=cfg, nthreads=nthreads)
    p2, k2, n2 = oracle.schedule_batched_incremental(b, sub, batch=batch, cfg=cfg, nthreads=nthreads)
    return (p1, k1, n1, a), (p2, k2, n2, b)


@pytest.mark.parametrize("config,n,p,batch", [(5, 1000, 20000, 64), (5, 300, 9000, 7), (5, 200, 2000, 1),
                                              (5, 64, 3000, 64), (2, 2000, 30000, 64), (4, 800, 12000, 64),
                                              (1, 100, 1000, 32)])
def test_batched_incremental_matches_brute_force(oracle, config, n, p, batch):
    """Per-type per-zone max trees + a best-first walk over the allowed zones give each pod the same
    64-entry list as the brute-force scan (hostname / zone anti-affinity, carried pods, tight
    clusters where most pods are unschedulable or carried)."""
    x, y = both_batched(oracle, *synth_generate(config, n, p), batch=batch)
    assert_equal(x, y)


def test_batched_incremental_tight_zones(oracle):
    """Few nodes per zone, many zone-anti-affinity pods: most lists run out of allowed zones."""
    nodes, pods = synth_generate(5, 120, 6000, seed=3)
    nodes["zone"][:] = np.arange(120) % 3
    pods["anti_affinity"][::2] = 2
    x, y = both_batched(oracle, nodes, pods)
    assert_equal(x, y)
    assert (x[0] < 0).mean() > 0.2


def test_batched_incremental_rejects_normalizing_profiles(oracle):
    nodes, pods = synth_generate(4, 100, 100)
    with pytest.raises(ValueError):
        oracle.schedule_batched_incremental({k: v.copy() for k, v in nodes.items()}, pods_from_struct(pods),
                                            cfg=dict(enable_taint=1))
