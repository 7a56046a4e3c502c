"""Batched mode (spec/semantics.md S11) on the CPU oracle: invariants and the exact-mode limit.

S11 is approximate by design (a node takes at most one pod per batch, pods score against the
batch-start table), so its checks are (i) the placements it makes are feasible and respect the
required anti-affinity (per node for hostname apps, per zone for zone apps), (ii) with batches of
one pod it IS the exact sequential stream, and (iii) the GPU reproduces it bit for bit
(tests/test_gpu_batched.py).
"""
import numpy as np
import pytest

from oracle import oracle as O


def check_invariants(nodes0, nodes, pods, placement):
    p = len(placement)
    assert (placement >= -1).all(), "every pod decided"
    for k in ("req_cpu", "req_mem"):
        alloc = nodes["alloc_cpu" if k == "req_cpu" else "alloc_mem"]
        assert (nodes[k] <= alloc).all(), k
    assert (nodes["pods"] <= nodes["max_pods"]).all()
    # the final table is the initial one plus the placed pods' requests
    placed = placement >= 0
    for k, pk in (("req_cpu", "req_cpu"), ("req_mem", "req_mem"), ("nz_cpu", "nz_cpu"), ("nz_mem", "nz_mem")):
        exp = nodes0[k].copy()
        np.add.at(exp, placement[placed], pods[pk][placed])
        assert np.array_equal(exp, nodes[k]), k
    app, aa, zone = pods["app"], pods["anti_affinity"], nodes["zone"]
    host = {}
    zon = {}
    for j in range(p):
        n = int(placement[j])
        if n < 0:
            continue
        if aa[j] == 1:
            key = (int(app[j]), n)
            assert key not in host, f"hostname anti-affinity violated by pods {host.get(key)} and {j}"
            host[key] = j
        if aa[j] == 2:
            key = (int(app[j]), int(zone[n]))
            assert key not in zon, f"zone anti-affinity violated by pods {zon.get(key)} and {j}"
            zon[key] = j


@pytest.mark.parametrize("batch", [1, 7, 64])
def test_batched_invariants_config5(batch):
    nodes, pods = O.generate(5, 150, 4000)
    n0, _ = O.copy_cluster(nodes, pods)
    pl, keys, nb = O.schedule_batched(nodes, pods, batch=batch, nthreads=4)
    check_invariants(n0, nodes, pods, pl)
    assert (pl == -1).any() and (pl >= 0).any()
    assert nb >= -(-len(pl) // batch)
    # a hostname-AA app never has two pods on one node even when the cluster is tight
    assert ((pods["anti_affinity"] == 1) & (pl >= 0)).sum() > 100


def test_batch_of_one_is_the_exact_stream():
    """Without anti-affinity, S11 with one pod per batch degenerates to spec S7/S8 exactly."""
    nodes, pods = O.generate(2, 120, 2500)
    a, _ = O.copy_cluster(nodes, pods)
    b, _ = O.copy_cluster(nodes, pods)
    pe, ke, _ = O.schedule(a, pods)
    pb, kb, _ = O.schedule_batched(b, pods, batch=1)
    assert np.array_equal(pe, pb) and np.array_equal(ke, kb)
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pods"):
        assert np.array_equal(a[k], b[k])


def test_batched_places_every_pod_of_a_roomy_cluster():
    nodes, pods = O.generate(2, 300, 2000)
    n0, _ = O.copy_cluster(nodes, pods)
    pl, _, nb = O.schedule_batched(nodes, pods, batch=64)
    check_invariants(n0, nodes, pods, pl)
    assert (pl >= 0).all()
    assert nb == -(-2000 // 64)  # nothing carried: every pod found a free candidate
