"""Cross-checks of the two oracle restatements and the three generator restatements.

* C oracle (liboracle.so) vs pure-Python oracle (oracle.py py_*): placements and best keys on
  hypothesis-fuzzed small clusters (ties, capacity edges, zero allocatable, config-4 masks).
* spec/synth.md generator: C oracle vs numpy restatement vs the product's qs_synth_generate
  (host code in libqsched.so; no GPU needed).
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import oracle as O
from rescfg import add_ext1, random_resource_cfg

MIB, GIB = 1 << 20, 1 << 30


def random_cluster(rng, n, p, features):
    nodes, pods = O.empty_cluster(n, p)
    nodes["alloc_cpu"][:] = rng.choice([0, 1000, 2000, 4000, 6000, 8000], n, p=[.05, .2, .2, .25, .15, .15])
    nodes["alloc_mem"][:] = rng.choice([0, 1, 2, 4, 8, 16], n, p=[.05, .15, .2, .3, .2, .1]) * GIB
    nodes["max_pods"][:] = rng.choice([1, 2, 5, 110], n)
    pods["qos"][:] = rng.integers(0, 3, p)
    cpu = rng.choice([0, 100, 250, 500, 1000, 2000, 4000], p)
    mem = rng.choice([0, 64, 128, 512, 1024, 4096], p) * MIB
    missing = rng.random(p) < 0.3
    pods["req_cpu"][:] = np.where(missing, 0, cpu)
    pods["req_mem"][:] = mem
    pods["nz_cpu"][:] = np.where(missing, 100, cpu)
    pods["nz_mem"][:] = np.where(mem == 0, 200 * MIB, mem)
    if features:
        nodes["alloc_ext"][:, 0] = rng.choice([0, 0, 4, 8], n)
        nodes["taint_hard"][:] = rng.choice([0, 0, 1, 2], n).astype(np.uint64)
        nodes["taint_soft"][:] = rng.choice([0, 4, 8, 12], n).astype(np.uint64)
        nodes["label_bits"][:, 0] = rng.integers(0, 16, n).astype(np.uint64)
        pods["req_ext"][:, 0] = rng.choice([0, 0, 0, 1, 2, 8], p)
        pods["tol_hard"][:] = rng.choice([0, 1, 3], p).astype(np.uint64)
        pods["tol_soft"][:] = rng.choice([0, 4], p).astype(np.uint64)
        pods["sel"][:, 0] = rng.choice([0, 0, 1], p).astype(np.uint64)
        pods["n_req_terms"][:] = rng.integers(0, 3, p)
        pods["req_terms"][:, :, 0] = rng.integers(0, 16, (p, 4)).astype(np.uint64)
        pods["n_pref_terms"][:] = rng.integers(0, 3, p)
        pods["pref_terms"][:, :, 0] = rng.integers(1, 16, (p, 4)).astype(np.uint64)
        pods["pref_weight"][:] = rng.integers(1, 101, (p, 4))
    return nodes, pods


CFG_FEATURES = dict(enable_taint=1, enable_affinity=1)


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 2**32 - 1), n=st.integers(1, 24), p=st.integers(0, 60),
       features=st.booleans(), qos_sort=st.booleans())
def test_c_oracle_equals_python_oracle(seed, n, p, features, qos_sort):
    rng = np.random.default_rng(seed)
    nodes, pods = random_cluster(rng, n, p, features)
    cfg = dict(O.DEFAULT_CONFIG, qos_sort=int(qos_sort), **(CFG_FEATURES if features else {}))
    n1, _ = O.copy_cluster(nodes, pods)
    n2, _ = O.copy_cluster(nodes, pods)
    pl_c, best_c, _ = O.schedule(n1, pods, cfg)
    pl_p, best_p = O.py_schedule(n2, pods, cfg)
    assert pl_c.tolist() == pl_p
    assert [int(x) for x in best_c] == best_p
    for k in n1:
        assert np.array_equal(n1[k], n2[k])


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 2**32 - 1), n=st.integers(1, 20), p=st.integers(0, 50), features=st.booleans())
def test_c_oracle_equals_python_oracle_resource_lists(seed, n, p, features):
    """Random LeastAllocated / Balanced resource lists (spec S5 "Scoring resources"), two extended
    resource columns, both oracles bit for bit."""
    rng = np.random.default_rng(seed)
    nodes, pods = random_cluster(rng, n, p, True)
    add_ext1(rng, nodes, pods)
    nodes["req_ext"][:, 0] = np.minimum(nodes["alloc_ext"][:, 0], rng.integers(0, 3, n))
    cfg = dict(O.DEFAULT_CONFIG, **random_resource_cfg(rng), **(CFG_FEATURES if features else {}))
    n1, _ = O.copy_cluster(nodes, pods)
    n2, _ = O.copy_cluster(nodes, pods)
    pl_c, best_c, _ = O.schedule(n1, pods, cfg)
    pl_p, best_p = O.py_schedule(n2, pods, cfg)
    assert pl_c.tolist() == pl_p
    assert [int(x) for x in best_c] == best_p


def test_openmp_arm_matches_sequential():
    nodes, pods = O.generate(2, 800, 3000)
    a, _ = O.copy_cluster(nodes, pods)
    b, _ = O.copy_cluster(nodes, pods)
    pa, ka, _ = O.schedule(a, pods, nthreads=1)
    pb, kb, _ = O.schedule(b, pods, nthreads=4)
    assert np.array_equal(pa, pb) and np.array_equal(ka, kb)


@pytest.mark.parametrize("config,n,p", [(1, 100, 1000), (2, 300, 2000), (4, 300, 3000), (5, 400, 3000)])
def test_generators_agree(config, n, p):
    import qsched
    a_nodes, a_pods = O.generate(config, n, p)
    b_nodes, b_pods = O.py_generate(config, n, p)
    c_nodes, c_pods_s = qsched.synth_generate(config, n, p)
    c_pods = qsched.pods_from_struct(c_pods_s)
    for k in a_nodes:
        assert np.array_equal(a_nodes[k], b_nodes[k]), k
        assert np.array_equal(a_nodes[k], c_nodes[k]), k
    for k in a_pods:
        assert np.array_equal(a_pods[k], b_pods[k]), k
        assert np.array_equal(a_pods[k], c_pods[k]), k


def test_config1_oracle_stable():
    """Config 1 (BASELINE configs[0]) end to end: every pod placed, capacity respected."""
    nodes, pods = O.generate(1, 100, 1000)
    n0, _ = O.copy_cluster(nodes, pods)
    pl, best, order = O.schedule(n0, pods)
    assert (pl >= 0).all()
    assert (n0["req_cpu"] <= n0["alloc_cpu"]).all() and (n0["req_mem"] <= n0["alloc_mem"]).all()
    assert (n0["pods"] <= 110).all()
    # QoSSort: Guaranteed first, then Burstable, then BestEffort
    q = pods["qos"][order]
    assert (np.diff(q) <= 0).all()
