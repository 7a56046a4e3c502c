"""qsched.checks.stream_invariants on oracle results (CPU): true invariants hold, and each check
catches the corruption it is meant for (a moved placement, a dropped Reserve, a pod wrongly left
unschedulable)."""
import numpy as np

from qsched import pods_from_struct, synth_generate
from qsched.checks import stream_invariants


def _run(oracle, config, n, p, cfg=None):
    nodes, pods = synth_generate(config, n, p)
    fin = {k: v.copy() for k, v in nodes.items()}
    pl, _, _ = oracle.schedule(fin, pods_from_struct(pods), cfg, nthreads=4)
    return nodes, pods, pl, fin


def test_invariants_hold(oracle):
    for config, n, p in [(2, 400, 8000), (3, 600, 12000), (4, 300, 4000)]:
        nodes, pods, pl, fin = _run(oracle, config, n, p)
        r = stream_invariants(nodes, pods, pl, fin)
        assert r["conservation"] and r["capacity"] and r["unschedulable_infeasible"], (config, r)
        assert r["placed"] == int((pl >= 0).sum())


def test_invariants_catch_corruption(oracle):
    nodes, pods, pl, fin = _run(oracle, 2, 300, 9000)
    assert (pl < 0).any()
    bad = pl.copy()
    j = int(np.nonzero(bad >= 0)[0][0])
    bad[j] = (bad[j] + 1) % 300  # placed on another node: the table no longer adds up
    assert not stream_invariants(nodes, pods, bad, fin)["conservation"]
    fin2 = {k: v.copy() for k, v in fin.items()}
    fin2["pods"][pl[j]] -= 1  # a Reserve lost
    assert not stream_invariants(nodes, pods, pl, fin2)["conservation"]
    # an unschedulable pod that fits somewhere in the final table: free one node up
    fin3 = {k: v.copy() for k, v in fin.items()}
    fin3["req_cpu"][:] = 0
    fin3["req_mem"][:] = 0
    fin3["pods"][0] = 0
    assert stream_invariants(nodes, pods, pl, fin3)["unschedulable_infeasible"] is False


def test_batched_invariants(oracle):
    """Batched mode (spec S11): the oracle's result satisfies conservation, capacity and required
    anti-affinity; two pods of one hostname-anti-affinity app forced onto one node break the last."""
    from qsched.checks import batched_invariants

    nodes, pods = synth_generate(5, 400, 6000)
    fin = {k: v.copy() for k, v in nodes.items()}
    pl, _, _ = oracle.schedule_batched(fin, pods_from_struct(pods), nthreads=4)
    r = batched_invariants(nodes, pods, pl, fin)
    assert r["conservation"] and r["capacity"] and r["anti_affinity"], r
    host = np.nonzero((pods["anti_affinity"] == 1) & (pl >= 0))[0]
    a = pods["app"][host]
    vals, cnt = np.unique(a, return_counts=True)
    two = host[a == vals[np.argmax(cnt)]][:2]
    assert two.size == 2
    bad = pl.copy()
    bad[two[1]] = bad[two[0]]
    assert not batched_invariants(nodes, pods, bad, fin)["anti_affinity"]
