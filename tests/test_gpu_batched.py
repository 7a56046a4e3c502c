"""GPU parity of batched mode (QS_MODE_BATCHED, spec/semantics.md S11, config 5) through the C ABI:
placements, claimed keys and the final node table bit-for-bit against the CPU oracle's
or_schedule_batched, plus the S11 invariants (capacity, hostname / zone anti-affinity) at the
full config-5 size where the oracle would take minutes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from qsched import Scheduler, pods_from_struct, synth_generate  # noqa: E402

from test_batched_model import check_invariants  # noqa: E402


def run_gpu_batched(nodes, pods, batch=0, cfg=None):
    with Scheduler(dict(cfg or {}, batch_pods=batch)) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods)
        stats = st.run(mode="batched")
        pl, keys = st.results()
        st.free()
        final = s.read_nodes()
    return pl, keys, final, stats


@pytest.mark.parametrize("config,n,p,batch", [(5, 1000, 20000, 64), (5, 300, 9000, 7), (5, 200, 2000, 1),
                                              (2, 2000, 30000, 64), (4, 800, 12000, 64)])
def test_batched_parity(oracle, config, n, p, batch):
    nodes, pods = synth_generate(config, n, p)
    g_pl, g_keys, g_final, stats = run_gpu_batched(nodes, pods, batch)
    assert stats["engine_used"] == "batched"
    on = {k: v.copy() for k, v in nodes.items()}
    o_pl, o_keys, o_nb = oracle.schedule_batched(on, pods_from_struct(pods), batch=batch or 64, nthreads=16)
    bad = np.nonzero(g_pl != o_pl)[0]
    assert bad.size == 0, f"{bad.size} placements differ; first at pod {bad[0]}: gpu {g_pl[bad[0]]} oracle {o_pl[bad[0]]}"
    assert np.array_equal(g_keys, o_keys)
    for k in ("req_cpu", "req_mem", "req_ext", "nz_cpu", "nz_mem", "pods"):
        assert np.array_equal(g_final[k], on[k]), k
    assert stats["batches"] == o_nb


@pytest.mark.parametrize("n,fused", [(3000, "0"), (20000, "1")])
def test_batched_merge_forms(oracle, monkeypatch, n, fused):
    """The two merge forms of a batch's chunk lists give the same lists: the merge inside the select
    launch (per-pod tickets, the default when G * L <= 512) switched off with
    QS_BATCH_FUSED_MERGE=0, and a 20,000-node table whose G * L > 512 takes the separate k_la_merge
    launch whatever the switch says."""
    monkeypatch.setenv("QS_BATCH_FUSED_MERGE", fused)
    nodes, pods = synth_generate(5, n, 4000)
    g_pl, g_keys, g_final, stats = run_gpu_batched(nodes, pods)
    on = {k: v.copy() for k, v in nodes.items()}
    o_pl, o_keys, o_nb = oracle.schedule_batched(on, pods_from_struct(pods), batch=64, nthreads=16)
    assert np.array_equal(g_pl, o_pl)
    assert np.array_equal(g_keys, o_keys)
    assert stats["batches"] == o_nb


def test_batched_full_config5_invariants():
    """BASELINE.json configs[4]: 10,000 nodes; 200,000 pods with 1,000 anti-affinity apps."""
    nodes, pods = synth_generate(5, 10000, 200000)
    pl, keys, final, stats = run_gpu_batched(nodes, pods)
    check_invariants(nodes, final, pods_from_struct(pods), pl)
    assert (pl >= 0).mean() > 0.5


def test_batched_full_config5_exact(oracle):
    """BASELINE.json configs[4] at full size, bit for bit: every placement, claimed key and the final
    table of the 10,000 x 200,000 batched stream against or_schedule_batched_incremental (identical to
    or_schedule_batched, tests/test_oracle_incremental.py), plus the batch count."""
    nodes, pods = synth_generate(5, 10000, 200000)
    g_pl, g_keys, g_final, stats = run_gpu_batched(nodes, pods)
    on = {k: v.copy() for k, v in nodes.items()}
    o_pl, o_keys, o_nb = oracle.schedule_batched_incremental(on, pods_from_struct(pods), nthreads=16)
    bad = np.nonzero(g_pl != o_pl)[0]
    assert bad.size == 0, f"{bad.size} placements differ; first at pod {bad[0]}: gpu {g_pl[bad[0]]} oracle {o_pl[bad[0]]}"
    assert np.array_equal(g_keys, o_keys)
    for k in on:
        assert np.array_equal(g_final[k], on[k]), k
    assert stats["batches"] == o_nb


def test_batched_then_exact_share_the_table(oracle):
    """A batched stream leaves the table (and its anti-affinity state) for the next stream."""
    nodes, pods = synth_generate(5, 500, 6000)
    with Scheduler({}) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods[:3000])
        st.run(mode="batched")
        pl1, _ = st.results()
        st.free()
        st = s.prepare(pods[3000:])
        st.run(mode="batched")
        pl2, _ = st.results()
        st.free()
        final = s.read_nodes()
    on = {k: v.copy() for k, v in nodes.items()}
    op = pods_from_struct(pods)
    sub1 = {k: v[:3000] for k, v in op.items()}
    sub2 = {k: v[3000:] for k, v in op.items()}
    o1, _, _ = oracle.schedule_batched(on, sub1, nthreads=16)
    assert np.array_equal(pl1, o1)
    # the oracle restarts its anti-affinity state per call: compare capacity state only
    for k in ("req_cpu", "pods"):
        assert (final[k] >= on[k]).all()
    del sub2, pl2
