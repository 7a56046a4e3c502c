"""GPU parity of the framework-embedded path through the C ABI, bit-exact vs the
oracle: qs_score_pod (PreFilter+Filter+Score+NormalizeScore for every node of one pod),
qs_reserve / qs_unreserve (Reserve / Unreserve), qs_node_upsert with Generation diffs.

Each case runs with the row table only and with the column-major (SoA) copy forced on
(``scan_soa_min_nodes = 1``), so the SoA scan kernel and its Reserve bookkeeping are checked on
small tables too.  The SCAN engine's exact stream over the SoA copy is checked here as well, and
at an HBM-resident table size (2^21 nodes) against the oracle on a short stream.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from qsched import Scheduler, pods_from_struct, synth_generate  # noqa: E402

from test_gpu_parity import CFG4, assert_same, run_oracle  # noqa: E402

LAYOUTS = {"rows": {}, "soa": {"scan_soa_min_nodes": 1}}


def oracle_scores(nodes, pods, j, cfg=None):
    from oracle import oracle as O
    keys, sc = O.score_pod(nodes, pods_from_struct(pods), j, cfg)
    feas = keys != 0
    total = np.where(feas, (keys >> np.uint64(32)).astype(np.int64) - 1, -1)
    best = int(0xFFFFFFFF - (int(keys.max()) & 0xFFFFFFFF)) if keys.max() else -1
    return feas, sc, total, best


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("config,n", [(1, 100), (2, 3000), (4, 2000)])
def test_score_pod_parity(layout, config, n):
    nodes, pods = synth_generate(config, n, 40)
    cfg = dict(LAYOUTS[layout])
    if config == 4:
        cfg.update(CFG4)
    with Scheduler(cfg) as s:
        s.load_nodes(nodes)
        for j in range(0, 40, 7):
            got = s.score_pod(pods[j])
            feas, sc, total, best = oracle_scores(nodes, pods, j, CFG4 if config == 4 else None)
            assert np.array_equal(got["feasible"], feas)
            assert np.array_equal(got["total"], total)
            assert got["best"] == best
            np.testing.assert_array_equal(got["scores"][feas], sc[feas])


@pytest.mark.parametrize("n", [1, 255, 257, 1023, 1024, 1025, 4096, 16383, 16384, 16385, 50000,
                               70001])
def test_score_pod_grid_edges_reused_buffers(n):
    """The multi-workgroup score launch (one node per thread, ceil(n/1024) workgroups of
    kScorePodGT = 1024 threads, the last arrival publishing best + done) at workgroup-count edges
    (1023/1024/1025, 16383/16384/16385) and beyond round 3's 16,384-node one-launch limit
    (50,000 = config 3's table; 70,001 keeps a SoA copy too), with the packed outputs unpacked 16
    nodes at a time (tails 1, 15, 1, 15, 0, 1, 0, 15, 0, 1, 0, 1) into caller buffers reused across
    calls and Reserves; every call diffed against the oracle and against a fresh-buffer call."""
    from oracle import oracle as O
    nodes, pods = synth_generate(2, n, 12)
    with Scheduler({}) as s:
        s.load_nodes(nodes)
        ref = {k: v.copy() for k, v in nodes.items()}
        op = pods_from_struct(pods)
        bufs = s.score_buffers()
        for j in range(6):
            got = s.score_pod(pods[j], out=bufs)
            assert got["total"] is bufs["total"]
            fresh = s.score_pod(pods[j])
            feas, sc, total, best = oracle_scores(ref, pods, j)
            for g in (got, fresh):
                assert np.array_equal(g["feasible"], feas)
                assert np.array_equal(g["total"], total)
                assert g["best"] == best
                np.testing.assert_array_equal(g["scores"][feas], sc[feas])
            if best >= 0:
                s.reserve(best, pods[j])
                O.lib().or_reserve(O.ctypes.byref(O._mk_nodes(ref)), O.ctypes.byref(O._mk_pods(op)), j, best, 1)


@pytest.mark.parametrize("layout", LAYOUTS)
def test_reserve_unreserve_roundtrip(layout):
    """Reserve changes the next pod's scores exactly like the oracle's Reserve; Unreserve restores."""
    from oracle import oracle as O
    nodes, pods = synth_generate(2, 500, 20)
    with Scheduler(LAYOUTS[layout]) as s:
        s.load_nodes(nodes)
        ref = {k: v.copy() for k, v in nodes.items()}
        op = pods_from_struct(pods)
        for j in range(10):
            best = s.score_pod(pods[j])["best"]
            assert best >= 0
            s.reserve(best, pods[j])
            O.lib().or_reserve(O.ctypes.byref(O._mk_nodes(ref)), O.ctypes.byref(O._mk_pods(op)), j, best, 1)
            got = s.score_pod(pods[j + 1])
            feas, _, total, b2 = oracle_scores(ref, pods, j + 1)
            assert np.array_equal(got["total"], total) and got["best"] == b2
        final = s.read_nodes()
        for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pods"):
            assert np.array_equal(final[k], ref[k]), k


@pytest.mark.parametrize("layout", LAYOUTS)
def test_unreserve_restores_table(layout):
    nodes, pods = synth_generate(2, 300, 12)
    with Scheduler(LAYOUTS[layout]) as s:
        s.load_nodes(nodes)
        before = s.read_nodes()
        wins = []
        for j in range(12):
            b = s.score_pod(pods[j])["best"]
            s.reserve(b, pods[j])
            wins.append(b)
        for j in reversed(range(12)):
            s.unreserve(wins[j], pods[j])
        after = s.read_nodes()
        for k in before:
            assert np.array_equal(before[k], after[k]), k
        # the device table (both layouts) is back too: scores equal the fresh-cluster scores
        got = s.score_pod(pods[0])
        _, _, total, best = oracle_scores(nodes, pods, 0)
        assert np.array_equal(got["total"], total) and got["best"] == best


@pytest.mark.parametrize("layout", LAYOUTS)
def test_upsert_generation_diff(layout):
    nodes, pods = synth_generate(2, 200, 4)
    with Scheduler(LAYOUTS[layout]) as s:
        s.load_nodes(nodes)
        row = {k: (v[7].tolist() if v.ndim > 1 else int(v[7])) for k, v in nodes.items()}
        row["req_cpu"] = row["alloc_cpu"] - 100  # node 7 nearly full on cpu
        s.upsert(7, row, generation=5)
        stale = dict(row, req_cpu=0)
        s.upsert(7, stale, generation=5)  # same generation: ignored (already applied)
        assert int(s.read_nodes()["req_cpu"][7]) == row["req_cpu"]
        ref = {k: v.copy() for k, v in nodes.items()}
        ref["req_cpu"][7] = row["req_cpu"]
        got = s.score_pod(pods[0])
        feas, _, total, best = oracle_scores(ref, pods, 0)
        assert np.array_equal(got["feasible"], feas) and np.array_equal(got["total"], total)


def test_scan_engine_soa_stream_parity(oracle):
    nodes, pods = synth_generate(2, 3000, 2000)
    with Scheduler(dict(engine="scan", scan_soa_min_nodes=1)) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods)
        st.run()
        pl, keys = st.results()
        st.free()
        final = s.read_nodes()
    o = run_oracle(oracle, nodes, pods, {})
    assert_same((pl, keys), o[:2], final, o[2])


def test_scan_engine_soa_after_lookahead(oracle):
    """A lookahead run updates the rows only; the next SCAN run must rebuild the SoA copy."""
    nodes, pods = synth_generate(2, 2000, 3000)
    with Scheduler(dict(engine="lookahead", scan_soa_min_nodes=1)) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods[:1500])
        st.run()
        st.free()
        best = s.score_pod(pods[1500])["best"]
    ref = {k: v.copy() for k, v in nodes.items()}
    oracle.schedule(ref, pods_from_struct(pods[:1500]), nthreads=16)
    _, _, _, b2 = oracle_scores(ref, pods, 1500)
    assert best == b2


def test_hbm_resident_scan_parity(oracle):
    """2^21 nodes (67 MB of SoA columns): the SCAN engine over the SoA copy, 24 pods."""
    n = 1 << 21
    nodes, pods = synth_generate(2, n, 24)
    with Scheduler(dict(engine="scan")) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods)
        st.run()
        pl, keys = st.results()
        st.free()
    o = run_oracle(oracle, nodes, pods, {}, nthreads=16)
    assert np.array_equal(pl, o[0]) and np.array_equal(keys, o[1])


@pytest.mark.parametrize("config,n", [(2, 5000), (4, 3000), (2, 20001)])
def test_score_pod_packed_words(config, n):
    """qs_score_pod_packed: the kernel's per-node words read in place (no copy-out) decode to the
    oracle's feasibility and plugin scores, the best node matches, and qs_score_pod's arrays are
    the same words unpacked (totals = the QoS-weighted sums)."""
    nodes, pods = synth_generate(config, n, 12)
    cfg = CFG4 if config == 4 else {}
    with Scheduler(cfg) as s:
        s.load_nodes(nodes)
        for j in range(0, 12, 3):
            best, pk = s.score_pod_packed(pods[j])
            feas, sc, total, obest = oracle_scores(nodes, pods, j, cfg or None)
            assert best == obest
            assert np.array_equal(pk != 0xFFFFFFFF, feas)
            dec = np.stack([(pk >> (8 * k)) & 255 for k in range(4)], axis=1).astype(np.int64)
            np.testing.assert_array_equal(dec[feas], sc[feas])
            got = s.score_pod(pods[j])
            assert np.array_equal(got["feasible"], feas) and np.array_equal(got["total"], total)
