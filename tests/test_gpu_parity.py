"""GPU parity: libqsched.so (through the C ABI) vs the CPU oracle, bit-exact.

Placements, per-pod best keys (spec S7 packed (total, index)) and the final node table must be
identical to oracle/ on the same seeded inputs (spec/synth.md generator).  Parity is unpinned by
the reference (it has no code); the oracle itself is pinned by spec/kat.md (tests/test_oracle_kat.py).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from qsched import Scheduler, pods_from_struct, synth_generate  # noqa: E402

CFG4 = dict(enable_taint=1, enable_affinity=1)


def run_gpu(nodes, pods, cfg, engine, lookahead=0):
    with Scheduler(dict(cfg, engine=engine, lookahead=lookahead)) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods)
        stats = st.run()
        pl, keys = st.results()
        st.free()
        final = s.read_nodes()
    return pl, keys, final, stats


def run_oracle(oracle, nodes, pods, cfg, nthreads=16):
    on = {k: v.copy() for k, v in nodes.items()}
    pl, keys, _ = oracle.schedule(on, pods_from_struct(pods), cfg, nthreads=nthreads)
    return pl, keys, on


def assert_same(g, o, final_g, final_o):
    pl_g, keys_g = g
    pl_o, keys_o = o
    bad = np.nonzero(pl_g != pl_o)[0]
    assert bad.size == 0, f"{bad.size} placements differ; first at pod {bad[0]}: gpu {pl_g[bad[0]]} oracle {pl_o[bad[0]]}"
    assert np.array_equal(keys_g, keys_o)
    for k in final_o:
        assert np.array_equal(final_g[k], final_o[k]), k


@pytest.mark.parametrize("engine", ["persistent", "scan", "lookahead"])
@pytest.mark.parametrize("config,n,p", [(1, 100, 1000), (2, 700, 9000), (2, 5000, 3000)])
def test_stream_parity(oracle, engine, config, n, p):
    nodes, pods = synth_generate(config, n, p)
    g = run_gpu(nodes, pods, {}, engine)
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("K", [1, 2, 7, 33, 64])
def test_lookahead_windows(oracle, K):
    nodes, pods = synth_generate(2, 1500, 6000)
    g = run_gpu(nodes, pods, {}, "lookahead", lookahead=K)
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("engine", ["persistent", "scan", "lookahead"])
def test_config4_parity(oracle, engine):
    nodes, pods = synth_generate(4, 2000, 6000)
    g = run_gpu(nodes, pods, CFG4, engine)
    o = run_oracle(oracle, nodes, pods, CFG4)
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("serial", [0, 1])
def test_config4_full_lookahead(oracle, serial):
    """BASELINE.json configs[3]: 5,000 nodes x 150,000 pods, Fit + Balanced + TaintToleration +
    NodeAffinity + amd.com/gpu, on the normalizing LOOKAHEAD engine (overlapped and serial)."""
    nodes, pods = synth_generate(4, 5000, 150000)
    g = run_gpu(nodes, pods, dict(CFG4, lookahead_serial=serial), "lookahead")
    o = run_oracle(oracle, nodes, pods, CFG4)
    assert_same(g[:2], o[:2], g[2], o[2])
    assert g[3]["engine_used"] == "lookahead"
    assert g[3]["resident"] == (1 if serial == 0 else 0)  # overlapped windows: one resident launch


@pytest.mark.parametrize("waves", ["4", "1"])
@pytest.mark.parametrize("K", [1, 5, 32, 64])
def test_config4_lookahead_windows(oracle, K, waves, monkeypatch):
    """Tight cluster (many nodes fill up): exercises the normalize-maximum safety test and the
    exact rescan fallback.  The rescan path must actually run (stats.truncations), and with the
    four-wave resolver (overlapped windows, K <= 32) so must the stop / resume hand-off
    (stats.resumed_windows); QS_NORM_WAVES=1 pins the single-wave kernel for comparison."""
    monkeypatch.setenv("QS_NORM_WAVES", waves)
    nodes, pods = synth_generate(4, 400, 14000)
    g = run_gpu(nodes, pods, CFG4, "lookahead", lookahead=K)
    o = run_oracle(oracle, nodes, pods, CFG4)
    assert_same(g[:2], o[:2], g[2], o[2])
    assert g[3]["truncations"] > 0
    if waves == "4" and K <= 32:
        assert g[3]["resumed_windows"] > 0
    else:
        assert g[3]["resumed_windows"] == 0


def test_config2_full_lookahead(oracle):
    """BASELINE.json configs[1]: 5,000 nodes x 100,000 pods, every placement bit-exact."""
    nodes, pods = synth_generate(2, 5000, 100000)
    g = run_gpu(nodes, pods, {}, "lookahead")
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])
    assert 0.01 <= (g[0] < 0).mean() <= 0.05  # spec/synth.md G4: 1-5 % unschedulable


@pytest.mark.parametrize("config,n,p,K", [(1, 100, 1000, 32), (2, 1500, 6000, 32), (2, 5000, 3000, 32),
                                          (2, 9000, 7000, 32), (2, 30000, 4000, 32), (2, 1500, 6000, 7),
                                          (2, 2000, 5000, 16), (2, 3000, 2000, 1), (2, 50000, 3000, 32),
                                          (4, 40000, 3000, 32), (2, 100000, 1500, 32)])
def test_resident_stream(oracle, monkeypatch, config, n, p, K):
    """The resident lookahead stream (the whole window sequence as one launch of a resolver and
    selector workgroups) across selector geometries (1 to 16 node chunks, 3 to 16
    nodes per lane, one or two keys per merging thread with two selector workgroups per CU, ext
    resources, partial last windows, K = 1..32): bit-exact vs the oracle, reported in
    stats.resident, and identical to the per-window launches (QS_RESIDENT=0)."""
    nodes, pods = synth_generate(config, n, p)
    g = run_gpu(nodes, pods, {}, "lookahead", lookahead=K)
    assert g[3]["resident"] == 1
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])
    monkeypatch.setenv("QS_RESIDENT", "0")
    w = run_gpu(nodes, pods, {}, "lookahead", lookahead=K)
    assert w[3]["resident"] == 0
    assert np.array_equal(w[0], g[0]) and np.array_equal(w[1], g[1])


def test_resident_declines_large_tables(oracle):
    """Beyond 15 chunks of 8,192 nodes (K = 32, two selector workgroups per CU) the stream runs as
    per-window launches."""
    nodes, pods = synth_generate(2, 130000, 600)
    g = run_gpu(nodes, pods, {}, "lookahead")
    assert g[3]["resident"] == 0
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])


def test_config2_full_persistent(oracle):
    nodes, pods = synth_generate(2, 5000, 100000)
    g = run_gpu(nodes, pods, {}, "persistent")
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("engine", ["persistent", "scan", "lookahead"])
def test_ext_resources_without_taints(oracle, engine):
    """amd.com/gpu requests in Filter with the Fit+Balanced profile (no taint/affinity plugins)."""
    nodes, pods = synth_generate(4, 1800, 5000)
    g = run_gpu(nodes, pods, {}, engine)
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("engine", ["persistent", "scan", "lookahead"])
def test_custom_weights_parity(oracle, engine):
    """Non-default plugin / resource weights (also exercises the 64-bit key reduction path)."""
    cfg = dict(w_fit=(10, 20, 30), w_bal=(5, 7, 9), fit_weight_cpu=2, fit_weight_mem=3)
    ocfg = dict(wc=2, wm=3, w_fit=(10, 20, 30), w_bal=(5, 7, 9))
    nodes, pods = synth_generate(2, 1500, 6000)
    g = run_gpu(nodes, pods, cfg, engine)
    o = run_oracle(oracle, nodes, pods, ocfg)
    assert_same(g[:2], o[:2], g[2], o[2])


def test_balanced_skip_besteffort(oracle):
    nodes, pods = synth_generate(2, 800, 4000)
    g = run_gpu(nodes, pods, dict(balanced_skip_besteffort=1), "lookahead")
    o = run_oracle(oracle, nodes, pods, dict(balanced_skip_besteffort=1))
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("n,p,K", [(400, 14000, 32), (2000, 6000, 32), (5000, 20000, 32), (9000, 8000, 16),
                                   (3000, 5000, 7), (600, 4000, 1), (20000, 3000, 32)])
def test_resident_stream_norm(oracle, monkeypatch, n, p, K):
    """Normalizing profiles (TaintToleration + NodeAffinity + amd.com/gpu, config 4) as ONE resident
    launch: selectors publish the chunks' partial maxima and combine them per pod
    before scoring, the resolver tests the maxima per pod and rescans a pod exactly with all eight
    waves when one may be lost.  Bit-exact vs the oracle, and identical to the per-window launches;
    the tight cluster (400 nodes) must take the rescan path."""
    nodes, pods = synth_generate(4, n, p)
    g = run_gpu(nodes, pods, CFG4, "lookahead", lookahead=K)
    assert g[3]["resident"] == 1
    o = run_oracle(oracle, nodes, pods, CFG4)
    assert_same(g[:2], o[:2], g[2], o[2])
    if n == 400:
        assert g[3]["truncations"] > 0 and g[3]["resumed_windows"] > 0
    monkeypatch.setenv("QS_RESIDENT", "0")
    w = run_gpu(nodes, pods, CFG4, "lookahead", lookahead=K)
    assert w[3]["resident"] == 0
    assert np.array_equal(w[0], g[0]) and np.array_equal(w[1], g[1])


@pytest.mark.parametrize("resident", ["1", "0"])
@pytest.mark.parametrize("prof", [dict(enable_taint=1), dict(enable_affinity=1)], ids=["taint-only", "affinity-only"])
def test_single_normalizing_plugin(oracle, monkeypatch, prof, resident):
    """Only one of TaintToleration / NodeAffinity enabled: the normalizing kernels evaluate both, so
    the disabled plugin's part of every pod record is neutral (all taints tolerated / no affinity
    terms) and its weight 0 — placements and keys as the oracle with that plugin off."""
    monkeypatch.setenv("QS_RESIDENT", resident)
    nodes, pods = synth_generate(4, 1500, 8000)
    g = run_gpu(nodes, pods, prof, "lookahead")
    assert g[3]["resident"] == int(resident)
    o = run_oracle(oracle, nodes, pods, prof)
    assert_same(g[:2], o[:2], g[2], o[2])
    s = run_gpu(nodes, pods, prof, "scan")
    assert_same(s[:2], o[:2], s[2], o[2])
