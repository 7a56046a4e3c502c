"""Failure recovery and rejected-update rollback (SURVEY.md §5 failure detection / recovery;
VERDICT r1 missing #6).

* The host mirror is authoritative and synced after every stream, so a device fault drops the
  device table and the next call rebuilds it from the mirror: the placements the caller was told
  about stay applied, the failed stream's do not.  Faults are injected with QS_INJECT_FAULT.
* A rejected qs_node_upsert / qs_unreserve (value outside the device range, a column driven
  negative) leaves qs_nodes_read and later placements unchanged.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from qsched import QschedError, Scheduler, pods_from_struct, synth_generate  # noqa: E402

from oracle import oracle as O  # noqa: E402


@pytest.mark.parametrize("engine", ["lookahead", "scan", "persistent"])
def test_device_fault_rebuilds_from_mirror(engine, monkeypatch):
    nodes, pods = synth_generate(2, 1200, 6000)
    op = pods_from_struct(pods)
    with Scheduler({"engine": engine}) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods[:3000])
        st.run()
        pl1, _ = st.results()
        st.free()
        after1 = s.read_nodes()
        st = s.prepare(pods[3000:])
        monkeypatch.setenv("QS_INJECT_FAULT", "stream_run")  # one-shot: the library unsets it
        with pytest.raises(QschedError, match="injected device fault"):
            st.run()
        # the failed stream is void: the table is the one after stream 1
        mid = s.read_nodes()
        for k in after1:
            assert np.array_equal(mid[k], after1[k]), k
        stats = st.run()  # re-run the same prepared stream on the rebuilt device table
        assert stats["device_faults"] == 1
        pl2, keys2 = st.results()
        st.free()
        final = s.read_nodes()
    on = {k: v.copy() for k, v in nodes.items()}
    o1, _, _ = O.schedule(on, {k: v[:3000] for k, v in op.items()}, nthreads=16)
    o2, ok2, _ = O.schedule(on, {k: v[3000:] for k, v in op.items()}, nthreads=16)
    assert np.array_equal(pl1, o1)
    assert np.array_equal(pl2, o2) and np.array_equal(keys2, ok2)
    for k in on:
        assert np.array_equal(final[k], on[k]), k


def test_rejected_upsert_leaves_table_unchanged():
    nodes, pods = synth_generate(2, 300, 200)
    with Scheduler({}) as s:
        s.load_nodes(nodes)
        before = s.read_nodes()
        bad = {k: (v[5].tolist() if v.ndim > 1 else int(v[5])) for k, v in nodes.items()}
        bad["alloc_cpu"] = 1 << 30  # outside the int32 cpu column range
        with pytest.raises(QschedError, match="alloc_cpu"):
            s.upsert(5, bad, generation=3)
        bad = dict(bad, alloc_cpu=4000, req_mem=-1)
        with pytest.raises(QschedError, match="req_mem"):
            s.upsert(5, bad, generation=4)
        after = s.read_nodes()
        for k in before:
            assert np.array_equal(before[k], after[k]), k
        pl = s.schedule(pods)
    on = {k: v.copy() for k, v in nodes.items()}
    o, _, _ = O.schedule(on, pods_from_struct(pods))
    assert np.array_equal(pl, o)


def test_rejected_unreserve_leaves_table_unchanged():
    nodes, pods = synth_generate(2, 200, 50)
    with Scheduler({}) as s:
        s.load_nodes(nodes)
        before = s.read_nodes()
        with pytest.raises(QschedError, match="negative|outside"):
            s.unreserve(3, pods[0])  # node 3 holds no pod: every column would go negative
        after = s.read_nodes()
        for k in before:
            assert np.array_equal(before[k], after[k]), k
        got = s.score_pod(pods[1])
    keys, _ = O.score_pod(nodes, pods_from_struct(pods), 1)
    assert got["best"] == int(0xFFFFFFFF - (int(keys.max()) & 0xFFFFFFFF))


def test_handoff_timeout_falls_back_to_events(monkeypatch):
    """A resolver that gives up waiting for its window's lists (the in-kernel hand-off, e.g. under
    a profiler that serialises the two streams) makes the run return QS_ETIMEOUT; the device table
    is rebuilt from the mirror and the context switches to cross-stream events, so re-running the
    prepared stream gives the oracle's placements (hand-off timeout injected with QS_INJECT_FAULT)."""
    nodes, pods = synth_generate(2, 1200, 4000)
    with Scheduler({"engine": "lookahead"}) as s:
        s.load_nodes(nodes)
        before = s.read_nodes()
        st = s.prepare(pods)
        monkeypatch.setenv("QS_INJECT_FAULT", "handoff")
        with pytest.raises(QschedError, match="QS_ETIMEOUT"):
            st.run()
        mid = s.read_nodes()
        for k in before:
            assert np.array_equal(mid[k], before[k]), k
        st.run()
        pl, keys = st.results()
        st.free()
    on = {k: v.copy() for k, v in nodes.items()}
    o, ok, _ = O.schedule(on, pods_from_struct(pods), nthreads=16)
    assert np.array_equal(pl, o) and np.array_equal(keys, ok)


def test_resident_stream_timeout_drains_on_device(monkeypatch):
    """The resident stream's in-kernel timeout path, driven for real (VERDICT r2 missing #5): a
    selector never delivers window 3 (QS_INJECT_FAULT=resident_stall, one-shot per context,
    DevCfg.inject), so the resolver's bounded wait raises werr, every other wait gives up on it, the
    launch drains and the run returns QS_ETIMEOUT within about the 0.5 s bound.  The device table is
    rebuilt from the mirror (unchanged); the next run uses per-window launches and gives the oracle's
    placements, and the run after that is the resident stream again (a timeout
    is not sticky), bit-exact too."""
    import time

    nodes, pods = synth_generate(2, 5000, 20000)
    with Scheduler({"engine": "lookahead"}) as s:
        s.load_nodes(nodes)
        before = s.read_nodes()
        st = s.prepare(pods)
        monkeypatch.setenv("QS_INJECT_FAULT", "resident_stall")
        t0 = time.perf_counter()
        with pytest.raises(QschedError, match="resident lookahead stream timed out"):
            st.run()
        assert time.perf_counter() - t0 < 5.0
        mid = s.read_nodes()
        for k in before:
            assert np.array_equal(mid[k], before[k]), k
        stats = st.run()
        assert stats["resident"] == 0 and stats["device_faults"] == 1
        pl, keys = st.results()
        st.free()
        s.load_nodes(nodes)  # the same context, from the empty cluster again
        st = s.prepare(pods)
        stats3 = st.run()
        assert stats3["resident"] == 1
        pl3, keys3 = st.results()
        st.free()
    on = {k: v.copy() for k, v in nodes.items()}
    o, ok, _ = O.schedule(on, pods_from_struct(pods), nthreads=16)
    assert np.array_equal(pl, o) and np.array_equal(keys, ok)
    assert np.array_equal(pl3, o) and np.array_equal(keys3, ok)


def test_resident_stream_second_timeout_sticks(monkeypatch):
    """Two consecutive resident timeouts (QS_INJECT_FAULT=resident_stall_always: every resident launch
    stalls) leave the context on per-window launches for good: timeout, per-window run, timeout again,
    then per-window runs only — each of them bit-exact."""
    nodes, pods = synth_generate(2, 3000, 6000)
    on = {k: v.copy() for k, v in nodes.items()}
    o, ok, _ = O.schedule(on, pods_from_struct(pods), nthreads=16)
    with Scheduler({"engine": "lookahead"}) as s:
        monkeypatch.setenv("QS_INJECT_FAULT", "resident_stall_always")
        seen = []
        for _ in range(5):
            s.load_nodes(nodes)  # from the empty cluster each time (a timeout drops the snapshot)
            st = s.prepare(pods)
            try:
                stats = st.run()
            except QschedError as e:
                assert "resident lookahead stream timed out" in str(e)
                seen.append("timeout")
                st.free()
                continue
            seen.append("resident" if stats["resident"] else "per-window")
            pl, keys = st.results()
            st.free()
            assert np.array_equal(pl, o) and np.array_equal(keys, ok)
    assert seen == ["timeout", "per-window", "timeout", "per-window", "per-window"], seen


def test_resident_timeouts_apart_do_not_stick(monkeypatch):
    """Only CONSECUTIVE resident timeouts keep per-window launches: timeout, per-window,
    a resident run that succeeds, a second timeout, then per-window once and resident again."""
    nodes, pods = synth_generate(2, 3000, 6000)
    on = {k: v.copy() for k, v in nodes.items()}
    o, ok, _ = O.schedule(on, pods_from_struct(pods), nthreads=16)
    seen = []
    with Scheduler({"engine": "lookahead"}) as s:
        plan = ["resident_stall", None, None, "resident_stall_always", None, None]
        for inj in plan:
            if inj:
                monkeypatch.setenv("QS_INJECT_FAULT", inj)
            else:
                monkeypatch.delenv("QS_INJECT_FAULT", raising=False)
            s.load_nodes(nodes)
            st = s.prepare(pods)
            try:
                stats = st.run()
            except QschedError as e:
                assert "resident lookahead stream timed out" in str(e)
                seen.append("timeout")
                st.free()
                continue
            seen.append("resident" if stats["resident"] else "per-window")
            pl, keys = st.results()
            st.free()
            assert np.array_equal(pl, o) and np.array_equal(keys, ok)
    assert seen == ["timeout", "per-window", "resident", "timeout", "per-window", "resident"], seen
