"""The peer-memory mailbox transport of the sharded engine through
the C ABI: qs_open_shard without an RCCL id + qs_dist_mailbox_export / _connect.

* world = 2 as two processes on the one GPU of the box: each rank scores its own node shard, writes
  its per-window lists (and, for TaintToleration/NodeAffinity, its partial maxima) into the other
  rank's mailbox through the IPC mapping and waits for the other's flags.  Both ranks must return
  the oracle's placements, keys and final table — the world > 1 library path, executed.
* world = 1 in one process: the same kernels with the rank's own mailbox only.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CFG4 = dict(enable_taint=1, enable_affinity=1)


def _rank(rank, world, qin, qout, cfg, config, n, p):
    import sys
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "custom-k8s-scheduler_amd")]
    import qsched

    try:
        nodes, pods = qsched.synth_generate(config, n, p)
        with qsched.Scheduler(dict(cfg, engine="lookahead"), device=0, shard=(rank, world, None)) as s:
            qout.put(("h", rank, s.mailbox_export()))
            s.mailbox_connect(qin.get(timeout=120))
            s.load_nodes(nodes)
            st = s.prepare(pods)
            stats = st.run()
            pl, keys = st.results()
            st.free()
            final = s.read_nodes()
        qout.put(("r", rank, pl, keys, final, stats["engine_used"]))
    except Exception as e:  # reported to the parent instead of hanging it
        qout.put(("e", rank, repr(e)))


def run_world(world, cfg, config, n, p):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    qout = ctx.Queue()
    qins = [ctx.Queue() for _ in range(world)]
    procs = [ctx.Process(target=_rank, args=(r, world, qins[r], qout, cfg, config, n, p)) for r in range(world)]
    for pr in procs:
        pr.start()
    handles, results = {}, {}
    try:
        while len(handles) < world:
            m = qout.get(timeout=180)
            assert m[0] != "e", m
            handles[m[1]] = m[2]
        for q in qins:
            q.put([handles[r] for r in range(world)])
        while len(results) < world:
            m = qout.get(timeout=300)
            assert m[0] != "e", m
            results[m[1]] = m[2:]
    finally:
        for pr in procs:
            pr.join(60)
            if pr.is_alive():
                pr.kill()
    return results


@pytest.mark.parametrize("cfg,config,n,p", [({}, 2, 3000, 12000), (CFG4, 4, 2000, 6000)],
                         ids=["config2", "config4"])
def test_mailbox_world2_two_processes(oracle, cfg, config, n, p):
    from qsched import pods_from_struct, synth_generate

    res = run_world(2, cfg, config, n, p)
    nodes, pods = synth_generate(config, n, p)
    on = {k: v.copy() for k, v in nodes.items()}
    o_pl, o_keys, _ = oracle.schedule(on, pods_from_struct(pods), cfg, nthreads=16)
    for rank in range(2):
        pl, keys, final, eng = res[rank]
        assert eng == "lookahead"
        bad = np.nonzero(pl != o_pl)[0]
        assert bad.size == 0, f"rank {rank}: {bad.size} placements differ, first at pod {bad[0]}"
        assert np.array_equal(keys, o_keys), rank
        for k in on:
            assert np.array_equal(final[k], on[k]), (rank, k)


def test_mailbox_world1_in_process(oracle):
    from qsched import Scheduler, pods_from_struct, synth_generate

    nodes, pods = synth_generate(2, 1500, 6000)
    with Scheduler({"engine": "lookahead"}, shard=(0, 1, None)) as s:
        s.mailbox_connect([s.mailbox_export()])
        s.load_nodes(nodes)
        for _ in range(2):  # a second run re-uses the mailbox with newer sequence numbers
            s.load_nodes(nodes)
            st = s.prepare(pods)
            st.run()
            pl, keys = st.results()
            st.free()
    on = {k: v.copy() for k, v in nodes.items()}
    o_pl, o_keys, _ = oracle.schedule(on, pods_from_struct(pods), {}, nthreads=16)
    assert np.array_equal(pl, o_pl) and np.array_equal(keys, o_keys)


def test_sharded_context_needs_a_transport():
    from qsched import QschedError, Scheduler, synth_generate

    nodes, pods = synth_generate(2, 500, 200)
    with Scheduler({"engine": "lookahead"}, shard=(0, 2, None)) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods)
        with pytest.raises(QschedError, match="transport"):
            st.run()
        st.free()
