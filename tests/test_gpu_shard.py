"""GPU parity of the node-sharded LOOKAHEAD engine.

Two ways to exercise the sharded layout on the single-GPU box:
  * ``virtual_shards = W``: one process runs the select of all W node shards into the
    [shard][pod][GLp] list layout the RCCL all-gather produces, then the same resolver — this is the
    multi-GPU data path minus the collective, checked bit-exact against the oracle for W up to 8;
  * ``qs_open_shard`` with world = 1 and a real RCCL unique id: the communicator is built and the
    in-place all-gather runs every window (one rank), so the RCCL call path itself is exercised.
The multi-rank protocol (lists gathered across processes, replicated resolve) is checked on CPU
with world-size-2 gloo in tests/test_lookahead_model.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from qsched import Scheduler, dist_unique_id, synth_generate  # noqa: E402

from test_gpu_parity import assert_same, run_oracle  # noqa: E402


def run_sharded(nodes, pods, cfg, shard=None):
    with Scheduler(dict({"engine": "lookahead"}, **cfg), shard=shard) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods)
        stats = st.run()
        pl, keys = st.results()
        st.free()
        final = s.read_nodes()
    return pl, keys, final, stats


@pytest.mark.parametrize("W", [2, 3, 4, 8])
@pytest.mark.parametrize("n,p", [(5000, 3000), (777, 4000)])
def test_virtual_shards_parity(oracle, W, n, p):
    nodes, pods = synth_generate(2, n, p)
    g = run_sharded(nodes, pods, dict(virtual_shards=W))
    assert g[3]["engine_used"] == "lookahead"
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("W,K", [(1, 32), (2, 32), (8, 32), (8, 64)])
def test_config3_scale_virtual_shards(oracle, W, K):
    """Config 3 generator (seed 0x5EED0003) at its full 50,000-node table, 3,000 pods."""
    nodes, pods = synth_generate(3, 50000, 3000)
    g = run_sharded(nodes, pods, dict(virtual_shards=W, lookahead=K))
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])


def test_ext_resources_virtual_shards(oracle):
    nodes, pods = synth_generate(4, 1800, 5000)
    g = run_sharded(nodes, pods, dict(virtual_shards=4))
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])


def test_rccl_one_rank_communicator(oracle):
    """qs_open_shard(rank 0, world 1, id): RCCL communicator + per-window all-gather on the GPU."""
    nodes, pods = synth_generate(3, 4000, 5000)
    g = run_sharded(nodes, pods, {}, shard=(0, 1, dist_unique_id()))
    o = run_oracle(oracle, nodes, pods, {})
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("W", [2, 4])
def test_config4_virtual_shards(oracle, W):
    """Normalizing profile, sharded: partial maxima of every shard combine into each pod's
    NormInfo before the shard selects (the RCCL path all-gathers them first)."""
    from test_gpu_parity import CFG4
    nodes, pods = synth_generate(4, 3000, 9000)
    g = run_sharded(nodes, pods, dict(CFG4, virtual_shards=W))
    o = run_oracle(oracle, nodes, pods, CFG4)
    assert_same(g[:2], o[:2], g[2], o[2])


def test_config4_rccl_one_rank(oracle):
    from test_gpu_parity import CFG4
    nodes, pods = synth_generate(4, 2000, 5000)
    g = run_sharded(nodes, pods, CFG4, shard=(0, 1, dist_unique_id()))
    o = run_oracle(oracle, nodes, pods, CFG4)
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("config,n,p,prof", [(2, 3000, 3000, {}), (3, 20000, 1500, {}), (4, 2000, 2000, "norm"),
                                             (4, 2500, 2000, "gpu-scoring")])
def test_allreduce_engine_one_rank(oracle, config, n, p, prof):
    """QS_ENGINE_ALLREDUCE (the as-is RCCL baseline): per pod the rank scans its
    node shard and one ncclAllReduce(u64 max) of the packed key decides (two u32 max all-reduces of
    the normalize maxima first for TaintToleration / NodeAffinity); at world 1 with a one-rank
    communicator, bit-exact vs the oracle, placements, keys and the final table."""
    from test_gpu_parity import CFG4
    from rescfg import GPU_CFG
    cfg = {} if not prof else (CFG4 if prof == "norm" else dict(CFG4, **GPU_CFG))
    nodes, pods = synth_generate(config, n, p)
    g = run_sharded(nodes, pods, dict(cfg, engine="allreduce"), shard=(0, 1, dist_unique_id()))
    assert g[3]["engine_used"] == "allreduce"
    o = run_oracle(oracle, nodes, pods, cfg)
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("V", [2, 3, 8])
@pytest.mark.parametrize("config,n,p,prof", [(2, 3000, 2000, {}), (4, 2000, 1500, "norm"), (4, 2500, 1500, "gpu-scoring")])
def test_allreduce_engine_virtual_world(oracle, V, config, n, p, prof):
    """The per-pod all-reduce engine of a V-rank world in one process: the one-rank
    context scans each rank's node range [r*n/V, (r+1)*n/V) in turn into the same scratch — partial
    normalize maxima by atomicMax, partial keys max-into-best, as ncclAllReduce(max) combines the
    ranks' values — then commits the one Reserve every rank would apply.  The shard partition, the
    max over shards (ties across a shard edge resolve to the lower node index through the packed
    key) and the replicated commit are checked bit-exact against the oracle, placements, keys and the
    final table.  (A real two-rank communicator needs two devices: test_gpu_rccl_world2.py.)"""
    from test_gpu_parity import CFG4
    from rescfg import GPU_CFG
    cfg = {} if not prof else (CFG4 if prof == "norm" else dict(CFG4, **GPU_CFG))
    nodes, pods = synth_generate(config, n, p)
    g = run_sharded(nodes, pods, dict(cfg, engine="allreduce", virtual_shards=V), shard=(0, 1, dist_unique_id()))
    assert g[3]["engine_used"] == "allreduce"
    o = run_oracle(oracle, nodes, pods, cfg)
    assert_same(g[:2], o[:2], g[2], o[2])


def test_allreduce_engine_needs_a_communicator():
    """Without an RCCL communicator the per-pod all-reduce engine refuses to run (QS_ESTATE)."""
    from qsched import QschedError, Scheduler
    nodes, pods = synth_generate(2, 500, 200)
    with Scheduler({"engine": "allreduce"}) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods)
        with pytest.raises(QschedError, match="RCCL communicator"):
            st.run()
        st.free()
