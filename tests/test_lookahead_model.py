"""CPU model of the exact top-K lookahead engine and of its sharded (multi-GPU) protocol.

The model mirrors k_la_select / k_la_resolve (custom-k8s-scheduler_amd/csrc/qs_kernels.hip):
window of K pods, per-pod top-L stale keys per node chunk computed against the window-start
table, then sequential resolution with the dirty set.  Scores come from the C oracle
(or_score_pod), so this checks the ALGORITHM (list sizes, dirty handling, tie order) against the
exact sequential oracle on CPU — the GPU tests check the kernels.  The sharded variant runs as
world_size-2 gloo processes: each rank builds the lists of its node shard, the lists are
all-gathered (the RCCL exchange of qs_open_shard), and every rank resolves identically.
"""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O


def topl_keys(keys, lo, hi, L):
    k = keys[lo:hi]
    k = k[k > 0]
    if len(k) > L:
        k = np.sort(k)[::-1][:L]
    return [int(x) for x in k]


def select_window(nodes, pods, order, s0, K, L, chunks):
    """Per pod of the window: union over chunks of the chunk's top-L stale keys."""
    lists = []
    for i in range(K):
        if s0 + i >= len(order):
            break
        keys, _ = O.score_pod(nodes, pods, int(order[s0 + i]))
        lst = []
        for lo, hi in chunks:
            lst += topl_keys(keys, lo, hi, L)
        lists.append(lst)
    return lists


def resolve_window(nodes, pods, order, s0, lists, placement):
    dirty = set()
    for i, lst in enumerate(lists):
        j = int(order[s0 + i])
        cand = max([e for e in lst if (0xFFFFFFFF - (e & 0xFFFFFFFF)) not in dirty], default=0)
        fresh, _ = O.score_pod(nodes, pods, j)  # fresh keys; only the dirty nodes' are used
        best = max([cand] + [int(fresh[d]) for d in dirty])
        if best == 0:
            placement[j] = -1
            continue
        w = 0xFFFFFFFF - (best & 0xFFFFFFFF)
        placement[j] = w
        O.lib().or_reserve(O.ctypes.byref(O._mk_nodes(nodes)), O.ctypes.byref(O._mk_pods(pods)), j, w, 1)
        dirty.add(w)


def chunks_of(n, G):
    per = -(-n // G)
    return [(g * per, min(n, (g + 1) * per)) for g in range(G) if g * per < n]


def model_schedule(nodes, pods, K, G):
    order = O.py_order(pods, O.DEFAULT_CONFIG)
    placement = np.full(len(order), -2, np.int32)
    for s0 in range(0, len(order), K):
        lists = select_window(nodes, pods, order, s0, K, K, chunks_of(len(nodes["alloc_cpu"]), G))
        resolve_window(nodes, pods, order, s0, lists, placement)
    return placement


@pytest.mark.parametrize("K,G", [(1, 1), (4, 3), (16, 1), (16, 5), (64, 2)])
def test_lookahead_model_is_exact(K, G):
    nodes, pods = O.generate(2, 120, 900)
    ref_nodes, _ = O.copy_cluster(nodes, pods)
    ref, _, _ = O.schedule(ref_nodes, pods)
    got = model_schedule(nodes, pods, K, G)
    assert np.array_equal(got, ref)
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pods"):
        assert np.array_equal(nodes[k], ref_nodes[k])


def test_short_lists_would_break_exactness():
    """L < K is not enough: with L = 1 the model diverges from the oracle on a spreading stream
    (guards against 'optimising' the list length below the dirty-set bound)."""
    nodes, pods = O.generate(2, 60, 400)
    ref_nodes, _ = O.copy_cluster(nodes, pods)
    ref, _, _ = O.schedule(ref_nodes, pods)
    order = O.py_order(pods, O.DEFAULT_CONFIG)
    placement = np.full(len(order), -2, np.int32)
    K = 16
    for s0 in range(0, len(order), K):
        lists = select_window(nodes, pods, order, s0, K, 1, [(0, 60)])
        resolve_window(nodes, pods, order, s0, lists, placement)
    assert not np.array_equal(placement, ref)


# ------------------------------------------------- merged lists + overlapped windows ----
def merged_select(nodes, pods, order, s0, K, L, shards):
    """k_la_select + k_la_merge: per pod, the top-L keys of each node shard (chunk lists merged)."""
    lists = []
    for i in range(K):
        if s0 + i >= len(order):
            break
        keys, _ = O.score_pod(nodes, pods, int(order[s0 + i]))
        lst = []
        for lo, hi in shards:
            lst += topl_keys(keys, lo, hi, L)
        lists.append(lst)
    return lists


def resolve_window_inherit(nodes, pods, order, s0, lists, placement, inherited):
    """k_la_resolve4 with dprev: nodes dirtied by the previous window start dirty.  Returns the
    nodes this window dirtied (its dcur)."""
    dirty, won = set(inherited), set()
    for i, lst in enumerate(lists):
        j = int(order[s0 + i])
        cand = max([e for e in lst if (0xFFFFFFFF - (e & 0xFFFFFFFF)) not in dirty], default=0)
        fresh, _ = O.score_pod(nodes, pods, j)
        best = max([cand] + [int(fresh[d]) for d in dirty])
        if best == 0:
            placement[j] = -1
            continue
        w = 0xFFFFFFFF - (best & 0xFFFFFFFF)
        placement[j] = w
        O.lib().or_reserve(O.ctypes.byref(O._mk_nodes(nodes)), O.ctypes.byref(O._mk_pods(pods)), j, w, 1)
        dirty.add(w)
        won.add(w)
    return won


def model_schedule_overlap(nodes, pods, K, L, shards):
    """The overlapped engine: window w+1's lists are selected against the table as it stood
    before window w (they run beside window w's resolve), so window w's dirtied nodes are
    inherited as dirty; lists must hold L >= 2K keys per shard."""
    order = O.py_order(pods, O.DEFAULT_CONFIG)
    placement = np.full(len(order), -2, np.int32)
    starts = list(range(0, len(order), K))
    pending = merged_select(nodes, pods, order, starts[0], K, L, shards)  # select(0)
    inherited = set()
    for w, s0 in enumerate(starts):
        lists = pending
        # select(w+1) reads the table before resolve(w) runs (the stalest view it can get)
        if w + 1 < len(starts):
            pending = merged_select(nodes, pods, order, starts[w + 1], K, L, shards)
        inherited = resolve_window_inherit(nodes, pods, order, s0, lists, placement, inherited)
    return placement


@pytest.mark.parametrize("K,W", [(1, 1), (4, 1), (8, 3), (16, 2), (32, 1)])
def test_overlapped_merged_model_is_exact(K, W):
    nodes, pods = O.generate(2, 150, 1200)
    ref_nodes, _ = O.copy_cluster(nodes, pods)
    ref, _, _ = O.schedule(ref_nodes, pods)
    got = model_schedule_overlap(nodes, pods, K, 2 * K, chunks_of(150, W))
    assert np.array_equal(got, ref)
    for k in ("req_cpu", "req_mem", "nz_cpu", "nz_mem", "pods"):
        assert np.array_equal(nodes[k], ref_nodes[k])


def test_overlap_needs_two_windows_of_list():
    """With overlapped windows, L = K is too short (up to 2K-1 nodes are dirty): the model
    diverges from the oracle on a spreading stream, so the engine uses L = 2K."""
    nodes, pods = O.generate(2, 60, 600)
    ref_nodes, _ = O.copy_cluster(nodes, pods)
    ref, _, _ = O.schedule(ref_nodes, pods)
    got = model_schedule_overlap(nodes, pods, 16, 16, [(0, 60)])
    assert not np.array_equal(got, ref)


# ---------------------------------------------------------------- sharded protocol (gloo) ----
def _shard_worker(rank, world, port, K, n, p, q):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nodes, pods = O.generate(2, n, p)
    order = O.py_order(pods, O.DEFAULT_CONFIG)
    lo, hi = rank * n // world, (rank + 1) * n // world  # contiguous node range of this rank
    placement = np.full(p, -2, np.int32)
    for s0 in range(0, p, K):
        kw = min(K, p - s0)
        mine = select_window(nodes, pods, order, s0, K, K, [(lo, hi)])
        buf = np.zeros((kw, K), np.uint64)
        for i, lst in enumerate(mine):
            buf[i, :len(lst)] = lst
        t = torch.from_numpy(buf.view(np.int64).copy())
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t)  # the per-window exchange (RCCL all-gather in qs_open_shard)
        merged = [[int(x) for x in np.concatenate([pp[i].numpy().view(np.uint64) for pp in parts]) if x]
                  for i in range(kw)]
        resolve_window(nodes, pods, order, s0, merged, placement)  # replicated on every rank
    q.put((rank, placement.tobytes()))
    dist.destroy_process_group()


def test_sharded_protocol_gloo_world2():
    n, p, K, world = 90, 600, 16, 2
    nodes, pods = O.generate(2, n, p)
    ref, _, _ = O.schedule(nodes, pods)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, K, n, p, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
    for r in range(world):
        assert np.array_equal(np.frombuffer(res[r], np.int32), ref), f"rank {r}"
