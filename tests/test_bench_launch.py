"""bench.py's multi-GPU launch, host only (ADVICE r1 --gpus):
* ``--gpus N`` without a launcher re-launches under torch.distributed.run with N ranks on a
  127.0.0.1 rendezvous (checked through ``--dry-run``, which never touches a GPU);
* a launcher's WORLD_SIZE that disagrees with --gpus is an error, not a silent 1-GPU run;
* world size 2 over gloo: the rank plumbing bench.py uses on the GPU box (process group, RCCL id
  broadcast from rank 0, max over ranks, barrier) up to the first HIP call, which reports a
  status (no device here) instead of crashing or hanging.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def dry(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, "--dry-run"] + args, capture_output=True, text=True,
                          env=env, timeout=120)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_gpus_n_relaunches_under_torchrun(n):
    r = dry(["--gpus", str(n), "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan["mode"] == "torchrun" and plan["world"] == n
    argv = plan["argv"]
    assert argv[1:3] == ["-m", "torch.distributed.run"]
    assert f"--nproc-per-node={n}" in argv and "--master-addr=127.0.0.1" in argv and "--nnodes=1" in argv
    i = argv.index(BENCH)
    assert argv[i + 1:] == ["--gpus", str(n), "--steps", "3", "--warmup", "1"]  # no --dry-run, no loop


def test_single_gpu_runs_in_process():
    r = dry([])
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"mode": "in-process", "world": 1}


def test_launcher_world_size_must_match():
    r = dry(["--gpus", "4"], {"WORLD_SIZE": "2"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
    r = dry(["--gpus", "2"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 0 and json.loads(r.stdout.strip().splitlines()[-1])["mode"] == "in-process"


def _rank(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "custom-k8s-scheduler_amd")]
    import bench
    import qsched

    # no RCCL unique id without a GPU: a fixed stand-in id exercises the broadcast from rank 0
    qsched.dist_unique_id = lambda: bytes(range(128))
    cx = bench.Ctx(backend="gloo")
    r, w, uid = cx.shard()
    top = cx.max(float(rank) + 0.5)
    cx.barrier()
    status = None
    try:
        bench.open_sched(cx, {"engine": "lookahead"}, True)  # qs_open_shard: first HIP call
    except qsched.QschedError as e:
        status = e.status
    cx.dist.destroy_process_group()
    q.put((rank, r, w, uid, top, status))


def test_world2_gloo_rank_plumbing():
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, (r, r_, w, uid, top, status) in enumerate(res):
        assert r == rank and r_ == rank and w == 2
        assert uid == bytes(range(128))  # rank 1 received rank 0's id
        assert top == 1.5                # max over ranks
        assert status == 2               # QS_EDEVICE: no HIP device in this container


def _rank_fallback(rank, port, q, mode):
    """bench.measure_sharded's decision at world 2 (gloo), with measure() stubbed: the mailbox
    transport fails on one rank only (mode "raise") or gives different placements on the two ranks
    (mode "differ"); both ranks must then fall back to RCCL together."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "custom-k8s-scheduler_amd")]
    import numpy as np

    import bench

    cx = bench.Ctx(backend="gloo")
    a = bench.parse(["--gpus", "2"])

    def fake_measure(cx_, a_, workload, steps, warmup, with_diag=True):
        name = bench.TRANSPORT["name"]
        if name == "mailbox":
            if mode == "raise" and rank == 1:
                raise RuntimeError("QS_ETIMEOUT: mailbox exchange timed out")
            if mode == "differ":
                return {"placement": np.full(4, rank, np.int32)}
        return {"placement": np.arange(4, dtype=np.int32)}

    bench.measure = fake_measure
    m = bench.measure_sharded(cx, a, "config3")
    cx.dist.destroy_process_group()
    q.put((rank, m["transport"], [t["transport"] for t in m["transport_tried"]]))


@pytest.mark.parametrize("mode", ["raise", "differ"])
def test_world2_transport_fallback(mode):
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_fallback, args=(r, port, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res == [(0, "rccl", ["mailbox"]), (1, "rccl", ["mailbox"])]


_RUNS = [0]  # stream runs of this process on the failing transport's schedulers


class _FakeStream:
    """A prepared stream of the fake scheduler: fixed placements (identical on both ranks), a
    configurable failure at the n-th run of the process (diagnostic runs included)."""

    def __init__(self, owner, pods):
        self.o, self.pods = owner, pods

    def run(self, mode="exact"):
        _RUNS[0] += 1
        if self.o.fail_at == ("run", _RUNS[0]):
            raise RuntimeError("QS_ETIMEOUT: resident lookahead stream timed out")
        eng = "allreduce" if self.o.cfg.get("engine") == "allreduce" else "lookahead"
        return {"engine_used": eng, "resident": 1, "table_layout": "compact", "wall_s": 1e-3,
                "kernels": {"resolve": {"s": 1e-3, "launches": 1}}}

    def results(self):
        import numpy as np
        p = len(self.pods)
        if self.o.cfg.get("engine") == "allreduce":
            # the all-reduce engine's stand-in returns the exact stream (the oracle's placements), so
            # the rank-0 line's rccl_per_pod check must come out True through bench's own plumbing
            from oracle import oracle as O
            import qsched
            on = {k: v.copy() for k, v in self.o.nodes.items()}
            ref, keys, _ = O.schedule_incremental(on, qsched.pods_from_struct(self.pods), {}, nthreads=1)
            return np.asarray(ref, np.int32), np.asarray(keys, np.uint64)
        return np.arange(p, dtype=np.int32) % 7, np.zeros(p, np.uint64)

    def stamps(self):
        import numpy as np
        return np.arange(len(self.pods), dtype=np.uint64) * 50

    def free(self):
        pass


def _fake_scheduler_cls(rank, fail):
    class FakeScheduler:
        def __init__(self, cfg, device=0, shard=None):
            self.cfg = dict(cfg)
            self.fail_at = fail if (fail and fail[2] == rank) else None
            self.fail_at = self.fail_at[:2] if self.fail_at else None
            if self.fail_at == ("open", 1):
                raise RuntimeError("QS_EDEVICE: hipIpcGetMemHandle failed")

        def mailbox_export(self):
            return bytes([rank]) * 8

        def mailbox_connect(self, handles):
            assert len(handles) == 2

        def load_nodes(self, nodes):
            self.nodes = nodes

        def prepare(self, pods):
            if self.fail_at == ("prepare", 1):
                raise RuntimeError("QS_EINVAL: pod out of range")
            return _FakeStream(self, pods)

        def save_table(self):
            pass

        def restore_table(self):
            pass

        def read_nodes(self):
            return {k: v.copy() for k, v in self.nodes.items()}

        def close(self):
            pass

    return FakeScheduler


def _rank_measure_fail(rank, port, q, fail):
    """bench.measure_sharded with the REAL measure() / open_sched() / diag_runs() at world 2 over
    gloo; only the library's Scheduler is a CPU fake whose rank fail[2] fails in phase fail[:2]
    (mailbox open, prepare, or the n-th stream run).  Every rank must end on the same transport
    (RCCL after a mailbox failure) without a collective mismatch (ADVICE r3 bench.py:339)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "custom-k8s-scheduler_amd")]
    import bench
    import qsched

    bench.WORKLOADS["config3"] = (3, 300, 2000, "config3 (small, fake scheduler)")
    qsched.dist_unique_id = lambda: bytes(range(128))
    fake = _fake_scheduler_cls(rank, fail)
    mailbox_only = fake

    class Sched:  # the mailbox transport fails as configured, the RCCL one never
        def __new__(cls, cfg, device=0, shard=None):
            if shard is not None and shard[2] is not None:
                return _fake_scheduler_cls(rank, None)(cfg, device, shard)
            return mailbox_only(cfg, device, shard)

    qsched.Scheduler = Sched
    cx = bench.Ctx(backend="gloo")
    a = bench.parse(["--gpus", "2", "--steps", "3", "--warmup", "1"])
    m = bench.measure_sharded(cx, a, "config3")
    cx.dist.destroy_process_group()
    q.put((rank, m["transport"], [t["transport"] for t in m["transport_tried"]]))


@pytest.mark.parametrize("fail", [("open", 1, 1), ("prepare", 1, 0), ("run", 1, 1), ("run", 3, 0), ("run", 5, 1)],
                         ids=["open-r1", "prepare-r0", "warmup-r1", "timed-step-r0", "diag-run-r1"])
def test_world2_measure_fails_on_one_rank(fail):
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_measure_fail, args=(r, port, q, fail)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res == [(0, "rccl", ["mailbox"]), (1, "rccl", ["mailbox"])]


def test_cpu_arms_capped_by_the_process_share(monkeypatch):
    """The nproc OpenMP arm uses the smallest of the affinity mask, the cgroup quota and
    OMP_NUM_THREADS (round 4: the GPU box's mask shows 256 CPUs against a 16-CPU share)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    monkeypatch.setattr(bench, "cgroup_cpus", lambda: 16)
    monkeypatch.setenv("OMP_NUM_THREADS", "64")
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(256)))
    assert bench.effective_cpus() == 16
    monkeypatch.setattr(bench, "cgroup_cpus", lambda: None)
    assert bench.effective_cpus() == 64
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.effective_cpus() == 256


def _rank_line(rank, port, q):
    """bench.main() at world 2 over gloo (config 3 small, a CPU fake of the library's Scheduler):
    the rank-0 line must carry the sharded mailbox measurement AND the per-pod RCCL all-reduce
    variant beside it."""
    import contextlib
    import io
    import json

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank), QS_BENCH_BACKEND="gloo")
    sys.path[:0] = [ROOT, os.path.join(ROOT, "custom-k8s-scheduler_amd")]
    import bench
    import qsched

    bench.WORKLOADS["config3"] = (3, 300, 2000, "config3 (small, fake scheduler)")
    qsched.dist_unique_id = lambda: bytes(range(128))
    qsched.Scheduler = _fake_scheduler_cls(rank, None)
    sys.argv = ["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--rccl-sample", "400"]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.main()
    lines = [x for x in buf.getvalue().splitlines() if x.startswith("{")]
    q.put((rank, rc, json.loads(lines[-1]) if lines else None))


def test_world2_line_carries_mailbox_and_rccl_variants():
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_line, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][1] == 0 and res[1][1] == 0
    line = res[0][2]
    assert res[1][2] is None  # one JSON line, from rank 0
    assert line["n_gpus"] == 2 and line["config"]["transport"] == "mailbox"
    r = line["rccl_per_pod"]
    assert r["engine"] == "allreduce" and r["n_gpus"] == 2 and r["value"] > 0
    assert "ncclAllReduce" in r["variant"] and r["placements_match"] is True
