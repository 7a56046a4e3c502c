"""bench.py — BASELINE.json metric: pods scheduled/s (+ pod×node evals/s, p99 pod latency) of the
exact sequential stream, measured through libqsched's C ABI on MI355X.

Workloads (BASELINE.json configs):
  * N = 1 (default): configs[1] — 5,000 nodes × 100,000 pods on one GPU (the metric's config).
    The line also carries a ``config3`` object: the 50,000-node × 1,000,000-pod stream on the same
    single GPU, the N = 1 point of the config-3 scaling curve.
  * N > 1 (torchrun, one rank per GPU): configs[2] — 50,000 nodes × 1,000,000 pods with the node
    table sharded across the N ranks (qs_open_shard: contiguous node ranges, one exchange of
    top-L lists per lookahead window over xGMI: the peer-memory mailbox by default, an RCCL
    all-gather with ``--transport rccl``).  Total work is fixed: ``scaling`` = "strong".
  ``--workload config2|config3`` overrides (config2 at N > 1 = independent replicas, weak scaling).

A *step* = restore the empty cluster on the device (qs_table_restore, a D2D copy) + run the whole
exact stream (qs_stream_run): inputs resident in HBM, every pod scheduled, placements left in HBM.
Timed: K steps bracketed by barrier + device sync on both sides; MAX over ranks.

``--gpus N`` (N > 1) without a launcher environment re-launches this script under
``torch.distributed.run`` (one rank per GPU, 127.0.0.1 rendezvous) as a child process before any
GPU call, and exits with its status; ``--dry-run`` prints that launch plan and exits.  Under a
launcher, WORLD_SIZE must equal --gpus.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "custom-k8s-scheduler_amd"))

import qsched  # noqa: E402  (ctypes binding: the library is loaded on first use, not at import)

WORKLOADS = {
    # name: (generator config, nodes, pods, description)
    "config2": (2, 5000, 100000, "config2: 5,000 nodes x 100,000 pods, exact sequential, "
                                 "Fit+Balanced+QoS weights, percentageOfNodesToScore=100"),
    "config3": (3, 50000, 1000000, "config3: 50,000 nodes x 1,000,000 pods, exact sequential, "
                                   "node table sharded across ranks (list exchange per window)"),
    "config4": (4, 5000, 150000, "config4: 5,000 nodes x 150,000 pods, exact sequential, Fit + "
                                 "Balanced + TaintToleration + NodeAffinity + amd.com/gpu"),
    "config4_gpu_scoring": (4, 5000, 150000, "config4 with the AMD-GPU scoring resources: 5,000 nodes x "
                                             "150,000 pods, LeastAllocated {cpu:1, memory:1, amd.com/gpu:5}, "
                                             "BalancedAllocation over [cpu, memory, amd.com/gpu], TaintToleration "
                                             "+ NodeAffinity"),
    "config5": (5, 10000, 200000, "config5: 10,000 nodes x 200,000 pods, BATCHED mode (spec S11: "
                                  "64-pod batches, one pod per node per batch, hostname/zone "
                                  "anti-affinity over 1,000 apps) - approximate, reported separately"),
}
MODE = {"config5": "batched"}
PROFILE = {"config4": {"enable_taint": 1, "enable_affinity": 1},  # plugin switches per workload
           # NodeResourcesFitArgs.ScoringStrategy.Resources / BalancedAllocationArgs.Resources of an
           # AMD-GPU cluster (BASELINE.json configs[3]; spec S5): the kFeatRes kernels
           "config4_gpu_scoring": {"enable_taint": 1, "enable_affinity": 1,
                                   "fit_resources": [("cpu", 1), ("memory", 1), ("ext0", 5)],
                                   "balanced_resources": ["cpu", "memory", "ext0"]}}
# algorithmic bytes per pod x node evaluation of the normalizing profiles: the 8 state columns (32 B),
# the two extended-resource columns (8 B) and the taint / label mask row (32 B)
B_NODE_NORM = 72
C4G_INST = "<23u,"  # k_la_stream_res<kFeatRes | kFeatExt | kFeatTaint | kFeatAffinity, ...> (qs_kernels_res.inc)
B_NODE = 32  # algorithmic bytes per pod×node evaluation (8 int32 columns)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md:36 (spec); 6,290 GB/s measured
KERNEL_NAMES = {"resolve": "k_la_resolve4", "select": "k_la_select", "persistent": "k_persistent",
                "scan": "k_scan_key", "stream": "k_la_stream_res"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="auto", choices=["auto", "config2", "config3"])
    ap.add_argument("--engine", default="auto")
    ap.add_argument("--lookahead", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="pods in the CPU-baseline sample (0 = the whole stream, diffed against the GPU)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-config3", action="store_true", help="skip the N=1 config-3 reference point")
    ap.add_argument("--no-scan", action="store_true", help="skip the HBM-resident scan roofline leg")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the end-to-end, framework-path and wide-layout legs")
    ap.add_argument("--transport", default="mailbox", choices=["mailbox", "rccl"],
                    help="sharded exchange (N > 1): peer-memory mailbox over xGMI, or RCCL all-gather")
    ap.add_argument("--leg", default=None, choices=["config2", "wide", "config3", "config4", "config4_gpu_scoring",
                                                    "config5", "framework"],
                    help="run only this sub-leg on one GPU and print its JSON object (iteration probe, "
                         "not the bench line)")
    ap.add_argument("--rccl-sample", type=int, default=20000,
                    help="pods of the per-pod RCCL all-reduce leg (config-3 cluster; 0 = skip the leg)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print the launch plan (torchrun argv for --gpus N > 1) and exit, no GPU touched")
    return ap.parse_args(argv)


def launch_plan(a, argv, env=None):
    """How this invocation runs: {"mode": "torchrun", "argv": [...]} when --gpus N > 1 and no
    launcher environment is present (re-launch as N ranks), {"mode": "in-process", ...} otherwise.
    Raises SystemExit when a launcher's WORLD_SIZE disagrees with --gpus."""
    env = os.environ if env is None else env
    world = env.get("WORLD_SIZE")
    if world is None:
        if a.gpus > 1:
            import socket
            with socket.socket() as sk:  # a free local port for the rendezvous
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
                   os.path.abspath(__file__)] + [x for x in argv if x != "--dry-run"]
            return {"mode": "torchrun", "argv": cmd, "world": a.gpus}
        return {"mode": "in-process", "world": 1}
    if int(world) != a.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} from the launcher but --gpus {a.gpus}")
    return {"mode": "in-process", "world": int(world)}


class Ctx:
    """Process-group plumbing: rank/world from the torchrun env, RCCL id broadcast, barriers."""

    def __init__(self, backend=None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        # QS_BENCH_ONE_GPU=1 (rehearsal on a one-GPU box, with QS_BENCH_BACKEND=gloo): every rank
        # uses device 0, so the sharded mailbox path runs end to end as N processes on one card
        if os.environ.get("QS_BENCH_ONE_GPU") == "1":
            self.local = 0
        # "nccl" (= RCCL) on the GPU box; "gloo" rehearses the plumbing on CPU (tests/test_bench_launch.py)
        self.backend = backend or os.environ.get("QS_BENCH_BACKEND", "nccl")
        self.dev = f"cuda:{self.local}" if self.backend == "nccl" else "cpu"
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist

            if self.backend == "nccl":
                torch.cuda.set_device(self.local)
            dist.init_process_group(self.backend, init_method="env://")
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            import torch
            self.dist.barrier()
            if self.backend == "nccl":
                torch.cuda.synchronize()

    def max(self, v):
        if self.dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def min(self, v):
        if self.dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return float(t.item())

    def shard(self):
        """(rank, world, RCCL unique id) for qs_open_shard; the id is made on rank 0."""
        import torch
        uid = qsched.dist_unique_id() if self.rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8, device=self.dev)
        self.dist.broadcast(t, 0)
        return (self.rank, self.world, bytes(t.cpu().numpy().tolist()))


TRANSPORT = {"name": "mailbox"}  # sharded exchange: peer-memory mailbox (default) or RCCL


class PeerFailed(RuntimeError):
    """Another rank failed a phase this rank completed (raised on every rank at the same point)."""


def agree(cx, err):
    """Fixed collective point: every rank learns whether all ranks completed the phase; a local
    error is re-raised, a peer's surfaces as PeerFailed, on every rank after the same all-reduce
    (a rank that fails must not leave its peers blocked in a different collective)."""
    if cx.min(0.0 if err is not None else 1.0) > 0:
        return
    raise err if err is not None else PeerFailed("failed on another rank")


def open_sched(cx, cfg, sharded):
    """Sharded runs use the peer-memory mailbox (every rank exports its mailbox handle, the handles
    are all-gathered over the process group) or, with --transport rccl, an RCCL communicator.  The
    mailbox path runs the same collectives on every rank whatever fails locally."""
    if not sharded:
        return qsched.Scheduler(cfg, device=cx.local)
    if TRANSPORT["name"] == "rccl":
        return qsched.Scheduler(cfg, device=cx.local, shard=cx.shard())
    s = h = err = None
    try:
        s = qsched.Scheduler(cfg, device=cx.local, shard=(cx.rank, cx.world, None))
        h = s.mailbox_export()
    except Exception as e:
        err = e
    allh = [None] * cx.world
    cx.dist.all_gather_object(allh, h)
    if err is None and all(x is not None for x in allh):
        try:
            s.mailbox_connect(allh)
        except Exception as e:
            err = e
    try:
        agree(cx, err)
    except Exception:
        if s is not None:
            s.close()
        raise
    return s


def run_phase(cx, fn):
    """Local work of one phase, then the agreement point; returns fn's value."""
    out, err = None, None
    try:
        out = fn()
    except Exception as e:
        err = e
    agree(cx, err)
    return out


def load_prepare(s, nodes, pods):
    s.load_nodes(nodes)
    return s.prepare(pods)


def diag_runs(cx, nodes, pods, cfg, sharded):
    """Untimed diagnostic runs: per-pod device timestamps (p50/p99 decision interval) and per-kernel
    HIP-event times on the library's own stream (config.profile_kernels)."""
    s2 = open_sched(cx, dict(cfg, record_timestamps=1), sharded)
    try:
        st2 = run_phase(cx, lambda: load_prepare(s2, nodes, pods))
        cx.barrier()  # every rank's first window within the exchange's wait bound

        def stamps():
            st2.run()
            d = np.diff(st2.stamps().astype(np.int64)) * 0.01  # 100 MHz s_memrealtime ticks -> us
            st2.free()
            # split by window position: the interval ending at a window's first pod
            # (the window boundary, 1 in K) against the ones inside a window
            K = int(cfg.get("lookahead") or 32)
            bnd = (np.arange(1, len(d) + 1) % K) == 0
            split = {"window_boundary": float(np.percentile(d[bnd], 99)) if bnd.any() else None,
                     "within_window": float(np.percentile(d[~bnd], 99)) if (~bnd).any() else None}
            return float(np.percentile(d, 50)), float(np.percentile(d, 99)), split
        p50, p99, split = run_phase(cx, stamps)
    finally:
        s2.close()
    s3 = open_sched(cx, dict(cfg, profile_kernels=1), sharded)
    try:
        st3 = run_phase(cx, lambda: load_prepare(s3, nodes, pods))
        cx.barrier()

        def prof():
            r3 = st3.run()
            kp = r3["kernels"]
            if r3.get("resident") and "resolve" in kp:  # one resident launch
                kp = {"stream": kp["resolve"]}
            st3.free()
            return kp
        kp = run_phase(cx, prof)
    finally:
        s3.close()
    return p50, p99, kp, split


def roofline(kp, n_nodes, n_pods, fallback_s, b_node=B_NODE, inst=None):
    """Dominant kernel (most device time in the profiled run): algorithmic bytes per launch =
    (pod x node evaluations it completes per launch) x B_node / mean launch time."""
    dom = max(kp, key=lambda k: kp[k]["s"]) if kp else None
    avg_s = kp[dom]["s"] / kp[dom]["launches"] if dom else fallback_s
    units = n_pods * n_nodes / (kp[dom]["launches"] if dom else 1)
    achieved = units * b_node / avg_s / 1e9
    kname = KERNEL_NAMES.get(dom, dom)
    traffic, tk = pmc_traffic(kname, inst) if dom else (None, None)
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": None if traffic is None else round(traffic),
            "kernel": kname, "avg_launch_us": round(avg_s * 1e6, 3),
            "bytes_per_launch": round(units * b_node), "bytes_per_eval": b_node, "traffic_kernel": tk}


def pmc_traffic(kernel_prefix, inst=None):
    """HBM bytes per launch of `kernel_prefix` (and, if given, the template-argument prefix `inst`,
    e.g. "<23u," for one feature class) from the committed rocprofv3 PMC summary
    (profiles/*_pmc_summary.csv, tools/summarize_pmc.py: separate FETCH_SIZE and WRITE_SIZE
    passes, 2 x FETCH_SIZE + WRITE_SIZE per MI355X_MICROARCH.md:298), with the matched row's
    kernel name.  (None, None) if not collected."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.csv")))
    if not files:
        return None, None
    for row in csv.DictReader(open(files[-1])):
        name = row["kernel"]
        base, _, targs = name.partition("<")
        if base.endswith(kernel_prefix) and (inst is None or ("<" + targs).startswith(inst)):
            return float(row["hbm_bytes_per_launch"]), name
    return None, None


_T0 = time.time()


def progress(msg):
    """A phase line on stderr (the JSON line alone goes to stdout): a full run takes minutes, and
    the GPU pool takes a command silent for 3 minutes to be hung."""
    print(f"bench [{time.time() - _T0:6.1f} s] {msg}", file=sys.stderr, flush=True)


def host_info():
    """The box the CPU arms ran on (north_star: "core count stated")."""
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "usable_cpus": usable,
            "cgroup_cpus": cgroup_cpus(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cgroup_cpus():
    """CPUs' worth of time the cgroup grants (cgroup v2 cpu.max quota / period; None = no quota).
    The GPU box's affinity mask shows every CPU of the machine while its share is 16: OpenMP at the
    mask's width oversubscribes the quota (ROUND 4: the 256-thread arm did not finish in 3 min)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:  # cgroup v1
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, -(-q // per))
    except (OSError, ValueError):
        return None


def effective_cpus():
    """min(affinity mask, cgroup quota, OMP_NUM_THREADS when the environment sets the share)."""
    h = host_info()
    omp = h["omp_num_threads"]
    cands = [x for x in (h["usable_cpus"], h["cgroup_cpus"], int(omp) if omp and omp.isdigit() else None) if x]
    return min(cands) if cands else (os.cpu_count() or 16)


def cpu_baseline(nodes, pods, n_nodes, n_pods, sample, threads=1, gpu_placement=None, repeats=5):
    """Oracle (C restatement) on the same stream: 1 thread, or the node-parallel OpenMP arm
    (SURVEY §8(d) arm 2: upstream's Parallelizer runs 16 workers).  sample = 0 runs the whole
    stream, and its placements are diffed against the GPU's (`placements_match`).  The value is the
    median of `repeats` runs (median of 5); every run's rate is listed."""
    from oracle import oracle as O

    whole = sample <= 0 or sample >= n_pods
    sample = n_pods if whole else sample
    sub = qsched.pods_from_struct(pods[:sample])
    times, placement = [], None
    for r in range(repeats):
        progress(f"cpu baseline: {sample:,} pods, {threads} thread(s), run {r + 1} of {repeats}")
        on = {k: v.copy() for k, v in nodes.items()}
        t0 = time.perf_counter()
        pl, _, _ = O.schedule(on, sub, nthreads=threads)
        times.append(time.perf_counter() - t0)
        placement = pl if placement is None else placement
    dt = float(np.median(times))
    how = "1 thread" if threads == 1 else f"{threads} OpenMP threads over the nodes of each pod"
    what = (f"the whole {n_pods:,}-pod stream" if whole else
            f"first {sample:,} of the {n_pods:,} pods (QoS-sorted within the sample)")
    out = {"value": round(sample / dt, 1), "unit": "pods/s", "cores": threads, "kind": "port",
           "host": host_info(),
           "sample": f"{what} onto the empty {n_nodes:,}-node cluster, oracle/qs_oracle.c {how}, "
                     f"median of {repeats} runs, {dt:.2f} s each",
           "runs_pods_per_s": [round(sample / t, 1) for t in times],
           "evals_per_s": round(sample * n_nodes / dt, 1)}
    if whole and gpu_placement is not None:
        out["placements_match"] = bool(np.array_equal(placement, gpu_placement))
    return out


def cpu_baseline_framework(n_nodes=5000, sample=4000, threads=16, repeats=5):
    """The north_star's baseline shape (BASELINE.json:5, configs[0] :7): the CPU reference plugins
    (host/cpu_plugins.cpp: NodeResourcesFit + LeastAllocated, BalancedAllocation, QoS-class profile
    weights) through the framework runtime (Run*Plugins, upstream's 16-worker node Parallelizer,
    deterministic selectHost) on config 2's cluster as k8s objects, timed by tools/cpu_framework.cpp
    (Go is absent: the plugin set is C++).  Median of `repeats`; placements diffed against the
    oracle on the same pods inside the tool."""
    import subprocess
    exe = os.path.join(ROOT, "custom-k8s-scheduler_amd", "cpu_framework")
    runs = []
    for rr in range(repeats):
        progress(f"cpu framework baseline: run {rr + 1} of {repeats}")
        r = subprocess.run([exe, "2", str(n_nodes), str(sample), str(threads)], capture_output=True, text=True,
                           timeout=300)
        runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    med = sorted(runs, key=lambda x: x["pods_per_s"])[len(runs) // 2]
    return {"value": med["pods_per_s"], "unit": "pods/s", "cores": threads, "kind": "port",
            "host": host_info(),
            "sample": f"first {sample:,} pods of config 2 (QoS-sorted) onto the empty {n_nodes:,}-node cluster "
                      "as k8s objects: CPU plugins through the framework runtime (tools/cpu_framework.cpp), "
                      f"{threads}-worker Parallelizer, median of {repeats} runs, {med['seconds']:.2f} s each",
            "runs_pods_per_s": [x["pods_per_s"] for x in runs],
            "evals_per_s": med["evals_per_s"],
            "placements_match": all(x["placements_match"] for x in runs)}


def measure(cx, a, workload, steps, warmup, with_diag=True):
    """Timed exact stream of `workload`; returns a dict of measurements (rank-0 meaningful).  Every
    rank runs the same collectives in the same order whatever fails locally: open (open_sched's
    agreement), load + prepare (agreement), the steps (a failed step skips the rest; barriers and an
    agreement after the loop), results (agreement)."""
    gen, n_nodes, n_pods, desc = WORKLOADS[workload]
    sharded = workload == "config3" and cx.world > 1
    seed = 0x5EED0000 + gen + (cx.rank if (cx.world > 1 and not sharded) else 0)
    nodes, pods = qsched.synth_generate(gen, n_nodes, n_pods, seed=seed)
    cfg = dict({"engine": a.engine, "lookahead": a.lookahead}, **PROFILE.get(workload, {}))
    mode = MODE.get(workload, "exact")
    s = open_sched(cx, cfg, sharded)
    try:
        def setup():
            s.load_nodes(nodes)
            st_ = s.prepare(pods)  # (may re-lay the table out for the pods' quantities: snapshot after)
            s.save_table()
            return st_
        st = run_phase(cx, setup)

        def step():
            s.restore_table()
            return st.run(mode=mode)

        # all ranks enter their first run together: a sharded rank's first window waits (bounded)
        # for its peers' lists, and a one-sided timeout would void only that rank's run
        err, last = None, None
        cx.barrier()
        for _ in range(warmup):
            if err is None:
                try:
                    step()
                except Exception as e:
                    err = e
        cx.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            if err is None:
                try:
                    last = step()
                except Exception as e:
                    err = e
        cx.barrier()
        dt = time.perf_counter() - t0
        agree(cx, err)
        elapsed = cx.max(dt)

        def collect():
            pl_, keys_ = st.results()
            final_ = s.read_nodes()  # the table after the last timed step (which started from the snapshot)
            st.free()
            return pl_, keys_, final_
        placement, keys, final = run_phase(cx, collect)
    finally:
        s.close()
    ranks_work = cx.world if (cx.world > 1 and not sharded) else 1  # replicas multiply the work
    value = n_pods * steps * ranks_work / elapsed
    out = {"value": value, "ms_per_step": elapsed / steps * 1e3, "engine": last["engine_used"],
           "launch": "resident" if last.get("resident") else "per-window",
           "table_layout": last["table_layout"],
           "unschedulable_frac": float((placement < 0).mean()), "n_nodes": n_nodes,
           "placement": placement.copy(), "keys": keys, "final": final, "cfg": cfg,
           "n_pods": n_pods, "desc": desc, "sharded": sharded, "nodes": nodes, "pods": pods,
           "replicas": ranks_work}
    if with_diag:
        out["p50"], out["p99"], out["kp"], out["p99_split"] = diag_runs(cx, nodes, pods, cfg, sharded)
        out["wall_fallback"] = last["wall_s"]
    return out


def measure_sharded(cx, a, workload):
    """N > 1 config 3: the requested transport (default: the peer-memory mailbox, which runs the
    sharded RESIDENT stream), falling back to the RCCL all-gather when any rank fails or the ranks'
    placements disagree.  measure() fails on every rank at the same agreement point, and the ranks
    then all-reduce an ok flag and the placement checksum, so a fallback never leaves ranks out of
    step (tests/test_bench_launch.py drives real measure() failures at world 2 over gloo)."""
    import zlib

    tried = []
    order = [a.transport] + (["rccl"] if a.transport != "rccl" else [])
    for name in order:
        TRANSPORT["name"] = name
        m, err = None, None
        try:
            m = measure(cx, a, workload, a.steps, a.warmup)
        except Exception as e:  # a timed-out or failed exchange on this rank
            err = repr(e)[:300]
        ok = cx.min(1.0 if m is not None else 0.0) > 0
        if ok:
            crc = float(zlib.crc32(np.ascontiguousarray(m["placement"]).tobytes()))
            ok = cx.min(crc) == cx.max(crc)
            if not ok:
                err = "placements differ across ranks"
        if ok:
            m["transport"] = name
            m["transport_tried"] = tried
            return m
        tried.append({"transport": name, "error": err or "failed on another rank"})
    raise SystemExit(f"bench.py: every transport failed: {tried}")


def measure_rccl_per_pod(cx, a):
    """SURVEY.md §8(e) C1, RCCL as-is: the config-3 cluster (50,000 nodes) and a
    bounded sample of its pod stream (the first --rccl-sample arrivals, same generator) on the per-pod
    all-reduce engine: each rank scans its node shard per pod and the ranks max-reduce one packed
    8-byte key with ncclAllReduce (QS_ENGINE_ALLREDUCE).  One warm-up and one timed step, MAX over
    ranks; reported beside the sharded line as the labelled baseline of the lookahead transports.
    Every rank runs the same collectives whatever fails locally (run_phase / agree)."""
    gen, n_nodes, _, _ = WORKLOADS["config3"]
    sample = a.rccl_sample
    nodes, pods = qsched.synth_generate(gen, n_nodes, sample)
    cfg = {"engine": "allreduce"}
    s = run_phase(cx, lambda: qsched.Scheduler(cfg, device=cx.local,
                                               shard=cx.shard() if cx.world > 1 else (0, 1, qsched.dist_unique_id())))
    try:
        def setup():
            s.load_nodes(nodes)
            st_ = s.prepare(pods)
            s.save_table()
            return st_
        st = run_phase(cx, setup)
        err, last = None, None
        cx.barrier()
        try:
            s.restore_table()
            st.run()
        except Exception as e:
            err = e
        cx.barrier()
        t0 = time.perf_counter()
        if err is None:
            try:
                s.restore_table()
                last = st.run()
            except Exception as e:
                err = e
        cx.barrier()
        dt = time.perf_counter() - t0
        agree(cx, err)
        elapsed = cx.max(dt)
        placement, _ = run_phase(cx, st.results)
        st.free()
    finally:
        s.close()
    return {"variant": "RCCL as-is: per pod one ncclAllReduce(count 1, ncclUint64, ncclMax) of the packed "
                       "(score, node) key over the node shards (SURVEY.md section 8(e) C1, QS_ENGINE_ALLREDUCE)",
            "workload": f"config3 cluster ({n_nodes:,} nodes), first {sample:,} pods of its stream",
            "value": round(sample / elapsed, 1), "unit": "pods/s", "ms_per_step": round(elapsed * 1e3, 3),
            "us_per_pod": round(elapsed / sample * 1e6, 3), "steps": 1, "engine": last["engine_used"],
            "n_gpus": cx.world, "nodes": nodes, "pods": pods, "placement": placement}


def check_rccl_sample(r):
    """The per-pod all-reduce sample against the oracle's incremental exact stream."""
    from oracle import oracle as O
    on = {k: v.copy() for k, v in r.pop("nodes").items()}
    ref, _, _ = O.schedule_incremental(on, qsched.pods_from_struct(r.pop("pods")), {}, nthreads=16)
    return bool(np.array_equal(r.pop("placement"), ref))


def check_stream(m):
    """Correctness of a timed leg: the oracle over the WHOLE stream, diffed
    against the GPU's placements, per-pod keys and final table, plus qsched.checks' size-independent
    invariants.  Fit + Balanced profiles use or_schedule_incremental (the brute-force oracle's
    node_key() with an incremental argmax: seconds for config 3's 1,000,000 x 50,000), normalizing
    profiles the brute-force oracle with 16 threads."""
    from oracle import oracle as O
    from qsched.checks import stream_invariants

    norm = bool(m["cfg"].get("enable_taint") or m["cfg"].get("enable_affinity"))
    ocfg = {k: m["cfg"][k] for k in ("enable_taint", "enable_affinity", "fit_resources", "balanced_resources")
            if k in m["cfg"]}
    on = {k: v.copy() for k, v in m["nodes"].items()}
    sub = qsched.pods_from_struct(m["pods"])
    t0 = time.perf_counter()
    if norm:
        ref, rkeys, _ = O.schedule(on, sub, ocfg, nthreads=16)
        how = "oracle/qs_oracle.c or_schedule, 16 OpenMP threads"
    else:
        ref, rkeys, _ = O.schedule_incremental(on, sub, ocfg, nthreads=16)
        how = "oracle/qs_oracle.c or_schedule_incremental, 16 OpenMP threads"
    dt = time.perf_counter() - t0
    inv = stream_invariants(m["nodes"], m["pods"], m["placement"], m["final"], fit_only=not norm)
    return {"placements_match": bool(np.array_equal(ref, m["placement"])),
            "keys_match": bool(np.array_equal(rkeys, m["keys"])),
            "table_match": all(bool(np.array_equal(on[k], m["final"][k])) for k in on),
            "oracle": how, "oracle_s": round(dt, 2),
            "invariants": {k: v for k, v in inv.items() if v is not None}}


def check_batched(m):
    """Correctness of the batched leg (config 5, spec S11): the incremental batched oracle over the
    WHOLE stream (or_schedule_batched_incremental, identical to or_schedule_batched: per pod type and
    zone a max tree, only claimed nodes re-scored), diffed against the GPU's placements, claimed keys
    and final table, plus conservation / capacity / anti-affinity invariants."""
    from oracle import oracle as O
    from qsched.checks import batched_invariants

    on = {k: v.copy() for k, v in m["nodes"].items()}
    t0 = time.perf_counter()
    ref, rkeys, _ = O.schedule_batched_incremental(on, qsched.pods_from_struct(m["pods"]), nthreads=16)
    dt = time.perf_counter() - t0
    inv = batched_invariants(m["nodes"], m["pods"], m["placement"], m["final"])
    return {"placements_match": bool(np.array_equal(ref, m["placement"])),
            "keys_match": bool(np.array_equal(rkeys, m["keys"])),
            "table_match": all(bool(np.array_equal(on[k], m["final"][k])) for k in on),
            "oracle": "oracle/qs_oracle.c or_schedule_batched_incremental, 16 OpenMP threads",
            "oracle_s": round(dt, 2), "invariants": inv}


def scan_roofline(cx, a, n_nodes=1 << 24, n_pods=32):
    """The scoring scan at an HBM-resident table (north_star's >= 50 % target):
    the SCAN engine's exact stream over 2^24 nodes (512 MiB of SoA columns, beyond the 256 MiB
    Infinity Cache), one full Filter+Score scan + argmax per pod, then Reserve.  Achieved =
    n_nodes x B_node / mean k_scan_soa launch time (HIP events on the library stream)."""
    nodes, pods = qsched.synth_generate(2, n_nodes, n_pods)
    cfg = {"engine": "scan"}
    s = qsched.Scheduler(cfg, device=cx.local)
    s.load_nodes(nodes)
    st = s.prepare(pods)
    s.save_table()
    st.run()  # warm-up
    walls = []
    for _ in range(3):
        s.restore_table()
        walls.append(st.run()["wall_s"])
    placement, _ = st.results()  # the last run started from the restored (empty) table
    st.free()
    s.close()
    from oracle import oracle as O
    on = {k: v.copy() for k, v in nodes.items()}
    t0 = time.perf_counter()
    ref, _, _ = O.schedule(on, qsched.pods_from_struct(pods), nthreads=16)
    oracle_s = time.perf_counter() - t0
    del on
    sp = qsched.Scheduler(dict(cfg, profile_kernels=1), device=cx.local)
    sp.load_nodes(nodes)
    stp = sp.prepare(pods)
    stp.run()
    kp = stp.run()["kernels"]["scan"]  # second run: table already advanced, same work per scan
    stp.free()
    sp.close()
    avg = kp["s"] / kp["launches"]
    achieved = n_nodes * B_NODE / avg / 1e9
    wall = min(walls)
    return {"workload": f"SCAN engine, {n_nodes:,} nodes (config-2 distribution, SoA columns) x "
                        f"{n_pods} pods: one full scoring scan + argmax + Reserve per pod",
            "pods_per_s": round(n_pods / wall, 1), "evals_per_s": round(n_pods * n_nodes / wall, 1),
            "placements_match": bool(np.array_equal(placement, ref)),
            "oracle_16t_s": round(oracle_s, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic("k_scan_soa")[0], "kernel": "k_scan_soa",
                         "avg_launch_us": round(avg * 1e6, 2),
                         "bytes_per_launch": n_nodes * B_NODE}}


def ki_decimal_cluster(n, p, seed):
    """Config-2 shaped cluster in real-world quantities: odd-Ki node allocatable (64-768 GiB, as
    kubelet reports it) and decimal pod requests (100M, 512M, 1G, 3G).  Needs the wide layout."""
    nodes, pods = qsched.synth_generate(2, n, p, seed=seed)
    rng = np.random.default_rng(seed)
    nodes["alloc_mem"][:] = (rng.integers(64 << 20, 768 << 20, n) | 1) * 1024
    dec = rng.choice([100 * 10**6, 512 * 10**6, 10**9, 3 * 10**9], p)
    has = pods["req_mem"] > 0
    pods["req_mem"] = np.where(has, dec, 0)
    pods["nz_mem"] = np.where(has, dec, 209715200)
    return nodes, pods


def wide_leg(cx, a, n_nodes=5000, n_pods=100000, steps=3):
    """Config-2 shape on the wide layout (f64 memory columns), placements diffed
    against the 16-thread oracle."""
    nodes, pods = ki_decimal_cluster(n_nodes, n_pods, seed=0x5EED0002)
    s = qsched.Scheduler({"engine": a.engine, "lookahead": a.lookahead}, device=cx.local)
    s.load_nodes(nodes)
    st = s.prepare(pods)
    s.save_table()
    stats = st.run()
    walls = []
    for _ in range(steps):
        s.restore_table()
        t0 = time.perf_counter()
        st.run()
        walls.append(time.perf_counter() - t0)
    placement, _ = st.results()
    st.free()
    s.close()
    from oracle import oracle as O
    on = {k: v.copy() for k, v in nodes.items()}
    ref, _, _ = O.schedule(on, qsched.pods_from_struct(pods), nthreads=16)
    wall = min(walls)
    return {"workload": f"{n_nodes:,} nodes (odd-Ki allocatable 64-768 GiB) x {n_pods:,} pods "
                        "(decimal requests 100M/512M/1G/3G): exact stream on the wide layout",
            "table_layout": stats["table_layout"], "engine": stats["engine_used"],
            "launch": "resident" if stats.get("resident") else "per-window",
            "value": round(n_pods / wall, 1), "unit": "pods/s", "ms_per_step": round(wall * 1e3, 3),
            "placements_match": bool(np.array_equal(placement, ref))}


def e2e_leg(cx, nodes, pods, gpu_placement):
    """qs_schedule_stream end to end on a freshly loaded table (SURVEY.md §8(d) GPU timing): host
    precompute (QoSSort, compaction) + H2D of the pod records + device run (incl. building the
    stream's HIP graph) + D2H of placements, with the phases reported separately."""
    out = []
    for _ in range(2):
        s = qsched.Scheduler({}, device=cx.local)
        s.load_nodes(nodes)
        t0 = time.perf_counter()
        placement, stats = s.schedule(pods, with_stats=True)
        e2e = time.perf_counter() - t0
        s.close()
        out.append((e2e, stats, placement))
    e2e, stats, placement = min(out, key=lambda x: x[0])
    n = len(placement)
    return {"what": "qs_schedule_stream wall on a freshly loaded table: prepare (QoSSort + compaction "
                    "+ H2D) + run (graph build + device stream) + D2H of placements",
            "pods_per_s": round(n / e2e, 1), "e2e_ms": round(e2e * 1e3, 3),
            "prepare_h2d_ms": round(stats["h2d_s"] * 1e3, 3), "device_run_ms": round(stats["wall_s"] * 1e3, 3),
            "d2h_ms": round(stats["d2h_s"] * 1e3, 3),
            "placements_match": bool(np.array_equal(placement, gpu_placement))}


def framework_leg(cx, n_nodes=5000, n_pods=5000):
    """The framework-embedded path (SURVEY.md §3.4, §5 p99 definition): per pod one qs_score_pod
    (PreFilter..NormalizeScore over all nodes, per-node feasible / plugin scores / totals copied
    back for Filter/Score lookups) + one qs_reserve of the chosen node, host wall per pod through
    the Python ctypes binding.  Arrival order; placements diffed against the oracle."""
    nodes, pods = qsched.synth_generate(2, n_nodes, n_pods)
    s = qsched.Scheduler({}, device=cx.local)
    s.load_nodes(nodes)
    lat = np.empty(n_pods)
    placement = np.empty(n_pods, np.int32)
    bufs = s.score_buffers()  # reused per call, as a plugin keeps its per-node arrays
    for j in range(n_pods):
        t0 = time.perf_counter()
        best = s.score_pod(pods[j], out=bufs)["best"]
        if best >= 0:
            s.reserve(best, pods[j])
        lat[j] = time.perf_counter() - t0
        placement[j] = best
    s.close()
    from oracle import oracle as O
    on = {k: v.copy() for k, v in nodes.items()}
    ref, _, _ = O.schedule(on, qsched.pods_from_struct(pods), {"qos_sort": 0}, nthreads=16)
    us = lat * 1e6
    out = {"workload": f"{n_nodes:,} nodes x {n_pods:,} pods, qs_score_pod + qs_reserve per pod, arrival "
                       "order; p50/p99 from the C++ caller (tools/fw_latency.cpp, every per-node output "
                       "copied out), python_ctypes = the same loop through the ctypes binding",
           "python_ctypes": {"p50_us": round(float(np.percentile(us, 50)), 2),
                             "p99_us": round(float(np.percentile(us, 99)), 2),
                             "mean_us": round(float(us.mean()), 2), "pods_per_s": round(n_pods / lat.sum(), 1),
                             "placements_match": bool(np.array_equal(placement, ref))}}
    import subprocess
    exe = os.path.join(ROOT, "custom-k8s-scheduler_amd", "fw_latency")
    # mode 1: every per-node output copied out; 0: best key only; 2: the packed per-node words read in
    # place (qs_score_pod_packed, §4.6); the 50,000-node rows: any table size takes the same launch
    for nn, npods, outputs, key in ((n_nodes, n_pods, 1, "native"), (n_nodes, n_pods, 0, "native_best_only"),
                                    (n_nodes, n_pods, 2, "native_packed"), (50000, 3000, 2, "native_50k_packed"),
                                    (50000, 3000, 1, "native_50k")):
        try:
            r = subprocess.run([exe, str(nn), str(npods), str(outputs)], capture_output=True, text=True,
                               timeout=120)
            out[key] = json.loads(r.stdout.strip().splitlines()[-1])
        except Exception as e:  # reported, not fatal: the ctypes numbers stand
            out[key] = {"error": repr(e)[:200]}
    nat = out.get("native", {})
    for k in ("p50_us", "p99_us", "mean_us", "pods_per_s", "placements_match"):
        out[k] = nat.get(k, out["python_ctypes"][k])
    return out


def run_leg(cx, a, leg):
    """One sub-leg alone (--leg), with its correctness check."""
    if leg == "wide":
        return wide_leg(cx, a)
    if leg == "framework":
        return framework_leg(cx)
    steps = 1 if leg == "config3" else 3
    gs = leg == "config4_gpu_scoring"
    m = measure(cx, a, leg, steps, 1, with_diag=gs)
    out = {"workload": m["desc"], "value": round(m["value"], 1), "unit": "pods/s",
           "ms_per_step": round(m["ms_per_step"], 3), "engine": m["engine"], "launch": m["launch"],
           "unschedulable_frac": round(m["unschedulable_frac"], 5)}
    if gs:
        out["roofline"] = roofline(m["kp"], m["n_nodes"], m["n_pods"], m["wall_fallback"], b_node=B_NODE_NORM,
                                   inst=C4G_INST)
    out["check"] = check_batched(m) if leg == "config5" else check_stream(m)
    return out


def main():
    argv = sys.argv[1:]
    a = parse(argv)
    TRANSPORT["name"] = a.transport
    plan = launch_plan(a, argv)
    if a.dry_run:
        print(json.dumps(plan), flush=True)
        return 0
    if plan["mode"] == "torchrun":
        # one rank per GPU; this parent never touches the GPU (no exec after GPU init)
        import subprocess
        return subprocess.run(plan["argv"]).returncode
    # stdout carries the JSON line alone: native libraries' banners (RCCL prints its version lines
    # on stdout at communicator init) and any other print go to stderr
    real_out = sys.stdout
    if real_out is sys.__stdout__:  # the process's fd 1: kept for the JSON line, fd 1 -> stderr
        sys.stdout.flush()
        real_out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
    emit = lambda obj: print(json.dumps(obj), file=real_out, flush=True)
    cx = Ctx()
    if a.leg:
        emit(run_leg(cx, a, a.leg))
        return 0
    workload = a.workload if a.workload != "auto" else ("config2" if cx.world == 1 else "config3")
    progress(f"{workload}: timed stream ({a.steps} steps, {a.warmup} warmup)")
    if cx.world > 1 and workload == "config3":
        m = measure_sharded(cx, a, workload)
    else:
        m = measure(cx, a, workload, a.steps, a.warmup)
    rccl = None
    if workload == "config3" or (cx.world == 1 and not a.no_config3):
        if a.rccl_sample > 0:
            progress(f"per-pod RCCL all-reduce leg ({a.rccl_sample} pods)")
            try:
                rccl = measure_rccl_per_pod(cx, a)
            except Exception as e:  # reported, not fatal (every rank fails it at the same point)
                rccl = {"error": repr(e)[:300]}
    c3 = c4 = c4g = c5 = scan = None
    if cx.world == 1 and workload == "config2" and not a.no_config3:
        progress("config3 leg")
        c3 = measure(cx, a, "config3", 1, 1, with_diag=False)
        progress("config4 leg")
        c4 = measure(cx, a, "config4", 3, 1, with_diag=False)
        progress("config4 leg with the AMD-GPU scoring resources")
        c4g = measure(cx, a, "config4_gpu_scoring", 3, 1, with_diag=True)
        progress("config5 leg")
        c5 = measure(cx, a, "config5", 3, 1, with_diag=False)
    if cx.world == 1 and not a.no_scan:
        progress("scan roofline leg")
        scan = scan_roofline(cx, a)
    e2e = fw = wide = None
    if cx.world == 1 and workload == "config2" and not a.no_extra:
        progress("end-to-end, framework and wide legs")
        e2e = e2e_leg(cx, m["nodes"], m["pods"], m["placement"])
        fw = framework_leg(cx)
        wide = wide_leg(cx, a)
    if cx.rank == 0:
        rl = roofline(m["kp"], m["n_nodes"], m["n_pods"], m["wall_fallback"],
                      inst="<0u," if not m["sharded"] and workload == "config2" else None)
        if m["sharded"]:
            how = ("RCCL all-gather per window" if TRANSPORT["name"] == "rccl" else
                   "peer-memory mailbox, shard lists exchanged in-launch" if m["launch"] == "resident" else
                   "peer-memory mailbox per window")
            par, scaling = f"node-sharded x{cx.world} ({how})", "strong"
        elif cx.world > 1:
            par, scaling = f"replicas x{cx.world}", "weak"
        else:
            par, scaling = "single", "weak"
        out = {
            "metric": f"pods scheduled/sec (exact sequential stream, {m['n_nodes']:,} nodes x "
                      f"{m['n_pods']:,} pods)",
            "value": round(m["value"], 1), "unit": "pods/s", "n_gpus": cx.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(m["ms_per_step"], 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "int32+f64",
            "data": f"synthetic (spec/synth.md generator, config {WORKLOADS[workload][0]})",
            "config": {"workload": m["desc"], "engine": m["engine"], "launch": m["launch"],
                       "table_layout": m["table_layout"],
                       "lookahead": a.lookahead or 32, "parallelism": par},
            "evals_per_s": round(m["value"] * m["n_nodes"], 1),
            "p50_pod_latency_us": round(m["p50"], 4), "p99_pod_latency_us": round(m["p99"], 4),
            "p99_pod_latency_split_us": {k: (round(v, 4) if v is not None else None)
                                         for k, v in (m.get("p99_split") or {}).items()},
            "unschedulable_frac": round(m["unschedulable_frac"], 5),
            "roofline": rl,
            "kernels_us_per_step": {k: round(v["s"] * 1e6, 1) for k, v in m["kp"].items()},
        }
        if m.get("transport"):
            out["config"]["transport"] = m["transport"]
            if m["transport_tried"]:
                out["config"]["transport_fallback_from"] = m["transport_tried"]
        if m["sharded"] or (cx.world == 1 and not a.no_cpu):
            progress("oracle check of the timed stream")
            out["check"] = check_stream(m)
        if rccl is not None:
            if "placement" in rccl:
                rccl["placements_match"] = check_rccl_sample(rccl)
            out["rccl_per_pod"] = rccl
        if c3 is not None:
            progress("oracle checks of the config 3 / 4 / 5 legs")
            out["config3"] = {"workload": c3["desc"] + " (1 GPU: the N=1 point of the curve)",
                              "value": round(c3["value"], 1), "unit": "pods/s",
                              "evals_per_s": round(c3["value"] * c3["n_nodes"], 1),
                              "ms_per_step": round(c3["ms_per_step"], 3), "steps": 1,
                              "engine": c3["engine"], "launch": c3["launch"],
                              "unschedulable_frac": round(c3["unschedulable_frac"], 5),
                              "check": check_stream(c3)}
        if c4 is not None:
            out["config4"] = {"workload": c4["desc"], "value": round(c4["value"], 1), "unit": "pods/s",
                              "evals_per_s": round(c4["value"] * c4["n_nodes"], 1),
                              "ms_per_step": round(c4["ms_per_step"], 3), "steps": 3,
                              "engine": c4["engine"], "launch": c4["launch"],
                              "unschedulable_frac": round(c4["unschedulable_frac"], 5),
                              "check": check_stream(c4)}
        if c4g is not None:
            out["config4_gpu_scoring"] = {
                "workload": c4g["desc"], "value": round(c4g["value"], 1), "unit": "pods/s",
                "evals_per_s": round(c4g["value"] * c4g["n_nodes"], 1),
                "ms_per_step": round(c4g["ms_per_step"], 3), "steps": 3, "engine": c4g["engine"],
                "launch": c4g["launch"], "unschedulable_frac": round(c4g["unschedulable_frac"], 5),
                "vs_config4": round(c4g["value"] / c4["value"], 4),
                "roofline": roofline(c4g["kp"], c4g["n_nodes"], c4g["n_pods"], c4g["wall_fallback"],
                                     b_node=B_NODE_NORM, inst=C4G_INST),
                "check": check_stream(c4g)}
        if c5 is not None:
            out["config5_batched"] = {"workload": c5["desc"], "value": round(c5["value"], 1),
                                      "unit": "pods/s", "evals_per_s": round(c5["value"] * c5["n_nodes"], 1),
                                      "ms_per_step": round(c5["ms_per_step"], 3), "steps": 3,
                                      "engine": c5["engine"],
                                      "unschedulable_frac": round(c5["unschedulable_frac"], 5),
                                      "check": check_batched(c5)}
        if scan is not None:
            out["scan"] = scan
        if e2e is not None:
            out["end_to_end"] = e2e
            out["framework_path"] = fw
            out["wide_layout"] = wide
        if cx.world == 1 and not a.no_cpu:
            out["cpu_baseline"] = cpu_baseline(m["nodes"], m["pods"], m["n_nodes"], m["n_pods"],
                                               a.cpu_sample, gpu_placement=m["placement"])
            out["cpu_baseline_parallel"] = cpu_baseline(m["nodes"], m["pods"], m["n_nodes"], m["n_pods"],
                                                        a.cpu_sample, threads=16,
                                                        gpu_placement=m["placement"])
            usable = effective_cpus()
            if usable != 16:  # the OpenMP arm at every CPU this process may use (a bounded sample)
                out["cpu_baseline_parallel_nproc"] = cpu_baseline(m["nodes"], m["pods"], m["n_nodes"], m["n_pods"],
                                                                  20000, threads=usable)
            else:
                out["cpu_baseline_parallel_nproc"] = {
                    "skipped": "this process may use 16 CPUs (affinity / cgroup quota / OMP_NUM_THREADS): "
                               "the nproc arm is cpu_baseline_parallel", "host": host_info()}
            out["cpu_baseline_framework"] = cpu_baseline_framework()
        emit(out)
    if cx.dist is not None:
        cx.dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
