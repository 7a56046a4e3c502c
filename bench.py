"""bench.py — BASELINE.json metric: pods scheduled/s (+ pod×node evals/s, p99 pod latency) of the
exact sequential stream, measured through libqsched's C ABI on MI355X.

Workloads (BASELINE.json configs):
  * N = 1 (default): configs[1] — 5,000 nodes × 100,000 pods on one GPU (the metric's config).
    The line also carries a ``config3`` object: the 50,000-node × 1,000,000-pod stream on the same
    single GPU, the N = 1 point of the config-3 scaling curve.
  * N > 1 (torchrun, one rank per GPU): configs[2] — 50,000 nodes × 1,000,000 pods with the node
    table sharded across the N ranks (qs_open_shard: contiguous node ranges, one RCCL all-gather of
    top-L lists per lookahead window over xGMI).  Total work is fixed: ``scaling`` = "strong".
  ``--workload config2|config3`` overrides (config2 at N > 1 = independent replicas, weak scaling).

A *step* = restore the empty cluster on the device (qs_table_restore, a D2D copy) + run the whole
exact stream (qs_stream_run): inputs resident in HBM, every pod scheduled, placements left in HBM.
Timed: K steps bracketed by barrier + device sync on both sides; MAX over ranks.
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

import qsched  # noqa: E402

WORKLOADS = {
    # name: (generator config, nodes, pods, description)
    "config2": (2, 5000, 100000, "config2: 5,000 nodes x 100,000 pods, exact sequential, "
                                 "Fit+Balanced+QoS weights, percentageOfNodesToScore=100"),
    "config3": (3, 50000, 1000000, "config3: 50,000 nodes x 1,000,000 pods, exact sequential, "
                                   "node table sharded across ranks (RCCL all-gather per window)"),
    "config4": (4, 5000, 150000, "config4: 5,000 nodes x 150,000 pods, exact sequential, Fit + "
                                 "Balanced + TaintToleration + NodeAffinity + amd.com/gpu"),
    "config5": (5, 10000, 200000, "config5: 10,000 nodes x 200,000 pods, BATCHED mode (spec S11: "
                                  "64-pod batches, one pod per node per batch, hostname/zone "
                                  "anti-affinity over 1,000 apps) - approximate, reported separately"),
}
MODE = {"config5": "batched"}
PROFILE = {"config4": {"enable_taint": 1, "enable_affinity": 1}}  # plugin switches per workload
B_NODE = 32  # algorithmic bytes per pod×node evaluation (8 int32 columns)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md:36 (spec); 6,290 GB/s measured
KERNEL_NAMES = {"resolve": "k_la_resolve4", "select": "k_la_select", "persistent": "k_persistent",
                "scan": "k_scan_key"}


def parse():
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
    return ap.parse_args()


class Ctx:
    """Process-group plumbing: rank/world from the torchrun env, RCCL id broadcast, barriers."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist

            torch.cuda.set_device(self.local)
            dist.init_process_group("nccl", init_method="env://")
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            import torch
            self.dist.barrier()
            torch.cuda.synchronize()

    def max(self, v):
        if self.dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=f"cuda:{self.local}")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def shard(self):
        """(rank, world, RCCL unique id) for qs_open_shard; the id is made on rank 0."""
        import torch
        uid = qsched.dist_unique_id() if self.rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8, device=f"cuda:{self.local}")
        self.dist.broadcast(t, 0)
        return (self.rank, self.world, bytes(t.cpu().numpy().tolist()))


def open_sched(cx, cfg, sharded):
    return qsched.Scheduler(cfg, device=cx.local, shard=cx.shard() if sharded else None)


def diag_runs(cx, nodes, pods, cfg, sharded):
    """Untimed diagnostic runs: per-pod device timestamps (p50/p99 decision interval) and per-kernel
    HIP-event times on the library's own stream (config.profile_kernels)."""
    p50 = p99 = None
    s2 = open_sched(cx, dict(cfg, record_timestamps=1), sharded)
    s2.load_nodes(nodes)
    st2 = s2.prepare(pods)
    st2.run()
    d = np.diff(st2.stamps().astype(np.int64)) * 0.01  # 100 MHz s_memrealtime ticks -> us
    p50, p99 = float(np.percentile(d, 50)), float(np.percentile(d, 99))
    st2.free()
    s2.close()
    s3 = open_sched(cx, dict(cfg, profile_kernels=1), sharded)
    s3.load_nodes(nodes)
    st3 = s3.prepare(pods)
    kp = st3.run()["kernels"]
    st3.free()
    s3.close()
    return p50, p99, kp


def roofline(kp, n_nodes, n_pods, fallback_s):
    """Dominant kernel (most device time in the profiled run): algorithmic bytes per launch =
    (pod x node evaluations it completes per launch) x B_node / mean launch time."""
    dom = max(kp, key=lambda k: kp[k]["s"]) if kp else None
    avg_s = kp[dom]["s"] / kp[dom]["launches"] if dom else fallback_s
    units = n_pods * n_nodes / (kp[dom]["launches"] if dom else 1)
    achieved = units * B_NODE / avg_s / 1e9
    kname = KERNEL_NAMES.get(dom, dom)
    traffic = pmc_traffic(kname) if dom else None
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": None if traffic is None else round(traffic),
            "kernel": kname, "avg_launch_us": round(avg_s * 1e6, 3),
            "bytes_per_launch": round(units * B_NODE)}


def pmc_traffic(kernel_prefix):
    """HBM bytes per launch of `kernel_prefix` from the committed rocprofv3 PMC summary
    (profiles/*_pmc_summary.csv, tools/summarize_pmc.py: separate FETCH_SIZE and WRITE_SIZE
    passes, 2 x FETCH_SIZE + WRITE_SIZE per MI355X_MICROARCH.md:298).  None if not collected."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.csv")))
    if not files:
        return None
    for row in csv.DictReader(open(files[-1])):
        if row["kernel"].split("<")[0].endswith(kernel_prefix):
            return float(row["hbm_bytes_per_launch"])
    return None


def cpu_baseline(nodes, pods, n_nodes, n_pods, sample, threads=1, gpu_placement=None):
    """Oracle (C restatement) on the same stream: 1 thread, or the node-parallel OpenMP arm
    (SURVEY §8(d) arm 2: upstream's Parallelizer runs 16 workers).  sample = 0 runs the whole
    stream, and its placements are diffed against the GPU's (`placements_match`)."""
    from oracle import oracle as O

    whole = sample <= 0 or sample >= n_pods
    sample = n_pods if whole else sample
    sub = qsched.pods_from_struct(pods[:sample])
    on = {k: v.copy() for k, v in nodes.items()}
    t0 = time.perf_counter()
    placement, _, _ = O.schedule(on, sub, nthreads=threads)
    dt = time.perf_counter() - t0
    how = "1 thread" if threads == 1 else f"{threads} OpenMP threads over the nodes of each pod"
    what = (f"the whole {n_pods:,}-pod stream" if whole else
            f"first {sample} of the {n_pods:,} pods (QoS-sorted within the sample)")
    out = {"value": round(sample / dt, 1), "unit": "pods/s", "cores": threads, "kind": "port",
           "sample": f"{what} onto the empty {n_nodes:,}-node cluster, oracle/qs_oracle.c {how}, "
                     f"{dt:.2f} s",
           "evals_per_s": round(sample * n_nodes / dt, 1)}
    if whole and gpu_placement is not None:
        out["placements_match"] = bool(np.array_equal(placement, gpu_placement))
    return out


def measure(cx, a, workload, steps, warmup, with_diag=True):
    """Timed exact stream of `workload`; returns a dict of measurements (rank-0 meaningful)."""
    gen, n_nodes, n_pods, desc = WORKLOADS[workload]
    sharded = workload == "config3" and cx.world > 1
    seed = 0x5EED0000 + gen + (cx.rank if (cx.world > 1 and not sharded) else 0)
    nodes, pods = qsched.synth_generate(gen, n_nodes, n_pods, seed=seed)
    cfg = dict({"engine": a.engine, "lookahead": a.lookahead}, **PROFILE.get(workload, {}))
    s = open_sched(cx, cfg, sharded)
    s.load_nodes(nodes)
    s.save_table()
    st = s.prepare(pods)

    mode = MODE.get(workload, "exact")

    def step():
        s.restore_table()
        return st.run(mode=mode)

    for _ in range(warmup):
        step()
    cx.barrier()
    t0 = time.perf_counter()
    last = None
    for _ in range(steps):
        last = step()
    cx.barrier()
    elapsed = cx.max(time.perf_counter() - t0)
    placement, _ = st.results()
    st.free()
    s.close()
    ranks_work = cx.world if (cx.world > 1 and not sharded) else 1  # replicas multiply the work
    value = n_pods * steps * ranks_work / elapsed
    out = {"value": value, "ms_per_step": elapsed / steps * 1e3, "engine": last["engine_used"],
           "unschedulable_frac": float((placement < 0).mean()), "n_nodes": n_nodes,
           "placement": placement.copy(),
           "n_pods": n_pods, "desc": desc, "sharded": sharded, "nodes": nodes, "pods": pods,
           "replicas": ranks_work}
    if with_diag:
        out["p50"], out["p99"], out["kp"] = diag_runs(cx, nodes, pods, cfg, sharded)
        out["wall_fallback"] = last["wall_s"]
    return out


def scan_roofline(cx, a, n_nodes=1 << 24, n_pods=32):
    """The scoring scan at an HBM-resident table (north_star's >= 50 % target):
    the SCAN engine's exact stream over 2^24 nodes (512 MiB of SoA columns, beyond the 256 MiB
    Infinity Cache), one full Filter+Score scan + argmax per pod, then Reserve.  Achieved =
    n_nodes x B_node / mean k_scan_soa launch time (HIP events on the library stream)."""
    nodes, pods = qsched.synth_generate(2, n_nodes, n_pods)
    cfg = {"engine": "scan"}
    s = qsched.Scheduler(cfg, device=cx.local)
    s.load_nodes(nodes)
    s.save_table()
    st = s.prepare(pods)
    st.run()  # warm-up
    walls = []
    for _ in range(3):
        s.restore_table()
        walls.append(st.run()["wall_s"])
    st.free()
    s.close()
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
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic("k_scan_soa"), "kernel": "k_scan_soa",
                         "avg_launch_us": round(avg * 1e6, 2),
                         "bytes_per_launch": n_nodes * B_NODE}}


def main():
    a = parse()
    cx = Ctx()
    workload = a.workload if a.workload != "auto" else ("config2" if cx.world == 1 else "config3")
    m = measure(cx, a, workload, a.steps, a.warmup)
    c3 = c4 = c5 = scan = None
    if cx.world == 1 and workload == "config2" and not a.no_config3:
        c3 = measure(cx, a, "config3", 1, 1, with_diag=False)
        c4 = measure(cx, a, "config4", 3, 1, with_diag=False)
        c5 = measure(cx, a, "config5", 3, 1, with_diag=False)
    if cx.world == 1 and not a.no_scan:
        scan = scan_roofline(cx, a)
    if cx.rank == 0:
        rl = roofline(m["kp"], m["n_nodes"], m["n_pods"], m["wall_fallback"])
        if m["sharded"]:
            par, scaling = f"node-sharded x{cx.world} (RCCL all-gather per window)", "strong"
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
            "config": {"workload": m["desc"], "engine": m["engine"],
                       "lookahead": a.lookahead or 32, "parallelism": par},
            "evals_per_s": round(m["value"] * m["n_nodes"], 1),
            "p50_pod_latency_us": round(m["p50"], 4), "p99_pod_latency_us": round(m["p99"], 4),
            "unschedulable_frac": round(m["unschedulable_frac"], 5),
            "roofline": rl,
            "kernels_us_per_step": {k: round(v["s"] * 1e6, 1) for k, v in m["kp"].items()},
        }
        if c3 is not None:
            out["config3"] = {"workload": c3["desc"] + " (1 GPU: the N=1 point of the curve)",
                              "value": round(c3["value"], 1), "unit": "pods/s",
                              "evals_per_s": round(c3["value"] * c3["n_nodes"], 1),
                              "ms_per_step": round(c3["ms_per_step"], 3), "steps": 1,
                              "engine": c3["engine"]}
        if c4 is not None:
            out["config4"] = {"workload": c4["desc"], "value": round(c4["value"], 1), "unit": "pods/s",
                              "evals_per_s": round(c4["value"] * c4["n_nodes"], 1),
                              "ms_per_step": round(c4["ms_per_step"], 3), "steps": 3,
                              "engine": c4["engine"],
                              "unschedulable_frac": round(c4["unschedulable_frac"], 5)}
        if c5 is not None:
            out["config5_batched"] = {"workload": c5["desc"], "value": round(c5["value"], 1),
                                      "unit": "pods/s", "evals_per_s": round(c5["value"] * c5["n_nodes"], 1),
                                      "ms_per_step": round(c5["ms_per_step"], 3), "steps": 3,
                                      "engine": c5["engine"],
                                      "unschedulable_frac": round(c5["unschedulable_frac"], 5)}
        if scan is not None:
            out["scan"] = scan
        if cx.world == 1 and not a.no_cpu:
            out["cpu_baseline"] = cpu_baseline(m["nodes"], m["pods"], m["n_nodes"], m["n_pods"],
                                               a.cpu_sample, gpu_placement=m["placement"])
            out["cpu_baseline_parallel"] = cpu_baseline(m["nodes"], m["pods"], m["n_nodes"], m["n_pods"],
                                                        a.cpu_sample, threads=16,
                                                        gpu_placement=m["placement"])
        print(json.dumps(out), flush=True)
    if cx.dist is not None:
        cx.dist.destroy_process_group()


if __name__ == "__main__":
    main()
