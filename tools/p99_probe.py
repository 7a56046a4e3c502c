"""Per-pod decision intervals of the resident stream, split by position in the lookahead window.

The p99 pod latency of BASELINE.json:2 is the 99th percentile of the interval between consecutive
decisions (in-kernel s_memrealtime stamps, 100 MHz).  A window of K pods has one boundary interval
(window w's last pod -> window w+1's first), so with K = 32 about 3.1 % of the intervals are
boundary ones: if they are the slow class, the p99 is a boundary percentile.  This prints the
percentiles per class (interval ending at window position k = 0 / 1 / 2..K-2 / K-1) and whether
the pod was won by a dirty slot (node already chosen earlier in the window) or a clean list entry.
Writes the raw intervals to gpurun_out/p99_intervals.npz.
Usage (GPU box): python tools/p99_probe.py   (env CFG=2|4, N, P, K, RUNS)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "custom-k8s-scheduler_amd"))
import numpy as np  # noqa: E402

import qsched  # noqa: E402

cfgno = int(os.environ.get("CFG", 2))
n = int(os.environ.get("N", 5000))
p = int(os.environ.get("P", 100000 if cfgno == 2 else 150000))
K = int(os.environ.get("K", 32))
runs = int(os.environ.get("RUNS", 3))
nodes, pods = qsched.synth_generate(cfgno, n, p)
prof = {"enable_taint": 1, "enable_affinity": 1} if cfgno == 4 else {}
s = qsched.Scheduler(dict({"engine": "lookahead", "lookahead": K, "record_timestamps": 1}, **prof))
s.load_nodes(nodes)
s.save_table()
st = s.prepare(pods)
allp = []
for r in range(runs):
    s.restore_table()
    stats = st.run()
    stamps = st.stamps().astype(np.int64)
    pl, keys = st.results()
    d = np.diff(stamps) * 0.01  # us; d[j] = interval ending at stream position j + 1
    pos = (np.arange(1, len(stamps)) % K)
    allp.append(d)
    print(f"run {r}: wall {stats['wall_s'] * 1e3:.2f} ms resident={stats['resident']} "
          f"p50 {np.percentile(d, 50):.3f} p99 {np.percentile(d, 99):.3f} max {d.max():.2f} us", flush=True)
    for name, m in [("k=0 (boundary)", pos == 0), ("k=1", pos == 1), ("k=2..K-2", (pos >= 2) & (pos <= K - 2)),
                    ("k=K-1", pos == K - 1)]:
        x = d[m]
        if len(x) == 0:
            continue
        print(f"  {name:16s} n={len(x):6d} mean {x.mean():.3f} p50 {np.percentile(x, 50):.3f} "
              f"p90 {np.percentile(x, 90):.3f} p99 {np.percentile(x, 99):.3f} max {x.max():.2f}", flush=True)
    nb = d[pos != 0]
    print(f"  without boundary intervals: p99 {np.percentile(nb, 99):.3f}; fraction of intervals > 1 us "
          f"that are boundary: {np.mean(pos[d > 1.0] == 0) if (d > 1.0).any() else 0:.3f}", flush=True)
    by_k = np.array([np.median(d[pos == k]) for k in range(K)])
    print("  median by k:", " ".join(f"{v:.2f}" for v in by_k), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"p99_intervals_cfg{cfgno}.npz"), d=np.stack(allp), K=K)
st.free()
s.close()
