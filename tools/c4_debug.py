"""Config-4 resident-stream debug: resident vs per-window keys in stream order, first mismatch."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "custom-k8s-scheduler_amd")]
import numpy as np
import qsched

def run(nodes, pods, cfg, resident):
    os.environ["QS_RESIDENT"] = "1" if resident else "0"
    with qsched.Scheduler(cfg) as s:
        s.load_nodes(nodes)
        st = s.prepare(pods)
        stats = st.run()
        pl, keys = st.results()
        st.free()
    return pl, keys, stats

CASES = [(400, 512, 32, "both"), (2000, 2000, 32, "both"), (400, 512, 32, "taint"),
         (400, 512, 32, "aff"), (400, 512, 1, "both"), (400, 512, 32, "fit")]
if os.environ.get("CASES"):
    CASES = [(int(a), int(b), int(c), d) for a, b, c, d in (x.split(":") for x in os.environ["CASES"].split(","))]
for n, p, K, prof in CASES:
    nodes, pods = qsched.synth_generate(4, n, p)
    cfg = {"engine": "lookahead", "lookahead": K}
    if prof in ("both", "taint"): cfg["enable_taint"] = 1
    if prof in ("both", "aff"): cfg["enable_affinity"] = 1
    g = run(nodes, pods, cfg, True)
    w = run(nodes, pods, cfg, False)
    order = np.lexsort((np.arange(p), -pods["priority"], -pods["qos"]))
    gk, wk = g[1][order], w[1][order]
    bad = np.nonzero(gk != wk)[0]
    print(f"n={n} p={p} K={K} {prof}: resident={g[2]['resident']} rescans={g[2]['truncations']}/{w[2]['truncations']} "
          f"stopped={g[2]['resumed_windows']}/{w[2]['resumed_windows']} mismatches={bad.size}", flush=True)
    if bad.size:
        s = int(bad[0])
        print(f"   first stream pos {s} (window {s // K}, pod {s % K}): res key {int(gk[s]):#x} node {int(g[0][order][s])} "
              f"| win key {int(wk[s]):#x} node {int(w[0][order][s])}", flush=True)
        for t in bad[1:6]:
            print(f"   next {int(t)}: {int(gk[t]):#x} vs {int(wk[t]):#x}")
