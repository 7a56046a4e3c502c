"""Sweep lookahead window sizes / engines on config 2; prints device ms per 100k-pod stream."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "custom-k8s-scheduler_amd"))
import numpy as np
import qsched

n, p = int(os.environ.get("N", 5000)), int(os.environ.get("P", 100000))
cfgno = int(os.environ.get("CFG", 2))
nodes, pods = qsched.synth_generate(cfgno, n, p)
ref = None
for eng, K in [(e.split(":")[0], int(e.split(":")[1])) for e in os.environ.get("RUNS", "lookahead:64").split(",")]:
    prof = {"enable_taint": 1, "enable_affinity": 1} if cfgno == 4 else {}
    s = qsched.Scheduler(dict({"engine": eng, "lookahead": K}, **prof))
    s.load_nodes(nodes); s.save_table()
    st = s.prepare(pods)
    walls = []
    for r in range(4):
        s.restore_table()
        stats = st.run()
        walls.append(stats["wall_s"])
    pl, _ = st.results()
    if ref is None: ref = pl
    print(f"{eng:10s} K={K:3d} ms/stream={1e3*min(walls[1:]):8.2f}  pods/s={p/min(walls[1:]):12.0f} same={np.array_equal(pl, ref)} resident={stats['resident']} rescans={stats['truncations']} stopped_windows={stats['resumed_windows']}", flush=True)
    st.free(); s.close()
