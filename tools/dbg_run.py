"""Debug helper: run a small lookahead stream, report the first placement that differs from the
oracle in processing order (stderr of the kernel's QS_RUN_DEBUG printf goes to the log)."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/custom-k8s-scheduler_amd")
import numpy as np, qsched
from oracle import oracle as O
cfg, n, p = (int(x) for x in sys.argv[1:4])
nodes, pods = qsched.synth_generate(cfg, n, p)
with qsched.Scheduler({"engine": "lookahead"}) as s:
    s.load_nodes(nodes); st = s.prepare(pods); st.run(); pl, keys = st.results(); st.free()
on = {k: v.copy() for k, v in nodes.items()}
opl, okeys, order = O.schedule(on, qsched.pods_from_struct(pods), None)
bad = [k for k, j in enumerate(order) if pl[j] != opl[j]]
print("MISMATCH", len(bad), "first processing position", bad[:1],
      [(int(order[k]), int(pl[order[k]]), int(opl[order[k]]), hex(int(keys[order[k]])), hex(int(okeys[order[k]]))) for k in bad[:3]], flush=True)
