"""Schedule a scheduler_perf-style workload file on the GPU and print one JSON line of stats
(pods scheduled/s over the device-resident stream, unschedulable count, engine).
usage: python tools/run_workload.py tests/golden/workloads/qos_mix.yaml [workload] [--check]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "custom-k8s-scheduler_amd"))
import numpy as np  # noqa: E402

import qsched  # noqa: E402
from qsched import workload as W  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path, wl = args[0], (args[1] if len(args) > 1 else None)
    nodes, pods, prof = W.load(path, wl)
    with qsched.Scheduler(dict(prof)) as s:
        s.load_nodes(nodes)
        s.save_table()
        st = s.prepare(pods)
        st.run()  # warm-up (graph capture)
        s.restore_table()
        stats = st.run()
        pl, keys = st.results()
        st.free()
    out = {"workload": f"{os.path.basename(path)}:{wl or 'default'}", "nodes": len(nodes["alloc_cpu"]),
           "pods": len(pods), "pods_per_s": round(len(pods) / stats["wall_s"], 1),
           "unschedulable": int((pl < 0).sum()), "engine": stats["engine_used"], **prof}
    if "--check" in sys.argv:  # bit-exact against the oracle (test infrastructure)
        from oracle import oracle as O
        on = {k: v.copy() for k, v in nodes.items()}
        po, ko, _ = O.schedule(on, qsched.pods_from_struct(pods), dict(prof), nthreads=16)
        out["parity"] = bool(np.array_equal(po, pl) and np.array_equal(ko, keys))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
