"""Per-kernel device time (config.profile_kernels) for a workload; QS_DIAG=1 adds the resolver's
per-wave busy cycles.  usage: CFG=2 N=5000 P=100000 K=32 VS=1 ENGINE=lookahead TA=0 python tools/kprof.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "custom-k8s-scheduler_amd"))
import qsched

cfgno, n, p = int(os.environ.get("CFG", 2)), int(os.environ.get("N", 5000)), int(os.environ.get("P", 100000))
K, vs = int(os.environ.get("K", 0)), int(os.environ.get("VS", 1))
eng, ta = os.environ.get("ENGINE", "lookahead"), int(os.environ.get("TA", 0))
mode = os.environ.get("MODE", "exact")
nodes, pods = qsched.synth_generate(cfgno, n, p)
for prof in (0, 1):
    s = qsched.Scheduler({"engine": eng if mode == "exact" else "auto", "lookahead": K, "profile_kernels": prof, "virtual_shards": vs,
                          "enable_taint": ta, "enable_affinity": ta})
    s.load_nodes(nodes); s.save_table()
    st = s.prepare(pods)
    for r in range(3 if p <= 200000 else 1):
        s.restore_table()
        stats = st.run(mode=mode)
    ks = {k: (v["s"] * 1e3, v["launches"], v["s"] / max(1, v["launches"]) * 1e6) for k, v in stats["kernels"].items()}
    print(f"cfg{cfgno} {eng} ta={ta} n={n} p={p} K={K} vs={vs} profile={prof}: wall {stats['wall_s']*1e3:.2f} ms "
          f"({p / stats['wall_s']:.0f} pods/s, rescans {stats['truncations']})  "
          + "  ".join(f"{k}: {a:.2f} ms / {b} = {c:.2f} us" for k, (a, b, c) in ks.items()), flush=True)
    st.free(); s.close()
