"""Mean k_scan_soa launch time and HBM rate on the 2^24-node SoA table (bench.py scan_roofline's
kernel, a few pods; HIP events).  QSCHED_LIB picks a variant library.  Usage: python tools/scan_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "custom-k8s-scheduler_amd"))
import qsched  # noqa: E402

n, p = 1 << 24, int(os.environ.get("P", 16))
nodes, pods = qsched.synth_generate(2, n, p)
s = qsched.Scheduler({"engine": "scan", "profile_kernels": 1})
s.load_nodes(nodes)
st = s.prepare(pods)
st.run()
for r in range(int(os.environ.get("RUNS", 3))):
    k = st.run()["kernels"]["scan"]
    avg = k["s"] / k["launches"]
    print(f"{os.path.basename(os.environ.get('QSCHED_LIB', 'libqsched.so'))}: k_scan_soa {avg * 1e6:.2f} us "
          f"-> {n * 32 / avg / 1e9:.1f} GB/s ({n * 32 / avg / 8e12:.3f} of 8 TB/s)", flush=True)
st.free()
s.close()
