"""Run only the bench's HBM-resident scan leg (for profiling passes)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
n = int(os.environ.get("N", 1 << 24))
print(json.dumps(bench.scan_roofline(bench.Ctx(), None, n_nodes=n)))
