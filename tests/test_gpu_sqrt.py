"""Device f64 arithmetic of configurable BalancedAllocation lists (spec/semantics.md S10
"Configurable scoring resources", VERDICT r4 next #1: "first prove that device sqrt(double) is
correctly rounded").  Runs tests/native/sqrt_sweep (built by `make -C custom-k8s-scheduler_amd`):
qs::sqrt_rn against the host's correctly rounded sqrt bit for bit on 32 M inputs, and the kernels'
ba_score<kFeatExt | kFeatRes> against the oracle's or_balanced_v on 2 M random (node, pod, list)
cases."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "sqrt_sweep")


def test_device_sqrt_and_balanced_lists():
    if not os.path.exists(EXE):
        raise FileNotFoundError(f"{EXE} missing: build with make -C custom-k8s-scheduler_amd")
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    m1 = re.search(r"sqrt mismatches (\d+) of (\d+)", r.stdout)
    m2 = re.search(r"balanced mismatches (\d+) of (\d+) \((\d+) with three", r.stdout)
    assert m1 and m2, r.stdout + r.stderr
    assert int(m1.group(1)) == 0 and int(m1.group(2)) >= 32 << 20
    assert int(m2.group(1)) == 0 and int(m2.group(2)) >= 2 << 20
    assert int(m2.group(3)) > 100000  # the >= 3-resource (sqrt) path is well covered
    assert r.returncode == 0
