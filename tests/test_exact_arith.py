"""spec S10 exactness of the device arithmetic, checked on the host.

tests/native/exact_arith.c restates the two division formulas the gfx950 kernels use
(custom-k8s-scheduler_amd/csrc/qs_device.hpp floor_div / fraction) with the same IEEE operations
(fma, -ffp-contract=off) and compares them with true integer and IEEE division: exhaustively over
every allocatable value of spec/synth.md, exhaustively for small divisors, and on 20M random pairs
over the whole compacted range [1, 2^24); and the scan kernel's reciprocal RN(1/a) (f32 estimate +
two f64 Newton steps) exhaustively over [1, 2^24) for every estimate within 2 f32 ulps.  Mode 4: the
wide layout's LeastAllocated (f64 quotient + one fma-exact integer correction) and Markstein
BalancedAllocation quotient on 12M pairs over every binade up to 2^46 bytes (all-ones significands,
requests near the allocatable and near multiples of a / 100).  Mode 5: BalancedAllocation's division
by the resource count (3 or 4) on 80M cases (scaling by 1/4; Markstein's correction with RN(1/3)).
The GPU parity tests then confirm the device agrees.
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("exact") / "exact_arith")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", out,
                    os.path.join(HERE, "native", "exact_arith.c"), "-lm"], check=True)
    return out


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4, 5])
def test_division_formulas_exact(exe, mode):
    r = subprocess.run([exe, str(mode)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout
