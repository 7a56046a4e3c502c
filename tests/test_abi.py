"""C-ABI boundary checks that need no GPU: libqsched.so loads, exports every symbol declared in
include/qsched.h, struct layouts agree with the binding, host helpers (spec S2/S3) behave like
upstream, and calls fail with status codes (never crashes) when no device exists."""
import ctypes
import os
import re

import numpy as np
import pytest

import qsched
from qsched import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "qsched.h")
MIB = 1 << 20


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(qs_[a-z_0-9]+)\s*\(", text)))


def test_every_declared_symbol_is_exported():
    lib = qsched.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/qsched.h but not exported"
    assert set(syms) == set(_abi.EXPORTED), "binding signature table out of sync with the header"


def test_struct_sizes():
    lib = qsched.load()
    assert lib.qs_struct_size(3) == 248  # qs_pod (ABI v2: app, anti_affinity)
    assert lib.qs_struct_size(99) == 0


def test_no_symbols_leak_torch():
    # the boundary is plain C: no torch/c10 symbols in the library's dynamic table
    names = [ln.split()[-1] for ln in os.popen(f"nm -D --defined-only {_abi.LIB_PATH}").read().splitlines()
             if ln.strip()]
    assert not any("c10" in n or "torch" in n for n in names)
    assert "qs_schedule_stream" in names
    # only the C ABI is exported (the library builds with -fvisibility=hidden)
    text_syms = [n for n in names if not n.startswith("_")]
    assert all(n.startswith("qs_") for n in text_syms), text_syms


def test_every_registered_kernel_has_device_code():
    """Each kernel the host side registers (by mangled name) has a kernel descriptor (<name>.kd)
    in the embedded gfx950 code object.  Guards against host/device name drift, e.g. a kernel
    signature that mangles an unnamed type ($_N is numbered per compilation pass)."""
    import subprocess
    strs = set(subprocess.run(["strings", "-n", "8", _abi.LIB_PATH], capture_output=True,
                              text=True).stdout.split())
    kernels = {s for s in strs if re.fullmatch(r"_ZN2qs\d+k_\w+", s.replace("$", "_"))}
    assert len(kernels) > 100
    assert not any("$_" in k for k in kernels)
    missing = [k for k in kernels if k + ".kd" not in strs]
    assert not missing, missing[:3]


def test_config_default():
    lib = qsched.load()
    c = _abi.QsConfig()
    lib.qs_config_default(ctypes.byref(c))
    assert c.abi_version == 3 and list(c.w_fit) == [1, 2, 3] and list(c.w_bal) == [1, 1, 1]
    assert c.w_taint == 3 and c.w_affinity == 2 and c.qos_sort == 1
    assert c.fit_weight_cpu == 1 and c.fit_weight_mem == 1


def test_open_without_device_returns_status():
    lib = qsched.load()
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    c = _abi.QsConfig()
    lib.qs_config_default(ctypes.byref(c))
    ctx = ctypes.c_void_p()
    st = lib.qs_open(ctypes.byref(c), 0, ctypes.byref(ctx))
    assert st in (_abi.QS_EDEVICE, _abi.QS_EINVAL)
    assert not ctx.value
    bad = _abi.QsConfig()
    lib.qs_config_default(ctypes.byref(bad))
    bad.abi_version = 7
    assert lib.qs_open(ctypes.byref(bad), 0, ctypes.byref(ctx)) == _abi.QS_EINVAL
    assert lib.qs_close(None) == _abi.QS_EINVAL
    # no context: qs_last_error(NULL) says why this thread's last qs_open failed
    assert b"abi_version" in lib.qs_last_error(None) or b"version" in lib.qs_last_error(None)


# ---- spec S2 / S3 (UP component-helpers/resource#PodRequests, qos.go#ComputePodQOS) ----------
def test_pod_requests_and_qos_guaranteed():
    p = qsched.pod_from_containers([dict(req_cpu=500, req_mem=256 * MIB, lim_cpu=500, lim_mem=256 * MIB)])
    assert (p["req_cpu"], p["req_mem"], p["nz_cpu"], p["nz_mem"], p["qos"]) == (500, 256 * MIB, 500, 256 * MIB, 2)


def test_pod_requests_defaults_only_for_missing():
    p = qsched.pod_from_containers([dict(req_cpu=0)])  # explicit 0 cpu, memory missing
    assert (p["req_cpu"], p["nz_cpu"], p["req_mem"], p["nz_mem"]) == (0, 0, 0, 200 * MIB)
    assert p["qos"] == 0  # zero quantities are ignored by ComputePodQOS
    p = qsched.pod_from_containers([{}])
    assert (p["nz_cpu"], p["nz_mem"], p["qos"]) == (100, 200 * MIB, 0)


def test_pod_requests_init_and_sidecars():
    # regular 100m; init 500m; sidecar 200m started before a second init of 400m:
    # sum = 100 + 200 = 300; init needs: 500 (first), 400 + 200 = 600 -> max(300, 600) = 600
    cs = [dict(kind="regular", req_cpu=100), dict(kind="init", req_cpu=500),
          dict(kind="sidecar", req_cpu=200), dict(kind="init", req_cpu=400)]
    p = qsched.pod_from_containers(cs)
    assert p["req_cpu"] == 600
    p = qsched.pod_from_containers(cs, overhead=(50, 10 * MIB))
    assert p["req_cpu"] == 650 and p["req_mem"] == 10 * MIB


@pytest.mark.parametrize("containers,qos", [
    ([{}], 0),
    ([dict(req_cpu=100)], 1),
    ([dict(lim_cpu=100, lim_mem=MIB)], 1),  # raw spec: len(requests) != len(limits) -> Burstable
    ([dict(req_cpu=100, req_mem=MIB, lim_cpu=100, lim_mem=MIB)], 2),  # post API defaulting
    ([dict(req_cpu=100, lim_cpu=100, lim_mem=MIB)], 1),
    ([dict(req_cpu=100, req_mem=MIB, lim_cpu=100, lim_mem=MIB), dict(req_cpu=1)], 1),
    ([dict(req_cpu=100, req_mem=MIB, lim_cpu=100, lim_mem=MIB),
      dict(req_cpu=5, req_mem=5, lim_cpu=5, lim_mem=5)], 2),
    ([dict(req_cpu=100, req_mem=MIB, lim_cpu=200, lim_mem=MIB)], 1),
])
def test_compute_qos(containers, qos):
    assert qsched.compute_qos(containers) == qos


def test_synth_generate_matches_spec_mix():
    nodes, pods = qsched.synth_generate(2, 5000, 100000)
    q = np.bincount(pods["qos"], minlength=3) / len(pods)
    assert abs(q[2] - 0.2) < 0.01 and abs(q[1] - 0.5) < 0.01 and abs(q[0] - 0.3) < 0.01
    assert set(np.unique(nodes["alloc_cpu"])) <= {4000, 8000, 16000, 32000, 64000, 96000}
    assert (nodes["alloc_mem"] % (1 << 30) == 0).all()
    assert (pods["req_mem"] % MIB == 0).all() and (pods["nz_mem"] % MIB == 0).all()
