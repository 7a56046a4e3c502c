"""The C++ framework layer (custom-k8s-scheduler_amd/host: the kube-scheduler framework surface
mirrored over the C ABI) through its native table-driven tests, tests/native/test_framework.cpp.
The binary is built in-tree by `make -C custom-k8s-scheduler_amd` (__graft_entry__.build)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "native", "test_framework")


def run(mode, timeout):
    assert os.path.exists(BIN), f"{BIN} missing: run `make -C custom-k8s-scheduler_amd`"
    r = subprocess.run([BIN, mode], capture_output=True, text=True, timeout=timeout)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


def test_framework_host_logic():
    """Quantities, taint/requirement interning, pod requests, QoSSort, FitError text (no GPU)."""
    run("--cpu", 60)


@pytest.mark.gpu
def test_framework_plugins_on_device():
    """QoSGPU filter/score tables and the ScheduleOne loop vs qs_schedule_stream and the oracle."""
    run("--gpu", 110)


def test_framework_host_logic_sanitized():
    """The same host checks built with -fsanitize=address,undefined (SURVEY §5 host sanitizers):
    quantity parsing, interning, pod requests, QoSSort and FitError text run clean."""
    root = os.path.join(os.path.dirname(HERE), "custom-k8s-scheduler_amd")
    b = subprocess.run(["make", "-C", root, "asan"], capture_output=True, text=True, timeout=1500)  # (a cold ASan build of the host library takes minutes)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    exe = os.path.join(root, "build", "test_framework_asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, "--cpu"], capture_output=True, text=True, timeout=900, env=env)  # (≈ 4.5 min under ASan)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "0 failures" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
