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
