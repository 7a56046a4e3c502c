"""GPU parity on scheduler_perf-style workload files: the loaded cluster and
pod stream (taints, tolerations, node selectors, required/preferred node affinity, amd.com/gpu,
three QoS classes, priorities) scheduled by every engine, bit-exact against the oracle."""
import os

import pytest

pytestmark = pytest.mark.gpu

from qsched import workload as W  # noqa: E402

from test_gpu_parity import assert_same, run_gpu, run_oracle  # noqa: E402

QOS_MIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "workloads", "qos_mix.yaml")


@pytest.mark.parametrize("engine", ["persistent", "scan", "lookahead"])
def test_workload_small(oracle, engine):
    nodes, pods, prof = W.load(QOS_MIX, "small")
    g = run_gpu(nodes, pods, prof, engine)
    o = run_oracle(oracle, nodes, pods, prof)
    assert_same(g[:2], o[:2], g[2], o[2])


@pytest.mark.parametrize("K", [8, 32])
def test_workload_500_nodes(oracle, K):
    nodes, pods, prof = W.load(QOS_MIX, "500Nodes")
    g = run_gpu(nodes, pods, prof, "lookahead", lookahead=K)
    o = run_oracle(oracle, nodes, pods, prof)
    assert_same(g[:2], o[:2], g[2], o[2])
    assert g[3]["engine_used"] == "lookahead"
