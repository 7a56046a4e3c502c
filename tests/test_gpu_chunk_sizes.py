"""Resident streams at table sizes whose selector chunks are 7 x 512 nodes (round 6: E = 7 is
instantiated beside 3 / 5 / 8 / 16).  The chunk plan (csrc/qs_kernels.hip,
la_stream_res_plan) picks E = 7 for Fit + Balanced tables of ~37k-44k nodes (two selector
workgroups per CU, G <= 15 chunks) and for normalizing tables of ~18k-21k nodes (G <= 7): every
layout / profile class that instantiates k_la_stream_res<F, 7, ...> runs here once, against the
oracle on placements, per-pod keys and the final table.
"""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rescfg import GPU_CFG  # noqa: E402
from test_gpu_parity import CFG4, assert_same, run_gpu, run_oracle  # noqa: E402
from test_gpu_wide import ki_cluster  # noqa: E402

from qsched import synth_generate  # noqa: E402


def _check(oracle, nodes, pods, cfg):
    g = run_gpu(nodes, pods, cfg, "lookahead")
    o = run_oracle(oracle, nodes, pods, cfg)
    assert_same(g[:2], o[:2], g[2], o[2])
    assert g[3]["engine_used"] == "lookahead" and g[3]["resident"] == 1


def test_fit_balanced_e7(oracle):
    nodes, pods = synth_generate(2, 40000, 12000)
    _check(oracle, nodes, pods, {})


def test_wide_layout_e7(oracle):
    nodes, pods = ki_cluster(40000, 12000)
    _check(oracle, nodes, pods, {})


@pytest.mark.parametrize("gpu_scoring", [False, True], ids=["norm", "norm-gpu-scoring"])
def test_normalizing_e7(oracle, gpu_scoring):
    cfg = dict(CFG4, **GPU_CFG) if gpu_scoring else dict(CFG4)
    nodes, pods = synth_generate(4, 20000, 12000)
    _check(oracle, nodes, pods, cfg)
