"""Scoring-resource configurations for the parity tests (spec S5 "Scoring resources";
NodeResourcesFitArgs.ScoringStrategy.Resources / NodeResourcesBalancedAllocationArgs.Resources).

``GPU_CFG`` is the AMD-GPU cluster configuration of VERDICT r4 (LeastAllocated {cpu:1, memory:1,
amd.com/gpu:5}, Balanced over [cpu, memory, amd.com/gpu]); ``random_resource_cfg`` draws lists of
1-4 distinct resources in random order with weights 1..100 (upstream's validation range).
"""
import numpy as np

RESOURCES = ["cpu", "memory", "ext0", "ext1"]
GPU_CFG = dict(fit_resources=[("cpu", 1), ("memory", 1), ("ext0", 5)],
               balanced_resources=["cpu", "memory", "ext0"])
# named configurations the GPU parity tests run (ids for parametrize)
NAMED = {
    "gpu5": GPU_CFG,
    "ext-only-fit": dict(fit_resources=[("ext0", 3)], balanced_resources=["ext0", "cpu"]),
    "four-res": dict(fit_resources=[("ext1", 2), ("memory", 7), ("cpu", 1), ("ext0", 100)],
                     balanced_resources=["ext1", "ext0", "memory", "cpu"]),
    "cpu-only": dict(fit_resources=[("cpu", 4)], balanced_resources=["cpu"]),
    "mem-cpu-swapped": dict(fit_resources=[("memory", 3), ("cpu", 2)], balanced_resources=["memory", "cpu"]),
}


def random_resource_cfg(rng):
    k = int(rng.integers(1, 5))
    fit = [(RESOURCES[i], int(rng.integers(1, 101))) for i in rng.permutation(4)[:k]]
    kb = int(rng.integers(1, 5))
    bal = [RESOURCES[i] for i in rng.permutation(4)[:kb]]
    return dict(fit_resources=fit, balanced_resources=bal)


def add_ext1(rng, nodes, pods, frac=0.3):
    """A second extended resource column (ext1) on some nodes and pods."""
    n, p = len(nodes["alloc_cpu"]), len(pods["req_cpu"])
    nodes["alloc_ext"][:, 1] = np.where(rng.random(n) < frac, rng.choice([1, 2, 4, 16, 100], n), 0)
    pods["req_ext"][:, 1] = np.where(rng.random(p) < frac, rng.choice([1, 2, 3], p), 0)
