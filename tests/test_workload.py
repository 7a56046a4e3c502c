"""scheduler_perf-style workload files: quantities, interning and the records
the loader builds, checked on the host; the GPU schedules the same file in test_gpu_workload.py.

Expected masks are worked out by hand from UP core/v1/toleration.go#ToleratesTaint and the
node-selector operator semantics (host/intern.cpp restates the same rules for the C++ layer)."""
import os
from fractions import Fraction

import numpy as np
import pytest

from qsched import workload as W

HERE = os.path.dirname(os.path.abspath(__file__))
QOS_MIX = os.path.join(HERE, "golden", "workloads", "qos_mix.yaml")


@pytest.mark.parametrize("q,want", [("500m", Fraction(1, 2)), ("2", 2), ("1.5", Fraction(3, 2)),
                                    ("2Gi", 2 * 2**30), ("1e3", 1000), ("128Mi", 128 * 2**20),
                                    ("1k", 1000), (4, 4), ("0.25", Fraction(1, 4))])
def test_parse_quantity(q, want):
    assert W.parse_quantity(q) == want


def test_quantity_rounding():  # Quantity.MilliValue / Value round up (UP resource.Quantity)
    assert W.milli_value("0.1m") == 1
    assert W.milli_value("1.5") == 1500
    assert W.value("1.5Ki") == 1536
    assert W.value("0.5") == 1
    with pytest.raises(ValueError):
        W.parse_quantity("12x")


def test_tolerates():
    taint = {"key": "k", "value": "v", "effect": "NoSchedule"}
    assert W.tolerates({"key": "k", "operator": "Equal", "value": "v"}, taint)
    assert W.tolerates({"key": "k", "value": "v"}, taint)            # default operator Equal
    assert not W.tolerates({"key": "k", "value": "w"}, taint)
    assert W.tolerates({"operator": "Exists"}, taint)                 # empty key: every taint
    assert not W.tolerates({"key": "k", "operator": "Exists", "effect": "NoExecute"}, taint)
    assert not W.tolerates({"key": "k", "operator": "Bogus"}, taint)


@pytest.mark.parametrize("req,labels,want", [
    (("z", "In", ("a", "b")), {"z": "a"}, True), (("z", "In", ("a",)), {}, False),
    (("z", "In", ()), {"z": "a"}, False),                             # invalid: no values
    (("z", "NotIn", ("a",)), {}, True), (("z", "NotIn", ("a",)), {"z": "a"}, False),
    (("z", "Exists", ()), {"z": ""}, True), (("z", "DoesNotExist", ()), {"z": "x"}, False),
    (("n", "Gt", ("5",)), {"n": "7"}, True), (("n", "Lt", ("5",)), {"n": "7"}, False),
    (("n", "Gt", ("x",)), {"n": "7"}, False), (("n", "Gt", ("5",)), {"n": "seven"}, False),
])
def test_requirement_matches(req, labels, want):
    assert W.requirement_matches(req, labels) is want


def test_load_qos_mix_records():
    nodes, pods, prof = W.load(QOS_MIX, "small")
    assert prof == {"enable_taint": 1, "enable_affinity": 1}
    n, p = len(nodes["alloc_cpu"]), len(pods)
    assert (n, p) == (60 + 8 + 20, 400 + 150 + 30 + 300)
    # nodes: general (zone round-robin), gpu (tainted, amd.com/gpu in ext slot 0), maintenance
    assert nodes["alloc_cpu"][0] == 32000 and nodes["alloc_mem"][0] == 128 * 2**30
    assert nodes["max_pods"][0] == 110
    assert nodes["alloc_ext"][60].tolist() == [8, 0] and nodes["alloc_ext"][0].tolist() == [0, 0]
    assert nodes["taint_hard"][60] == 1 and nodes["taint_soft"][60] == 0        # taint bit 0
    assert nodes["taint_hard"][-1] == 0 and nodes["taint_soft"][-1] == 2        # taint bit 1
    # requirement bits in first-seen order: zone In{z1,z2}=0, disktype Exists=1, pool=gpu=2,
    # zone NotIn{z0}=3
    lb = nodes["label_bits"][:, 0]
    assert lb[0] == 0                      # general, z0
    assert lb[1] == 0b1001                 # general, z1
    assert lb[60] == 0b1111                # gpu, z1, ssd
    assert lb[61] == 0b1111                # gpu, z2, ssd
    assert lb[-1] == 0b1010                # maintenance: z3, ssd
    assert (nodes["label_bits"][:, 1] == 0).all()
    web, db, gpu, batch = pods[0], pods[400], pods[550], pods[580]
    assert (web["qos"], web["req_cpu"], web["req_mem"]) == (1, 500, 2**30)
    assert (db["qos"], db["priority"], db["n_pref_terms"]) == (2, 100, 2)
    assert db["pref_weight"].tolist() == [50, 20, 0, 0]
    assert db["pref_terms"][0].tolist() == [1, 0] and db["pref_terms"][1].tolist() == [2, 0]
    assert gpu["req_ext"].tolist() == [2, 0] and gpu["tol_hard"] == 1 and gpu["tol_soft"] == 0
    assert gpu["sel"].tolist() == [4, 0] and gpu["qos"] == 1
    assert (batch["qos"], batch["req_cpu"], batch["nz_cpu"], batch["nz_mem"]) == (0, 0, 100, 200 * 2**20)
    assert batch["tol_soft"] == 2 and batch["tol_hard"] == 0   # tolerates the maintenance taint only
    assert batch["n_req_terms"] == 1 and batch["req_terms"][0].tolist() == [8, 0]


def test_workload_params_and_counts():
    nodes, pods, _ = W.load(QOS_MIX, "500Nodes")
    assert len(nodes["alloc_cpu"]) == 440 + 40 + 20 and len(pods) == 6000 + 2500 + 200 + 3000
    with pytest.raises(KeyError):
        W.load(QOS_MIX, "nope")


def test_empty_term_and_limits():
    text = """
- name: T
  workloadTemplate:
  - {opcode: createNodes, count: 2, nodeTemplate: {status: {allocatable: {cpu: "4", memory: 8Gi}}}}
  - opcode: createPods
    count: 1
    podTemplate:
      spec:
        affinity: {nodeAffinity: {requiredDuringSchedulingIgnoredDuringExecution: {nodeSelectorTerms: [{}]}}}
        containers: [{name: c}]
"""
    nodes, pods, prof = W.load(text)
    assert pods[0]["n_req_terms"] == 1
    assert pods[0]["req_terms"][0].tolist() == [0, 1 << 63]   # the reserved never-bit 127
    assert (nodes["label_bits"] == 0).all() and prof["enable_affinity"] == 1


def test_oracle_schedules_loaded_workload(oracle):
    """The loaded records are valid oracle input; both oracles agree on them (S7/S8)."""
    import qsched
    nodes, pods, prof = W.load(QOS_MIX, "small")
    on = {k: v.copy() for k, v in nodes.items()}
    pl, keys, _ = oracle.schedule(on, qsched.pods_from_struct(pods), dict(prof), nthreads=4)
    assert (pl >= -1).all() and (pl < len(nodes["alloc_cpu"])).all()
    gpu_pods = np.arange(550, 580)
    assert ((pl[gpu_pods] >= 60) & (pl[gpu_pods] < 68)).all()   # only the tainted gpu pool fits
    batch = np.arange(580, 880)
    zones = np.array([["z0", "z1", "z2", "z3"][i % 4] for i in range(60)] + ["z1", "z2"] * 4 + ["z3"] * 20)
    placed = pl[batch][pl[batch] >= 0]
    assert (zones[placed] != "z0").all()                         # required NotIn z0
