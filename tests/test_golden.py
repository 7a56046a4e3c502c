"""Golden fixtures (tests/golden/*.npz, written by tests/golden/make_golden.py from both oracle
restatements): the generator reproduces the recorded inputs bit-for-bit (C oracle, numpy oracle and
the product's qs_synth_generate), the C oracle reproduces the recorded outputs, and — on the GPU —
every engine of libqsched.so reproduces them through the C ABI."""
import json
import os

import numpy as np
import pytest

import qsched
from oracle import oracle as O

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INDEX = json.load(open(os.path.join(HERE, "index.json")))


def _digest(nodes, pods, full=False):
    import hashlib
    h = hashlib.sha256()
    for d in (nodes, pods):
        for k in sorted(d):
            if not full and k in ("zone", "app", "anti_affinity"):  # ABI-v2 columns (input_sha256_full)
                continue
            h.update(k.encode())
            h.update(np.ascontiguousarray(d[k]).tobytes())
    return h.hexdigest()


def _batched(meta):
    return meta["profile"].get("mode") == "batched"


def _profile(meta):
    return {k: v for k, v in meta["profile"].items() if k not in ("mode", "batch")}


def _load(meta):
    return dict(np.load(os.path.join(HERE, meta["name"] + ".npz"), allow_pickle=False))


@pytest.mark.parametrize("meta", INDEX, ids=[m["name"] for m in INDEX])
def test_inputs_reproduce(meta):
    c, n, p = meta["config"], meta["nodes"], meta["pods"]
    assert _digest(*O.generate(c, n, p)) == meta["input_sha256"]
    assert _digest(*O.py_generate(c, n, p)) == meta["input_sha256"]
    nodes, pods = qsched.synth_generate(c, n, p)
    assert _digest(nodes, qsched.pods_from_struct(pods)) == meta["input_sha256"]
    # every column, the zone / app / anti-affinity ones included
    assert _digest(*O.generate(c, n, p), full=True) == meta["input_sha256_full"]
    assert _digest(nodes, qsched.pods_from_struct(pods), full=True) == meta["input_sha256_full"]


@pytest.mark.parametrize("meta", INDEX, ids=[m["name"] for m in INDEX])
def test_oracle_reproduces_outputs(meta):
    g = _load(meta)
    nodes, pods = O.generate(meta["config"], meta["nodes"], meta["pods"])
    cfg = dict(O.DEFAULT_CONFIG, **_profile(meta))
    if _batched(meta):
        pl, best, nb = O.schedule_batched(nodes, pods, batch=meta["profile"]["batch"], cfg=cfg)
        assert nb == meta["batches"]
        order = g["order"]
    else:
        pl, best, order = O.schedule(nodes, pods, cfg)
    assert np.array_equal(pl, g["placement"])
    assert np.array_equal(best, g["best_key"])
    assert np.array_equal(order, g["order"])
    for k in ["req_cpu", "req_mem", "req_ext", "nz_cpu", "nz_mem", "pods"]:
        assert np.array_equal(nodes[k], g["final_" + k]), k


def _engines(meta):
    if _batched(meta):
        return ["batched"]
    return ["persistent", "scan", "lookahead", "auto"]


@pytest.mark.gpu
@pytest.mark.parametrize("meta", INDEX, ids=[m["name"] for m in INDEX])
def test_gpu_reproduces_golden(meta):
    g = _load(meta)
    nodes, pods = qsched.synth_generate(meta["config"], meta["nodes"], meta["pods"])
    for eng in _engines(meta):
        if eng == "batched":
            prof, mode = dict(_profile(meta), batch_pods=meta["profile"]["batch"]), "batched"
        else:
            prof, mode = dict(_profile(meta), engine=eng), "exact"
        with qsched.Scheduler(prof) as s:
            s.load_nodes(nodes)
            st = s.prepare(pods)
            stats = st.run(mode=mode)
            if eng == "batched":
                assert stats["batches"] == meta["batches"]
            pl, keys = st.results()
            st.free()
            fin = s.read_nodes()
        assert np.array_equal(pl, g["placement"]), eng
        assert np.array_equal(keys, g["best_key"]), eng
        for k in ["req_cpu", "req_mem", "req_ext", "nz_cpu", "nz_mem", "pods"]:
            assert np.array_equal(fin[k], g["final_" + k]), (eng, k)
