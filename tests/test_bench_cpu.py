"""bench.py's CPU-baseline leg (SURVEY §8(d) CPU timing arm), host only: the 1-thread and the
node-parallel OpenMP arms of the C oracle place the same stream identically, and the leg's
`placements_match` flag compares against the placement it is handed."""
import numpy as np

import bench
import qsched


def test_cpu_arms_agree_and_flag_mismatch():
    nodes, pods = qsched.synth_generate(2, 300, 4000, seed=0x5EED0002)
    from oracle import oracle as O

    ref, _, _ = O.schedule({k: v.copy() for k, v in nodes.items()}, qsched.pods_from_struct(pods))
    one = bench.cpu_baseline(nodes, pods, 300, 4000, 0, threads=1, gpu_placement=ref)
    par = bench.cpu_baseline(nodes, pods, 300, 4000, 0, threads=4, gpu_placement=ref)
    assert one["placements_match"] and par["placements_match"]
    assert one["cores"] == 1 and par["cores"] == 4 and one["kind"] == "port"
    bad = ref.copy()
    bad[np.flatnonzero(bad >= 0)[0]] += 1
    assert not bench.cpu_baseline(nodes, pods, 300, 4000, 0, gpu_placement=bad)["placements_match"]
    # a bounded sample is timed but not diffed
    assert "placements_match" not in bench.cpu_baseline(nodes, pods, 300, 4000, 1000, gpu_placement=ref)


def test_roofline_of_the_resident_stream():
    """A resident stream is one launch of k_la_stream_res: the roofline prices the whole stream's
    algorithmic bytes (pods x nodes x 32 B) against that launch's duration, and reads its HBM
    traffic from the committed PMC summary."""
    kp = {"stream": {"s": 0.054, "launches": 1}}
    rl = bench.roofline(kp, 5000, 100000, 0.054)
    assert rl["kernel"] == "k_la_stream_res"
    assert rl["bytes_per_launch"] == 100000 * 5000 * 32
    assert abs(rl["achieved"] - 16e9 / 0.054 / 1e9) < 1e-6 * rl["achieved"] + 0.01
    assert rl["frac"] == round(rl["achieved"] / rl["peak"], 5)
    assert rl["traffic"] is None or rl["traffic"] > 0
    # per-window launches: the dominant kernel's mean launch
    kp = {"resolve": {"s": 0.070, "launches": 3125}, "select": {"s": 0.040, "launches": 3125}}
    rl = bench.roofline(kp, 5000, 100000, 0.09)
    assert rl["kernel"] == "k_la_resolve4" and rl["bytes_per_launch"] == 32 * 5000 * 32
