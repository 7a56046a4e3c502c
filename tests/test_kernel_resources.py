"""Code-object metadata of the built gfx950 kernels, CPU only: every kernel in
libqsched.so — the resident stream ``k_la_stream_res`` of every feature class / geometry above all
(its resolver runs one dependent chain per pod, where a scratch round trip is ~1 µs) — must have

* no private (scratch) segment: ``.private_segment_fixed_size == 0`` (no alloca left in memory);
* no VGPR spills: ``.vgpr_spill_count == 0``;
* at most 256 VGPRs (``.vgpr_count``; 512-thread workgroups: two waves per SIMD).

(The per-window normalizing fallbacks — k_la_resolve4 / k_la_resolve_norm of the wide and
configurable-resource classes, k_persistent — still spill; they run only for tables or sharded
modes the resident stream does not cover)

SGPR spills (``.sgpr_spill_count``) are reported, not asserted: the compiler parks uniform values
beyond the 106 addressable SGPRs in VGPR lanes (v_writelane / v_readlane, no memory traffic); every
resident kernel has them.  The metadata is read from the library's .hip_fatbin
section (one offload bundle per translation unit) with the ROCm LLVM tools; the test skips when the
library or the tools are absent.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "custom-k8s-scheduler_amd", "libqsched.so")
LLVM = "/opt/rocm/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernel_metadata(lib=LIB):
    """[(kernel name, {field: int})] for every gfx950 kernel of every bundle in lib's .hip_fatbin."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, a in enumerate(starts):
            b = starts[i + 1] if i + 1 < len(starts) else len(data)
            part = os.path.join(d, f"b{i}.bin")
            co = os.path.join(d, f"b{i}.co")
            open(part, "wb").write(data[a:b].rstrip(b"\0") if i + 1 < len(starts) else data[a:b])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode != 0:
                # (bundles are 4 KiB-aligned; a stripped tail can cut a code object: retry unstripped)
                open(part, "wb").write(data[a:b])
                subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True,
                               capture_output=True)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            for blk in re.split(r"\n\s+- \.agpr_count", notes)[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk).group(1)
                f = {k: int(re.search(r"\." + k + r":\s+(\d+)", blk).group(1))
                     for k in ("vgpr_count", "sgpr_count", "sgpr_spill_count", "vgpr_spill_count",
                               "private_segment_fixed_size")}
                out.append((name, f))
    return out


@pytest.fixture(scope="module")
def meta():
    if not os.path.exists(LIB) or not shutil.which(f"{LLVM}/llvm-readelf"):
        pytest.skip("libqsched.so or the ROCm LLVM tools are absent")
    return kernel_metadata()


def test_every_resident_stream_instantiation_is_present(meta):
    res = [n for n, _ in meta if "k_la_stream_res" in n]
    # four translation units (compact / wide rows x default / configurable scoring), both feature
    # classes each, every selector geometry
    assert len(res) >= 100, len(res)
    feats = {re.search(r"k_la_stream_resILj(\d+)E", n).group(1) for n in res}
    assert feats >= {"0", "4", "7", "12", "15", "20", "23", "28", "31"}, feats


def test_resident_stream_kernels_have_no_scratch_and_no_vgpr_spills(meta):
    bad = [(n[:120], f) for n, f in meta if "k_la_stream_res" in n and
           (f["private_segment_fixed_size"] or f["vgpr_spill_count"] or f["vgpr_count"] > 256)]
    assert not bad, bad
