"""Build a timing variant of the compact kernels (libqsched_<name>.so) from text substitutions of
csrc/qs_kernels.hpp (or qs_device.hpp), without touching the product sources (DESIGN.md §4.1e method: measure a
variant against the product in the same gpurun call, keep it only if it wins).

Usage: python tools/exp_variant.py NAME 'old1' 'new1' ['old2' 'new2' ...]
The product objects must be built (make -C custom-k8s-scheduler_amd).  Each `old` must occur.
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "custom-k8s-scheduler_amd")


def main():
    name, subs = sys.argv[1], sys.argv[2:]
    assert len(subs) % 2 == 0, "pairs of old / new"
    src = os.path.join(PKG, "csrc")
    dst = os.path.join(PKG, "build", f"var_{name}")
    if os.path.exists(dst):
        shutil.rmtree(dst)
    shutil.copytree(src, dst)
    # each substitution applies to the first of these headers that holds its `old` text
    files = [os.path.join(dst, f) for f in ("qs_kernels.hpp", "qs_device.hpp", "qs_kernels.hip")]
    text = {f: open(f).read() for f in files}
    for old, new in zip(subs[0::2], subs[1::2]):
        f = next((f for f in files if old in text[f]), None)
        assert f is not None, f"not found: {old[:80]!r}"
        text[f] = text[f].replace(old, new)
    for f in files:
        open(f, "w").write(text[f])
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-ffp-contract=off",
             "-Wno-unused-function", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
             f"-I{os.path.join(ROOT, 'include')}"] + os.environ.get("EXP_DEFS", "").split()
    obj = os.path.join(dst, "qs_kernels.o")
    subprocess.run(["/opt/rocm/bin/hipcc"] + flags + ["-c", os.path.join(dst, "qs_kernels.hip"), "-o", obj], check=True)
    # EXP_DEFS="-DQS_RES_DIAG_BLOCK" EXP_OBJS=build_diag: a diagnostic variant (tools/diag_build.sh objects)
    objs = os.environ.get("EXP_OBJS", "build")
    others = [os.path.join(PKG, objs, f) for f in ("qs_kernels_wide.o", "qs_kernels_res.o", "qs_kernels_res_wide.o",
                                                   "qs_host.o", "qs_helpers.o", "qs_dist.o")]
    out = os.path.join(PKG, f"libqsched_{name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, obj] + others +
                   ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    print(out)


if __name__ == "__main__":
    main()
