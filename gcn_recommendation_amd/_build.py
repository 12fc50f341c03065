"""Build liblgcn_engine.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with
the repo snapshot to the GPU box)."""
import os
import shutil
import subprocess

_PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_PKG)
SRCS = [os.path.join(_PKG, "csrc", f) for f in ("lgcn_engine.hip", "lgcn_eval.hip", "lgcn_bpr.hip")]
HDR = os.path.join(ROOT, "include", "lgcn.h")
OUT = os.path.join(_PKG, "liblgcn_engine.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the engine)")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in SRCS + [HDR, __file__])


def build(force=False, verbose=False):
    if not force and not needs_build():
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-Wall", "-I", os.path.join(ROOT, "include")] + SRCS + \
          ["-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
