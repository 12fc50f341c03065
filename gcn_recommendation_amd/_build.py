"""Build liblgcn_engine.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with
the repo snapshot to the GPU box). Each .hip translation unit compiles to an object in
parallel (the k_layer instantiations are split by epilogue mode), then one link."""
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

_PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_PKG)
CSRC = os.path.join(_PKG, "csrc")
SRCS = [os.path.join(CSRC, f) for f in (
    "lgcn_layer_add_sparse.hip", "lgcn_layer_add_div.hip", "lgcn_layer_add.hip",
    "lgcn_layer_mean.hip", "lgcn_layer_store.hip", "lgcn_engine.hip", "lgcn_eval.hip",
    "lgcn_bpr.hip", "lgcn_fusion.hip", "lgcn_exact.hip")]
HDRS = [os.path.join(ROOT, "include", "lgcn.h"), os.path.join(CSRC, "lgcn_kernels.h")]
OUT = os.path.join(_PKG, "liblgcn_engine.so")
OBJ_DIR = os.path.join(_PKG, "_obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the engine)")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in SRCS + HDRS + [__file__])


def build(force=False, verbose=False, jobs=None, variant=None, defines=()):
    """variant: build an A/B copy (extra -D defines) as _variants/liblgcn_<variant>.so, loaded by
    engine.load_library when LGCN_LIB points at it; the product library is untouched."""
    out, obj_dir, flags = OUT, OBJ_DIR, FLAGS + [f"-D{d}" for d in defines]
    if variant:
        out = os.path.join(_PKG, "_variants", f"liblgcn_{variant}.so")
        obj_dir = os.path.join(_PKG, "_variants", variant)
    elif not force and not needs_build():
        return OUT
    os.makedirs(obj_dir, exist_ok=True)
    cc = hipcc()
    inc = ["-I", os.path.join(ROOT, "include"), "-I", CSRC]

    def compile_one(src):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if not force and os.path.exists(obj) and all(
                os.path.getmtime(obj) > os.path.getmtime(p) for p in [src] + HDRS + [__file__]):
            return obj  # up to date (incremental rebuild)
        cmd = [cc] + flags + inc + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        return obj

    n = jobs or min(len(SRCS), max(1, min(8, (os.cpu_count() or 2))))
    with ThreadPoolExecutor(n) as pool:
        objs = list(pool.map(compile_one, SRCS))
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + ["-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def build_capture_host(verbose=False):
    """tools/capture_host: the C host that captures the library's two-lane schedule into a HIP
    graph (tests/test_gpu_sides.py::test_c_host_captures_full_schedule), linked against the
    in-tree liblgcn_engine.so (rpath $ORIGIN/../gcn_recommendation_amd)."""
    src = os.path.join(ROOT, "tools", "capture_host.cpp")
    exe = os.path.join(ROOT, "tools", "capture_host")
    if os.path.exists(exe) and all(os.path.getmtime(exe) > os.path.getmtime(p)
                                   for p in (src, OUT, HDRS[0])):
        return exe
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O2", "-I", os.path.join(ROOT, "include"), src,
           "-L", _PKG, "-llgcn_engine", "-Wl,-rpath,$ORIGIN/../gcn_recommendation_amd",
           "-o", exe]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return exe


if __name__ == "__main__":
    # python -m gcn_recommendation_amd._build [variant DEFINE=VALUE ...]
    import sys
    if len(sys.argv) > 1:
        print(build(variant=sys.argv[1], defines=sys.argv[2:], verbose=False))
    else:
        print(build(force=True, verbose=True))
