"""Bisect HIP-graph capture of the sided forward by stream budget (LGCN_AUX_STREAMS=$1)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gcn_recommendation_amd import engine  # noqa: E402
import test_gpu_sides as T  # noqa: E402

SEGV = None
if os.environ.get("LGCN_SEGV_TRACE"):  # native backtrace of a host crash (tools/segv_trace.c)
    import ctypes
    SEGV = ctypes.CDLL(os.path.join(ROOT, "tools", "libsegv_trace.so"))
os.environ["LGCN_SIDES_MIN_NNZ"] = "0"
os.environ["LGCN_AUX_STREAMS"] = sys.argv[1]
dev = torch.device("cuda:0")
r, c, v, n = T._brand_graph(np.random.default_rng(21))
adj = T._adj(r, c, v, n, dev)
g = engine.graph_from_coo(adj, sides=(T.U, T.U + T.I))
x = T._segs(T._e0(np.random.default_rng(8), "xavier", n, 64), dev)
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ref = engine.propagate_forward(g, x, K, hub_threshold=128)
print("eager ok", flush=True)
if SEGV is not None:  # the runtime may have installed its own handlers since
    SEGV.segv_install()
cap = engine.CapturedForward(g, x, K, hub_threshold=128)
print("captured", flush=True)
print("replay bitwise", bool(torch.equal(cap.replay(), ref)), flush=True)
