"""C2 (Books-subset shape) forward probe: single-row lane groups (the default below 131k rows)
vs row bundles forced by LGCN_TUNE_MIN_GROUPS, and HIP-graph replay (engine.CapturedForward).
Measured round 1: 0.200 ms default; bundles 0.27-1.78 ms (too few waves); graph replay 0.203 ms.

    python tools/c2_probe.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402

cfg = bench.CONFIGS["c2"]
dev = torch.device("cuda", 0)
lib = engine.load_library()
r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
U, I, K = cfg["users"], cfg["items"], cfg["K"]
n = U + I
adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v), (n, n)).to(dev)
g = engine.graph_from_coo(adj)
gen = torch.Generator().manual_seed(42)
segs = [bench.xavier(U, 64, gen).to(dev), bench.xavier(I, 64, gen).to(dev)]
def t(reps=50):
    for _ in range(5): engine.propagate_forward(g, segs, K)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): engine.propagate_forward(g, segs, K)
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps
ref = engine.propagate_forward(g, segs, K).clone()
for mg in (0, 32768, 16384, 8192, 4096):
    lib.lgcn_tune(engine.TUNE_MIN_GROUPS, mg)
    ms = [t() for _ in range(3)]
    same = torch.equal(engine.propagate_forward(g, segs, K), ref)
    print(json.dumps({"min_groups": mg, "ms": round(min(ms), 4), "bitwise_same": same}), flush=True)
lib.lgcn_tune(engine.TUNE_MIN_GROUPS, 0)
cg = engine.CapturedForward(g, segs, K)
def tg(reps=50):
    for _ in range(5): cg.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): cg.replay()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps
print(json.dumps({"hipgraph_ms": round(min(tg() for _ in range(3)), 4)}), flush=True)
