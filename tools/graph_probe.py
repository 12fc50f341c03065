"""HIP-graph replay (engine.CapturedForward) vs eager launches of the K-layer forward on a
small graph (C1 shape, launch-bound) and on C2. Prints one JSON line per graph.

    python tools/graph_probe.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gcn_recommendation_amd import engine, graph  # noqa: E402


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda", 0)
    cases = {"c1": dict(users=1000, items=1000, interactions=10000, d=64, K=2, seed=0),
             "c2": bench.CONFIGS["c2"]}
    for name, cfg in cases.items():
        U, I, d, K = cfg["users"], cfg["items"], cfg["d"], cfg["K"]
        u, i = graph.uniform_interactions(U, I, cfg["interactions"], cfg["seed"])
        rows, cols = graph.edge_lists(u, i, U, I, use_brand=False)
        r, c, v = graph.normalise(rows, cols, U + I)
        n = U + I
        adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                      (n, n)).to(dev)
        g = engine.graph_from_coo(adj)
        gen = torch.Generator().manual_seed(42)
        segs = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
        eager = engine.propagate_forward(g, segs, K)
        cap = engine.CapturedForward(g, segs, K)
        same = torch.equal(cap.replay(), eager)
        te = timed(lambda: engine.propagate_forward(g, segs, K))
        tg = timed(cap.replay)
        print(json.dumps({"graph": name, "nnz": len(v), "eager_ms": round(te, 4),
                          "hipgraph_ms": round(tg, 4), "bitwise": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
