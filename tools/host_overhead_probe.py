"""Host enqueue time vs GPU time of the C3 forward and backwards (is a call host-bound?): wall
time of 20 back-to-back calls until the last returns (host side) and until the GPU is done.
    python tools/host_overhead_probe.py
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402


def main():
    cfg = bench.CONFIGS[os.environ.get("CFG", "c3")]
    dev = torch.device("cuda:0")
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I = cfg["users"], cfg["items"]
    n, d, K = U + I, cfg["d"], cfg["K"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    g = engine.graph_from_coo(adj, sides=(U, U + I))
    gen = torch.Generator().manual_seed(42)
    segs = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
    G = [torch.randn(U, d, device=dev), torch.randn(I, d, device=dev)]
    Gs = [torch.zeros(U, d, device=dev), torch.zeros(I, d, device=dev)]
    rs = np.random.default_rng(1)
    Gs[0][torch.from_numpy(rs.integers(0, U, 2048)).to(dev)] = 1e-3
    Gs[1][torch.from_numpy(rs.integers(0, I, 4096)).to(dev)] = -1e-3
    runs = [("forward", lambda: engine.propagate_forward(g, segs, K)),
            ("backward_dense", lambda: engine.propagate_backward(g, G, K)),
            ("backward_bpr", lambda: engine.propagate_backward(g, Gs, K))]
    for name, f in runs:
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            f()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        # one call alone: host time to return, then GPU completion
        s0 = time.perf_counter()
        f()
        s1 = time.perf_counter()
        torch.cuda.synchronize()
        s2 = time.perf_counter()
        print(f"{name}: 20 calls host {1e3 * (t1 - t0) / 20:.3f} ms/call, wall {1e3 * (t2 - t0) / 20:.3f}"
              f" ms/call; one call: host {1e3 * (s1 - s0):.3f} ms, done at {1e3 * (s2 - s0):.3f} ms",
              flush=True)


if __name__ == "__main__":
    main()
