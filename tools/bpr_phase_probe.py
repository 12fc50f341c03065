"""Phase log of one C3 BPR-batch backward on the sided schedule (engine.side_trace: per half-layer
(k, segment) the library's marks — start, part 0 / part 1 block passes done, layer kernel done,
chains done, part 0 / part 1 walks done, joined), in ms from an event recorded just before the
call; also the same for the forward. Marks a half-layer does not reach are left out.
    python tools/bpr_phase_probe.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402


def main():
    cfg = bench.CONFIGS["c3"]
    dev = torch.device("cuda:0")
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I = cfg["users"], cfg["items"]
    n, d, K = U + I, cfg["d"], cfg["K"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    g = engine.graph_from_coo(adj, sides=(U, U + I))
    gen = torch.Generator().manual_seed(42)
    segs = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
    Gs = [torch.zeros(U, d, device=dev), torch.zeros(I, d, device=dev)]
    rs = np.random.default_rng(1)
    Gs[0][torch.from_numpy(rs.integers(0, U, 2048)).to(dev)] = 1e-3
    Gs[1][torch.from_numpy(rs.integers(0, I, 4096)).to(dev)] = -1e-3
    for name, f in (("forward", lambda: engine.propagate_forward(g, segs, K)),
                    ("backward_bpr", lambda: engine.propagate_backward(g, Gs, K))):
        for _ in range(4):
            f()
            torch.cuda.synchronize()
        engine.side_trace = []
        ref = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        ref.record()
        f()
        end.record()
        torch.cuda.synchronize()
        tr = engine.side_trace[-1]
        engine.side_trace = None
        print(f"== {name}: {ref.elapsed_time(end):.3f} ms", flush=True)
        for (k, seg) in sorted(tr):
            marks = [(ph, ref.elapsed_time(ev)) for ph, ev in tr[(k, seg)]]
            marks = [f"{ph} {t:.3f}" for ph, t in marks if t >= 0]
            print(f"  layer {k} segment {seg}: " + ", ".join(marks), flush=True)


if __name__ == "__main__":
    main()
