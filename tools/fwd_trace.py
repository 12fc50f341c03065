"""A C3 forward, dense backward and BPR-batch backward, each run once after warm-up and separated
by 50-ms idle gaps, for a rocprofv3 kernel trace whose dispatch timeline tools/timeline.py splits
at the gaps (which kernel runs when, on which queue: the exact plan's critical path).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/fwd_trace.py
    python tools/timeline.py OUT
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("LGCN_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["LGCN_HW_QUEUES"]
import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402


def main():
    cfg = bench.CONFIGS[os.environ.get("CFG", "c3")]
    dev = torch.device("cuda:0")
    lib = engine.load_library()
    for kv in filter(None, os.environ.get("TUNE", "").split(",")):  # A/B: lgcn_tune knob:value
        k, val = (int(t) for t in kv.split(":"))
        lib.lgcn_tune(k, val)
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
            ("backward", lambda: engine.propagate_backward(g, G, K)),
            ("backward_bpr", lambda: engine.propagate_backward(g, Gs, K))]
    if os.environ.get("FWD_ONLY"):  # A/B timing: median of REPS forwards (and BPR backwards)
        reps = int(os.environ.get("REPS", "10"))
        sel = (runs[0], runs[1], runs[2]) if os.environ.get("DENSE") else (runs[0], runs[2])
        for name, fn in sel:
            for _ in range(3):
                fn()
            ts = []
            for _ in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                fn()
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b))
            print(f"{name}: median {np.median(ts):.3f} ms min {min(ts):.3f} "
                  f"[{os.environ.get('LGCN_LIB', 'product')} {os.environ.get('TUNE', '')}]"
                  f" all {' '.join(f'{t:.2f}' for t in ts)}", flush=True)
        return
    for name, fn in runs:
        for _ in range(3):  # warm-up right before: the backward's schedule follows G's sparsity
            fn()
        torch.cuda.synchronize()
        time.sleep(0.05)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        print(f"{name}: {a.elapsed_time(b):.3f} ms", flush=True)
        time.sleep(0.05)


if __name__ == "__main__":
    main()
