"""Where the hub walk's time goes beside the other lane vs alone: the walker's
phase timers (s_memtime per phase of the row-0 / column-0 wave of every walk launch, summed) of
one C3 forward on the two-lane schedule and of one forward with every part in order on one
stream (LGCN_EMU_OVERLAP=0: each walk runs alone). Needs the LGCN_EMU_STATS build:
    python -m gcn_recommendation_amd._build emustats LGCN_EMU_STATS=1
    LGCN_LIB=gcn_recommendation_amd/_variants/liblgcn_emustats.so python tools/walk_phase_probe.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
from exact_probe import phase_stats, stats  # noqa: E402


def main():
    cfg = bench.CONFIGS["c3"]
    dev = torch.device("cuda:0")
    lib = engine.load_library()
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I = cfg["users"], cfg["items"]
    n, d, K = U + I, cfg["d"], cfg["K"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    gen = torch.Generator().manual_seed(42)
    segs = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
    for mode in ("two lanes", "alone"):
        if mode == "alone":
            os.environ["LGCN_EMU_OVERLAP"] = "0"
        g = engine.graph_from_coo(adj, sides=(U, U + I))
        for _ in range(3):
            engine.propagate_forward(g, segs, K)
        torch.cuda.synchronize()
        stats(lib)
        import ctypes
        buf = (ctypes.c_ulonglong * 16)()
        assert lib.lgcn_emu_phase(buf) == 0  # reset
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        engine.propagate_forward(g, segs, K)
        b.record()
        torch.cuda.synchronize()
        print(f"== {mode}: forward {a.elapsed_time(b):.2f} ms; walker decisions {stats(lib)}",
              flush=True)
        phase_stats(lib)


if __name__ == "__main__":
    main()
