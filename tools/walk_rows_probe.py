"""Per-row walk statistics of one C3 forward (why part 1's longest row walks slower
per block than part 0's): for the part-0 row (slot 0) and part 1's rows (slots 1..), summed over
the forward's walk launches: translated / resolved blocks per column, cycles per resolved block
and the longest wave, on the two-lane schedule and with every part alone (LGCN_EMU_OVERLAP=0).
Needs the LGCN_EMU_STATS build with tools/patches/walk_rows_stats.patch applied (it keys the
per-row counters by part: slot 0 = part 0's row, slots 1.. = part 1's rows):
    git apply tools/patches/walk_rows_stats.patch
    bash tools/variant_one.sh emustats lgcn_exact.hip -DLGCN_EMU_STATS=1
    git apply -R tools/patches/walk_rows_stats.patch
    LGCN_LIB=gcn_recommendation_amd/_variants/liblgcn_emustats.so python tools/walk_rows_probe.py
"""
import ctypes
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
    lib = engine.load_library()
    lib.lgcn_emu_row_stats.argtypes = [ctypes.c_void_p]
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I = cfg["users"], cfg["items"]
    n, d, K = U + I, cfg["d"], cfg["K"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    gen = torch.Generator().manual_seed(42)
    segs = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
    buf = (ctypes.c_ulonglong * 1024)()
    for mode in ("two lanes", "alone"):
        if mode == "alone":
            os.environ["LGCN_EMU_OVERLAP"] = "0"
        g = engine.graph_from_coo(adj, sides=(U, U + I))
        for _ in range(3):
            engine.propagate_forward(g, segs, K)
        torch.cuda.synchronize()
        lib.lgcn_emu_row_stats(buf)  # reset
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        engine.propagate_forward(g, segs, K)
        t1.record()
        torch.cuda.synchronize()
        assert lib.lgcn_emu_row_stats(buf) == 0
        a = np.array(buf, dtype=np.float64).reshape(256, 4)
        print(f"== {mode}: forward {t0.elapsed_time(t1):.2f} ms (sums over the forward's walks)",
              flush=True)
        for k in range(12):
            f, s_, ts, tmax = a[k]
            if f + s_ == 0:
                continue
            print(f"  slot {k}: blocks {(f + s_) / d:.0f} per col, translated {f / d:.0f}, resolved "
                  f"{s_ / d:.0f} ({100 * s_ / (f + s_):.1f}%), cycles/resolved {ts / max(s_, 1):.0f}"
                  f", longest wave {tmax / 2.1e3:.0f} us (s_memtime cycles at 2.1 GHz)", flush=True)


if __name__ == "__main__":
    main()
