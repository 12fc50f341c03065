"""Timing of the sequential-chain kernel (lgcn_chain_rows) alone, per row length: one item row of
each degree in --degrees over a synthetic user pool, each run by itself (one row: one wave per
32-column slice), reported as us per row and ns / cycles per step (chain step = one edge).

    python tools/chain_probe.py [--degrees 1024,4096,16384,65536,262144] [--d 64] [--reps 5]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gcn_recommendation_amd import engine  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--degrees", default="1024,4096,16384,65536,262144")
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--clock-ghz", type=float, default=2.1)
    a = ap.parse_args()
    degs = [int(t) for t in a.degrees.split(",")]
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    U = max(degs) + 1000
    users = np.concatenate([rng.permutation(U)[:k] for k in degs])
    items = np.concatenate([np.full(k, i, np.int64) for i, k in enumerate(degs)])
    r, c, v, n = oracle.build_norm_adj(users, items, U, len(degs), 0, use_brand=False)
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([r, c])), torch.from_numpy(v),
                                  (n, n)).to(dev)
    g = engine.graph_from_coo(adj)
    lib = engine.load_library()
    hp = g.hubs(128, mode="exact", emu_min=128)  # every hub row in the emulated-row list
    er = hp.emu_rows.cpu().numpy()
    d = a.d
    x = torch.empty((n, d), device=dev).uniform_(-1e-3, 1e-3)
    y = torch.empty((n, d), device=dev)
    ep = engine._epilogue(engine.LGCN_EPI_STORE)
    xs = engine.rows_desc([x], d)
    st = engine._stream(dev)
    rb = hp.emu_rows.element_size() * 4
    deg_of = dict(zip(range(n), g.degrees()))
    for i in range(er.shape[0]):
        row = int(er[i, 0])
        k = deg_of[row]

        def run():
            assert lib.lgcn_chain_rows(engine._ptr(g.edges), hp.emu_blocks.data_ptr(),
                                       hp.emu_rows.data_ptr() + i * rb, 1, xs, 1.0,
                                       engine._ptr(y), d, d, ctypes.byref(ep), st) == 0
        run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        t = float(np.median(ts)) * 1e3
        print(f"row of {k:>8,} edges: {t:9.1f} us  {1e3 * t / k:7.2f} ns/step  "
              f"{a.clock_ghz * 1e3 * t / k:6.1f} cycles/step", flush=True)


if __name__ == "__main__":
    main()
