"""Timing probe of the backward's first layer on the C3 graph: dense G vs row-sparse G (BPR
batch) vs an all-zero G, in degree-ordered slots and in row-id order. One process, HIP events
around each lgcn_spmm_layer launch; prints one JSON line per case.

    python tools/bwd_probe.py [--config c3] [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402


def time_layer(g, x, y, d, ep, thr, reps, x_div, x_nz):
    hp = g.hubs(thr)
    for _ in range(2):
        engine.spmm_layer(g, x, y, d, ep, thr, hp, x_div=x_div, x_nz=x_nz)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        engine.spmm_layer(g, x, y, d, ep, thr, hp, x_div=x_div, x_nz=x_nz)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def time_parts(g, X, y, d, ep, thr, reps, x_div, x_nz):
    """(hub chunks only, rows only) of one lgcn_spmm_layer launch: n_rows = 0 keeps only the
    hub blocks of the grid; n_hub_items = 0 keeps only the row bundles (hub rows skipped)."""
    lib = engine.load_library()
    hp = g.hubs(thr)
    partials = torch.empty(max(hp.n_slots, 1) * d, device=g.device)
    stream = engine._stream(g.device)
    x = engine.rows_desc([X], d)
    out = []
    for n_rows, n_items in ((0, hp.n_items), (g.n_rows, 0)):
        def go():
            engine._check(lib.lgcn_spmm_layer(
                engine._ptr(g.rowptr), engine._ptr(g.edges), engine._ptr(g.row_ids), n_rows,
                thr, engine._ptr(hp.items), n_items, engine._ptr(partials), x, x_div,
                engine._ptr(x_nz), engine._ptr(y), y.stride(0), d, __import__("ctypes").byref(ep),
                stream), "probe")
        go()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(reps):
            go()
        b.record()
        torch.cuda.synchronize()
        out.append(round(a.elapsed_time(b) / reps, 3))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I, d, K = cfg["users"], cfg["items"], cfg["d"], cfg["K"]
    n = U + I
    thr = engine.hub_threshold_from_env()
    rowptr = np.searchsorted(r, np.arange(n + 1)).astype(np.int32)
    rs = np.random.default_rng(1)
    G = torch.zeros((n, d), device=dev)
    G[torch.from_numpy(rs.integers(0, U, 2048)).to(dev)] = 1e-3
    G[U + torch.from_numpy(rs.integers(0, I, 4096)).to(dev)] = -1e-3
    Z = torch.zeros_like(G)
    D = torch.randn_like(G)
    y = torch.empty_like(G)
    for order in ("degree", "stored"):
        g = engine.graph_from_host_csr(rowptr, c, v, n, dev, order=order)
        for name, X in (("dense", D), ("bpr", G), ("zero", Z)):
            nz, cnt = engine.rows_nonzero([X], d, dev)
            ep = engine._epilogue(engine.LGCN_EPI_ADD, addend=engine.rows_desc([X], d),
                                  div=float(K + 1))
            row = {"order": order, "G": name, "live_rows": int(cnt.item())}
            row["dense_ms"] = round(time_layer(g, [X], y, d, ep, thr, args.reps, K + 1.0, None), 3)
            ep.addend_nz = nz.data_ptr()
            row["masked_ms"] = round(time_layer(g, [X], y, d, ep, thr, args.reps, K + 1.0, nz), 3)
            row["masked_hub_rows_ms"] = time_parts(g, X, y, d, ep, thr, args.reps, K + 1.0, nz)
            print(json.dumps(row), flush=True)
        st = engine._epilogue(engine.LGCN_EPI_STORE)
        mean = engine._epilogue(engine.LGCN_EPI_MEAN, prev0=engine.rows_desc([D], d),
                                prev_dense=[Z, G], ld_prev=d, div=float(K + 1))
        print(json.dumps({"order": order, "mean_ms": round(
            time_layer(g, [D], y, d, mean, thr, args.reps, 1.0, None), 3)}), flush=True)
        print(json.dumps({"order": order, "store_ms": round(
            time_layer(g, [D], y, d, st, thr, args.reps, 1.0, None), 3)}), flush=True)
        del g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
