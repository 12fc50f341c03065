"""Per-rank cost of the featsplit decomposition, measured on ONE GPU: at P ranks every rank runs
the full K-layer propagation over the whole C3 graph on d/P columns, with no exchange. Timing
the single-GPU forward at d = d_config/P for P in 1, 2, 4, 8 predicts the strong-scaling curve of
`bench.py --gpus P --mode featsplit` (the ranks do not share anything but the node's power).

    python tools/featsplit_sweep.py [--config c3] [--steps 10]
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


def relabel(rowptr, c, v, U, I, order):
    """Node relabelling experiment: returns (rowptr', c', v') of P·Â·Pᵀ with every row's edges
    kept in their stored order (so each output row is the same fp32 chain, bitwise)."""
    n = U + I
    deg = np.diff(rowptr).astype(np.int64)
    if order in ("degree", "degree_rows"):
        perm = np.argsort(-deg, kind="stable")
    elif order.startswith("cluster"):
        # items by popularity first; then users grouped by one of their items (cluster: the
        # least popular, cluster_hot: the most popular), so an item row's users sit in
        # consecutive ids (4 rows of d=8 per 128-B line). *_deg: degree-major, the item key
        # only orders users of equal degree (keeps the bundles' rows of equal length)
        items = U + np.argsort(-deg[U:], kind="stable")
        new_item = np.empty(n, np.int64)
        new_item[items] = np.arange(I)
        ue = c[:rowptr[U]].astype(np.int64)
        key = np.full(U, -1, np.int64)
        has = deg[:U] > 0
        red = np.minimum if "hot" in order else np.maximum
        key[has] = red.reduceat(new_item[ue], rowptr[:U][has].astype(np.int64))
        if order.endswith("_deg"):
            users = np.lexsort((key, -deg[:U]))
        else:
            users = np.argsort(key, kind="stable")
        perm = np.concatenate([items, users])
    elif order in ("degkey", "degkey_rows"):
        # generic (no user/item split): degree-descending, ties by the highest degree-rank among
        # the row's neighbours — the node-agnostic form of cluster_deg
        rank0 = np.empty(n, np.int64)
        rank0[np.argsort(-deg, kind="stable")] = np.arange(n)
        key = np.full(n, -1, np.int64)
        has = deg > 0
        key[has] = np.maximum.reduceat(rank0[c.astype(np.int64)], rowptr[:-1][has].astype(np.int64))
        perm = np.lexsort((key, -deg))
    else:
        return rowptr, c, v
    new_id = np.empty(n, np.int64)
    new_id[perm] = np.arange(n)
    dn = deg[perm]
    rp = np.zeros(n + 1, np.int64)
    np.cumsum(dn, out=rp[1:])
    idx = np.arange(rp[-1], dtype=np.int64) - np.repeat(rp[:-1], dn) + \
        np.repeat(rowptr[:-1][perm].astype(np.int64), dn)
    if order in ("degree_rows", "degkey_rows"):  # processing order only: columns stay in the original ids
        return rp.astype(np.int32), c[idx], v[idx]
    return rp.astype(np.int32), new_id[c[idx]].astype(np.int32), v[idx]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--gen", default="powerlaw")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--dims", default="64,32,16,8")
    ap.add_argument("--variants", default="none:1:-",
                    help="comma list of order:slot_space:proc_order (order: none | degree | "
                         "degree_rows | cluster[_hot][_deg]; proc_order: - | degree | stored)")
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    engine.load_library()
    r, c0, v0, _, _, _ = bench.make_graph(cfg, args.gen, 16)
    U, I = cfg["users"], cfg["items"]
    n, K, nnz = U + I, cfg["K"], len(v0)
    rowptr0 = np.searchsorted(r, np.arange(n + 1)).astype(np.int32)
    del r
    thr = engine.hub_threshold_from_env()
    for var in args.variants.split(","):
        order, slot_space, proc = var.split(":")
        proc = None if proc == "-" else proc
        rowptr, c, v = relabel(rowptr0, c0, v0, U, I, order)
        if int(slot_space):  # what bench.py --mode featsplit runs (dist.FeatSplitPlan)
            from gcn_recommendation_amd import dist
            # LGCN_SIDES_FEATSPLIT=1: the shards on the two-lane schedule (bench.py's N > 1 path)
            sides = (U, U + I) if os.environ.get("LGCN_SIDES_FEATSPLIT") == "1" else None
            g = dist.FeatSplitPlan(rowptr, c, v, n, dev, sides=sides).graph
        else:
            g = engine.graph_from_host_csr(rowptr, c, v, n, dev, order=proc)
        del rowptr, c, v
        g.hubs(thr)
        out = []
        for d in [int(x) for x in args.dims.split(",")]:
            gen = torch.Generator().manual_seed(42)
            segs = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
            for _ in range(3):
                engine.propagate_forward(g, segs, K, thr)
            torch.cuda.synchronize()
            evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    for _ in range(K)] for _ in range(args.steps)]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for s in range(args.steps):  # (a sided graph: whole steps, no layer events)
                engine.propagate_forward(g, segs, K, thr,
                                         layer_events=None if g.split is not None else evs[s])
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.steps
            lay = (np.full(K, ms / K) if g.split is not None else
                   np.array([[x.elapsed_time(y) for x, y in st] for st in evs]).mean(0))
            b_layer = nnz * (4 * d + 8) + 4 * (n + 1) + 4 * n * d
            p = cfg["d"] // d
            row = {"variant": var, "d": d, "ranks": p, "ms_per_step": round(ms, 3),
                   "per_layer_ms": [round(float(x), 3) for x in lay],
                   "store_layer_GBps": round(b_layer / (lay[:-1].mean() / 1e3) / 1e9, 1),
                   "edges_per_s": round(K * nnz / (ms / 1e3), 1)}
            out.append(row)
            print(json.dumps(row), flush=True)
            del segs
            torch.cuda.empty_cache()
        del g
        torch.cuda.empty_cache()
        base = out[0]["ms_per_step"]
        print(json.dumps({"variant": var, "predicted_featsplit_speedup": {
            str(r_["ranks"]): round(base / r_["ms_per_step"], 2) for r_ in out}}),
            flush=True)


if __name__ == "__main__":
    main()
