"""A/B timing of the two-level hub combine (engine.DEFAULT_HUB_PRE_GROUP; 0 = one level) on C3:
forward (per layer) and dense backward, rounds interleaved in ONE process; d=64 in row-id
layout and d=8 in slot space (a featsplit rank at P=8). Prints one JSON line per setting.

    python tools/hub_probe.py [--caps 0,64,256,1024] [--rounds 3]
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
from gcn_recommendation_amd import dist, engine  # noqa: E402


def timed(fn, reps=5):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--caps", default="0,64,256,1024")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    cfg = bench.CONFIGS["c3"]
    dev = torch.device("cuda", 0)
    engine.load_library()
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I, K = cfg["users"], cfg["items"], cfg["K"]
    n = U + I
    rowptr = np.searchsorted(r, np.arange(n + 1)).astype(np.int32)
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    g = engine.graph_from_coo(adj)
    gs = dist.FeatSplitPlan(rowptr, c, v, n, dev).graph
    gen = torch.Generator().manual_seed(42)
    x64 = [bench.xavier(U, 64, gen).to(dev), bench.xavier(I, 64, gen).to(dev)]
    x8 = torch.rand((n, 8), device=dev) * 1e-3
    G = torch.randn((n, 64), device=dev)
    thr = engine.hub_threshold_from_env()
    caps = [int(x) for x in args.caps.split(",")]
    res = {cap: [] for cap in caps}
    for _ in range(args.rounds):
        for cap in caps:
            engine.DEFAULT_HUB_PRE_GROUP = cap
            hp = g.hubs(thr)
            gs.hubs(thr)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(K)]
            f64 = timed(lambda: engine.propagate_forward(g, x64, K, thr, layer_events=ev))
            lay = [a.elapsed_time(b) for a, b in ev]
            b64 = timed(lambda: engine.propagate_backward(g, [G], K, thr))
            f8 = timed(lambda: engine.propagate_forward(gs, [x8], K, thr))
            res[cap].append((f64, b64, f8, lay, hp.n_slots))
    for cap, rows in res.items():
        a = np.array([x[:3] for x in rows])
        print(json.dumps({"pre_group": cap, "hub_slots": rows[0][4],
                          "fwd_d64_ms": round(float(np.median(a[:, 0])), 3),
                          "bwd_d64_ms": round(float(np.median(a[:, 1])), 3),
                          "fwd_d8_slot_ms": round(float(np.median(a[:, 2])), 3),
                          "fwd_d64_layers_last_round": [round(x, 3) for x in rows[-1][3]]}),
              flush=True)


if __name__ == "__main__":
    main()
