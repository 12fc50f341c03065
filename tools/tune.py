"""Interleaved A/B timing of k_layer variants (rows per group x gathers in flight) and hub
thresholds on the bench graphs, in ONE process (guide §5.4 rule 24). Writes gpurun_out/tune.json.

    python tools/tune.py [--config c3] [--gens powerlaw,uniform] [--rounds 5]
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

VARIANTS = [(0, 0), (1, 8), (8, 4), (15, 4), (8, 6), (15, 6), (8, 8), (15, 8)]


def time_forward(g, segs, K, thr, reps=3):
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for _ in range(K)] for _ in range(reps)]
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for r in range(reps):
        out = engine.propagate_forward(g, segs, K, thr, layer_events=evs[r])
    b.record()
    torch.cuda.synchronize()
    lay = np.array([[x.elapsed_time(y) for x, y in st] for st in evs]).mean(0)
    return a.elapsed_time(b) / reps, lay.tolist(), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--gens", default="powerlaw,uniform")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--thresholds", default="128,256,512")
    ap.add_argument("--chunks", default="128,256,512")
    args = ap.parse_args()
    lib = engine.load_library()
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS[args.config]
    res = {}
    for gen in args.gens.split(","):
        r, c, v, _, _, _ = bench.make_graph(cfg, gen, 16)
        U, I = cfg["users"], cfg["items"]
        n = U + I
        adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                      (n, n)).to(dev)
        g = engine.graph_from_coo(adj)
        gg = torch.Generator().manual_seed(42)
        segs = [bench.xavier(U, 64, gg).to(dev), bench.xavier(I, 64, gg).to(dev)]
        K = cfg["K"]
        nnz = len(v)
        thrs = [int(t) for t in args.thresholds.split(",")]
        times = {}
        ref = {}
        chunks = [int(t) for t in args.chunks.split(",")]
        combos = [(thr, ch, rpg, u) for thr in thrs for ch in chunks for rpg, u in VARIANTS
                  if (rpg, u) == (0, 0) or ch == 256]
        for rnd in range(args.rounds):
            for thr, ch, rpg, u in combos:
                    engine.DEFAULT_HUB_CHUNK = ch
                    g._plans.clear()
                    lib.lgcn_tune(engine.TUNE_ROWS_PER_GROUP, rpg)
                    lib.lgcn_tune(engine.TUNE_UNROLL, u)
                    g.hubs(thr)  # re-plan outside the timed region
                    ms, lay, out = time_forward(g, segs, K, thr)
                    key = f"thr{thr}_ch{ch}_rpg{rpg}_u{u}"
                    times.setdefault(key, []).append((ms, lay))
                    if rnd == 0:
                        h = out[::997].cpu()
                        if (thr, ch) not in ref:
                            ref[(thr, ch)] = h
                        elif not torch.equal(ref[(thr, ch)], h):
                            print(f"!! {gen} {key}: result differs from first variant", flush=True)
        lib.lgcn_tune(engine.TUNE_ROWS_PER_GROUP, 0)
        lib.lgcn_tune(engine.TUNE_UNROLL, 0)
        summ = {}
        for k, lst in times.items():
            ms = [x[0] for x in lst]
            lay = np.array([x[1] for x in lst]).mean(0)
            summ[k] = {"ms_med": float(np.median(ms)), "ms_min": float(np.min(ms)),
                       "layers": [round(x, 4) for x in lay],
                       "gedges_s": K * nnz / (np.median(ms) / 1e3) / 1e9}
        best = sorted(summ.items(), key=lambda kv: kv[1]["ms_med"])
        for k, s in best:
            print(f"{gen:9s} {k:28s} {s['ms_med']:8.3f} ms  {s['gedges_s']:6.2f} Gedges/s  "
                  f"layers {[round(float(x), 3) for x in s['layers']]}", flush=True)
        res[gen] = {"nnz": nnz, "variants": summ}
        del adj, g, segs
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "tune.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
