"""The bipartite two-lane schedule on the C3 power-law graph against the one-operator schedule:
forward and backward ms per step for each stream budget (LGCN_AUX_STREAMS 3 / 7), bitwise
agreement of the two, and the per-half-layer phase log of one sided forward (ms from its start:
fork, part 0 / part 1 block passes, layer kernel, chains, part 0 / part 1 walks, joined) written
as JSON (--trace-out) — the "per-chain phase log" of profiles/.

    GPU_MAX_HW_QUEUES=8 python tools/sides_probe.py [--config c3] [--steps 5] [--trace-out f]
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


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--aux", default="3,7")
    ap.add_argument("--trace-out", default="")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    engine.load_library()
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I = cfg["users"], cfg["items"]
    n, d, K = U + I, cfg["d"], cfg["K"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    del r, c, v
    g1 = engine.graph_from_coo(adj)
    g2 = engine.graph_from_coo(adj, sides=(U, U + I))
    print(f"hw queues {engine.hw_queues()}; sided split {g2.split} "
          f"(side 1 = items [{U}, {U + I}))", flush=True)
    hps = g2.side_hubs(128)
    for s, hp in enumerate(hps):
        print(f"  side {s}: emulated rows {hp.n_emu_rows} ({hp.n_emu_blocks} blocks), walk parts "
              f"{hp.walk_parts(g2.nnz)}", flush=True)
    gen = torch.Generator().manual_seed(42)
    segs = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
    G = [t.clone() for t in segs]
    res = {}
    ref_f = ref_b = None
    for nx in [int(t) for t in a.aux.split(",")]:
        os.environ["LGCN_AUX_STREAMS"] = str(nx)
        for name, g in (("one_operator", g1), ("sides", g2)):
            if name == "one_operator" and nx > 3:
                continue
            tf = timed(lambda: engine.propagate_forward(g, segs, K), a.steps)
            tb = timed(lambda: engine.propagate_backward(g, G, K), a.steps)
            of = engine.propagate_forward(g, segs, K)
            ob = engine.propagate_backward(g, G, K)
            if ref_f is None:
                ref_f, ref_b = of, ob
            same = bool(torch.equal(of.view(torch.int32), ref_f.view(torch.int32)) and
                        torch.equal(ob.view(torch.int32), ref_b.view(torch.int32)))
            res[f"{name}_aux{nx}"] = {"forward_ms": round(tf, 3), "backward_ms": round(tb, 3),
                                      "bitwise_vs_first": same}
            print(f"{name:13s} aux {nx}: forward {tf:7.3f} ms  backward {tb:7.3f} ms  "
                  f"bitwise {same}", flush=True)
            del of, ob
    # phase log of one sided forward and one sided backward at the largest stream budget
    logs = {}
    for what in ("forward", "backward"):
        engine.side_trace = []
        engine.side_timing = []
        if what == "forward":
            engine.propagate_forward(g2, segs, K)
        else:
            engine.propagate_backward(g2, G, K)
        torch.cuda.synchronize()
        tr, tm = engine.side_trace[0], engine.side_timing[0]
        engine.side_trace = engine.side_timing = None
        t0 = tr[(1, 0)][0][1]
        for (k, s) in sorted(tr):
            ph = {nm: round(t0.elapsed_time(ev), 3) for nm, ev in tr[(k, s)]}
            ph["layer_kernel_ms"] = round(tm[(k, s)][0].elapsed_time(tm[(k, s)][1]), 3)
            ph["lane"] = (k + s) % 2
            logs.setdefault(what, {})[f"layer{k}_side{s}"] = ph
            print(f"{what} half-layer (k={k}, side={s}, lane {(k + s) % 2}): " +
                  ", ".join(f"{nm} {val}" for nm, val in ph.items()), flush=True)
    res["phases_ms_from_start"] = logs
    res["note"] = ("side 0 = users (+brands), side 1 = items; half-layer (k, side) runs on lane "
                   "(k + side) % 2; phase events are recorded on the stream of each part (a "
                   "part absent from a half-layer records at its fork)")
    if a.trace_out:
        os.makedirs(os.path.dirname(a.trace_out) or ".", exist_ok=True)
        json.dump(res, open(a.trace_out, "w"), indent=1)


if __name__ == "__main__":
    main()
