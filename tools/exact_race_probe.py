"""Repeat the exact-plan forward/backward of the few-bits case of tests/test_gpu_exact.py and report
which rows differ from the oracle, grouped by the path that computed them (bundle, whole long
row, emulated part, chain rows): localises a nondeterministic mismatch to one kernel.

    python tools/exact_race_probe.py [--reps 5] [--chain 1]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gcn_recommendation_amd import engine  # noqa: E402
from oracle import oracle  # noqa: E402
import test_gpu_exact as t  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chain", default="1")
    ap.add_argument("--order", default="degree")
    ap.add_argument("--kind", default="few_bits")
    a = ap.parse_args()
    os.environ["LGCN_CHAIN"] = a.chain
    os.environ["LGCN_ROW_ORDER"] = a.order
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(11)
    r, c, v, n = t._powerlaw(rng, 40_000, 3_000, 200_000)
    g = engine.graph_from_coo(t._adj(r, c, v, n, dev))
    d, K = 64, 3
    e0 = t._e0(rng, a.kind, n, d)
    G = t._e0(rng, "xavier", n, d)
    kw = dict(hub_threshold=128, hub_mode="exact", emu_min=512)
    hp = g.hubs(128, mode="exact", emu_min=512)
    deg = g.degrees()
    bounds = tuple(int(b) for b in os.environ.get("LGCN_EMU_PART_BOUNDS", "8192,1024").split(","))
    parts = hp.emu_parts(bounds)
    emu_rows = hp.emu_rows.cpu().numpy()
    where = np.full(n, "bundle", dtype=object)
    where[deg > 128] = "long"
    for (r0, r1, _, _, short) in parts:
        where[emu_rows[r0:r1, 0]] = "chain" if short and a.chain == "1" else f"emu[{r0}:{r1})"
    def report(tag, got, want):
        bad = np.nonzero((got.view(np.uint32) != want.view(np.uint32)).any(1))[0]
        if bad.size:
            kinds = {}
            for b in bad:
                kinds.setdefault(where[b], []).append(int(b))
            print(f"{tag}: {bad.size} rows differ: " + "; ".join(
                f"{k}: {len(v_)} rows (degrees {sorted(deg[v_])[-3:]})"
                for k, v_ in kinds.items()), flush=True)
        else:
            print(f"{tag}: bitwise", flush=True)

    # the backward layer by layer: h_k = G/(K+1) + Â h_{k-1}, h_0 = G/(K+1) gathered on load
    c4 = (G / np.float32(K + 1)).astype(np.float32)
    want = []
    h = c4
    o = np.argsort(c, kind="stable")  # Âᵀ with each row in Â's stored order (torch's t())
    rt, ct, vt = c[o], r[o], v[o]
    for k in range(K):
        h = (c4 + oracle.spmm(rt, ct, vt, n, h)).astype(np.float32)
        want.append(h)
    gt = g.transpose
    hpt = gt.hubs(128, mode="exact", emu_min=512)
    Gd = torch.from_numpy(G).to(dev)
    for rep in range(a.reps):
        for sparse in ("off", "on"):
            nz = engine.rows_nonzero([Gd], d, dev)[0] if sparse == "on" else None
            ep = engine._epilogue(engine.LGCN_EPI_ADD, addend=engine.rows_desc([Gd], d),
                                  div=float(K + 1))
            ep.addend_nz = None if nz is None else nz.data_ptr()
            hs = [Gd]
            for k in range(K):
                y = torch.empty((n, d), device=dev)
                engine.spmm_layer(gt, hs, y, d, ep, 128, hpt, x_div=float(K + 1) if k == 0 else 1.0,
                                  x_nz=nz if k == 0 else None)
                report(f"rep {rep} bwd-{sparse} layer {k + 1}", y.cpu().numpy(), want[k])
                hs = [torch.from_numpy(want[k]).to(dev)]  # next layer from the exact input


if __name__ == "__main__":
    main()
