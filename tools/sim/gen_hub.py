"""Dump the longest rows of the C3 power-law graph (bench.py's generator) with layer-1 and
layer-2 X columns, for the CPU simulation of the walk's resolve (tools/sim/resolve_sim.c).

    python tools/sim/gen_hub.py OUT_DIR [--cols 8] [--rows 0,1,5,20,42]
Writes OUT_DIR/row<k>_l<layer>.bin: int32 n, int32 d, float v[n], float x[n][d] (x row j = the
X row of edge j's column).
"""
import argparse
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from gcn_recommendation_amd import graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--cols", type=int, default=8)
    ap.add_argument("--rows", default="0,1,5,20,42")
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    U, I, E = graph.books_shape(a.scale)
    u, i = graph.powerlaw_interactions(U, I, E, 3)
    rows, cols = graph.edge_lists(u, i, U, I, use_brand=False)
    r, c, v = graph.normalise(rows, cols, U + I)
    n = U + I
    A = sp.csr_matrix((v, (r, c)), shape=(n, n))
    A.sort_indices()
    deg = np.diff(A.indptr)
    order = np.argsort(-deg, kind="stable")
    d = a.cols
    rng = np.random.default_rng(11)
    e0 = np.empty((n, d), np.float32)
    e0[:U] = (rng.random((U, d), dtype=np.float32) * 2 - 1) * np.float32(np.sqrt(6.0 / (U + 64)))
    e0[U:] = (rng.random((I, d), dtype=np.float32) * 2 - 1) * np.float32(np.sqrt(6.0 / (I + 64)))
    e1 = (A @ e0.astype(np.float64)).astype(np.float32)  # approximate layer 1 (stats only)
    for k in [int(t) for t in a.rows.split(",")]:
        row = order[k]
        b, e = A.indptr[row], A.indptr[row + 1]
        cc, vv = A.indices[b:e], A.data[b:e].astype(np.float32)
        for layer, X in ((1, e0), (2, e1)):
            with open(os.path.join(a.out, f"row{k}_l{layer}.bin"), "wb") as f:
                np.array([e - b, d], np.int32).tofile(f)
                vv.tofile(f)
                np.ascontiguousarray(X[cc]).tofile(f)
        print(f"row rank {k}: id {row} degree {e - b}", flush=True)


if __name__ == "__main__":
    main()
