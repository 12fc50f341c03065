"""TEST INFRASTRUCTURE ONLY — the CPU parity oracle for the LightGCN propagation path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
module; the product (`gcn_recommendation_amd/`, `models/`) never does. It is the checker, never
the thing measured or shipped.

Contents, each restating a reference function (paths relative to the reference repo):
  * build_norm_adj      main.py:282-336   edge list -> symmetric D^-1/2 A D^-1/2 COO (numpy,
                                           the exact fp32 operation order of the scipy path)
  * spmm / forward / backward             models/lightgcn.py:40-54 + autograd, in C
                                           (oracle/lgcn_oracle.c, sequential fmaf = ATen's CPU
                                           addmm_sparse_dense loop)
  * reference_forward_torch               models/lightgcn.py:37-59 as torch CPU ops (the
                                           reference's own algorithm; timed as cpu_baseline)
  * evaluate            main.py:404-439   Recall@K / NDCG@K with the -1e10 train mask and topk

Pinning: tests/test_oracle_golden.py checks all of them against tests/golden/*.npz, which
tests/golden/gen_golden.py produced by importing the reference itself (bitwise: sha1 of every
layer output, final embedding and gradient; the adjacency arrays; Recall/NDCG exactly).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liblgcn_oracle.so")
_lib = None


def build():
    """Compile oracle/lgcn_oracle.c with gcc (oracle/Makefile)."""
    subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
    return _SO


def _load():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(_HERE, "lgcn_oracle.c")
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(src):
        build()
    lib = ctypes.CDLL(_SO)
    p = ctypes.c_void_p
    i64 = ctypes.c_int64
    lib.oracle_spmm_coo.argtypes = [i64, p, p, p, i64, i64, p, p]
    lib.oracle_forward.argtypes = [i64, p, p, p, i64, i64, i64, p, p, p]
    lib.oracle_backward.argtypes = [i64, p, p, p, i64, i64, i64, p, p]
    lib.oracle_forward_f64.argtypes = [i64, p, p, p, i64, i64, i64, p, p]
    lib.oracle_spmm_rows.argtypes = [p, p, p, i64, p, i64, p, p]
    for f in (lib.oracle_spmm_coo, lib.oracle_forward, lib.oracle_backward,
              lib.oracle_forward_f64, lib.oracle_spmm_rows):
        f.restype = None
    _lib = lib
    return lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _coo(rows, cols, vals):
    return (np.ascontiguousarray(rows, dtype=np.int64), np.ascontiguousarray(cols, dtype=np.int64),
            np.ascontiguousarray(vals, dtype=np.float32))


# ----------------------------------------------------------------------------------------------
# main.py:282-336 — the normalised adjacency
# ----------------------------------------------------------------------------------------------
def build_norm_adj(train_user, train_item, U, I, B, ib_item=None, ib_brand=None, use_brand=True):
    """Return (rows int64, cols int64, vals float32, n_nodes) in the reference's stored order.

    main.py:283-311 edge list (both directions; item<->brand only with use_brand),
    :321 coo_matrix of ones (duplicates later summed), :326-329 rowsum^-1/2 in fp32 with inf->0,
    :330-331 D·A·D via scipy CSR products -> value = fp32((d_r * m) * d_c), entries sorted by
    (row, col) with duplicates merged, :334-336 int64 indices / fp32 values.
    """
    item_offset, brand_offset = U, U + I
    n = U + I + B
    u = np.asarray(train_user, dtype=np.int64)
    it = np.asarray(train_item, dtype=np.int64) + item_offset
    if use_brand:
        ibi = np.asarray(ib_item, dtype=np.int64) + item_offset
        ibb = np.asarray(ib_brand, dtype=np.int64) + brand_offset
        rows = np.concatenate([u, it, ibi, ibb])
        cols = np.concatenate([it, u, ibb, ibi])
    else:
        rows = np.concatenate([u, it])
        cols = np.concatenate([it, u])
    # rowsum of the ones matrix (duplicates counted), fp32 like scipy's float32 sum
    rowsum = np.bincount(rows, minlength=n).astype(np.float32)
    with np.errstate(divide="ignore"):
        dinv = np.power(rowsum, np.float32(-0.5))
    dinv[np.isinf(dinv)] = np.float32(0.0)
    key = rows * np.int64(n) + cols
    ukey, mult = np.unique(key, return_counts=True)       # sorted by (row, col), dup-merged
    r = ukey // n
    c = ukey % n
    vals = (dinv[r] * mult.astype(np.float32)) * dinv[c]
    return r.astype(np.int64), c.astype(np.int64), vals.astype(np.float32), n


# ----------------------------------------------------------------------------------------------
# models/lightgcn.py:40-54 (+ autograd) — C oracle
# ----------------------------------------------------------------------------------------------
def spmm(rows, cols, vals, n_rows, x):
    rows, cols, vals = _coo(rows, cols, vals)
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty((n_rows, x.shape[1]), np.float32)
    _load().oracle_spmm_coo(len(vals), _ptr(rows), _ptr(cols), _ptr(vals), n_rows, x.shape[1],
                            _ptr(x), _ptr(y))
    return y


def spmm_rows(rowptr, cols, vals, x, sel):
    """Rows `sel` of Â·X for a row-sorted COO given as CSR (rowptr int64 [n+1] over the stored
    order): each row is the same sequential fmaf chain `spmm` runs for it."""
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    cols = np.ascontiguousarray(cols, dtype=np.int64)
    vals = np.ascontiguousarray(vals, dtype=np.float32)
    x = np.ascontiguousarray(x, dtype=np.float32)
    sel = np.ascontiguousarray(sel, dtype=np.int64)
    assert sel.size == 0 or (sel.min() >= 0 and sel.max() < rowptr.size - 1)
    y = np.empty((sel.size, x.shape[1]), np.float32)
    _load().oracle_spmm_rows(_ptr(rowptr), _ptr(cols), _ptr(vals), x.shape[1], _ptr(x), sel.size,
                             _ptr(sel), _ptr(y))
    return y


def forward(rows, cols, vals, e0, K, return_layers=False):
    """final = mean(E0..EK); optionally also [E1..EK]."""
    rows, cols, vals = _coo(rows, cols, vals)
    e0 = np.ascontiguousarray(e0, dtype=np.float32)
    n, d = e0.shape
    out = np.empty_like(e0)
    layers = np.empty((K, n, d), np.float32) if return_layers else None
    _load().oracle_forward(len(vals), _ptr(rows), _ptr(cols), _ptr(vals), n, d, K, _ptr(e0),
                           _ptr(out), _ptr(layers))
    return (out, layers) if return_layers else out


def backward(rows, cols, vals, g, K):
    """dE0 for an upstream gradient g of the final embeddings."""
    rows, cols, vals = _coo(rows, cols, vals)
    g = np.ascontiguousarray(g, dtype=np.float32)
    n, d = g.shape
    out = np.empty_like(g)
    _load().oracle_backward(len(vals), _ptr(rows), _ptr(cols), _ptr(vals), n, d, K, _ptr(g),
                            _ptr(out))
    return out


def forward_f64(rows, cols, vals, e0, K):
    """fp64 arbiter of the forward (row-sorted COO): exact-arithmetic yardstick, not a restatement."""
    rows, cols, vals = _coo(rows, cols, vals)
    e0 = np.ascontiguousarray(e0, dtype=np.float32)
    n, d = e0.shape
    out = np.empty((n, d), np.float64)
    _load().oracle_forward_f64(len(vals), _ptr(rows), _ptr(cols), _ptr(vals), n, d, K, _ptr(e0),
                               _ptr(out))
    return out


def reference_forward_torch(adj, ego, K, layer_times=None):
    """models/lightgcn.py:41-54 with torch CPU ops, exactly as the reference runs them.
    layer_times: optional list that receives each torch.sparse.mm's wall seconds."""
    import time
    import torch
    with torch.no_grad():
        all_e = [ego]
        x = ego
        for _ in range(K):
            t0 = time.perf_counter()
            x = torch.sparse.mm(adj, x)
            if layer_times is not None:
                layer_times.append(time.perf_counter() - t0)
            all_e.append(x)
        return torch.mean(torch.stack(all_e, dim=0), dim=0)


# ----------------------------------------------------------------------------------------------
# main.py:404-439 — Recall@K / NDCG@K
# ----------------------------------------------------------------------------------------------
def evaluate(user_emb, item_emb, val_user, val_item, train_user, train_item, k, batch_size=1024):
    import torch
    user_emb = torch.as_tensor(np.asarray(user_emb, dtype=np.float32))
    item_emb = torch.as_tensor(np.asarray(item_emb, dtype=np.float32))
    test_user_items = dict(zip(np.asarray(val_user).tolist(), np.asarray(val_item).tolist()))
    train_map = {}
    for uu, ii in zip(np.asarray(train_user).tolist(), np.asarray(train_item).tolist()):
        train_map.setdefault(uu, []).append(ii)
    users = list(test_user_items.keys())
    recalls, ndcgs = [], []
    with torch.no_grad():
        for i in range(0, len(users), batch_size):
            bu = users[i:i + batch_size]
            scores = torch.matmul(user_emb[torch.LongTensor(bu)], item_emb.T)
            for j, uu in enumerate(bu):
                if uu in train_map:
                    scores[j, train_map[uu]] = -1e10
            _, top = torch.topk(scores, k=k)
            top = top.numpy()
            for j, uu in enumerate(bu):
                pred, true = top[j], test_user_items[uu]
                hit = true in pred
                recalls.append(1 if hit else 0)
                ndcgs.append(1 / np.log2(np.where(pred == true)[0][0] + 2) if hit else 0)
    return float(np.mean(recalls)), float(np.mean(ndcgs))
