"""Host-side graph construction: the reference's normalised adjacency (main.py:282-336) and the
synthetic interaction generators for BASELINE.json's configs.

`build_norm_adj` produces the same `torch.sparse_coo_tensor` the reference passes to the model
(bitwise: same stored order, same fp32 values), vectorised with numpy instead of scipy so it
scales to the Books-size graphs. Checked against the reference-built Â in
tests/test_graph_builder.py (golden fixtures).
"""
import numpy as np
import torch


def edge_lists(train_user, train_item, U, I, ib_item=None, ib_brand=None, use_brand=True):
    """main.py:283-311 — both directions of user<->item (+ item<->brand with use_brand)."""
    item_offset, brand_offset = U, U + I
    u = np.asarray(train_user, dtype=np.int64)
    it = np.asarray(train_item, dtype=np.int64) + item_offset
    if use_brand:
        ibi = np.asarray(ib_item, dtype=np.int64) + item_offset
        ibb = np.asarray(ib_brand, dtype=np.int64) + brand_offset
        return np.concatenate([u, it, ibi, ibb]), np.concatenate([it, u, ibb, ibi])
    return np.concatenate([u, it]), np.concatenate([it, u])


def normalise(rows, cols, n):
    """main.py:313-331: ones -> duplicate-merged multiplicity m, rowsum in fp32, d = rowsum^-1/2
    (inf -> 0), value fp32((d_r * m) * d_c); entries ordered by (row, col)."""
    rowsum = np.bincount(rows, minlength=n).astype(np.float32)
    with np.errstate(divide="ignore"):
        dinv = np.power(rowsum, np.float32(-0.5))
    dinv[np.isinf(dinv)] = np.float32(0.0)
    key = rows * np.int64(n) + cols
    key.sort(kind="stable")
    if key.size:
        start = np.concatenate([[True], key[1:] != key[:-1]])
        ukey = key[start]
        mult = np.diff(np.concatenate([np.nonzero(start)[0], [key.size]]))
    else:
        ukey = key
        mult = np.zeros(0, np.int64)
    r = ukey // n
    c = ukey - r * n
    vals = (dinv[r] * mult.astype(np.float32)) * dinv[c]
    return r, c, vals.astype(np.float32)


def build_norm_adj(train_user, train_item, U, I, B, ib_item=None, ib_brand=None, use_brand=True,
                   device="cpu"):
    """The reference's `norm_adj_tensor` (main.py:282-336) as a torch sparse COO on `device`."""
    n = U + I + B
    rows, cols = edge_lists(train_user, train_item, U, I, ib_item, ib_brand, use_brand)
    r, c, v = normalise(rows, cols, n)
    idx = torch.from_numpy(np.vstack((r, c)))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(v), torch.Size((n, n))).to(device)


def build_norm_adj_device(train_user, train_item, U, I, B, ib_item=None, ib_brand=None,
                          use_brand=True, device="cuda"):
    """main.py:282-336 on the HIP device: the same `norm_adj_tensor`
    (bitwise: stored order, duplicate merge, fp32 values) as build_norm_adj, plus the engine's
    CSR plan attached to it, so the first model call does no conversion.

    Device work: degree histogram (integer atomics), 64-bit radix sort of row*n+col keys,
    run-length encode (multiplicity m), values fp32((d_r*m)*d_c), COO + CSR in one pass.
    Host work: the edge-list concat (main.py:300-311) and d = rowsum^-1/2 with numpy's float32
    power (main.py:326-329) — numpy's power is not correctly rounded, so only numpy reproduces
    the reference's d bitwise; it is N floats, the rest is O(nnz) on the device.
    """
    import ctypes
    from . import engine
    lib = engine.load_library()
    dev = torch.device(device)
    n = U + I + B
    rows, cols = edge_lists(train_user, train_item, U, I, ib_item, ib_brand, use_brand)
    ne = int(rows.size)
    if n > engine.INT32_MAX - 1 or ne > engine.INT32_MAX:
        raise engine.LgcnError("graph too large for int32 CSR")
    P = engine._ptr
    with torch.cuda.device(dev):
        st = engine._stream(dev)
        r_d = torch.from_numpy(rows).to(dev)
        c_d = torch.from_numpy(cols).to(dev)
        m = max(ne, 1)
        keys_a = torch.empty(m, dtype=torch.int64, device=dev)
        keys_b = torch.empty(m, dtype=torch.int64, device=dev)
        uniq = torch.empty(m, dtype=torch.int64, device=dev)
        counts = torch.empty(m, dtype=torch.int32, device=dev)
        n_unique = torch.zeros(1, dtype=torch.int32, device=dev)
        nbytes = ctypes.c_size_t(0)
        engine._check(lib.lgcn_adj_sort_unique(P(r_d), P(c_d), ne, n, P(keys_a), P(keys_b),
                                               P(uniq), P(counts), P(n_unique), None,
                                               ctypes.byref(nbytes), st), "lgcn_adj_sort_unique")
        temp = torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=dev)
        engine._check(lib.lgcn_adj_sort_unique(P(r_d), P(c_d), ne, n, P(keys_a), P(keys_b),
                                               P(uniq), P(counts), P(n_unique), P(temp),
                                               ctypes.byref(nbytes), st), "lgcn_adj_sort_unique")
        del temp, keys_a, r_d, c_d
        deg = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        engine._check(lib.lgcn_adj_degree(P(keys_b), ne, n, P(deg), st), "lgcn_adj_degree")
        rowsum = deg[:n].cpu().numpy().astype(np.float32)
        with np.errstate(divide="ignore"):
            dinv = np.power(rowsum, np.float32(-0.5))
        dinv[np.isinf(dinv)] = np.float32(0.0)
        dinv_d = torch.from_numpy(dinv).to(dev)
        del keys_b
        nnz = int(n_unique.item())
        idx = torch.empty((2, max(nnz, 1)), dtype=torch.int64, device=dev)
        vals = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
        rowptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
        edges = torch.empty(max(nnz, 1), dtype=torch.int64, device=dev)
        engine._check(lib.lgcn_adj_finish(P(uniq), P(counts), nnz, n, P(dinv_d), P(idx[0]),
                                          P(idx[1]), P(vals), P(rowptr), P(edges), st),
                      "lgcn_adj_finish")
        idx, vals = idx[:, :nnz], vals[:nnz]
        adj = torch.sparse_coo_tensor(idx, vals, (n, n))
        # users and brands link only to items (main.py:295-311): the item rows are one side
        sides = (U, U + I)
        g = engine._finish_graph(lib, adj._indices()[0], adj._indices()[1], adj._values(), rowptr,
                                 edges, n, nnz, dev, st, cols_sorted=True, sides=sides)
    return engine.attach_graph(adj, g, sides)


# ----------------------------------------------------------------------------------------------
# synthetic interactions (BASELINE.json configs)
# ----------------------------------------------------------------------------------------------
def uniform_interactions(U, I, E, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, U, E), rng.integers(0, I, E)


def _zipf_draw(rng, n_cat, alpha, size):
    """Draw `size` category ids with P(rank k) ∝ (k+1)^-alpha; ranks map to a random id order."""
    w = np.power(np.arange(1, n_cat + 1, dtype=np.float64), -alpha)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    ranks = np.searchsorted(cdf, rng.random(size), side="right")
    ranks = np.minimum(ranks, n_cat - 1)
    perm = rng.permutation(n_cat)
    return perm[ranks]


def powerlaw_interactions(U, I, E, seed, item_alpha=1.1, user_alpha=0.6):
    """Power-law bipartite interactions: item popularity is rank-Zipf(item_alpha) (SURVEY §8d:
    a≈1.1); every user has >= 1 interaction and the remaining E-U are spread by
    rank-Zipf(user_alpha) activity. Ids are randomly permuted (no popularity/id correlation)."""
    rng = np.random.default_rng(seed)
    base = rng.permutation(U)[:min(U, E)]
    extra = E - base.size
    users = np.concatenate([base, _zipf_draw(rng, U, user_alpha, extra)]) if extra > 0 else base
    items = _zipf_draw(rng, I, item_alpha, users.size)
    order = rng.permutation(users.size)
    return users[order], items[order]


def books_shape(scale=1.0):
    """Amazon Reviews 2023 Books (public card): ≈10.3M users, ≈4.4M items, ≈29.5M ratings."""
    return int(10_300_000 * scale), int(4_400_000 * scale), int(29_500_000 * scale)
