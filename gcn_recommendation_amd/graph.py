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
