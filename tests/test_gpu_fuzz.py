"""Seeded fuzz of the HIP propagation against the oracle (the reference's CPU arithmetic):
random sizes (1..4000 rows), widths (d = 1..256, aligned and not), depths (K = 0..4), COO
shapes (symmetric row-sorted like main.py's Â, unsorted with duplicate coordinates, skewed with
hub rows, mostly-empty rows), both storage orders, single-row and bundled lane groups. The plain
chain mode and the default exact hub plan (long rows as whole-row chains, longer rows emulated by
blocks — thresholds lowered so these small graphs exercise both) must be bitwise for the forward
and the backward (dense and row-sparse upstream gradients); the optional hub chunking must stay
within the north_star tolerance."""
import numpy as np
import pytest
import torch

from gcn_recommendation_amd import engine
from oracle import oracle
from util import assert_close_normwise

pytestmark = pytest.mark.gpu

N_CASES = 24
DIMS = [1, 2, 3, 4, 8, 12, 16, 20, 32, 64, 96, 128, 256]


def _coo(rng, kind, n):
    nnz = int(rng.integers(0, 12 * n + 1))
    if kind == 2:    # skewed: a few hub columns/rows
        hubs = rng.integers(0, n, max(1, n // 200))
        r = rng.integers(0, n, nnz)
        c = np.where(rng.random(nnz) < 0.5, rng.choice(hubs, nnz), rng.integers(0, n, nnz))
    elif kind == 3:  # most rows empty
        live = rng.choice(n, max(1, n // 10), replace=False)
        r, c = rng.choice(live, nnz), rng.choice(live, nnz)
    else:
        r, c = rng.integers(0, n, nnz), rng.integers(0, n, nnz)
    v = rng.standard_normal(nnz).astype(np.float32)
    if kind in (0, 2, 3):  # the reference's layout: symmetric values, row-sorted, unique
        r, c = np.concatenate([r, c]), np.concatenate([c, r])
        key = np.unique(r * n + c)
        r, c = key // n, key % n
        lo = np.minimum(r, c) * n + np.maximum(r, c)
        _, inv = np.unique(lo, return_inverse=True)
        v = rng.standard_normal(inv.max() + 1 if inv.size else 0).astype(np.float32)[inv]
    return r, c, v    # kind 1: unsorted, duplicates kept (torch sums them in stored order)


@pytest.mark.parametrize("case", range(N_CASES))
def test_fuzz_forward_backward(gpu_device, monkeypatch, case):
    rng = np.random.default_rng(5000 + case)
    kind = case % 4
    n = int(rng.integers(1, 4001))
    d = int(rng.choice(DIMS))
    K = int(rng.integers(0, 5))
    monkeypatch.setenv("LGCN_ROW_ORDER", "degree" if case % 2 == 0 else "stored")
    r, c, v = _coo(rng, kind, n)
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([r, c]).astype(np.int64)),
                                  torch.from_numpy(v), (n, n)).to(gpu_device)
    g = engine.graph_from_coo(adj)
    e0 = rng.standard_normal((n, d)).astype(np.float32)
    G = rng.standard_normal((n, d)).astype(np.float32)
    x = [torch.from_numpy(e0).to(gpu_device)]
    lib = engine.load_library()
    old = lib.lgcn_tune(engine.TUNE_MIN_GROUPS, 1 if case % 3 == 0 else 0)  # force bundles
    try:
        want = oracle.forward(r, c, v, e0, K)
        got = engine.propagate_forward(g, x, K, hub_threshold=engine.INT32_MAX).cpu().numpy()
        assert np.array_equal(got, want), (case, n, d, K, kind)
        want_b = oracle.backward(r, c, v, G, K)
        got_b = engine.propagate_backward(g, torch.from_numpy(G).to(gpu_device), K,
                                          engine.INT32_MAX, sparse="off").cpu().numpy()
        assert np.array_equal(got_b, want_b), (case, "backward")
        # a row-sparse upstream gradient through the masked path: same bits as the oracle
        Gs = np.zeros_like(G)
        live = rng.choice(n, max(1, n // 50), replace=False)
        Gs[live] = G[live]
        got_s = engine.propagate_backward(g, torch.from_numpy(Gs).to(gpu_device), K,
                                          engine.INT32_MAX, sparse="on").cpu().numpy()
        assert np.array_equal(got_s, oracle.backward(r, c, v, Gs, K)), (case, "sparse backward")
        # the default exact hub plan with low thresholds: rows above 8 edges are whole-row
        # chains, above 16 emulated — bitwise, forward and both backward paths
        kw = dict(hub_threshold=8, hub_mode="exact", emu_min=16)
        got = engine.propagate_forward(g, x, K, **kw).cpu().numpy()
        assert np.array_equal(got, want), (case, "exact plan forward")
        got_b = engine.propagate_backward(g, torch.from_numpy(G).to(gpu_device), K, sparse="off",
                                          **kw).cpu().numpy()
        assert np.array_equal(got_b, want_b), (case, "exact plan backward")
        got_s = engine.propagate_backward(g, torch.from_numpy(Gs).to(gpu_device), K, sparse="on",
                                          **kw).cpu().numpy()
        assert np.array_equal(got_s, oracle.backward(r, c, v, Gs, K)), (case, "exact sparse bwd")
        # optional hub chunking: deterministic and within the north_star tolerance
        f1 = engine.propagate_forward(g, x, K, hub_threshold=8, hub_mode="chunk").cpu().numpy()
        f2 = engine.propagate_forward(g, x, K, hub_threshold=8, hub_mode="chunk").cpu().numpy()
        assert np.array_equal(f1, f2)
        if want.size and np.abs(want).max() > 0:
            assert_close_normwise(f1, want, what=f"case {case} chunked")
    finally:
        lib.lgcn_tune(engine.TUNE_MIN_GROUPS, old)
