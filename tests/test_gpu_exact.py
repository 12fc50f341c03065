"""GPU parity of the exact hub path — hub rows reproduced by block emulation, and the shorter
of them (<= 512 blocks) by the latency-hidden sequential chain (LGCN_CHAIN=1, the default;
both in gcn_recommendation_amd/csrc/lgcn_exact.hip) — against the oracle's sequential fmaf chain
(oracle/lgcn_oracle.c, the arithmetic of models/lightgcn.py:45's torch.sparse.mm on CPU).

Bar: BITWISE, forward and backward, for every input. The cases aim at the emulation's proof
obligations: random-walk accumulators that cross binades and zero (xavier E0), drifting
accumulators that climb many binades (biased E0), products with few mantissa bits (possible
exact ties), rows of mostly zero products (row-sparse G), huge dynamic range (subnormal and
near-overflow values), every width class and both storage orders."""
import numpy as np
import pytest
import torch

from gcn_recommendation_amd import engine
from oracle import oracle

pytestmark = pytest.mark.gpu


def _powerlaw(rng, U, I, n_inter):
    """Bipartite graph with Zipf item popularity (a few items hold most edges) + main.py's Â."""
    p = 1.0 / np.arange(1, I + 1) ** 1.1
    items = rng.choice(I, n_inter, p=p / p.sum())
    users = rng.integers(0, U, n_inter)
    r, c, v, n = oracle.build_norm_adj(users, items, U, I, 0, use_brand=False)
    return r, c, v, n


def _e0(rng, kind, n, d):
    b = np.sqrt(6.0 / (n + d))
    if kind == "xavier":
        return rng.uniform(-b, b, (n, d)).astype(np.float32)
    if kind == "drift":  # every column biased: accumulators climb through many binades
        return (rng.uniform(-b, b, (n, d)) * 0.3 + b * 0.5 * np.sign(np.arange(d) % 2 - 0.5)
                ).astype(np.float32)
    if kind == "few_bits":  # k/64: exact products, exact-tie candidates everywhere
        return (rng.integers(-32, 33, (n, d)) / 64.0).astype(np.float32)
    if kind == "range":  # subnormal to 1e30 magnitudes, sign flips
        mag = 10.0 ** rng.uniform(-40, 30, (n, d))
        return (mag * rng.choice([-1.0, 1.0], (n, d))).astype(np.float32)
    if kind == "sparse_rows":
        x = rng.standard_normal((n, d)).astype(np.float32)
        x[rng.random(n) > 0.01] = 0.0
        return x
    raise ValueError(kind)


def _adj(r, c, v, n, dev):
    return torch.sparse_coo_tensor(torch.from_numpy(np.vstack([r, c])), torch.from_numpy(v),
                                   (n, n)).to(dev)


@pytest.mark.parametrize("chain", ["1", "0"])
@pytest.mark.parametrize("order", ["degree", "stored"])
@pytest.mark.parametrize("kind", ["xavier", "drift", "few_bits", "range", "sparse_rows"])
def test_emulated_hubs_bitwise(gpu_device, monkeypatch, kind, order, chain):
    monkeypatch.setenv("LGCN_ROW_ORDER", order)
    monkeypatch.setenv("LGCN_CHAIN", chain)
    rng = np.random.default_rng(11)
    r, c, v, n = _powerlaw(rng, 40_000, 3_000, 200_000)
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device))
    d, K = 64, 3
    e0 = _e0(rng, kind, n, d)
    want = oracle.forward(r, c, v, e0, K)
    x = [torch.from_numpy(e0).to(gpu_device)]
    kw = dict(hub_threshold=128, hub_mode="exact", emu_min=512)
    assert g.hubs(128, mode="exact", emu_min=512).n_emu_rows >= 5
    got = engine.propagate_forward(g, x, K, **kw).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), kind
    G = _e0(rng, "sparse_rows" if kind == "sparse_rows" else "xavier", n, d)
    want_b = oracle.backward(r, c, v, G, K)
    for sparse in ("off", "on"):
        got_b = engine.propagate_backward(g, torch.from_numpy(G).to(gpu_device), K,
                                          sparse=sparse, **kw).cpu().numpy()
        assert np.array_equal(got_b.view(np.uint32), want_b.view(np.uint32)), (kind, sparse)


@pytest.mark.parametrize("chain", ["1", "0"])
@pytest.mark.parametrize("d", [1, 8, 12, 16, 32, 100, 128, 256])
def test_emulated_hubs_widths(gpu_device, monkeypatch, d, chain):
    monkeypatch.setenv("LGCN_CHAIN", chain)
    rng = np.random.default_rng(100 + d)
    r, c, v, n = _powerlaw(rng, 8_000, 600, 40_000)
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device))
    e0 = _e0(rng, "xavier", n, d)
    for K in (1, 2, 4):
        want = oracle.forward(r, c, v, e0, K)
        got = engine.propagate_forward(g, [torch.from_numpy(e0).to(gpu_device)], K,
                                       hub_threshold=64, hub_mode="exact", emu_min=256)
        assert np.array_equal(got.cpu().numpy(), want), (d, K)


@pytest.mark.parametrize("chain", ["1", "0"])
def test_one_giant_row(gpu_device, monkeypatch, chain):
    """A 300k-edge item row (1,172 blocks: several 64-block walker chunks), first block ragged
    by the planner's cut, plus a row of exactly 256 and 257 edges (sequential chains: one
    window + a partial one, and the ring's dummy windows past the row)."""
    monkeypatch.setenv("LGCN_CHAIN", chain)
    rng = np.random.default_rng(3)
    U = 300_000
    users = np.concatenate([np.arange(U), rng.integers(0, U, 256), rng.integers(0, U, 257),
                            rng.integers(0, U, 50_000)])
    items = np.concatenate([np.zeros(U, np.int64), np.ones(256, np.int64),
                            np.full(257, 2, np.int64), rng.integers(3, 2_000, 50_000)])
    r, c, v, n = oracle.build_norm_adj(users, items, U, 2_000, 0, use_brand=False)
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device))
    for kind in ("xavier", "drift"):
        e0 = _e0(rng, kind, n, 64)
        want = oracle.forward(r, c, v, e0, 3)
        got = engine.propagate_forward(g, [torch.from_numpy(e0).to(gpu_device)], 3,
                                       hub_threshold=128, hub_mode="exact", emu_min=255)
        assert np.array_equal(got.cpu().numpy(), want), kind


def test_exact_is_default_and_deterministic(gpu_device, monkeypatch):
    monkeypatch.delenv("LGCN_HUB_MODE", raising=False)
    monkeypatch.delenv("LGCN_HUB_THRESHOLD", raising=False)
    monkeypatch.setenv("LGCN_EMU_MIN_DEGREE", "300")
    rng = np.random.default_rng(5)
    r, c, v, n = _powerlaw(rng, 20_000, 1_000, 100_000)
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device))
    e0 = _e0(rng, "xavier", n, 64)
    x = [torch.from_numpy(e0).to(gpu_device)]
    a = engine.propagate_forward(g, x, 3).cpu().numpy()
    b = engine.propagate_forward(g, x, 3).cpu().numpy()
    assert g.hubs(engine.hub_threshold_from_env()).n_emu_rows > 0
    assert np.array_equal(a, b) and np.array_equal(a, oracle.forward(r, c, v, e0, 3))


@pytest.mark.parametrize("sides", [False, True])
def test_live_edge_chains_bpr_gradient(gpu_device, monkeypatch, sides):
    """The backward of a BPR batch's gradient (a few live rows): every emulated row of the first
    layer runs as a chain over its live edges (lgcn_live_rows: device compaction + chain kernel),
    bitwise the oracle's full chain — on a 300k-edge item row and power-law hubs, rows with no
    live edge at all included, on one operator and on the bipartite two-lane schedule."""
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "1")
    rng = np.random.default_rng(21)
    U, I = 300_000, 3_000
    users = np.concatenate([np.arange(U), rng.integers(0, U, 200_000)])
    p = 1.0 / np.arange(1, I) ** 1.1
    items = np.concatenate([np.zeros(U, np.int64), 1 + rng.choice(I - 1, 200_000, p=p / p.sum())])
    r, c, v, n = oracle.build_norm_adj(users, items, U, I, 0, use_brand=False)
    adj = _adj(r, c, v, n, gpu_device)
    g = engine.graph_from_coo(adj, sides=(U, U + I) if sides else None)
    assert (g.split is not None) == sides
    d, K = 64, 3
    G = np.zeros((n, d), np.float32)
    live_u = rng.integers(0, U, 2048)
    live_i = U + rng.integers(0, I, 4096)
    G[live_u] = rng.standard_normal((live_u.size, d)).astype(np.float32) * 1e-3
    G[live_i] = rng.standard_normal((live_i.size, d)).astype(np.float32) * 1e-3
    want = oracle.backward(r, c, v, G, K)
    gt = torch.from_numpy(G).to(gpu_device)
    kw = dict(hub_threshold=128, hub_mode="exact")
    got = engine.propagate_backward(g, gt, K, sparse="on", **kw).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    monkeypatch.setenv("LGCN_LIVE", "0")
    got0 = engine.propagate_backward(g, gt, K, sparse="on", **kw).cpu().numpy()
    assert np.array_equal(got0.view(np.uint32), want.view(np.uint32))
    # an all-zero gradient: every live-edge row is empty
    z = engine.propagate_backward(g, torch.zeros_like(gt), K, sparse="on", **kw)
    assert not bool(z.any())
