"""GPU parity of the bipartite two-lane schedule (lgcn_propagate_forward_sides / _backward_sides,
gcn_recommendation_amd/csrc/lgcn_engine.hip): the reference graph links users and brands only to
items (main.py:295-311), so every layer runs as two half-layers — the item rows and the rest — on
two lanes, the walks of the longest item rows of consecutive layers side by side.

Bar: BITWISE against the oracle's sequential fmaf chain (models/lightgcn.py:45's torch.sparse.mm
on CPU), forward and backward, with hub rows on both sides (brand rows are the side-0 hubs), for
every stream budget: two lanes with their own aux streams (7), a lane without aux streams (4),
both lanes on one stream set (3), no schedule at all; and through autograd (propagate_blocks) and
a captured HIP graph."""
import numpy as np
import pytest
import torch

from gcn_recommendation_amd import engine
from oracle import oracle

from test_gpu_exact import _adj, _e0

pytestmark = pytest.mark.gpu

U, I, B = 40_000, 3_000, 200


def _brand_graph(rng, n_inter=200_000):
    """Zipf item popularity (item hubs up to ~25k edges: walked) and Zipf brand sizes (brand rows
    of several hundred items: side-0 hubs)."""
    p = 1.0 / np.arange(1, I + 1) ** 1.1
    items = rng.choice(I, n_inter, p=p / p.sum())
    users = rng.integers(0, U, n_inter)
    pb = 1.0 / np.arange(1, B + 1) ** 1.1
    ib_item = np.arange(I)
    ib_brand = rng.choice(B, I, p=pb / pb.sum())
    return oracle.build_norm_adj(users, items, U, I, B, ib_item, ib_brand, use_brand=True)


@pytest.fixture(scope="module")
def brand_graph():
    rng = np.random.default_rng(21)
    return _brand_graph(rng)


def _segs(x, dev):
    return [torch.from_numpy(np.ascontiguousarray(a)).to(dev)
            for a in (x[:U], x[U:U + I], x[U + I:])]


KW = dict(hub_threshold=128, hub_mode="exact", emu_min=256)


@pytest.mark.parametrize("n_aux", [7, 4, 3, 0])
@pytest.mark.parametrize("kind", ["xavier", "few_bits"])
def test_sides_bitwise(gpu_device, monkeypatch, brand_graph, n_aux, kind):
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    if n_aux == 0:
        monkeypatch.setenv("LGCN_EMU_OVERLAP", "0")
    else:
        monkeypatch.setenv("LGCN_AUX_STREAMS", str(n_aux))
    r, c, v, n = brand_graph
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device), sides=(U, U + I))
    assert g.split == n - I and g.sides == (U, U + I)
    ids = g.row_ids.cpu().numpy()
    assert ((ids[g.split:] >= U) & (ids[g.split:] < U + I)).all()
    hps = g.side_hubs(128, mode="exact", emu_min=256)
    assert hps[1].n_emu_rows >= 5 and hps[0].n_emu_rows >= 1   # item and brand hubs
    rng = np.random.default_rng(5)
    e0 = _e0(rng, kind, n, 64)
    x = _segs(e0, gpu_device)
    for K in (1, 2, 3):
        want = oracle.forward(r, c, v, e0, K)
        got = engine.propagate_forward(g, x, K, **KW).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (kind, K)
    G = _e0(rng, "xavier", n, 64)
    G[rng.random(n) > 0.05] = 0.0   # a BPR batch's row-sparse gradient
    for K in (1, 3):
        want_b = oracle.backward(r, c, v, G, K)
        for sparse in ("off", "on"):
            got_b = engine.propagate_backward(g, _segs(G, gpu_device), K, sparse=sparse,
                                              **KW).cpu().numpy()
            assert np.array_equal(got_b.view(np.uint32), want_b.view(np.uint32)), (K, sparse)


def test_sides_autograd_and_capture(gpu_device, monkeypatch, brand_graph):
    """The model's entry (propagate_blocks: sides from the segment sizes) forward + autograd
    backward, and the forward captured in a HIP graph on the two lanes (the caller's stream, its
    3 aux streams and lane 1's main stream forked and joined)."""
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    monkeypatch.setenv("LGCN_AUX_STREAMS", "7")
    r, c, v, n = brand_graph
    adj = _adj(r, c, v, n, gpu_device)
    rng = np.random.default_rng(8)
    e0 = _e0(rng, "xavier", n, 64)
    w = [t.clone().requires_grad_(True) for t in _segs(e0, gpu_device)]
    out = engine.propagate_blocks(adj, w, 3, hub_threshold=128)
    g = engine.graph_from_coo(adj, sides=(U, U + I))
    assert g.split is not None
    want = oracle.forward(r, c, v, e0, 3)
    got = torch.cat([o.detach() for o in out]).cpu().numpy()
    assert np.array_equal(got, want)
    G = _e0(rng, "xavier", n, 64)
    torch.autograd.backward(list(out), _segs(G, gpu_device))
    got_b = torch.cat([t.grad for t in w]).cpu().numpy()
    assert np.array_equal(got_b, oracle.backward(r, c, v, G, 3))
    x = [t.detach() for t in w]
    cap = engine.CapturedForward(g, x, 3, hub_threshold=128)
    # the capture ran the two lanes (lane 1 without its own aux streams: make_lanes' rule)
    assert engine.last_schedule == {"sided": True, "aux_streams": 7, "lanes": 2, "captured": True}
    for _ in range(2):
        assert np.array_equal(cap.replay().cpu().numpy(), want)


def test_sides_refused_when_not_bipartite(gpu_device, monkeypatch):
    """An edge inside one side (user-user) keeps the one-operator schedule: same bits."""
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    rng = np.random.default_rng(2)
    users = rng.integers(0, 500, 5_000)
    items = rng.integers(0, 50, 5_000)
    r, c, v, n = oracle.build_norm_adj(users, items, 500, 50, 0, use_brand=False)
    r = np.concatenate([r, [0, 1]])
    c = np.concatenate([c, [1, 0]])
    v = np.concatenate([v, np.float32([0.5, 0.5])])
    o = np.lexsort((c, r))
    r, c, v = r[o], c[o], v[o]
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device), sides=(500, 550))
    assert g.split is None
    e0 = _e0(rng, "xavier", n, 16)
    got = engine.propagate_forward(g, [torch.from_numpy(e0).to(gpu_device)], 2,
                                   **KW).cpu().numpy()
    assert np.array_equal(got, oracle.forward(r, c, v, e0, 2))


@pytest.mark.parametrize("P", [2, 8])
def test_featsplit_shards_on_two_lanes(gpu_device, monkeypatch, brand_graph, P):
    """dist.FeatSplitPlan with the item rows as sides (what bench.py --gpus P runs per rank): the
    slot-space operator stays side-major, every rank's d/P columns propagate on the two-lane
    schedule (d/P = 8 at P = 8: the chain kernel's 8-column slices), forward and backward
    bitwise against the oracle per column block."""
    from gcn_recommendation_amd import dist as D
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    r, c, v, n = brand_graph
    d, K = 64, 3
    rowptr = np.searchsorted(r, np.arange(n + 1)).astype(np.int32)
    plan = D.FeatSplitPlan(rowptr, c, v, n, gpu_device, sides=(U, U + I))
    assert plan.graph.split is not None and plan.sides == (U, U + I)
    plan.attach_transpose(rowptr, c, v)
    assert plan.graph.transpose.split is not None
    rng = np.random.default_rng(31)
    e0 = _e0(rng, "xavier", n, d)
    segs = [torch.from_numpy(e0)]
    want = oracle.forward(r, c, v, e0, K)
    G = _e0(rng, "xavier", n, d)
    want_g = oracle.backward(r, c, v, G, K)
    cols, cols_b = [], []
    for p in range(P):
        x, (c0, c1) = plan.shard(segs, P, p)
        assert c1 - c0 == d // P
        cols.append(plan.unshard(plan.forward(x, K, 128, hub_mode="exact")).cpu().numpy())
        gs = torch.from_numpy(np.ascontiguousarray(G[:, c0:c1])).to(gpu_device)[plan.perm]
        cols_b.append(plan.unshard(plan.backward(gs.contiguous(), K, 128, sparse="off"))
                      .cpu().numpy())
    assert np.array_equal(np.concatenate(cols, 1), want)
    assert np.array_equal(np.concatenate(cols_b, 1), want_g)


def test_default_environment_runs_two_lanes(gpu_device, monkeypatch, brand_graph):
    """What main.py gets (models/lightgcn.py forward under HIP's default hardware queues, no
    LGCN_* stream knob): the drop-in forward runs the two-lane schedule with 7 aux streams (the
    second lane's high-priority streams take their own queue pool), bitwise."""
    import os
    monkeypatch.delenv("LGCN_AUX_STREAMS", raising=False)
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    assert os.environ.get("GPU_MAX_HW_QUEUES") in (None, "", "4"), "not the default environment"
    assert engine.n_aux_streams() == 7
    r, c, v, n = brand_graph
    adj = _adj(r, c, v, n, gpu_device)
    e0 = _e0(np.random.default_rng(12), "xavier", n, 64)
    w = _segs(e0, gpu_device)
    out = engine.propagate_blocks(adj, w, 3, hub_threshold=128)
    assert engine.last_schedule == {"sided": True, "aux_streams": 7, "lanes": 2,
                                    "captured": False}
    got = torch.cat([o.detach() for o in out]).cpu().numpy()
    assert np.array_equal(got, oracle.forward(r, c, v, e0, 3))
