"""GPU parity of the bipartite two-lane schedule (lgcn_propagate_forward_sides / _backward_sides,
gcn_recommendation_amd/csrc/lgcn_engine.hip): the reference graph links users and brands only to
items (main.py:295-311), so every layer runs as two half-layers — the item rows and the rest — on
two lanes, the walks of the longest item rows of consecutive layers side by side.

Bar: BITWISE against the oracle's sequential fmaf chain (models/lightgcn.py:45's torch.sparse.mm
on CPU), forward and backward, with hub rows on both sides (brand rows are the side-0 hubs), for
every stream budget: two lanes with their own aux streams (7), a lane without aux streams (4),
both lanes on one stream set (3), no schedule at all; and through autograd (propagate_blocks) and
a captured HIP graph. The side-0 classes (lgcn_csr_side_classes: users linked to the walked
item rows of part 0 / part 1 / neither) and the dependency schedule built on them are checked
with all three classes populated, and with classes off (graph and schedule)."""
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


def _classes_env(monkeypatch, classes):
    """Walk cuts small enough for the brand graph to have all three side-0 classes: part 0 =
    item rows of more than 40 blocks (~10k edges), part 1 = more than 8 (2048-edge chain cut)."""
    monkeypatch.setenv("LGCN_EMU_PART0", "40")
    monkeypatch.setenv("LGCN_CHAIN_MAX", "2048")
    monkeypatch.setenv("LGCN_CLASSES", "0" if classes == "graph_off" else "1")
    if classes == "graph_off":
        monkeypatch.setenv("LGCN_CLASSES", "0")
    if classes == "sched_off":
        monkeypatch.setenv("LGCN_SCHED_CLASSES", "0")


def _check_classes(g, r, c, n, both=False):
    """The class-major slot order: side 0 = users + brands in classes 0 / 1 / 2 by the walked
    item rows they link to, each class degree-descending; side 1 untouched. both: linked in
    either direction (an operator that is not structurally symmetric)."""
    ids = g.row_ids.cpu().numpy()
    rp = g.rowptr_host().astype(np.int64)
    deg = np.diff(rp)
    c0, c1 = g.class_end
    p0, p01 = g.class_parts
    assert 0 < c0 < c1 < g.split and 0 < p0 < p01   # every class populated
    part = {int(x): (0 if k < p0 else 1) for k, x in enumerate(ids[g.split:g.split + p01])}
    for cls, (a, b) in enumerate(((0, c0), (c0, c1), (c1, g.split))):
        assert (np.diff(deg[a:b]) <= 0).all()
        for s_ in range(a, b, max(1, (b - a) // 200)):   # a sample of each class
            row = ids[s_]
            nb = c[np.searchsorted(r, row):np.searchsorted(r, row + 1)]
            if both:
                nb = np.concatenate([nb, r[c == row]])
            got = min([part[int(x)] for x in nb if int(x) in part], default=2)
            assert got == cls, (s_, row, got, cls)


@pytest.mark.parametrize("n_aux", [7, 4, 3, 0])
@pytest.mark.parametrize("kind", ["xavier", "few_bits"])
@pytest.mark.parametrize("classes", ["on", "graph_off", "sched_off"])
def test_sides_bitwise(gpu_device, monkeypatch, brand_graph, n_aux, kind, classes):
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    if n_aux == 0:
        monkeypatch.setenv("LGCN_EMU_OVERLAP", "0")
    else:
        monkeypatch.setenv("LGCN_AUX_STREAMS", str(n_aux))
    _classes_env(monkeypatch, classes)
    r, c, v, n = brand_graph
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device), sides=(U, U + I))
    assert g.split == n - I and g.sides == (U, U + I)
    ids = g.row_ids.cpu().numpy()
    assert ((ids[g.split:] >= U) & (ids[g.split:] < U + I)).all()
    assert ((ids[:g.split] < U) | (ids[:g.split] >= U + I)).all()
    assert np.array_equal(np.sort(ids), np.arange(n))
    if classes == "graph_off":
        assert g.class_end in (None, (g.split, g.split))
    else:
        _check_classes(g, r, c, n)
    hps = g.side_hubs(128, mode="exact", emu_min=256)
    assert hps[3].n_emu_rows >= 5 and sum(h.n_emu_rows for h in hps[:3]) >= 1  # item, brand hubs
    rng = np.random.default_rng(5)
    e0 = _e0(rng, kind, n, 64)
    x = _segs(e0, gpu_device)
    for K in (1, 2, 3, 4):
        want = oracle.forward(r, c, v, e0, K)
        got = engine.propagate_forward(g, x, K, **KW).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (kind, K)
        if n_aux:  # the library reports what it ran
            assert engine.last_schedule["lanes"] == (2 if n_aux >= 4 else 1)
            assert engine.last_schedule["classes"] == (classes == "on" and n_aux > 0)
    G = _e0(rng, "xavier", n, 64)
    G[rng.random(n) > 0.05] = 0.0   # a BPR batch's row-sparse gradient
    for K in (1, 3, 4):
        want_b = oracle.backward(r, c, v, G, K)
        for sparse in ("off", "on"):
            got_b = engine.propagate_backward(g, _segs(G, gpu_device), K, sparse=sparse,
                                              **KW).cpu().numpy()
            assert np.array_equal(got_b.view(np.uint32), want_b.view(np.uint32)), (K, sparse)


def test_classes_directed_operator(gpu_device, monkeypatch, brand_graph):
    """the side-0 classes of an operator that is bipartite but not structurally
    symmetric. Half of the item -> user edges are dropped, so many users read a walked item row
    that does not read them; lgcn_csr_side_classes marks classes from both directions, and the
    class schedule (classes on, two lanes with their aux streams) stays bitwise."""
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    monkeypatch.setenv("LGCN_AUX_STREAMS", "7")
    _classes_env(monkeypatch, "on")
    r, c, v, n = brand_graph
    rng = np.random.default_rng(3)
    drop = (r >= U) & (r < U + I) & (c < U) & (rng.random(r.size) < 0.5)
    r, c, v = r[~drop], c[~drop], v[~drop]
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device), sides=(U, U + I))
    assert g.split == n - I
    _check_classes(g, r, c, n, both=True)
    e0 = _e0(rng, "xavier", n, 64)
    for K in (2, 3):
        got = engine.propagate_forward(g, _segs(e0, gpu_device), K, **KW).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), oracle.forward(r, c, v, e0, K).view(np.uint32))
        assert engine.last_schedule["classes"]
    G = _e0(rng, "xavier", n, 64)
    got_b = engine.propagate_backward(g, _segs(G, gpu_device), 3, sparse="off", **KW)
    assert np.array_equal(got_b.cpu().numpy().view(np.uint32),
                          oracle.backward(r, c, v, G, 3).view(np.uint32))


def test_library_streams():
    """lgcn_stream_create: the schedule's own streams (not torch's pooled ones) at both
    priorities; torch work on them completes."""
    import ctypes
    lib = engine.load_library()
    dev = torch.device("cuda:0")
    for high in (0, 1):
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            assert lib.lgcn_stream_create(high, ctypes.byref(h)) == 0
        st = torch.cuda.ExternalStream(h.value, device=dev)
        with torch.cuda.stream(st):
            x = torch.arange(1 << 20, device=dev, dtype=torch.float32).sum()
        st.synchronize()
        assert float(x) == float((1 << 20) * ((1 << 20) - 1) // 2)
        assert lib.lgcn_stream_destroy(h) == 0


def test_backward_hint_ring(gpu_device, monkeypatch, brand_graph):
    """The backward's asynchronous live-row hints (engine._hint_*): 12 back-to-back calls (more
    than the ring's 8 slots in flight) on a dense G end with the dense decision, on a BPR-like G
    with the row-sparse one; every call bitwise either way."""
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    r, c, v, n = brand_graph
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device), sides=(U, U + I))
    rng = np.random.default_rng(13)
    G = _e0(rng, "xavier", n, 64)
    Gs = np.where(rng.random((n, 1)) < 0.01, G, 0.0).astype(np.float32)
    for Gx, dense in ((G, True), (Gs, False), (G, True)):
        want = oracle.backward(r, c, v, Gx, 3)
        segs = _segs(Gx, gpu_device)
        outs = [engine.propagate_backward(g, segs, 3, **KW) for _ in range(12)]
        torch.cuda.synchronize()
        for o in outs:
            assert np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32))
        assert engine._hint_dense(gpu_device, n) is dense


def test_sparse_backward_part0_cut(gpu_device, monkeypatch, brand_graph):
    """The row-sparse backward's own part-0 cut (engine.PART0_SPARSE_BACKWARD, 2048 blocks at
    C3; here 16 so that the brand graph's item hubs move from part 1 to part 0): once the hint
    ring says G is row-sparse the backward's plans take it, the dense calls keep the forward's
    cut, and every call is bitwise against the oracle."""
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    monkeypatch.setenv("LGCN_CHAIN_MAX", "2048")
    monkeypatch.setenv("LGCN_CLASSES", "0")
    monkeypatch.setattr(engine, "PART0_SPARSE_BACKWARD", 16)
    seen = []
    orig = engine._side_plans

    def spy(*a, **kw):
        seen.append(kw.get("part0"))
        return orig(*a, **kw)

    monkeypatch.setattr(engine, "_side_plans", spy)
    r, c, v, n = brand_graph
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device), sides=(U, U + I))
    hp = g.side_hubs(128, mode="exact", emu_min=256)[3]
    rows16, _ = hp.walk_parts(g.nnz, backward=True, part0=16)
    rows_fwd, _ = hp.walk_parts(g.nnz, backward=True)
    assert rows16[0] > rows_fwd[0] and rows16[1] == rows_fwd[1]  # the cut moves rows to part 0
    rng = np.random.default_rng(17)
    G = _e0(rng, "xavier", n, 64)
    Gs = np.where(rng.random((n, 1)) < 0.01, G, 0.0).astype(np.float32)
    for Gx in (Gs, G, Gs):
        want = oracle.backward(r, c, v, Gx, 3)
        segs = _segs(Gx, gpu_device)
        seen.clear()
        for _ in range(10):
            got = engine.propagate_backward(g, segs, 3, **KW)
            torch.cuda.synchronize()  # the hint of each call lands before the next
            assert np.array_equal(got.cpu().numpy().view(np.uint32), want.view(np.uint32))
        assert seen[-1] == (16 if Gx is Gs else None), seen


def test_lane1_shared_bitwise(gpu_device, monkeypatch, brand_graph):
    """LGCN_SCHED_LANE1_SHARED: lane 1 on the caller's stream and lane 0's aux streams reversed
    (two lanes of half-layers on three aux streams): forward and row-sparse / dense backward
    bitwise."""
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    sc = engine.Sched(gpu_device, 3, "backward", lane1_shared=True)
    monkeypatch.setattr(engine, "sched_for", lambda dev, n_aux=None, role="forward": sc)
    r, c, v, n = brand_graph
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device), sides=(U, U + I))
    rng = np.random.default_rng(12)
    e0 = _e0(rng, "xavier", n, 64)
    got = engine.propagate_forward(g, _segs(e0, gpu_device), 3, **KW).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), oracle.forward(r, c, v, e0, 3).view(np.uint32))
    assert (engine.last_schedule["lanes"], engine.last_schedule["lane1_aux"]) == (2, 3)
    G = _e0(rng, "xavier", n, 64)
    for frac in (0.03, 1.0):
        Gm = np.where(rng.random((n, 1)) < frac, G, 0.0).astype(np.float32)
        got_b = engine.propagate_backward(g, _segs(Gm, gpu_device), 3, **KW).cpu().numpy()
        assert np.array_equal(got_b.view(np.uint32), oracle.backward(r, c, v, Gm, 3).view(np.uint32))


def test_c_host_captures_full_schedule():
    """tools/capture_host.cpp (built by __graft_entry__.build() against liblgcn_engine.so; no torch
    in its process, /opt/rocm's HIP runtime): the two-lane forward and backward with lane 1's own
    aux streams, captured, instantiated and replayed bitwise equal to the eager calls."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                       "capture_host")
    if not os.path.exists(exe):
        pytest.skip("tools/capture_host not built (__graft_entry__.build())")
    env = {k: v for k, v in os.environ.items() if k != "LD_LIBRARY_PATH"}
    out = subprocess.run([exe, "3", "both"], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "lane-1 aux streams under the capture 3" in out.stdout, out.stdout
    assert "replays bitwise equal to eager" in out.stdout, out.stdout


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
    # the capture ran the two lanes; lane 1 keeps its own aux streams only on a HIP runtime that
    # captures the full schedule (>= 7.2; the torch wheel's 7.0 does not: DESIGN §4e)
    full = bool(engine.load_library().lgcn_capture_full_schedule())
    s = engine.last_schedule
    assert (s["lanes"], s["lane1_aux"], s["captured"], s["aux_streams"], s["capture_full"]) == \
        (2, 3 if full else 0, True, 7, full)
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
    if os.environ.get("GPU_MAX_HW_QUEUES") not in (None, "", "4"):
        pytest.skip("GPU_MAX_HW_QUEUES is set: not the default environment")
    assert engine.n_aux_streams() == 7
    r, c, v, n = brand_graph
    adj = _adj(r, c, v, n, gpu_device)
    e0 = _e0(np.random.default_rng(12), "xavier", n, 64)
    w = _segs(e0, gpu_device)
    out = engine.propagate_blocks(adj, w, 3, hub_threshold=128)
    s = engine.last_schedule
    assert (s["lanes"], s["lane1_aux"], s["captured"], s["aux_streams"]) == (2, 3, False, 7)
    got = torch.cat([o.detach() for o in out]).cpu().numpy()
    assert np.array_equal(got, oracle.forward(r, c, v, e0, 3))


@pytest.mark.parametrize("classes", ["on", "graph_off"])
def test_c_host_plans_sided_bitwise(gpu_device, monkeypatch, brand_graph, classes):
    """What a C host runs: plans from the C planner alone (lgcn_plan_items for
    the whole-row items, lgcn_plan_exact for the emulated / chain rows, lgcn_plan_scratch_bytes;
    tools/c_host_plans.py), the slot layout in lgcn_sides_t, one lgcn_propagate_forward_sides /
    _backward_sides call each — bitwise against the oracle and the Python binding."""
    import ctypes
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    from c_host_plans import c_host_side_plans
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    monkeypatch.setenv("LGCN_AUX_STREAMS", "7")
    _classes_env(monkeypatch, classes)
    r, c, v, n = brand_graph
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device), sides=(U, U + I))
    lib = engine.load_library()
    d, K = 64, 3
    chain_max = int(engine.chain_max_degree(g.nnz))   # (LGCN_CHAIN_MAX of _classes_env)
    plans, keep = c_host_side_plans(lib, g.rowptr_host(), g.row_ids_host(), g.segments(), g.nnz,
                                    d, gpu_device, emu_min=256, chain_max=chain_max)
    assert sum(plans[2 * s].n_items for s in range(4)) > 0       # whole-row items present
    assert plans[6].emu_part_rows[1] > 0                          # walked item rows
    rng = np.random.default_rng(23)
    e0 = _e0(rng, "xavier", n, d)
    x = _segs(e0, gpu_device)
    sides = g.sides_struct()
    sc = engine.sched_for(gpu_device)
    layers = [torch.empty((n, d), device=gpu_device) for _ in range(K - 1)]
    out = torch.empty((n, d), device=gpu_device)
    bufs = (ctypes.c_void_p * (K - 1))(*[t.data_ptr() for t in layers])
    P = engine._ptr
    st = engine._stream(gpu_device)
    rc = lib.lgcn_propagate_forward_sides(P(g.rowptr), P(g.edges), P(g.row_ids),
                                          ctypes.byref(sides), plans, engine.rows_desc(x, d), d, K,
                                          bufs, P(out), sc.handle, st)
    assert rc == 0
    want = oracle.forward(r, c, v, e0, K)
    assert np.array_equal(out.cpu().numpy(), want)
    assert torch.equal(out, engine.propagate_forward(g, x, K, hub_threshold=128, hub_mode="exact",
                                                     emu_min=256))
    gt = g.transpose
    G = _e0(rng, "xavier", n, d)
    plans_t, keep_t = c_host_side_plans(lib, gt.rowptr_host(), gt.row_ids_host(), gt.segments(),
                                        gt.nnz, d, gpu_device, emu_min=256, chain_max=chain_max)
    work = torch.empty((n, d), device=gpu_device)
    ge0 = torch.empty((n, d), device=gpu_device)
    sides_t = gt.sides_struct()
    rc = lib.lgcn_propagate_backward_sides(P(gt.rowptr), P(gt.edges), P(gt.row_ids),
                                           ctypes.byref(sides_t), plans_t,
                                           engine.rows_desc(_segs(G, gpu_device), d), None, d, K,
                                           P(work), P(ge0), sc.handle, st)
    assert rc == 0
    assert np.array_equal(ge0.cpu().numpy(), oracle.backward(r, c, v, G, K))


@pytest.mark.parametrize("defer", ["0", "1"])
@pytest.mark.parametrize("classes", ["on", "graph_off"])
def test_mean_epilogue_deferred(gpu_device, monkeypatch, brand_graph, defer, classes):
    """The final mean half-layers' walks and chains write their rows' sums to emu_out and the
    mean of those rows follows once the other lane's layer K-1 is done (LGCN_EMU_DEFER=1, the
    default), or they wait for it (0): bitwise either way, K = 2..4."""
    monkeypatch.setenv("LGCN_SIDES_MIN_NNZ", "0")
    monkeypatch.setenv("LGCN_AUX_STREAMS", "7")
    monkeypatch.setenv("LGCN_EMU_DEFER", defer)
    _classes_env(monkeypatch, classes)
    r, c, v, n = brand_graph
    g = engine.graph_from_coo(_adj(r, c, v, n, gpu_device), sides=(U, U + I))
    e0 = _e0(np.random.default_rng(29), "drift", n, 64)
    x = _segs(e0, gpu_device)
    for K in (2, 3, 4):
        got = engine.propagate_forward(g, x, K, **KW).cpu().numpy()
        assert np.array_equal(got, oracle.forward(r, c, v, e0, K)), K
