"""Multi-GPU LightGCN propagation on one node: one process per GPU, torch.distributed over RCCL
(backend "nccl" on ROCm) for the exchange steps, the HIP engine for every local layer.

Two decompositions of E_{k+1} = Â·E_k (models/lightgcn.py:44-46) over P ranks:

rowpart (north_star): Â's rows are cut into P contiguous blocks balanced by nnz + per-row cost;
    rank p owns rows [R_p, R_{p+1}) with global columns. Layer 1 gathers E0 (replicated
    parameters) in place; its output slice goes straight into the rank's chunk of a rank-major
    buffer [P * n_max x d] that one in-place all_gather_into_tensor completes; layers >= 2 read
    that buffer through column ids remapped to the padded layout once at plan time. The last
    layer's fused mean reads E0 and the local slices of E1..E_{K-1}; the final slice is
    all-gathered so every rank holds the full table, as the single-GPU forward returns it.
    Exchange per layer: (P-1)/P * N * d * 4 bytes per rank.

featsplit: every rank holds the whole CSR (0.45 GB at Books scale) and d/P embedding columns
    (column-parallel embedding tables); columns of an SpMM are independent, so the K layers
    need NO exchange. The output stays column-sharded; consumers reduce partial dot products
    (bpr_loss_featsplit: one all_reduce of B floats per loss).

On a CPU tensor the local layer is the reference's ATen op (used by the gloo tests of the
orchestration); a HIP tensor always runs the engine.
"""
import os

import numpy as np
import torch
import torch.distributed as dist

from . import engine


# ----------------------------------------------------------------------------------------------
# process group
# ----------------------------------------------------------------------------------------------
def init(device_type="cuda", backend=None):
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # LGCN_DIST_BACKEND=gloo rehearses the multi-process GPU path on a one-GPU box
    backend = backend or os.environ.get("LGCN_DIST_BACKEND") or (
        "nccl" if device_type == "cuda" else "gloo")
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend, **kw)
    return dist.get_rank(), dist.get_world_size()


def shutdown():
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


# ----------------------------------------------------------------------------------------------
# row partition planning (host)
# ----------------------------------------------------------------------------------------------
# a walked row (above the chain cut: block pass + walk, one wave per column) costs its rank
# ~20x a bandwidth-bound edge: the C3 2.77M-edge item row's walk takes ~3.0 ms alone while a layer
# kernel moves ~18 edges/ns
WALK_FACTOR = 20.0


def row_costs(deg, row_cost=4.0, walk_deg=None, walk_factor=WALK_FACTOR):
    """Per-row cost of a rank's exact-plan layer: nnz + row_cost for the rows the layer kernel
    and the chain kernel run, walk_factor x nnz for the walked rows (degree > walk_deg)."""
    deg = np.asarray(deg, dtype=np.float64)
    cost = deg + row_cost
    if walk_deg is not None:
        w = deg > walk_deg
        cost[w] = deg[w] * walk_factor + row_cost
    return cost


def _equal_cost_bounds(cum, lo, hi, k):
    """k contiguous blocks of rows [lo, hi) with near-equal cost (cum: prefix sums of the costs)."""
    t = cum[lo] + (cum[hi] - cum[lo]) * np.arange(k + 1) / k
    b = np.searchsorted(cum, t, side="left").astype(np.int64)
    b[0], b[-1] = lo, hi
    return np.maximum.accumulate(np.clip(b, lo, hi))


def balanced_row_bounds(deg, world, row_cost=4.0, walk_deg=None, walk_factor=WALK_FACTOR,
                        max_rows_factor=1.25):
    """Contiguous row blocks of near-equal cost (row_costs: nnz + row_cost per row, walked rows
    at walk_factor x nnz): P+1 boundaries. A row costing more than a rank's share (a walked hub
    row) gets a rank of its own when the ranks allow it, and the rows between such rows share the
    other ranks in proportion to their cost — so the rank that owns the 2.77M-edge row carries no
    other rows (rowpart balanced by walk cost). The exchange buffer is padded to the
    largest block (n_max rows per rank), so with walk costs the per-row cost doubles until no
    block holds more than max_rows_factor x N/P rows."""
    n = len(deg)
    b = _balanced_row_bounds(deg, world, row_cost, walk_deg, walk_factor)
    for _ in range(12):
        if walk_deg is None or world <= 1 or n == 0 or \
                np.diff(b).max() <= max_rows_factor * n / world:
            break
        row_cost *= 2.0
        b = _balanced_row_bounds(deg, world, row_cost, walk_deg, walk_factor)
    return b


def _balanced_row_bounds(deg, world, row_cost, walk_deg, walk_factor):
    cost = row_costs(deg, row_cost, walk_deg, walk_factor)
    n = cost.size
    if world <= 1 or n == 0:
        return np.asarray([0] + [n] * world, dtype=np.int64)
    cum = np.concatenate([[0.0], np.cumsum(cost)])
    giants = np.flatnonzero(cost > cum[-1] / world)
    # the non-giant row ranges between the giants
    edges_ = np.concatenate([[-1], giants, [n]])
    segs = [(int(a) + 1, int(b)) for a, b in zip(edges_[:-1], edges_[1:]) if b > a + 1]
    spare = world - giants.size
    if giants.size == 0 or spare < len(segs):
        return _equal_cost_bounds(cum, 0, n, world)
    # ranks per segment: at least 1, the rest by cost (largest remainder), capped by its rows
    sc = np.asarray([cum[b] - cum[a] for a, b in segs])
    k = np.ones(len(segs), dtype=np.int64)
    for _ in range(spare - len(segs)):
        room = np.asarray([b - a for a, b in segs]) > k
        if not room.any():
            break
        i = int(np.argmax(np.where(room, sc / k, -1.0)))
        k[i] += 1
    b = [0]
    pieces = sorted([(a, b_, int(kk)) for (a, b_), kk in zip(segs, k)] +
                    [(int(g), int(g) + 1, 1) for g in giants])
    for a, b_, kk in pieces:
        b.extend(_equal_cost_bounds(cum, a, b_, kk)[1:].tolist())
    while len(b) < world + 1:  # fewer rows than ranks somewhere: empty trailing blocks
        b.append(n)
    return np.asarray(b, dtype=np.int64)


def layout_positions(bounds, n_max, ids):
    """Global row id -> position in the rank-major padded buffer [P * n_max]."""
    ids = np.asarray(ids, dtype=np.int64)
    owner = np.searchsorted(bounds, ids, side="right") - 1
    return owner * n_max + (ids - bounds[owner])


def feature_bounds(d, world):
    """Column blocks per rank, multiples of 4 floats where d allows (16-B aligned gathers)."""
    unit = 4 if d % 4 == 0 and d // 4 >= world else 1
    units = d // unit
    cuts = [(units * p) // world * unit for p in range(world + 1)]
    cuts[-1] = d
    return np.asarray(cuts, dtype=np.int64)


class RowPartPlan:
    """Rank-local row block of a row-sorted global COO (r, c, v) with n nodes."""

    def __init__(self, r, c, v, n, world, rank, device, row_cost=4.0, walk_deg="auto"):
        rowptr_g = np.searchsorted(r, np.arange(n + 1)).astype(np.int64)
        if walk_deg == "auto":  # the engine's chain cut for the whole graph: rows above it walk
            walk_deg = engine.chain_max_degree(len(v)) if torch.device(device).type == "cuda" \
                else None
        self.bounds = balanced_row_bounds(np.diff(rowptr_g), world, row_cost, walk_deg)
        self.n, self.world, self.rank, self.device = n, world, rank, device
        self.n_max = int(np.diff(self.bounds).max())
        self.r0, self.r1 = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.n_local = self.r1 - self.r0
        e0, e1 = rowptr_g[self.r0], rowptr_g[self.r1]
        self.rowptr = (rowptr_g[self.r0:self.r1 + 1] - e0).astype(np.int32)
        self.cols = np.asarray(c[e0:e1], dtype=np.int64)
        self.cols_layout = layout_positions(self.bounds, self.n_max, self.cols)
        self.vals = np.asarray(v[e0:e1], dtype=np.float32)
        self.nnz_local = int(e1 - e0)
        if torch.device(device).type == "cuda":
            self.g1 = engine.graph_from_host_csr(self.rowptr, self.cols, self.vals, n, device)
            self.gk = engine.graph_from_host_csr(self.rowptr, self.cols_layout, self.vals,
                                                 world * self.n_max, device)
        else:
            self.g1 = self._cpu_coo(self.cols, n)
            self.gk = self._cpu_coo(self.cols_layout, world * self.n_max)

    def _cpu_coo(self, cols, n_cols):
        rows = np.repeat(np.arange(self.n_local), np.diff(self.rowptr))
        idx = torch.from_numpy(np.vstack([rows, cols]))
        return torch.sparse_coo_tensor(idx, torch.from_numpy(self.vals), (self.n_local, n_cols))

    def exchange_bytes_per_layer(self, d):
        return (self.world - 1) * self.n_max * d * 4


def allgather_into(out, inp):
    """all_gather_into_tensor; with the gloo backend and HIP tensors (the 2-process GPU test on a
    one-GPU box) the exchange bounces through host memory."""
    if out.device.type == "cuda" and dist.get_backend() == "gloo":
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu())
        out.copy_(o)
        return
    dist.all_gather_into_tensor(out, inp)


def _local_layer(graph, xs, y, d, ep, hub_thr):
    """y[:n_local] = epilogue(Â_local · X): engine on HIP, the reference ATen op on CPU."""
    if y.device.type == "cuda":
        return engine.spmm_layer(graph, xs, y, d, ep, hub_thr)
    x = torch.cat(xs, 0) if len(xs) > 1 else xs[0]
    y.copy_(torch.sparse.mm(graph, x))
    return y


def rowpart_buffers(plan, K, d, dev):
    """Layer buffers in the rank-major padded layout + this rank's (padded) final rows."""
    bufs = [torch.empty((plan.world * plan.n_max, d), dtype=torch.float32, device=dev)
            for _ in range(K - 1)]
    return bufs, torch.empty((plan.n_max, d), dtype=torch.float32, device=dev)


def rowpart_layer(plan, k, K, segments, bufs, out_local, hub_thr):
    """Local part of layer k (1-based): writes this rank's slice of E_k into bufs[k-1], or, for
    k == K, the fused mean of its rows into out_local[:n_local]."""
    d = segments[0].shape[1]
    on_gpu = segments[0].device.type == "cuda"
    rk, nm, nl = plan.rank, plan.n_max, plan.n_local
    g = plan.g1 if k == 1 else plan.gk
    xs = segments if k == 1 else [bufs[k - 2]]
    if k < K:
        mine = bufs[k - 1][rk * nm: rk * nm + nl]
        _local_layer(g, xs, mine, d, engine._epilogue(engine.LGCN_EPI_STORE) if on_gpu else None,
                     hub_thr)
        return
    prev = [b[rk * nm: rk * nm + nl] for b in bufs]
    if on_gpu:
        ep = engine._epilogue(engine.LGCN_EPI_MEAN, prev0=engine.rows_desc_from(segments, plan.r0, d),
                              prev_dense=prev, ld_prev=d, div=float(K + 1))
        _local_layer(g, xs, out_local[:nl], d, ep, hub_thr)
    else:  # reference order ((E0 + E1) + ...) + E_K, then / (K+1)
        last = torch.empty((nl, d), dtype=torch.float32)
        _local_layer(g, xs, last, d, None, hub_thr)
        s_ = torch.cat(segments, 0)[plan.r0:plan.r1].clone()
        for p_ in prev:
            s_ = s_ + p_
        out_local[:nl].copy_((s_ + last) / (K + 1))


def rowpart_forward(plan, segments, K, hub_thr=None, gather_final=True, layer_events=None):
    """K-layer propagation + mean over a row partition. segments: replicated E0 blocks
    (user, item[, brand]) in global row order. Returns the final table in layout order
    [P * n_max x d] (gather_final) or the local final rows [n_local x d]."""
    if hub_thr is None:
        hub_thr = engine.hub_threshold_from_env()
    d = segments[0].shape[1]
    dev = segments[0].device
    W, rk, nm, nl = plan.world, plan.rank, plan.n_max, plan.n_local
    bufs, out_local = rowpart_buffers(plan, K, d, dev)
    if K == 0:
        out_local[:nl].copy_(torch.cat(segments, 0)[plan.r0:plan.r1])
    for k in range(1, K + 1):
        if layer_events is not None:
            layer_events[k - 1][0].record()
        rowpart_layer(plan, k, K, segments, bufs, out_local, hub_thr)
        if layer_events is not None:
            layer_events[k - 1][1].record()
        if k < K:  # in-place all-gather: this rank's chunk is already in place
            allgather_into(bufs[k - 1], bufs[k - 1][rk * nm:(rk + 1) * nm])
    if not gather_final:
        return out_local[:nl]
    full = torch.empty((W * nm, d), dtype=torch.float32, device=dev)
    allgather_into(full, out_local)
    return full


def layout_to_global(plan, table):
    """Rows of a layout-ordered table [P * n_max x d] back in global order [n x d] (a copy)."""
    parts = [table[p * plan.n_max: p * plan.n_max + int(plan.bounds[p + 1] - plan.bounds[p])]
             for p in range(plan.world)]
    return torch.cat(parts, 0)


# ----------------------------------------------------------------------------------------------
# feature split
# ----------------------------------------------------------------------------------------------
def featsplit_slices(segments, world, rank):
    """This rank's column block of every E0 segment (contiguous copies: the parameter shard)."""
    d = segments[0].shape[1]
    cb = feature_bounds(d, world)
    c0, c1 = int(cb[rank]), int(cb[rank + 1])
    return [t[:, c0:c1].contiguous() for t in segments], (c0, c1)


def featsplit_forward(graph, seg_slices, K, hub_thr=None, layer_events=None):
    """K layers + mean on this rank's columns: no exchange at all."""
    if seg_slices[0].device.type == "cuda":
        return engine.propagate_forward(graph, seg_slices, K, hub_thr, layer_events=layer_events)
    ego = torch.cat(seg_slices, 0)
    all_e, x = [ego], ego
    for _ in range(K):
        x = torch.sparse.mm(graph, x)
        all_e.append(x)
    return torch.mean(torch.stack(all_e, 0), 0)


class FeatSplitPlan:
    """featsplit on a HIP device with the operator in slot space (engine.relabel_slots): rows
    and columns renumbered in degree-descending order, so the rank's parameter shard, the layer
    buffers and the output are all indexed by slot and every layer writes sequentially. At
    d/P = 8 columns (P = 8) a row is 32 B — a quarter of a 128-B line — and this layout is what
    keeps the per-rank layers near the line-granular HBM floor. perm[s] = node id of slot s;
    results are bitwise those of the row-id layout (every row keeps its fp32 chain)."""

    def __init__(self, rowptr, cols, vals, n, device, sides=None):
        """sides=(lo, hi): the item rows — a bipartite operator is stored side-major and each
        rank's shard runs the two-lane schedule (engine.propagate_forward without per-layer
        events), as the single-GPU path does."""
        g = engine.graph_from_host_csr(rowptr, cols, vals, n, device, order="degree",
                                       sides=sides)
        self.sides = g.sides
        self.graph, self.perm = engine.relabel_slots(g)
        self.inv = torch.empty_like(self.perm)
        self.inv[self.perm] = torch.arange(n, dtype=self.perm.dtype, device=device)
        self.n, self.device = n, device

    def shard(self, segments, world, rank):
        """Columns [c0, c1) of E0 = cat(segments) for this rank, rows in slot order: the rank's
        parameter shard (built once; the training state lives in this layout)."""
        d = segments[0].shape[1]
        cb = feature_bounds(d, world)
        c0, c1 = int(cb[rank]), int(cb[rank + 1])
        e0 = torch.cat([t[:, c0:c1] for t in segments], 0).to(self.device)
        return e0[self.perm].contiguous(), (c0, c1)

    def forward(self, x_slot, K, hub_thr=None, layer_events=None, hub_mode=None):
        """mean(E0..EK) of this rank's columns, in slot order. No exchange."""
        return engine.propagate_forward(self.graph, [x_slot], K, hub_thr,
                                        layer_events=layer_events, hub_mode=hub_mode)

    def attach_transpose(self, rowptr, cols, vals):
        """Âᵀ in the same slot space, for the backward of a shard (dE0 = Σ_k (Âᵀ)^k G/(K+1)):
        the CSR of Âᵀ with each row in the order autograd sums it (stable by column), ordered
        by degree — the same slot order as Â's, since the pattern is symmetric — and relabelled."""
        n = self.n
        rowptr = np.asarray(rowptr, dtype=np.int64)
        cols = np.asarray(cols, dtype=np.int64)
        vals = np.asarray(vals, dtype=np.float32)
        rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rowptr))
        order = np.argsort(cols, kind="stable")
        rt = cols[order]
        rpt = np.searchsorted(rt, np.arange(n + 1)).astype(np.int32)
        gt = engine.graph_from_host_csr(rpt, rows[order], vals[order], n, self.device,
                                        order="degree", sides=self.sides)
        if not torch.equal(gt.row_ids.long(), self.perm):
            raise engine.LgcnError("featsplit: the transpose's slot order differs from Â's "
                                   "(non-symmetric pattern)")
        self.graph.transpose, _ = engine.relabel_slots(gt)
        return self

    def backward(self, g_slot, K, hub_thr=None, sparse=None):
        """dE0 of this rank's columns (slot order) for its columns of the upstream gradient
        (slot order): the engine backward on Âᵀ in slot space. No exchange."""
        if self.graph.transpose is None:
            raise engine.LgcnError("FeatSplitPlan.backward needs attach_transpose() first")
        return engine.propagate_backward(self.graph, [g_slot], K, hub_thr, sparse=sparse)

    def slots(self, ids):
        """Slot positions of node ids (for gathering batch rows out of a slot-space table)."""
        return self.inv[ids]

    def unshard(self, y_slot):
        """A slot-space table back in node-id order."""
        return y_slot[self.inv]


class _AllReduceSum(torch.autograd.Function):
    """Sum of every rank's partials (one all_reduce). Every rank then evaluates the same loss
    of the same sums, so d loss / d (local partial) is the incoming gradient itself: the
    backward passes it through unchanged, with no collective."""

    @staticmethod
    def forward(ctx, part):
        out = part.clone()
        dist.all_reduce(out)
        return out

    @staticmethod
    def backward(ctx, g):
        return g


def bpr_loss_featsplit(u_slice, p_slice, n_slice, u0_slice, p0_slice, n0_slice, lambda_reg):
    """bpr_loss_reg (main.py:366-402) on column-sharded rows: partial dot products and partial
    squared norms are summed over ranks with ONE all_reduce of 2B+1 floats; differentiable —
    loss.backward() on every rank gives each rank the gradient of its own columns."""
    B = u_slice.shape[0]
    part = torch.cat([(u_slice * p_slice).sum(1), (u_slice * n_slice).sum(1),
                      (u0_slice.pow(2).sum() + p0_slice.pow(2).sum() +
                       n0_slice.pow(2).sum()).reshape(1)])
    part = _AllReduceSum.apply(part)
    pos, neg, sq = part[:B], part[B:2 * B], part[2 * B]
    bpr = -torch.mean(torch.log(torch.sigmoid(pos - neg) + 1e-8))
    return bpr + lambda_reg * sq / float(B)


# ----------------------------------------------------------------------------------------------
# bench driver (bench.py, N > 1)
# ----------------------------------------------------------------------------------------------
def _timed(fn, steps, warmup, dev):
    for _ in range(warmup):
        fn(None)
    torch.cuda.synchronize(dev)
    dist.barrier()
    evs = []
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(steps):
        ev = fn(True)
        evs.append(ev)
    t1.record()
    torch.cuda.synchronize(dev)
    dist.barrier()
    ms = t0.elapsed_time(t1)
    lay = np.array([[a.elapsed_time(b) for a, b in e] for e in evs])
    return ms, lay


def _max_over_ranks(t):
    tmax = t.clone()
    if dist.get_backend() == "gloo":  # rehearsal on one GPU: reduce on the host
        tmax = tmax.cpu()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    return tuple(float(x) for x in tmax.tolist())


C4_D, C4_K = 256, 4


def featsplit_backward_timing(plan, rowptr, c, v, x_slot, K, args, dev, hub_thr):
    """The training backward of a featsplit rank (its d/P columns of dE0 through Âᵀ in slot
    space, no exchange) for a dense upstream gradient, max over ranks. Reported, never fatal:
    the headline forward line is printed either way."""
    err = None
    try:
        plan.attach_transpose(rowptr, c, v)
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    # every rank takes the same branch (a one-sided failure must not strand the others in a
    # collective): proceed only if the transpose was built everywhere
    (failed,) = _max_over_ranks(torch.tensor([1.0 if err else 0.0], dtype=torch.float64,
                                             device=dev))
    if failed:
        plan.graph.transpose = None
        return {"error": err or "the transpose failed on another rank"}
    g = torch.randn_like(x_slot)
    ms, _ = _timed(lambda timed: (plan.backward(g, K, hub_thr, sparse="off"),
                                  [] if timed else None)[1], args.steps, args.warmup, dev)
    (ms_max,) = _max_over_ranks(torch.tensor([ms / args.steps], dtype=torch.float64, device=dev))
    del g
    out = {"ms_per_step": round(ms_max, 4),
           "propagated_edges_per_s": round(K * plan.graph.nnz / (ms_max / 1e3), 1),
           "what": "dE0 = sum_k (Â^T)^k G/(K+1) on each rank's columns (dense G)"}
    if getattr(args, "train_steps", 0) > 0:
        out["train_step"] = featsplit_train_timing(plan, x_slot, K, args, dev, hub_thr)
    plan.graph.transpose = None
    torch.cuda.empty_cache()
    return out


class ShardPropagate(torch.autograd.Function):
    """A featsplit rank's forward (its columns, slot space) with the engine backward."""

    @staticmethod
    def forward(ctx, plan, K, hub_thr, x_slot):
        ctx.plan, ctx.K, ctx.thr = plan, K, hub_thr
        return plan.forward(x_slot.detach(), K, hub_thr)

    @staticmethod
    def backward(ctx, g):
        return None, None, None, ctx.plan.backward(g.contiguous(), ctx.K, ctx.thr)


class ShardPropagateSides(torch.autograd.Function):
    """ShardPropagate on a side-major shard held as two blocks — slots [0, split) (users and
    brands) and [split, n) (items) — as the model holds its user and item weights: the batch
    gathers main.py makes (main.py:496-497) then index the block they read, so their gradients
    are dense over that block only (a single [n x d] shard made every gather's IndexBackward
    zero-fill and sum the whole table)."""

    @staticmethod
    def forward(ctx, plan, K, hub_thr, w0, w1):
        ctx.plan, ctx.K, ctx.thr, ctx.split = plan, K, hub_thr, int(w0.shape[0])
        out = engine.propagate_forward(plan.graph, [w0.detach(), w1.detach()], K, hub_thr)
        return tuple(torch.split(out, [ctx.split, out.shape[0] - ctx.split], 0))

    @staticmethod
    def backward(ctx, g0, g1):
        n = ctx.plan.graph.n_rows
        d = next(g.shape[1] for g in (g0, g1) if g is not None)
        gs = [g.contiguous() if g is not None else
              torch.zeros((rows, d), dtype=torch.float32, device=ctx.plan.graph.device)
              for g, rows in ((g0, ctx.split), (g1, n - ctx.split))]
        g = engine.propagate_backward(ctx.plan.graph, gs, ctx.K, ctx.thr)
        return None, None, None, g[:ctx.split], g[ctx.split:]


def featsplit_train_timing(plan, x_slot, K, args, dev, hub_thr, batch=2048):
    """main.py's training step (main.py:488-531) on P ranks: every rank propagates its columns,
    gathers the batch rows of its shard, the sharded BPR loss reduces partial dots (one
    all_reduce), the backward runs on the shard's columns, Adam updates the shard. Identical
    batches on every rank (same seed). Edges/s = 2K·nnz / t, max over ranks."""
    U, I = args.users, args.items
    rng = np.random.default_rng(0)
    batches = [tuple(plan.slots(torch.from_numpy(a).to(dev)) for a in (
        rng.integers(0, U, batch), U + rng.integers(0, I, batch), U + rng.integers(0, I, batch)))
        for _ in range(args.train_steps + 2)]
    it = iter(batches)
    sp_ = plan.graph.split
    if sp_ is not None:  # side-major shard: two blocks, as the model's user / item weights
        w0 = torch.nn.Parameter(x_slot[:sp_].clone())
        w1 = torch.nn.Parameter(x_slot[sp_:].clone())
        opt = torch.optim.Adam([w0, w1], lr=1e-3)
    else:
        w = torch.nn.Parameter(x_slot.clone())
        opt = torch.optim.Adam([w], lr=1e-3)

    def step(timed):
        su, sp, sn = next(it)
        opt.zero_grad()
        if sp_ is not None:
            o0, o1 = ShardPropagateSides.apply(plan, K, hub_thr, w0, w1)
            sp1, sn1 = sp - sp_, sn - sp_
            loss = bpr_loss_featsplit(o0[su], o1[sp1], o1[sn1], w0[su], w1[sp1], w1[sn1], 1e-4)
        else:
            out = ShardPropagate.apply(plan, K, hub_thr, w)
            loss = bpr_loss_featsplit(out[su], out[sp], out[sn], w[su], w[sp], w[sn], 1e-4)
        loss.backward()
        opt.step()
        loss.item()  # main.py:527 reads the loss back every batch
        return [] if timed else None
    ms, _ = _timed(step, args.train_steps, 2, dev)
    (ms_max,) = _max_over_ranks(torch.tensor([ms / args.train_steps], dtype=torch.float64,
                                             device=dev))
    del opt
    return {"ms_per_step": round(ms_max, 3),
            "propagated_edges_per_s": round(2 * K * plan.graph.nnz / (ms_max / 1e3), 1),
            "batch": batch, "optimizer": "Adam(lr=1e-3) on the rank's shard",
            "what": "main.py:488-531 on P ranks: shard forward + batch gathers + sharded BPR loss "
                    "(one all_reduce) + shard backward + Adam"}


def featsplit_c4(plan, world, rank, nnz, n, args, dev, hub_thr):
    """BASELINE configs[3] on the same graph (full Books shape, d=256, K=4 — the configuration
    BASELINE.md sets the >= 6x 8-GPU target on): this rank's d/P = 256/P columns, timed like
    the headline (warm-up, barrier, K-layer forwards, max over ranks). Weights are uniform
    random on the device (the timing does not depend on their values; parity is the C3 path's)."""
    c0, c1 = (int(x) for x in feature_bounds(C4_D, world)[rank:rank + 2])
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    bound = float(np.sqrt(6.0 / (n + C4_D)))
    x = (torch.rand((n, c1 - c0), generator=gen, device=dev) * 2 - 1) * bound

    sided = plan.graph.split is not None

    def fn(timed):
        if sided:  # whole steps: per-layer events would force the one-operator schedule
            ev = [(torch.cuda.Event(enable_timing=True),
                   torch.cuda.Event(enable_timing=True))] if timed else None
            if ev:
                ev[0][0].record()
            plan.forward(x, C4_K, hub_thr)
            if ev:
                ev[0][1].record()
            return ev
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(C4_K)] if timed else None
        plan.forward(x, C4_K, hub_thr, layer_events=ev)
        return ev
    ms, lay = _timed(fn, args.steps, args.warmup, dev)
    if lay.shape[1] == 1 and C4_K > 1:  # sided: a layer's share of the step
        lay = np.repeat(lay / C4_K, C4_K, axis=1)
    ms_max, store_ms = _max_over_ranks(torch.tensor([ms, float(lay[:, :-1].mean())],
                                                    dtype=torch.float64, device=dev))
    del x
    torch.cuda.empty_cache()
    return {"d": C4_D, "layers": C4_K, "columns_per_rank": c1 - c0,
            "ms_per_step": round(ms_max / args.steps, 4),
            "edges_per_s": round(C4_K * nnz * args.steps / (ms_max / 1e3), 1),
            "store_layer_ms": round(store_ms, 4),
            "schedule": "bipartite two-lane (whole steps timed)" if sided else "one operator"}


def profiled_traffic(cfg, args, mode, d_rank):
    """HBM bytes per launch of a featsplit rank's STORE layer at this column width, from the
    committed PMC profiles (profiles/traffic_c3_featsplit_*.json; C3 power-law only), or None."""
    if mode != "featsplit" or cfg.get("name", "").split()[0] != "C3" or args.gen != "powerlaw":
        return None
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    import json
    try:
        if d_rank == 8:
            return json.load(open(os.path.join(root, "traffic_c3_featsplit_d8.json")))[
                "hbm_bytes_per_launch"]
        if d_rank in (16, 32):
            ks = json.load(open(os.path.join(root, "traffic_c3_featsplit_d16_d32.json")))["kernels"]
            return int(next(v["hbm_bytes_per_launch"] for k, v in ks.items()
                            if k.startswith(f"d={d_rank} STORE")))
    except (OSError, KeyError, StopIteration, ValueError):
        return None
    return None


def _sided_store_launches(graph, x_slot, K, hub_thr, hub_mode, d, run, steps):
    """(ms per STORE layer-kernel segment launch, algorithmic bytes per launch) of a sided graph:
    `steps` calls of run() with engine.side_timing on (each segment's layer kernel timed on its
    lane's stream), bytes = the SURVEY 8d model over the rows the layer kernel runs (bundle rows
    and, in the exact plan, whole-row items up to emu_min_degree), as bench.py's N = 1 line."""
    engine.side_timing = []
    try:
        for _ in range(steps):
            run()
        torch.cuda.synchronize()
        tm = engine.side_timing
    finally:
        engine.side_timing = None
    ker = np.array([[[t[(k, g)][0].elapsed_time(t[(k, g)][1]) if (k, g) in t else 0.0
                      for g in range(engine.N_SEGS)] for k in range(1, K + 1)] for t in tm])
    rp = graph.rowptr_host().astype(np.int64)
    emu_min = engine.emu_min_degree_from_env(graph.nnz)
    thr = min(hub_thr if hub_thr is not None else engine.hub_threshold_from_env(),
              engine.INT32_MAX)
    cut = max(thr, emu_min if hub_mode == "exact" else 0)

    def kernel_bytes(a, b):
        deg = np.diff(rp[a:b + 1])
        run_ = deg <= cut
        return int(deg[run_].sum()) * (4 * d + 8) + 4 * (b - a + 1) + 4 * int(run_.sum()) * d
    segs = graph.segments()
    live = [g for g, (a, b) in enumerate(segs) if b > a]
    st = ker[:, :-1, :] if K > 1 else ker
    n_launch = max(len(live) * st.shape[1], 1)
    store_ms = float(st.sum(axis=(1, 2)).mean()) / n_launch
    b_launch = sum(kernel_bytes(*segs[g]) for g in live) * st.shape[1] / n_launch
    return store_ms, b_launch


def bench_distributed(args, cfg, r, c, v, emb_host, dev, hub_thr):
    rank, world = init("cuda")
    d, K = cfg["d"], cfg["K"]
    U, I = cfg["users"], cfg["items"]
    n = U + I
    nnz = len(v)
    mode = args.mode

    def mk_events():
        return [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(K)]

    if mode == "featsplit":
        rowptr = np.searchsorted(r, np.arange(n + 1)).astype(np.int32)
        plan = FeatSplitPlan(rowptr, c, v, n, dev, sides=(U, U + I))
        x_slot, (c0, c1) = plan.shard(emb_host, world, rank)
        dl = c1 - c0
        sided = plan.graph.split is not None
        if not sided:
            plan.graph.hubs(hub_thr)

        def fn(timed):
            if sided:  # the two-lane schedule has no layer boundary: one event pair per step
                ev = [(torch.cuda.Event(enable_timing=True),
                       torch.cuda.Event(enable_timing=True))] if timed else None
                if ev:
                    ev[0][0].record()
                plan.forward(x_slot, K, hub_thr)
                if ev:
                    ev[0][1].record()
                return ev
            ev = mk_events() if timed else None
            plan.forward(x_slot, K, hub_thr, layer_events=ev)
            return ev
        b_layer = nnz * (4 * dl + 8) + 4 * (n + 1) + 4 * n * dl
        comm = 0
        extra = {"columns": [int(c0), int(c1)],
                 "schedule": "bipartite two-lane" if sided else "one operator"}
    else:
        plan = RowPartPlan(r, c, v, n, world, rank, dev)
        segs = [t.to(dev) for t in emb_host]

        def fn(timed):
            ev = mk_events() if timed else None
            rowpart_forward(plan, segs, K, hub_thr, gather_final=True, layer_events=ev)
            return ev
        b_layer = plan.nnz_local * (4 * d + 8) + 4 * (plan.n_local + 1) + 4 * plan.n_local * d
        comm = K * plan.exchange_bytes_per_layer(d)
        extra = {"rows": [plan.r0, plan.r1], "nnz_local": plan.nnz_local}

    ms, lay = _timed(fn, args.steps, args.warmup, dev)
    if lay.shape[1] == 1 and K > 1:  # sided featsplit: whole steps; a layer's share of one
        lay = np.repeat(lay / K, K, axis=1)
    hub_mode = engine.hub_mode_from_env()
    if mode == "featsplit" and sided:
        # the N = 1 line's basis (bench.py): the STORE layer-kernel segment launches, each timed on
        # its lane's stream in a second loop, algorithmic bytes over the rows the kernel runs
        store_ms, b_layer = _sided_store_launches(plan.graph, x_slot, K, hub_thr, hub_mode, dl,
                                                  lambda: plan.forward(x_slot, K, hub_thr),
                                                  min(args.steps, 5))
        basis = ("algorithmic bytes (SURVEY 8d) of the rows the layer kernel runs / its segment "
                 "launch time (STORE layers 1..K-1, each timed on its lane's stream), per GPU, "
                 "max over ranks — the N = 1 line's basis")
    else:
        store_ms = float(lay[:, :-1].mean() if K > 1 else lay.mean())
        basis = "algorithmic bytes (SURVEY 8d) / whole-layer time (store layers), per GPU, " \
                "max over ranks"
    t = torch.tensor([ms, store_ms, float(lay.mean())], dtype=torch.float64, device=dev)
    ms_max, kern_ms, all_ms = _max_over_ranks(t)
    c4 = rp = bwd = chunk = None
    if mode == "featsplit" and hub_mode == "exact":
        # secondary: the same shard forward with chunked hub rows (fixed-order partial sums, not
        # the reference's rounding on hub rows): the throughput the split gets when the
        # sequential hub chains (whose walk does not shrink with P) are not reproduced
        def fn_c(timed):
            if sided:  # as fn: per-layer events would force the one-operator schedule
                ev = [(torch.cuda.Event(enable_timing=True),
                       torch.cuda.Event(enable_timing=True))] if timed else None
                if ev:
                    ev[0][0].record()
                plan.forward(x_slot, K, hub_thr, hub_mode="chunk")
                if ev:
                    ev[0][1].record()
                return ev
            ev = mk_events() if timed else None
            plan.forward(x_slot, K, hub_thr, layer_events=ev, hub_mode="chunk")
            return ev
        ms_c, _ = _timed(fn_c, args.steps, args.warmup, dev)
        (ms_c,) = _max_over_ranks(torch.tensor([ms_c], dtype=torch.float64, device=dev))
        chunk = {"ms_per_step": round(ms_c / args.steps, 4),
                 "edges_per_s": round(K * nnz * args.steps / (ms_c / 1e3), 1),
                 "what": "hub_mode=chunk on the same shards (not bitwise on hub rows)"}
    if mode == "featsplit" and getattr(args, "backward", True):
        bwd = featsplit_backward_timing(plan, rowptr, c, v, x_slot, K, args, dev, hub_thr)
    if mode == "featsplit" and getattr(args, "c4", True):
        c4 = featsplit_c4(plan, world, rank, nnz, n, args, dev, hub_thr)
    if mode == "featsplit" and getattr(args, "rowpart", True):
        del plan
        torch.cuda.empty_cache()
        rp = rowpart_secondary(r, c, v, n, nnz, K, d, emb_host, world, rank, args, dev, hub_thr)
    value = K * nnz * args.steps / (ms_max / 1e3)
    achieved = b_layer / (kern_ms / 1e3) / 1e9
    dw = dl if mode == "featsplit" else d
    b_fwd = K * (nnz * (4 * dw + 8) + 4 * (n + 1) + 4 * n * dw) if mode == "featsplit" else \
        K * b_layer
    fwd_rate = b_fwd / (ms_max / args.steps / 1e3) / 1e9
    return {
        "metric": "propagated edges/sec (SpMM) + Recall@20, Amazon-Books 3-layer d=64",
        "value": round(value, 1), "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_max / args.steps, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": cfg["name"], "generator": args.gen, "users": U, "items": I,
                   "interactions": cfg["interactions"], "nnz": nnz, "d": d, "layers": K,
                   "hub_threshold": hub_thr, "hub_mode": hub_mode,
                   "parallelism": f"{mode}{world}",
                   "exchange_bytes_per_step_per_rank": int(comm), **extra},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0,
                     "unit": "GB/s", "frac": round(achieved / 8000.0, 4), "traffic": None,
                     "basis": basis + "; no PMC pass of this build at N > 1",
                     "forward": {"bytes": int(b_fwd), "achieved": round(fwd_rate, 1),
                                 "frac": round(fwd_rate / 8000.0, 4),
                                 "note": "the rank's K x SURVEY 8d bytes per forward / "
                                         "ms_per_step (as the N = 1 line's roofline.forward)"},
                     "round1_pmc_traffic_chunk_mode": profiled_traffic(
                         cfg, args, mode, d // world if mode == "featsplit" else None),
                     "kernel": "k_layer store layers, per GPU (max over ranks)",
                     "bytes_per_launch": int(b_layer), "avg_launch_ms": round(kern_ms, 4)},
        **({"chunk_mode": chunk} if chunk else {}),
        **({"backward": bwd} if bwd else {}),
        **({"c4_same_graph": c4} if c4 else {}),
        **({"rowpart": rp} if rp else {}),
    }


def rowpart_secondary(r, c, v, n, nnz, K, d, emb_host, world, rank, args, dev, hub_thr,
                      steps=5):
    """The north_star decomposition measured beside the default one in the same run: row blocks
    balanced by nnz, every layer's slice all-gathered in place over RCCL (xGMI on one node), the
    final table gathered too. Local-layer time and exchange time are split by HIP events (max
    over ranks); the exchange rate is the bytes a rank receives per step / exchange time."""
    plan = RowPartPlan(r, c, v, n, world, rank, dev)
    segs = [t.to(dev) for t in emb_host]

    def fn(timed):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(K)] if timed else None
        rowpart_forward(plan, segs, K, hub_thr, gather_final=True, layer_events=ev)
        return ev
    st = min(steps, args.steps)
    ms, lay = _timed(fn, st, 1, dev)
    ms_max, local_ms = _max_over_ranks(torch.tensor([ms / st, float(lay.sum(1).mean())],
                                                    dtype=torch.float64, device=dev))
    recv = K * (world - 1) * plan.n_max * d * 4  # K-1 layer gathers + the final gather
    ex_ms = max(ms_max - local_ms, 1e-6)
    out = {"ms_per_step": round(ms_max, 3), "edges_per_s": round(K * nnz / (ms_max / 1e3), 1),
           "local_layers_ms": round(local_ms, 3), "exchange_ms": round(ex_ms, 3),
           "received_bytes_per_step_per_rank": int(recv),
           "padding_ratio": round(world * plan.n_max / n, 4),
           "exchange_bytes_per_layer_per_rank": int(plan.exchange_bytes_per_layer(d)),
           "exchange_GBps_per_rank": round(recv / (ex_ms / 1e3) / 1e9, 1),
           "what": "rowpart (north_star): row blocks + in-place all_gather_into_tensor of every "
                   "layer's slice (RCCL); exchange = step time - local layer kernels"}
    del plan, segs
    torch.cuda.empty_cache()
    return out
