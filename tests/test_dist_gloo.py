"""Multi-process (world_size 2, gloo, CPU) tests of the distributed orchestration in
gcn_recommendation_amd.dist: row-partition planning, the padded rank-major layout + column
remap, the in-place all-gather exchange, the fused mean's operand slices, the feature split and
its sharded BPR loss. On CPU the local layer is the reference's ATen op, so the distributed
result must be bitwise equal to the single-process oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, case_dims, load_case

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        from gcn_recommendation_amd import dist as D
        from oracle import oracle
        D.init("cpu")
        z = load_case(name)
        U, I, B, d, K = case_dims(z)
        n = U + I + B
        r, c, v = z["adj_row"].astype(np.int64), z["adj_col"].astype(np.int64), z["adj_val"]
        segs = [torch.from_numpy(z["param/user_embedding.weight"]),
                torch.from_numpy(z["param/item_embedding.weight"]),
                torch.from_numpy(z["param/brand_embedding.weight"])]
        e0 = torch.cat(segs).numpy()
        want = oracle.forward(r, c, v, e0, K)
        out = {}
        # row partition
        plan = D.RowPartPlan(r, c, v, n, world, rank, "cpu")
        full = D.rowpart_forward(plan, segs, K)
        got = D.layout_to_global(plan, full).numpy()
        out["rowpart_bitwise"] = bool(np.array_equal(got, want))
        out["bounds"] = plan.bounds.tolist()
        # feature split
        adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([r, c])), torch.from_numpy(v),
                                      (n, n))
        sl, (c0, c1) = D.featsplit_slices(segs, world, rank)
        mine = D.featsplit_forward(adj, sl, K)
        widths = np.diff(D.feature_bounds(d, world))
        wmax = int(widths.max())
        padded = torch.zeros((n, wmax))
        padded[:, :mine.shape[1]] = mine
        parts = [torch.empty((n, wmax)) for _ in widths]
        dist.all_gather(parts, padded)
        cat = torch.cat([p_[:, :int(w)] for p_, w in zip(parts, widths)], 1).numpy()
        out["featsplit_bitwise"] = bool(np.array_equal(cat, want))
        # sharded BPR loss == bpr_loss_reg on full rows
        from gcn_recommendation_amd.loss import bpr_loss_reg
        bu, bp, bn = (torch.from_numpy(z[k]) for k in ("bpr_users", "bpr_pos", "bpr_neg"))
        fin = torch.from_numpy(want)
        fu, fi = fin[:U], fin[U:U + I]
        u0, i0 = segs[0], segs[1]
        fu = fu.clone().requires_grad_()
        fi = fi.clone().requires_grad_()
        u0, i0 = u0.clone().requires_grad_(), i0.clone().requires_grad_()
        ref = bpr_loss_reg(fu[bu], fi[bp], fi[bn], u0[bu], i0[bp], i0[bn], 1e-4)
        ref.backward()
        mu = mine[:U].clone().requires_grad_()
        mi = mine[U:U + I].clone().requires_grad_()
        su0, si0 = sl[0].clone().requires_grad_(), sl[1].clone().requires_grad_()
        loss = D.bpr_loss_featsplit(mu[bu], mi[bp], mi[bn], su0[bu], si0[bp], si0[bn], 1e-4)
        loss.backward()
        out["bpr_rel_err"] = float(abs(loss.item() - ref.item()) / abs(ref.item()))
        # each rank's gradients == its columns of the full-row gradients
        gerr = 0.0
        for got, full in ((mu.grad, fu.grad), (mi.grad, fi.grad), (su0.grad, u0.grad),
                          (si0.grad, i0.grad)):
            w = full[:, c0:c1]
            gerr = max(gerr, float((got - w).abs().max() / max(float(full.abs().max()), 1e-30)))
        out["bpr_grad_err"] = gerr
        D.shutdown()
        q.put((rank, out))
    except Exception as e:  # surface worker failures to the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise


@pytest.mark.parametrize("name", ["c1_brand", "micro_d12", "hub_d32"])
def test_rowpart_and_featsplit_world2(name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, name, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(WORLD))
    for p in procs:
        p.join(60)
    for rk, out in res.items():
        assert "error" not in out, out.get("error")
        assert out["rowpart_bitwise"], (rk, out)
        assert out["featsplit_bitwise"], (rk, out)
        assert out["bpr_rel_err"] < 1e-6, out
        assert out["bpr_grad_err"] < 1e-5, out


def test_balanced_bounds_and_layout():
    from gcn_recommendation_amd import dist as D
    deg = np.array([100, 0, 0, 1, 1, 1, 50, 50, 2, 3])
    for world in (1, 2, 3, 4, 8):
        b = D.balanced_row_bounds(deg, world)
        assert b[0] == 0 and b[-1] == len(deg) and np.all(np.diff(b) >= 0)
        n_max = int(np.diff(b).max())
        pos = D.layout_positions(b, n_max, np.arange(len(deg)))
        assert len(np.unique(pos)) == len(deg)
        owner = pos // n_max
        assert np.all(np.diff(owner) >= 0)
    # walk cost: the rank holding a walked hub row gets few other rows, every rank some
    rng = np.random.default_rng(0)
    deg = rng.integers(1, 40, 10_000)
    deg[3_000] = 30_000   # below a rank's share by nnz, far above it as a walk
    for world in (4, 8):
        b0 = D.balanced_row_bounds(deg, world)
        b1 = D.balanced_row_bounds(deg, world, walk_deg=20_000, max_rows_factor=2.0)
        bc = D.balanced_row_bounds(deg, world, walk_deg=20_000)   # default row cap
        assert np.diff(bc).max() <= 1.25 * deg.size / world
        assert len(b1) == world + 1 and b1[0] == 0 and b1[-1] == deg.size
        assert np.all(np.diff(b1) >= 1)
        own0 = np.searchsorted(b0, 3_000, side="right") - 1
        own1 = np.searchsorted(b1, 3_000, side="right") - 1
        assert np.diff(b1)[own1] == 1 < np.diff(b0)[own0]   # the walked row alone
        cost = D.row_costs(deg, walk_deg=20_000)
        blk = [cost[b1[i]:b1[i + 1]].sum() for i in range(world) if i != own1]
        assert max(blk) <= 1.15 * (cost.sum() - cost[3_000]) / (world - 1)
    cb = D.feature_bounds(64, 8)
    assert list(np.diff(cb)) == [8] * 8
    cb = D.feature_bounds(12, 8)
    assert cb[-1] == 12 and np.all(np.diff(cb) >= 1)


def test_package_import_raises_hw_queues_under_torchrun():
    """A `torchrun main.py` rank (WORLD_SIZE > 1) gets GPU_MAX_HW_QUEUES=16 from importing the
    package (RCCL's streams would otherwise share the schedule's hardware queues);
    a single process is left alone, and a larger setting is kept."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "import os, gcn_recommendation_amd; print(os.environ.get('GPU_MAX_HW_QUEUES'))"
    for env, want in (({"WORLD_SIZE": "2"}, "16"), ({"WORLD_SIZE": "1"}, "None"),
                      ({"WORLD_SIZE": "4", "GPU_MAX_HW_QUEUES": "24"}, "24")):
        e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "GPU_MAX_HW_QUEUES")}
        e.update(env)
        out = subprocess.run([sys.executable, "-c", code], cwd=root, env=e, capture_output=True,
                             text=True, timeout=120)
        assert out.returncode == 0, out.stderr
        assert out.stdout.strip() == want, (env, out.stdout)
