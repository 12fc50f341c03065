"""Two real processes on the one GPU of the test box, gloo for the exchange (RCCL needs one GPU
per rank): the multi-process GPU code path of gcn_recommendation_amd.dist — per-rank plans,
engine layers on each rank's row block, the in-place all-gather step, the fused mean on local
slices, the final gather; and the feature split — bitwise against the oracle (exact mode)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT, case_dims, case_e0, load_case

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    try:
        import torch.distributed as dist
        from gcn_recommendation_amd import dist as D, engine
        from oracle import oracle
        dev = torch.device("cuda:0")
        D.init("cuda", backend="gloo")
        z = load_case("hub_d32")
        U, I, B, d, K = case_dims(z)
        n = U + I + B
        r, c, v = z["adj_row"].astype(np.int64), z["adj_col"].astype(np.int64), z["adj_val"]
        segs = [torch.from_numpy(z[f"param/{k}_embedding.weight"]).to(dev)
                for k in ("user", "item", "brand")]
        want = oracle.forward(r, c, v, case_e0(z), K)
        plan = D.RowPartPlan(r, c, v, n, world, rank, dev)
        full = D.rowpart_forward(plan, segs, K, hub_thr=engine.INT32_MAX)
        got = D.layout_to_global(plan, full).cpu().numpy()
        out = {"rowpart": bool(np.array_equal(got, want))}
        rowptr = np.searchsorted(r, np.arange(n + 1)).astype(np.int32)
        g = engine.graph_from_host_csr(rowptr, c, v, n, dev)
        sl, (c0, c1) = D.featsplit_slices(segs, world, rank)
        mine = D.featsplit_forward(g, sl, K, engine.INT32_MAX).cpu()
        out["featsplit"] = bool(np.array_equal(mine.numpy(), want[:, c0:c1]))
        fs = D.FeatSplitPlan(rowptr, c, v, n, dev)      # slot-space shards (bench.py's path)
        x, (c0, c1) = fs.shard(segs, world, rank)
        mine = fs.unshard(fs.forward(x, K, engine.INT32_MAX)).cpu()
        out["featsplit"] &= bool(np.array_equal(mine.numpy(), want[:, c0:c1]))
        D.shutdown()
        q.put((rank, out))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise


def test_two_processes_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(rk, 2, port, q)) for rk in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(60)
    for rk, out in res.items():
        assert "error" not in out, out["error"]
        assert out["rowpart"] and out["featsplit"], (rk, out)
