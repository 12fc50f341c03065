"""The C host path vs the Python path at C3: the forward as a C host drives it (one
lgcn_propagate_forward_sides call with the plans from lgcn_plan_exact and a 7-stream
lgcn_sched_t) against engine.propagate_forward, same graph, median of
REPS; and their outputs compared bitwise.

    python tools/c_abi_timing.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402


def median_ms(fn, reps):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    cfg = bench.CONFIGS[os.environ.get("CFG", "c3")]
    reps = int(os.environ.get("REPS", "10"))
    dev = torch.device("cuda:0")
    lib = engine.load_library()
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I = cfg["users"], cfg["items"]
    n, d, K = U + I, cfg["d"], cfg["K"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    g = engine.graph_from_coo(adj, sides=(U, U + I))
    assert g.split is not None
    gen = torch.Generator().manual_seed(42)
    segs = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
    # the C host's objects: 4 plans (2 sides x 2 scratch sets), the schedule, the buffers
    # (the plans the engine builds: at C3 scale rows of 129..1024 edges are whole-row items of
    # the layer kernel, emu_min = engine.emu_min_degree_from_env(nnz))
    plans, _ = engine._side_plans(g, d, 128, "exact", engine.emu_min_degree_from_env(g.nnz), True)
    sc = engine.sched_for(dev)
    layers = [torch.empty((n, d), device=dev) for _ in range(K - 1)]
    out_c = torch.empty((n, d), device=dev)
    bufs = (ctypes.c_void_p * (K - 1))(*[t.data_ptr() for t in layers])
    e0 = engine.rows_desc(segs, d)
    P = engine._ptr

    def c_host():
        rc = lib.lgcn_propagate_forward_sides(
            P(g.rowptr), P(g.edges), P(g.row_ids), n, g.split, plans, e0, d, K, bufs, P(out_c),
            sc.handle, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, lib.lgcn_error_string(rc)
    out_py = [None]

    def python():
        out_py[0] = engine.propagate_forward(g, segs, K)
    t_c = median_ms(c_host, reps)
    t_py = median_ms(python, reps)
    same = bool(torch.equal(out_c, out_py[0]))
    print(f"C host lgcn_propagate_forward_sides: {t_c:.3f} ms; engine.propagate_forward: "
          f"{t_py:.3f} ms; ratio {t_c / t_py:.3f}; outputs bitwise equal: {same}", flush=True)


if __name__ == "__main__":
    main()
