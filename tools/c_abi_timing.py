"""The C host path vs the Python path at C3: the forward as a C host drives it (one
lgcn_propagate_forward_sides call with plans built by the C planner alone — lgcn_plan_items +
lgcn_plan_exact per segment, tools/c_host_plans.py — and a 7-stream lgcn_sched_t,
INTEGRATION.md §2) against engine.propagate_forward, same graph, median of REPS; and their
outputs compared bitwise.

    python tools/c_abi_timing.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
from c_host_plans import c_host_side_plans  # noqa: E402
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
    # the C host's objects: 8 plans (4 segments x 2 scratch sets) from the C planner alone, the
    # schedule, the buffers
    plans, keep = c_host_side_plans(lib, g.rowptr_host(), g.row_ids_host(), g.segments(), g.nnz,
                                    d, dev)
    sides = g.sides_struct()
    sc = engine.sched_for(dev)
    out_c = torch.empty((n, d), device=dev)
    e0 = engine.rows_desc(segs, d)
    P = engine._ptr

    py_plans, _ = engine._side_plans(g, d, 128, "exact", None, True)

    def c_host(pl=plans):
        # fresh output buffers per call, as the Python binding allocates them (same allocator)
        lay = [torch.empty((n, d), device=dev) for _ in range(K - 1)]
        bf = (ctypes.c_void_p * (K - 1))(*[t.data_ptr() for t in lay])
        out_c.data = torch.empty((n, d), device=dev)
        rc = lib.lgcn_propagate_forward_sides(
            P(g.rowptr), P(g.edges), P(g.row_ids), ctypes.byref(sides), pl, e0, d, K, bf,
            P(out_c), sc.handle, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, lib.lgcn_error_string(rc)
    out_py = [None]

    def python():
        out_py[0] = engine.propagate_forward(g, segs, K)
    # interleaved: box-to-box and run-to-run drift hits both sides alike
    t_c, t_py, t_cp = [], [], []
    for _ in range(3):
        t_c.append(median_ms(c_host, reps))
        t_py.append(median_ms(python, reps))
        t_cp.append(median_ms(lambda: c_host(py_plans), reps))
    t_c, t_py, t_cp = (float(np.median(t)) for t in (t_c, t_py, t_cp))
    c_host()
    same = bool(torch.equal(out_c, out_py[0]))
    print(f"C host lgcn_propagate_forward_sides (C-planner plans): {t_c:.3f} ms; the same call "
          f"with the Python binding's plans: {t_cp:.3f} ms; engine.propagate_forward: {t_py:.3f} "
          f"ms; ratio C/Python {t_c / t_py:.3f}; outputs bitwise equal: {same}", flush=True)


if __name__ == "__main__":
    main()
