"""The torch side of the round-6 capture investigation: the sided forward over the
brand graph of tests/test_gpu_sides.py captured under torch.cuda.graph in a fresh process —
engine.CapturedForward, the same with capture_error_mode="relaxed", or the bare library call
with every buffer allocated before the capture (argv[1]: engine | relaxed | prealloc). With the
full schedule under the capture (the investigation's LGCN_CAPTURE_AUX_EXP build) every mode
segfaulted in hipStreamEndCapture — the torch process runs the 7.0 HIP runtime of the torch wheel,
and tools/capture_host.cpp crashes the same way on it. The library now restricts a capture on
runtimes before 7.2 (lgcn_capture_full_schedule), so this probe replays bitwise with lane 1 on its
main stream."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gcn_recommendation_amd import engine  # noqa: E402
from oracle import oracle  # noqa: E402
from test_gpu_sides import U, I, _brand_graph, _segs  # noqa: E402
from test_gpu_exact import _adj, _e0  # noqa: E402


def main():
    """argv[1]: engine (CapturedForward: buffers allocated inside the capture), prealloc (the
    library call alone under torch.cuda.graph, buffers allocated before), relaxed (as engine,
    capture_error_mode="relaxed")."""
    import ctypes
    mode = sys.argv[1] if len(sys.argv) > 1 else "engine"
    os.environ.setdefault("LGCN_SIDES_MIN_NNZ", "0")
    os.environ.setdefault("LGCN_AUX_STREAMS", "7")
    dev = torch.device("cuda:0")
    lib = engine.load_library()
    r, c, v, n = _brand_graph(np.random.default_rng(21))
    g = engine.graph_from_coo(_adj(r, c, v, n, dev), sides=(U, U + I))
    rng = np.random.default_rng(8)
    e0 = _e0(rng, "xavier", n, 64)
    x = _segs(e0, dev)
    K, d = 3, 64
    want = oracle.forward(r, c, v, e0, K)
    got = engine.propagate_forward(g, x, K, hub_threshold=128).cpu().numpy()
    print(mode, "eager bitwise:", np.array_equal(got, want), engine.last_schedule, flush=True)
    if mode in ("engine", "relaxed"):
        kw = {"capture_error_mode": "relaxed"} if mode == "relaxed" else {}
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            engine.propagate_forward(g, x, K, hub_threshold=128)
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        print("capturing ...", flush=True)
        with torch.cuda.graph(graph, **kw):
            out = engine.propagate_forward(g, x, K, hub_threshold=128)
    else:
        out = torch.empty((n, d), dtype=torch.float32, device=dev)
        layers = [torch.empty((n, d), dtype=torch.float32, device=dev) for _ in range(K - 1)]
        plans, _ = engine._side_plans(g, d, 128, None, None, engine._aligned16(x))
        sc = engine.sched_for(dev)
        bufs = (ctypes.c_void_p * (K - 1))(*[t.data_ptr() for t in layers])
        sides = g.sides_struct()
        e0d = engine.rows_desc(x, d)
        P = engine._ptr

        def call():
            return lib.lgcn_propagate_forward_sides(
                P(g.rowptr), P(g.edges), P(g.row_ids), ctypes.byref(sides), plans, e0d, d, K,
                bufs, P(out), sc.handle, engine._stream(dev))
        assert call() == 0
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        print("capturing ...", flush=True)
        with torch.cuda.graph(graph):
            rc = call()
        assert rc == 0, rc
        print("lane-1 aux under the capture:", sc.state(engine.SCHED_STATE_L1_AUX), flush=True)
    print("captured:", engine.last_schedule if mode != "prealloc" else "", flush=True)
    ok = True
    for _ in range(2):
        out.fill_(float("nan"))
        graph.replay()
        ok = ok and np.array_equal(out.cpu().numpy(), want)
    print(mode, "replays bitwise:", ok, flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
