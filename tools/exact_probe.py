"""Probe of the exact hub path on the C3 power-law graph: plan sizes, per-layer times, and (with
a LGCN_EMU_STATS build loaded through LGCN_LIB) the walker's fast/slow block decisions.

    python tools/exact_probe.py [--emu-min N] [--config c3] [--reps 3]
    python -m gcn_recommendation_amd._build emustats LGCN_EMU_STATS=1  # then LGCN_LIB=... --stats
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402

NAMES = ["translated", "resolved", "-", "not predicted", "resolve iterations", "-", "-", "-"]


def stats(lib):
    buf = (ctypes.c_ulonglong * 8)()
    assert lib.lgcn_emu_stats(buf) == 0
    return dict(zip(NAMES, list(buf)))


PHASES = ["tables", "predict", "slot wait", "scans", "resolve", "on-demand fetch", "-", "-",
          "chunks", "predicted", "resolved", "not predicted", "resolve iterations"]


def phase_stats(lib):
    buf = (ctypes.c_ulonglong * 16)()
    assert lib.lgcn_emu_phase(buf) == 0
    t = sum(buf[:8])
    print("  row 0 col 0 walker phases (s_memtime ticks, share): " + ", ".join(
        f"{n} {buf[k]} ({100 * buf[k] / max(t, 1):.0f}%)" for k, n in enumerate(PHASES[:6])) +
        "; " + ", ".join(f"{n} {buf[k]}" for k, n in enumerate(PHASES) if k >= 8), flush=True)


def row_stats(lib, hp, d, quiet=False):
    buf = (ctypes.c_ulonglong * 1024)()
    assert lib.lgcn_emu_row_stats(buf) == 0
    if quiet:
        return
    a = np.array(buf, dtype=np.float64).reshape(256, 4)
    rows = hp.emu_rows.cpu().numpy()
    for k in list(range(min(8, len(rows)))) + [min(len(rows), 256) - 1]:
        f, s_, ts, tmax = a[k]
        nb = rows[k, 2]
        print(f"  row {k}: {nb} blocks x {d} cols: translated {f / d:.0f} resolved {s_ / d:.0f} per "
              f"col ({100 * s_ / max(f + s_, 1):.1f}%), cycles/resolved block "
              f"{ts / max(s_, 1):.0f}, max wave time {tmax / 2.1e3:.0f} us (at 2.1 GHz)",
              flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--gen", default="powerlaw")
    ap.add_argument("--emu-min", type=int, default=None)
    ap.add_argument("--thr", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--walk", action="store_true", help="time layer 1's walk on row subsets")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    lib = engine.load_library()
    if a.stats:
        lib.lgcn_emu_stats.argtypes = [ctypes.c_void_p]
        lib.lgcn_emu_row_stats.argtypes = [ctypes.c_void_p]
        lib.lgcn_emu_set_mode.argtypes = [ctypes.c_int]
        lib.lgcn_emu_phase.argtypes = [ctypes.c_void_p]
    r, c, v, _, _, _ = bench.make_graph(cfg, a.gen, 16)
    U, I, B = cfg["users"], cfg["items"], cfg.get("brands", 0)
    n, d, K = U + I + B, cfg["d"], cfg["K"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    g = engine.graph_from_coo(adj)
    gen = torch.Generator().manual_seed(42)
    segs = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
    hp = g.hubs(a.thr, mode="exact", emu_min=a.emu_min)
    deg = np.sort(g.degrees())[::-1]
    print(f"plan: long rows {hp.n_long}, emulated rows {hp.n_emu_rows} ({hp.n_emu_blocks} blocks, "
          f"{int(deg[:hp.n_emu_rows].sum()):,} edges), emu_min {hp.emu_min}; top degrees "
          f"{deg[:6].tolist()}", flush=True)
    for rep in range(a.reps):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(K)]
        torch.cuda.synchronize()
        t0 = time.time()
        engine.propagate_forward(g, segs, K, a.thr, layer_events=ev, hub_mode="exact",
                                 emu_min=a.emu_min)
        torch.cuda.synchronize()
        print(f"rep {rep}: {1e3 * (time.time() - t0):.2f} ms wall; per layer "
              f"{[round(x.elapsed_time(y), 3) for x, y in ev]}", flush=True)
        if a.stats:
            print("  walker decisions (all layers):", stats(lib), flush=True)
            row_stats(lib, hp, d)
    if a.stats:
        per_layer_stats(lib, g, segs, d, K, a.thr, a.emu_min, hp)
    if a.walk:
        walk_timing(g, segs, d, a.thr, a.emu_min)




def per_layer_stats(lib, g, segs, d, K, thr, emu_min, hp):
    """Walker decisions of each layer of one forward (row 0 and all rows)."""
    n = g.n_rows
    stats(lib)
    row_stats(lib, hp, d, quiet=True)
    phase_stats(lib)
    layers = [torch.empty((n, d), device=g.device) for _ in range(K)]
    xs = segs
    for k in range(K):
        engine.spmm_layer(g, xs, layers[k], d, engine._epilogue(engine.LGCN_EPI_STORE), thr,
                          hubs=g.hubs(thr, mode="exact", emu_min=emu_min))
        torch.cuda.synchronize()
        st = stats(lib)
        buf = (ctypes.c_ulonglong * 1024)()
        lib.lgcn_emu_row_stats(buf)
        r0 = np.array(buf[:4], dtype=np.float64)
        print(f"  layer {k + 1}: all rows {st}; row 0 fast {r0[0] / d:.0f} slow {r0[1] / d:.0f} "
              f"per column", flush=True)
        phase_stats(lib)
        xs = [layers[k]]


def walk_timing(g, segs, d, thr, emu_min):
    """Layer 1's emulation walk timed on subsets of the emulated rows (isolated critical path
    vs the crowd); with a LGCN_EMU_STATS build also row 0's decisions and the timing
    experiments (1: re-run blocks skip their chain, 2: every block translates)."""
    lib = engine.load_library()
    hp = g.hubs(thr, mode="exact", emu_min=emu_min)
    plan = hp.struct(d, g.device)
    x = engine.rows_desc(segs, d)
    st = engine._stream(g.device)
    y = torch.empty((g.n_rows, d), device=g.device)
    ep = engine._epilogue(engine.LGCN_EPI_STORE)
    assert lib.lgcn_emu_blocks(engine._ptr(g.edges), plan.emu_blocks, hp.n_emu_blocks, x, 1.0, None,
                               d, plan.emu_rel, plan.emu_meta, plan.emu_stage, None, st) == 0
    has_modes = bool(os.environ.get("LGCN_LIB")) and hasattr(lib, "lgcn_emu_set_mode")
    has_stats = has_modes and hasattr(lib, "lgcn_emu_stats")
    if has_modes:
        lib.lgcn_emu_set_mode.argtypes = [ctypes.c_int]
    for mode in ([0, 1, 2, 3, 4, 5] if has_modes else [0]):
        if has_modes:
            lib.lgcn_emu_set_mode(mode)
            torch.cuda.synchronize()
        if has_stats:
            stats(lib)
            row_stats(lib, hp, d, quiet=True)
            if hasattr(lib, "lgcn_emu_phase"):
                buf = (ctypes.c_ulonglong * 16)()
                lib.lgcn_emu_phase(buf)  # reset
        if has_modes:
            print(f" walker mode {mode} (0 normal, 1 re-run blocks skip the chain, 2 all translate, "
                  f"3 all resolved, 4 all fail, none resolved)")
        for lo, hi in ((0, 1), (1, 2), (0, 8)) + (((8, hp.n_emu_rows), (0, hp.n_emu_rows))
                                                if mode == 0 else ()):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            assert lib.lgcn_emu_walk(engine._ptr(g.edges), plan.emu_blocks,
                                     hp.emu_rows[lo:].data_ptr(), hi - lo, plan.emu_rel,
                                     plan.emu_meta, plan.emu_stage, x, 1.0, None, engine._ptr(y),
                                     d, d, ctypes.byref(ep), engine.emu_slots()[0], None, st) == 0
            b.record()
            torch.cuda.synchronize()
            print(f"  walk rows [{lo}, {hi}): {a.elapsed_time(b):.3f} ms", flush=True)
            if has_stats and (lo, hi) == (0, 1):
                print("   row 0 decisions:", stats(lib), flush=True)
                row_stats(lib, hp, d, quiet=True)
                phase_stats(lib)
    if has_modes:
        lib.lgcn_emu_set_mode(0)

if __name__ == "__main__":
    main()
