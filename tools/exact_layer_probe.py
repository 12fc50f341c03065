"""Component timing of one exact-mode layer on the C3 power-law graph, per emulation threshold:
the emulation block pass, the layer kernel (bundles + whole long rows), the walk (all rows and
the longest row alone), each serialised on one stream, then the layer as spmm_layer runs it
(emulation on side streams beside the layer kernel).

    python tools/exact_layer_probe.py [--emu-min 4096,65536,...] [--layers 2]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gcn_recommendation_amd import engine  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--emu-min", default="0")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--blk-modes", default="",
                    help="with a LGCN_EMU_MODES/STATS build (LGCN_LIB): block-pass timing with "
                         "parts switched off, e.g. 1,2,4,7 (1 stage, 2 candidates, 4 lsb)")
    a = ap.parse_args()
    cfg = bench.CONFIGS[a.config]
    dev = torch.device("cuda:0")
    lib = engine.load_library()
    r, c, v, _, _, _ = bench.make_graph(cfg, "powerlaw", 16)
    U, I = cfg["users"], cfg["items"]
    n, d = U + I, cfg["d"]
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.vstack((r, c))), torch.from_numpy(v),
                                  (n, n)).to(dev)
    g = engine.graph_from_coo(adj)
    gen = torch.Generator().manual_seed(42)
    e0 = [bench.xavier(U, d, gen).to(dev), bench.xavier(I, d, gen).to(dev)]
    st = engine._stream(dev)
    P = engine._ptr
    ep = engine._epilogue(engine.LGCN_EPI_STORE)
    y = torch.empty((n, d), device=dev)
    deg = np.sort(g.degrees())[::-1]
    chunk_ms = None
    for emu_min in [int(t) for t in a.emu_min.split(",")]:
        hp = g.hubs(128, mode="exact", emu_min=emu_min)
        plan = hp.struct(d, dev)
        rest = engine.PlanT.from_buffer_copy(plan)
        rest.n_emu_rows = rest.n_emu_blocks = rest.emu_scratch_blocks = 0
        rest.emu_part_rows[0] = rest.emu_part_rows[1] = 0
        rest.emu_part_blocks[0] = rest.emu_part_blocks[1] = 0
        args = (P(g.rowptr), P(g.edges), P(g.row_ids), g.n_rows)
        print(f"emu_min {emu_min}: long rows {hp.n_long}, emulated rows {hp.n_emu_rows} "
              f"({hp.n_emu_blocks} blocks, {int(deg[:hp.n_emu_rows].sum()):,} edges)", flush=True)
        xs = e0
        for layer in range(1, a.layers + 1):
            x = engine.rows_desc(xs, d)
            t = {}
            t["layer_kernel"] = timed(lambda: lib.lgcn_layer(*args, ctypes.byref(rest), x, 1.0,
                                                             None, P(y), d, d, ctypes.byref(ep),
                                                             None, st))
            if hp.n_emu_rows:
                (r0, r1), (b0, b1) = hp.walk_parts(g.nnz)
                nb_all = hp.n_emu_blocks

                def blocks(k0, k1):
                    assert lib.lgcn_emu_blocks(
                        P(g.edges), plan.emu_blocks + k0 * 16, k1 - k0, x, 1.0, None, d,
                        plan.emu_rel + k0 * d * engine.LGCN_EMU_CANDS * 4,
                        plan.emu_meta + k0 * d * engine.LGCN_EMU_META_BYTES,
                        plan.emu_stage + k0 * (d + 1) * engine.LGCN_EMU_BLOCK * 4, None, st) == 0
                t["part0_blocks"] = timed(lambda: blocks(0, b0))
                t["part1_blocks"] = timed(lambda: blocks(b0, b1))
                for m in [int(k) for k in a.blk_modes.split(",") if k.strip()]:
                    lib.lgcn_emu_set_blk_mode(m)
                    t[f"part0_blocks_off{m}"] = timed(lambda: blocks(0, b0))
                    t[f"part1_blocks_off{m}"] = timed(lambda: blocks(b0, b1))
                    lib.lgcn_emu_set_blk_mode(0)
                t["blocks_all_walked"] = timed(lambda: blocks(0, b1))
                slots = engine.emu_slots()

                def walk(lo, hi, sl):
                    assert lib.lgcn_emu_walk(P(g.edges), plan.emu_blocks,
                                             hp.emu_rows[lo:].data_ptr(), hi - lo, plan.emu_rel,
                                             plan.emu_meta, plan.emu_stage, x, 1.0, None, P(y),
                                             d, d, ctypes.byref(ep), sl, None, st) == 0
                blocks(0, b1)
                t["walk_row0"] = timed(lambda: walk(0, 1, slots[0]))
                if r0 > 0:
                    t["walk_part0"] = timed(lambda: walk(0, r0, slots[0]))
                if r1 > r0:
                    t["walk_part1"] = timed(lambda: walk(r0, r1, slots[-1]))
                if hp.n_emu_rows > r1:
                    rb = hp.emu_rows.element_size() * 4
                    t["chain_rows"] = timed(lambda: lib.lgcn_chain_rows(
                        P(g.edges), plan.emu_blocks, plan.emu_rows + r1 * rb, hp.n_emu_rows - r1,
                        x, 1.0, P(y), d, d, ctypes.byref(ep), st))
                print(f"  parts: rows {r0}/{r1 - r0}/{hp.n_emu_rows - r1} (walk part 0 / walk "
                      f"part 1 / chain), walked blocks {b1} of {nb_all}; chain max degree "
                      f"{engine.chain_max_degree(g.nnz)}", flush=True)
            t["layer_overlapped"] = timed(lambda: engine.spmm_layer(g, xs, y, d, ep, 128, hp))
            os.environ["LGCN_EMU_OVERLAP"] = "0"
            t["layer_serial"] = timed(lambda: engine.spmm_layer(g, xs, y, d, ep, 128, hp))
            del os.environ["LGCN_EMU_OVERLAP"]
            if chunk_ms is None or layer not in chunk_ms:
                chunk_ms = chunk_ms or {}
                hc = g.hubs(128, mode="chunk")
                chunk_ms[layer] = timed(lambda: engine.spmm_layer(g, xs, y, d, ep, 128, hc))
            t["chunk_mode_layer"] = chunk_ms[layer]
            engine.emu_trace = []
            engine.spmm_layer(g, xs, y, d, ep, 128, hp)
            torch.cuda.synchronize()
            ev0 = engine.emu_trace[0][1]
            print(f"  layer {layer} phases (ms from start): " + ", ".join(
                f"{nm} {ev0.elapsed_time(e):.3f}" for nm, e in engine.emu_trace[1:]), flush=True)
            engine.emu_trace = None
            print(f"  layer {layer}: " + ", ".join(f"{k} {val:.3f}" for k, val in t.items()),
                  flush=True)
            if layer < a.layers:
                nxt = torch.empty((n, d), device=dev)
                engine.spmm_layer(g, xs, nxt, d, ep, 128, hp)
                xs = [nxt]
        del plan, rest
        hp._scratch.clear()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
