"""The hub plans of the sided propagation built the way a C host builds them:
only the C planner entry points — lgcn_emu_min_default, lgcn_chain_max_default, lgcn_plan_items,
lgcn_plan_exact, lgcn_plan_scratch_bytes — on the host copies of the slot-order row pointers and
row ids, device memory for the lists and scratch (hipMalloc in C; torch tensors here, which is
all the Python binding adds). Used by tools/c_abi_timing.py and tests/test_gpu_parity.py."""
import ctypes

import numpy as np
import torch

from gcn_recommendation_amd import engine


def c_host_side_plans(lib, rowptr_host, row_ids_host, segments, nnz_total, d, device,
                      threshold=128, emu_min=None, chain_max=None):
    """lgcn_hub_plan_t[2 * len(segments)] (two scratch sets per segment) and the device buffers
    they point at (keep them alive). emu_min / chain_max: the library defaults for the whole
    graph's nonzeros unless given."""
    rp_all = np.ascontiguousarray(rowptr_host, dtype=np.int32)
    ids_all = np.ascontiguousarray(row_ids_host, dtype=np.int32)
    if emu_min is None:
        emu_min = int(lib.lgcn_emu_min_default(int(nnz_total)))
    if chain_max is None:
        chain_max = int(lib.lgcn_chain_max_default(int(nnz_total)))
    plans = (engine.PlanT * (2 * len(segments)))()
    keep = []
    for g, (a, b) in enumerate(segments):
        rp = np.ascontiguousarray(rp_all[a:b + 1])
        ids = np.ascontiguousarray(ids_all[a:b])
        n = b - a
        m = ctypes.c_int32(0)
        items = None
        if n > 0:
            engine._check(lib.lgcn_plan_items(rp.ctypes.data, ids.ctypes.data, n, threshold,
                                              emu_min, None, ctypes.byref(m)), "lgcn_plan_items")
        if m.value:
            h = np.empty((m.value, 4), np.int32)
            engine._check(lib.lgcn_plan_items(rp.ctypes.data, ids.ctypes.data, n, threshold,
                                              emu_min, h.ctypes.data, ctypes.byref(m)),
                          "lgcn_plan_items")
            items = torch.from_numpy(h).to(device)
        base = engine.PlanT()
        if n > 0:
            engine._check(lib.lgcn_plan_exact(rp.ctypes.data, ids.ctypes.data, n,
                                              max(threshold, emu_min), chain_max, 0, None, None,
                                              ctypes.byref(base)), "lgcn_plan_exact(size)")
        er = eb = None
        if base.n_emu_rows:
            hr = np.empty((base.n_emu_rows, 4), np.int32)
            hb = np.empty((base.n_emu_blocks, 4), np.int32)
            engine._check(lib.lgcn_plan_exact(rp.ctypes.data, ids.ctypes.data, n,
                                              max(threshold, emu_min), chain_max, 0,
                                              hr.ctypes.data, hb.ctypes.data,
                                              ctypes.byref(base)), "lgcn_plan_exact")
            er, eb = torch.from_numpy(hr).to(device), torch.from_numpy(hb).to(device)
        sz = (ctypes.c_size_t * 3)()
        engine._check(lib.lgcn_plan_scratch_bytes(ctypes.byref(base), d, 0, sz),
                      "lgcn_plan_scratch_bytes")
        keep += [items, er, eb]
        for j in (0, 1):
            p = engine.PlanT()
            ctypes.memmove(ctypes.byref(p), ctypes.byref(base), ctypes.sizeof(p))
            p.threshold = threshold
            p.items, p.n_items = (items.data_ptr() if items is not None else None), m.value
            p.emu_rows = er.data_ptr() if er is not None else None
            p.emu_blocks = eb.data_ptr() if eb is not None else None
            if sz[0]:
                bufs = [torch.empty(int(x), dtype=torch.uint8, device=device) for x in sz]
                keep += bufs
                p.emu_rel, p.emu_meta, p.emu_stage = (t.data_ptr() for t in bufs)
            if base.n_emu_rows:  # the deferred mean's row sums (lgcn_hub_plan_t emu_out)
                eo = torch.empty(base.n_emu_rows * d, dtype=torch.float32, device=device)
                keep.append(eo)
                p.emu_out = eo.data_ptr()
            plans[2 * g + j] = p
    return plans, keep
