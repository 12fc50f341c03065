"""Host planner for long ("hub") rows: chunks tile each hub row exactly, in order; the exact plan
covers every hub row once (whole-row items or emulation blocks of <= 256 edges, in edge order)."""
import numpy as np

from gcn_recommendation_amd import engine


def test_plan_covers_hub_rows_exactly():
    deg = np.array([0, 3, 700, 1, 2000, 512, 513])
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    hp = engine.plan_hubs(rowptr, 512, 256, "cpu", pre_group=0, mode="chunk")
    items = hp.items.numpy()
    rows = hp.rows.numpy()
    assert hp.n_pre == 0 and hp.n_rows == hp.n_entries == 3
    assert list(rows[:, 0]) == [2, 4, 6]
    assert hp.n_slots == items.shape[0] == 3 + 8 + 3
    for r, first, n, _ in rows:
        it = items[first:first + n]
        assert (it[:, 0] == r).all()
        assert it[0, 1] == rowptr[r] and it[-1, 2] == rowptr[r + 1]
        assert (it[1:, 1] == it[:-1, 2]).all()
        assert (it[:, 3] == np.arange(first, first + n)).all()
        assert ((it[:, 2] - it[:, 1]) <= 256).all()


def test_two_level_combine_plan():
    """Rows with more than pre_group chunks: leading pre-reduction entries sum consecutive runs
    of the row's chunk slots into new slots (after all chunk slots); the row's final entry sums
    exactly those new slots; rows with few chunks are untouched."""
    deg = np.array([5, 300, 10 ** 5 + 7, 4096, 1000])
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    hp = engine.plan_hubs(rowptr, 128, 256, "cpu", pre_group=8, mode="chunk")
    items, tab = hp.items.numpy(), hp.rows.numpy()
    n_chunks = items.shape[0]
    assert n_chunks == 2 + 391 + 16 + 4
    pre, fin = tab[:hp.n_pre], tab[hp.n_pre:]
    assert hp.n_rows == 4 and list(fin[:, 0]) == [1, 2, 3, 4]
    assert (pre[:, 3] == 1).all() and (fin[:, 3] == 0).all()
    assert hp.n_pre == 49 + 2 and hp.n_slots == n_chunks + hp.n_pre
    assert (pre[:, 0] == n_chunks + np.arange(hp.n_pre)).all()
    covered = np.zeros(n_chunks, int)
    for tgt, first, n, _ in pre:
        assert 1 <= n <= 8
        covered[first:first + n] += 1
    for r, first, n, _ in fin:
        if first >= n_chunks:  # two-level row: its slots are pre-reduction targets, in order
            it = items[(items[:, 0] == r)]
            src = pre[(pre[:, 0] >= first) & (pre[:, 0] < first + n)]
            assert src[0, 1] == it[0, 3] and src[-1, 1] + src[-1, 2] == it[-1, 3] + 1
            assert (src[1:, 1] == src[:-1, 1] + src[:-1, 2]).all()
        else:
            assert n <= 8
            covered[first:first + n] += 1
    assert (covered == 1).all()  # every chunk partial is summed exactly once


def test_two_level_plan_without_big_rows():
    rowptr = np.array([0, 300, 301, 900], dtype=np.int32)
    hp = engine.plan_hubs(rowptr, 128, 256, "cpu", pre_group=8, mode="chunk")
    assert hp.n_pre == 0 and hp.n_rows == 2 and hp.n_slots == 2 + 3


def test_exact_plan_covers_every_hub_row_once():
    deg = np.array([0, 3, 700, 1, 2000, 512, 513, 256 * 70 + 1, 129, 128])
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    row_ids = np.arange(deg.size)[::-1].astype(np.int32)  # slot s holds row n-1-s
    hp = engine.plan_hubs(rowptr, 128, None, "cpu", row_ids_host=row_ids, mode="exact",
                          emu_min=600)
    items = hp.items.numpy()
    assert (items[:, 3] == -1).all() and hp.n_rows == 0 and hp.n_slots == 0
    long_slots = [s for s in range(deg.size) if 128 < deg[s] <= 600]
    assert list(items[:, 0]) == [row_ids[s] for s in long_slots]
    assert list(items[:, 1]) == [rowptr[s] for s in long_slots]
    assert list(items[:, 2]) == [rowptr[s + 1] for s in long_slots]
    blocks, rows = hp.emu_blocks.numpy(), hp.emu_rows.numpy()
    # emulated rows are stored longest first whatever the slot order (the walks of the longest
    # rows are a layer's critical path; emu_parts cuts the rows by length)
    emu_slots = sorted([s for s in range(deg.size) if deg[s] > 600], key=lambda s: -deg[s])
    assert list(rows[:, 0]) == [row_ids[s] for s in emu_slots]
    assert list(hp.emu_nb) == [-(-deg[s] // 256) for s in emu_slots]
    for k, s in enumerate(emu_slots):
        _, first, nb, _ = rows[k]
        b = blocks[first:first + nb]
        assert (b[:, 0] == k).all() and b[0, 3] == 1 and (b[1:, 3] == 0).all()
        assert b[0, 1] == rowptr[s] and b[-1, 2] == rowptr[s + 1]
        assert (b[1:, 1] == b[:-1, 2]).all() and ((b[:, 2] - b[:, 1]) <= 256).all()
        assert nb == -(-deg[s] // 256)
    assert hp.n_emu_blocks == sum(-(-deg[s] // 256) for s in emu_slots)


def test_exact_mode_has_no_hubs():
    rowptr = np.array([0, 10 ** 6], dtype=np.int32)
    hp = engine.plan_hubs(rowptr, engine.INT32_MAX, 256, "cpu")
    assert hp.n_items == 0 and hp.n_rows == 0


def test_env_threshold(monkeypatch):
    monkeypatch.setenv("LGCN_HUB_THRESHOLD", "exact")
    assert engine.hub_threshold_from_env() == engine.INT32_MAX
    monkeypatch.setenv("LGCN_HUB_THRESHOLD", "64")
    assert engine.hub_threshold_from_env() == 64
    monkeypatch.delenv("LGCN_HUB_THRESHOLD")
    assert engine.hub_threshold_from_env() == engine.DEFAULT_HUB_THRESHOLD


def test_rows_desc_from_addresses_global_rows():
    """Host check of the segment descriptor a rank uses to read E0 rows in place: local row i
    must address global row start+i of cat(segments) (a GPU fault in round 1 came from a
    sign error here)."""
    import torch
    d = 8
    segs = [torch.zeros(5, d), torch.zeros(7, d), torch.zeros(3, d)]
    glob = [(t, r) for t in segs for r in range(t.shape[0])]
    for start in (0, 2, 5, 6, 12, 14):
        desc = engine.rows_desc_from(segs, start, d)
        ptrs, ends = [desc.p0, desc.p1, desc.p2], [desc.end0, desc.end1]
        for i in range(15 - start):
            s = 0 if i < ends[0] else (1 if i < ends[1] else 2)
            if s == 0:
                addr = ptrs[0] + i * d * 4
            elif s == 1:
                addr = ptrs[1] + (i - ends[0]) * d * 4
            else:
                addr = ptrs[2] + (i - ends[1]) * d * 4
            t, r = glob[start + i]
            assert addr == t.data_ptr() + r * d * 4, (start, i)


def test_c_planner_parts_and_scratch():
    """lgcn_plan_exact (the C host planner a C caller uses; engine.plan_hubs calls it): part cuts
    by block count agree with walk_parts, scratch sizes follow lgcn.h, bad input is refused."""
    import ctypes
    lib = engine.load_library()
    deg = np.array([5, 9000, 256 * 9000 + 3, 70_000, 129, 256 * 300, 256 * 8193 + 1, 128])
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    plan = engine.PlanT()
    rc = lib.lgcn_plan_exact(rowptr.ctypes.data, None, deg.size, 128, 60_000, 8192, None, None,
                             ctypes.byref(plan))
    assert rc == 0
    nb = sorted([-(-int(x) // 256) for x in deg if x > 128], reverse=True)
    assert plan.n_emu_rows == len(nb) and plan.n_emu_blocks == sum(nb)
    b1 = -(-60_000 // 256)
    assert list(plan.emu_part_rows) == [sum(x > 8192 for x in nb), sum(x > b1 for x in nb)]
    assert plan.emu_part_blocks[0] == sum(x for x in nb if x > 8192)
    assert plan.emu_part_blocks[1] == plan.emu_scratch_blocks == sum(x for x in nb if x > b1)
    # the longest row of each walked part (the pieced schedule's chunk windows reach it)
    assert list(plan.emu_part_max_blocks) == [max(x for x in nb if x > 8192),
                                              max(x for x in nb if b1 < x <= 8192)]
    rows = np.empty((plan.n_emu_rows, 4), np.int32)
    blocks = np.empty((plan.n_emu_blocks, 4), np.int32)
    assert lib.lgcn_plan_exact(rowptr.ctypes.data, None, deg.size, 128, 60_000, 8192,
                               rows.ctypes.data, blocks.ctypes.data, ctypes.byref(plan)) == 0
    assert list(rows[:, 2]) == nb
    hp = engine.HubPlan(128, emu_nb=np.array(nb))
    pr, pb = hp.walk_parts(60_000 * 256)  # chain_max_degree(nnz) = 60_000 (the forward's)
    assert pr[0] == plan.emu_part_rows[0]
    assert list(pr) == list(plan.emu_part_rows) and list(pb) == list(plan.emu_part_blocks)
    # the backward's operator: its own default, nnz / 512
    assert lib.lgcn_chain_max_default(60_000 * 256) == 60_000
    assert lib.lgcn_chain_max_backward_default(60_000 * 512) == 60_000
    assert list(hp.walk_parts(60_000 * 512, backward=True)[0]) == list(plan.emu_part_rows)
    assert hp.struct(64, "cpu", nnz=60_000 * 256).emu_part_max_blocks[0] == \
        plan.emu_part_max_blocks[0]
    sizes = (ctypes.c_size_t * 3)()
    assert lib.lgcn_plan_scratch_bytes(ctypes.byref(plan), 64, 0, sizes) == 0
    nbw = plan.emu_part_blocks[1]
    assert list(sizes) == [nbw * 64 * 16 * 4, nbw * 64 * 16, nbw * 65 * 256 * 4]
    assert lib.lgcn_plan_scratch_bytes(ctypes.byref(plan), 64, 1, sizes) == 0
    assert sizes[0] == plan.n_emu_blocks * 64 * 16 * 4
    # refused: decreasing row pointers, rows without blocks
    bad = np.array([0, 10, 5], np.int32)
    assert lib.lgcn_plan_exact(bad.ctypes.data, None, 2, 0, 0, 0, None, None,
                               ctypes.byref(plan)) == -1
    assert lib.lgcn_plan_exact(rowptr.ctypes.data, None, deg.size, 128, 0, 0, rows.ctypes.data,
                               None, ctypes.byref(plan)) == -1
    assert lib.lgcn_chain_max_default(1_600_000) == 8192
    assert lib.lgcn_chain_max_default(56_300_000) == 56_300_000 // 256
    assert lib.lgcn_chain_max_default(10 ** 10) == 262144
    assert lib.lgcn_chain_max_backward_default(1_600_000) == 8192
    assert lib.lgcn_chain_max_backward_default(56_300_000) == 56_300_000 // 512
    assert lib.lgcn_chain_max_backward_default(10 ** 10) == 131072
