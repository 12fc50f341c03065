"""The C-ABI library: loads on a CPU host, exports every symbol include/lgcn.h declares, its
struct layouts match the ctypes mirror, and host-side argument validation answers without
touching a GPU."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT
from gcn_recommendation_amd import _build, engine

HEADER = os.path.join(ROOT, "include", "lgcn.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+(lgcn_\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    _build.build()
    return engine.load_library()


def test_library_exports_every_declared_symbol(lib):
    syms = declared_symbols()
    assert len(syms) >= 12
    out = subprocess.check_output(["nm", "-D", "--defined-only", engine.LIB_PATH], text=True)
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    bound = set(name for name, _, _ in engine.ABI)
    assert set(syms) == bound, set(syms) ^ bound


def test_library_is_gfx950_code_object(lib):
    blob = open(engine.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_version_and_errors(lib):
    assert lib.lgcn_abi_version() == engine.ABI_VERSION == 14
    assert b"invalid" in lib.lgcn_error_string(-1)
    assert lib.lgcn_error_string(0) == b"success"


def test_argument_validation_without_gpu(lib):
    ep = engine.EpilogueT()
    ep.mode = 7
    rows = engine.RowsT()
    # bad epilogue / bad d / negative sizes return before any HIP call
    assert lib.lgcn_spmm_layer(None, None, None, 0, 0, None, 0, None, rows, 1.0, None, None, 0,
                               64, ctypes.byref(ep), None) == -1
    ep.mode = engine.LGCN_EPI_STORE
    assert lib.lgcn_spmm_layer(None, None, None, 10, 0, None, 0, None, rows, 1.0, None, None, 0,
                               0, ctypes.byref(ep), None) == -1
    assert lib.lgcn_spmm_layer(None, None, None, -1, 0, None, 0, None, rows, 1.0, None, None, 0,
                               64, ctypes.byref(ep), None) == -1
    assert lib.lgcn_spmm_layer(None, None, None, 0, 0, None, 0, None, rows, 0.0, None, None, 64,
                               64, ctypes.byref(ep), None) == -1
    ep.mode = engine.LGCN_EPI_MEAN
    ep.n_prev = 18
    ep.div = 2.0
    assert lib.lgcn_hub_combine(None, 0, 0, None, None, 64, 64, ctypes.byref(ep), None) == -3
    ep.n_prev = 2
    assert lib.lgcn_hub_combine(None, 4, 5, None, None, 64, 64, ctypes.byref(ep), None) == -1
    assert lib.lgcn_rows_nonzero(engine.RowsT(), 10, 64, None, None, None) == -1
    assert lib.lgcn_rows_nonzero(engine.RowsT(), 10, 0, None, None, None) == -1
    assert lib.lgcn_propagate_forward(None, None, None, 5, None, rows, 64, -1,
                                      None, None, None, None, None) == -1
    plan = engine.PlanT()
    plan.n_emu_rows = 3  # emulated rows without their buffers
    ep.mode = engine.LGCN_EPI_STORE
    assert lib.lgcn_layer(None, None, None, 0, ctypes.byref(plan), rows, 1.0, None, None, 64, 64,
                          ctypes.byref(ep), None, None) == -1
    assert lib.lgcn_layer(None, None, None, 0, None, rows, 1.0, None, None, 64, 64,
                          ctypes.byref(ep), None, None) == -1
    plan.n_emu_rows, plan.n_emu_blocks = 0, 0
    plan.emu_part_rows[0], plan.emu_part_rows[1] = 1, 0  # parts out of order
    assert lib.lgcn_layer(None, None, None, 0, ctypes.byref(plan), rows, 1.0, None, None, 64, 64,
                          ctypes.byref(ep), None, None) == -1
    # the schedule: 1..7 auxiliary streams (4..7: a second lane); its knobs validated before
    # any HIP call
    h = ctypes.c_void_p()
    assert lib.lgcn_sched_create(None, 2, ctypes.byref(h)) == -1
    arr = (ctypes.c_void_p * 8)()
    assert lib.lgcn_sched_create(arr, 4, ctypes.byref(h)) == -1   # null streams
    assert lib.lgcn_sched_create(arr, 8, ctypes.byref(h)) == -1
    assert lib.lgcn_sched_create(arr, 0, ctypes.byref(h)) == -1
    assert lib.lgcn_sched_set(None, engine.SCHED_SLOTS0, 4) == -1
    assert lib.lgcn_sched_destroy(None) == 0
    assert lib.lgcn_emu_blocks(None, None, -1, rows, 1.0, None, 64, None, None, None, None,
                               None) == -1
    assert lib.lgcn_emu_blocks(None, None, 0, rows, 1.0, None, 64, None, None, None, None,
                               None) == 0
    assert lib.lgcn_emu_walk(None, None, None, 2, None, None, None, rows, 1.0, None, None, 64, 64,
                             ctypes.byref(ep), 0, None, None) == -1
    assert lib.lgcn_emu_walk(None, None, None, 0, None, None, None, rows, 1.0, None, None, 64, 64,
                             ctypes.byref(ep), 64, None, None) == -1   # slots out of range
    assert [lib.lgcn_chain_supported(d) for d in (4, 8, 12, 16, 24, 32, 64, 100, 192, 256)] == \
        [0, 1, 0, 1, 1, 1, 1, 0, 1, 1]
    assert lib.lgcn_chain_rows(None, None, None, 0, rows, 1.0, None, 64, 64, ctypes.byref(ep),
                               None) == 0     # nothing to do
    assert lib.lgcn_chain_rows(None, None, None, 2, rows, 1.0, None, 64, 12, ctypes.byref(ep),
                               None) == -1    # unsupported width
    # (+ padding, emu_live, emu_part_max_blocks, emu_out)
    assert ctypes.sizeof(engine.PlanT) == 8 * 8 + 6 * 4 + 5 * 4 + 4 + 8 + 8 + 8
    # live-edge rows: the row mask and the scratch are required, widths as the chain kernel's
    assert lib.lgcn_live_rows(None, None, 4, None, 2, rows, 1.0, None, None, 64, 64,
                              ctypes.byref(ep), 0, 0, ctypes.c_void_p(256), None) == -1   # no x_nz
    assert lib.lgcn_live_rows(None, None, 4, None, 2, rows, 1.0, ctypes.c_void_p(8), None, 64, 12,
                              ctypes.byref(ep), 0, 0, ctypes.c_void_p(256), None) == -1   # width
    assert lib.lgcn_live_rows(None, None, 0, None, 0, rows, 1.0, ctypes.c_void_p(8), None, 64, 64,
                              ctypes.byref(ep), 0, 0, None, None) == 0   # nothing to do
    assert lib.lgcn_live_scratch_bytes(3, 10) >= 10 * 256 * 8 + 10 * 4 + 3 * 32
    nbytes = ctypes.c_size_t(0)
    assert lib.lgcn_coo_sort_perm(None, -5, 10, None, None, None, None, None,
                                  ctypes.byref(nbytes), None) == -1
    assert lib.lgcn_csr_order_by_degree(None, None, -1, 0, 0, 0, None, None, None, None, None,
                                        None, None, None, None, ctypes.byref(nbytes), None) == -1
    assert lib.lgcn_csr_order_by_degree(None, None, 10, 0, 0, 0, None, None, None, None, None,
                                        None, None, None, ctypes.c_void_p(1), ctypes.byref(nbytes),
                                        None) == -1
    # the two key buffers come together or not at all
    assert lib.lgcn_csr_order_by_degree(None, None, 10, 0, 0, 0, None, None, None, None, None,
                                        None, ctypes.c_void_p(8), None, None, ctypes.byref(nbytes),
                                        None) == -1
    # sides must lie inside [0, n_rows]
    for lo, hi in ((-1, 3), (5, 4), (2, 11)):
        assert lib.lgcn_csr_order_by_degree(None, None, 10, 0, lo, hi, None, None, None, None,
                                            None, None, None, None, None, ctypes.byref(nbytes),
                                            None) == -1
    assert lib.lgcn_csr_check_bipartite(None, None, None, 10, 5, 3, 2, None, None) == -1
    assert lib.lgcn_csr_check_bipartite(None, None, None, 10, 0, 2, 3, ctypes.c_void_p(4),
                                        None) == 0   # no edges: nothing to check
    # the sided entry points: the slot layout, eight plans and the slot order are required
    sd = engine.SidesT()
    sd.n, sd.split = 5, 2
    sd.class_end[0], sd.class_end[1] = 2, 2
    assert lib.lgcn_propagate_forward_sides(None, None, None, None, None, rows, 64, 2,
                                            None, ctypes.c_void_p(8), None, None) == -1
    assert lib.lgcn_propagate_forward_sides(None, None, None, ctypes.byref(sd), None, rows, 64, 2,
                                            None, ctypes.c_void_p(8), None, None) == -1
    assert lib.lgcn_propagate_backward_sides(None, None, None, ctypes.byref(sd), None, rows, None,
                                             64, 1, None, ctypes.c_void_p(8), None, None) == -1
    # side classes: ranges checked before anything runs
    for split, p0, p1 in ((11, 0, 0), (4, 3, 2), (4, 0, 7)):
        assert lib.lgcn_csr_side_classes(None, None, None, 10, 0, split, p0, p1, None, None, None,
                                         None, None, None, ctypes.byref(nbytes), None) == -1
    assert lib.lgcn_sched_state(None, engine.SCHED_STATE_LANES) == -1


def test_struct_layout_matches_header():
    """Compile a probe against include/lgcn.h with gcc and compare sizeof/offsetof."""
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "lgcn.h"
int main(void){
 printf("%zu %zu %zu %zu\n", sizeof(lgcn_rows_t), sizeof(lgcn_epilogue_t),
        sizeof(lgcn_hub_item_t), sizeof(lgcn_hub_row_t));
 printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(lgcn_hub_plan_t),
        offsetof(lgcn_hub_plan_t, emu_live), offsetof(lgcn_epilogue_t, prev0),
        offsetof(lgcn_epilogue_t, prev_dense), offsetof(lgcn_epilogue_t, ld_prev),
        offsetof(lgcn_epilogue_t, addend), offsetof(lgcn_epilogue_t, addend_nz));
 return 0;}
"""
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "probe.c")
        exe = os.path.join(td, "probe")
        open(c, "w").write(src)
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        l1, l2 = subprocess.check_output([exe], text=True).split("\n")[:2]
    sizes = [int(x) for x in l1.split()]
    offs = [int(x) for x in l2.split()]
    assert sizes == [ctypes.sizeof(engine.RowsT), ctypes.sizeof(engine.EpilogueT), 16, 16]
    E = engine.EpilogueT
    assert offs == [ctypes.sizeof(engine.PlanT), engine.PlanT.emu_live.offset, E.prev0.offset,
                    E.prev_dense.offset, E.ld_prev.offset, E.addend.offset, E.addend_nz.offset]


def test_engine_refuses_missing_library(tmp_path):
    with pytest.raises(engine.LgcnError):
        engine._lib, saved = None, engine._lib
        try:
            engine.load_library(str(tmp_path / "nope.so"))
        finally:
            engine._lib = saved


def test_tune_knobs(lib):
    """lgcn_tune: every knob answers its previous value (a negative value only queries), an
    unknown knob is refused; knobs never change results (tested on the GPU)."""
    for knob in (engine.TUNE_ROWS_PER_GROUP, engine.TUNE_UNROLL, engine.TUNE_MEAN_PREFETCH,
                 engine.TUNE_MIN_GROUPS, engine.TUNE_EMU_MARGIN):
        old = lib.lgcn_tune(knob, -1)
        assert old >= 0
        assert lib.lgcn_tune(knob, 7) == old
        assert lib.lgcn_tune(knob, old) == 7
        assert lib.lgcn_tune(knob, -1) == old
    assert lib.lgcn_tune(99, 1) == -1
