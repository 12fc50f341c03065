"""Host side of the MI355X LightGCN propagation engine: ctypes binding of liblgcn_engine.so
(include/lgcn.h), the cached COO->CSR graph plan, and the autograd Function that replaces

    ego = torch.cat([user, item, brand]); for k < K: ego = torch.sparse.mm(adj, ego)
    final = torch.mean(torch.stack(all_layers), 0)           (models/lightgcn.py:37-54)

on a HIP device. There is no fallback: if the extension is missing or a launch fails, the call
raises. The library is loaded after `import torch`, so its libamdhip64.so.7 dependency binds to
the HIP runtime torch already loaded.
"""
import ctypes
import os
import threading

import numpy as np
import torch

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "liblgcn_engine.so")

# ---- ABI mirrors (include/lgcn.h) -------------------------------------------------------------
LGCN_EPI_STORE, LGCN_EPI_MEAN, LGCN_EPI_ADD = 0, 1, 2
LGCN_MAX_LAYERS = 16
COO_ROWS_UNSORTED, COO_OUT_OF_RANGE, COO_COLS_UNSORTED = 1, 2, 4
INT32_MAX = 2 ** 31 - 1
TUNE_ROWS_PER_GROUP, TUNE_UNROLL, TUNE_MEAN_PREFETCH, TUNE_MIN_GROUPS = 1, 2, 3, 4
TUNE_EMU_MARGIN = 6
SCHED_SLOTS0, SCHED_SLOTS1, SCHED_CHAIN, SCHED_TIMING_START, SCHED_TIMING_END, SCHED_TRACE = \
    1, 2, 3, 4, 5, 6
SCHED_TRACE_SIDES, SCHED_TIMING_SIDES = 7, 8
SCHED_CLASSES = 16
SCHED_LK_NORMAL = 17
SCHED_LANE1_SHARED = 18
SCHED_STATE_LANES, SCHED_STATE_L1_AUX, SCHED_STATE_CAPTURING, SCHED_STATE_CLASSES = 1, 2, 3, 4
SCHED_STATE_CAPTURE_FULL = 5
# segments of a sided propagation: the three side-0 classes, then side 1
N_SEGS = 4
# phases of one exact layer recorded under SCHED_TRACE (lgcn.h)
TRACE_PHASES = ("start", "part0_blocks", "part1_blocks", "layer_kernel", "chain_rows",
                "part0_walk", "part1_walk", "joined")
ABI_VERSION = 14
LGCN_EMU_CANDS, LGCN_EMU_META_BYTES, LGCN_EMU_BLOCK = 16, 16, 256

# Rows up to this degree run as row bundles in the layer kernel (one sequential fmaf chain each,
# bitwise = reference CPU path). Longer rows ("hubs") follow the hub mode:
#   exact (default): rows up to EMU_MIN_DEGREE are whole-row chains of their own, longer rows are
#                    reproduced exactly by block emulation (lgcn_exact.hip) — bitwise everywhere;
#   chunk:           rows are cut into HUB_CHUNK-edge chunks summed in a fixed order (fast,
#                    deterministic, NOT bitwise to the reference on long rows).
# LGCN_HUB_THRESHOLD=exact puts every row in the bundles (the plain sequential chain; slow on
# power-law hubs, kept as the unoptimised reference mode).
DEFAULT_HUB_THRESHOLD = 128
HUB_MODES = ("exact", "chunk")
# Rows above the bundle threshold and up to this degree run inside the layer kernel as one lane
# group's chain each (LGCN_EMU_MIN_DEGREE; hub items dispatched first in its grid); longer rows go
# to the emulated-row list, where the shorter ones run as sequential chains of their own
# (lgcn_chain_rows, beside the layer kernel) and the longest are block-emulated (emu_parts).
# Default by graph size (lgcn_emu_min_default): 0 (none) below 2^23 nonzeros, 1024 above — at C3
# the rows of 129..1024 edges (most of the ~12k chain rows) were a chain kernel whose grid waited
# behind the layer kernel's on a shared dispatch pipe; inside the layer kernel: forward 14.0-14.4
# -> 12.6-13.0 ms (sweep 512 / 1024 / 1536 / 2048: 12.9-13.0 / 12.6-13.0 / 12.7-13.1 / 12.7-13.3)


def hub_mode_from_env():
    m = os.environ.get("LGCN_HUB_MODE", "exact").lower()
    if m not in HUB_MODES:
        raise LgcnError(f"LGCN_HUB_MODE={m!r} ({' | '.join(HUB_MODES)})")
    return m


def emu_defer_enabled():
    """A final mean half-layer's walks and chains write their rows' sums to scratch and the mean
    of those rows follows once the other lane's layer K-1 is done (lgcn_hub_plan_t emu_out), so
    they start as soon as their block passes are done; LGCN_EMU_DEFER=0 makes them wait (same
    bits)."""
    return os.environ.get("LGCN_EMU_DEFER", "1") != "0"


def emu_min_degree_from_env(nnz=None):
    """LGCN_EMU_MIN_DEGREE, else the library's default for a graph of nnz nonzeros
    (lgcn_emu_min_default; None: small)."""
    v = os.environ.get("LGCN_EMU_MIN_DEGREE", "")
    if v:
        return int(v)
    return int(load_library().lgcn_emu_min_default(int(nnz or 0)))


def chain_max_degree(nnz, backward=False):
    """Rows of the emulated-row list up to this degree run as sequential chains (lgcn_chain_rows,
    ~16 ns per edge), longer ones are block-emulated (block pass + walk): env LGCN_CHAIN_MAX, else
    by graph size (lgcn_chain_max_default: a chain must stay short against the whole layer; the
    backward's operator Âᵀ: lgcn_chain_max_backward_default)."""
    v = os.environ.get("LGCN_CHAIN_MAX", "")
    if v:
        return int(v)
    lib = load_library()
    f = lib.lgcn_chain_max_backward_default if backward else lib.lgcn_chain_max_default
    return int(f(int(nnz)))


# Edges per hub chunk (chunk mode): DEFAULT_HUB_CHUNK when set (tests, tools/tune.py), else by
# graph size (hub_chunk_for). A chunk is one lane group's sequential chain, so it must stay short
# against the whole layer: on the C2 graph (1.6M nonzeros, 0.07-0.1 ms per layer) 128-edge
# chunks run the forward 0.318 -> 0.224 ms, on C3 (56M) 256 is best (tools/tune.py).
DEFAULT_HUB_CHUNK = None


def hub_chunk_for(nnz):
    if DEFAULT_HUB_CHUNK:
        return DEFAULT_HUB_CHUNK
    return 256 if nnz >= 8_000_000 else 128
# Hub rows with more chunks than this are combined in two levels (plan_hubs); 0 = one level
DEFAULT_HUB_PRE_GROUP = 256


class RowsT(ctypes.Structure):
    _fields_ = [("p0", ctypes.c_void_p), ("p1", ctypes.c_void_p), ("p2", ctypes.c_void_p),
                ("end0", ctypes.c_int32), ("end1", ctypes.c_int32), ("ld", ctypes.c_int64)]


class EpilogueT(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("n_prev", ctypes.c_int32), ("div", ctypes.c_float),
                ("pad", ctypes.c_int32), ("prev0", RowsT),
                ("prev_dense", ctypes.c_void_p * LGCN_MAX_LAYERS), ("ld_prev", ctypes.c_int64),
                ("addend", RowsT), ("addend_nz", ctypes.c_void_p)]


class PlanT(ctypes.Structure):
    """lgcn_hub_plan_t"""
    _fields_ = [("items", ctypes.c_void_p), ("rows", ctypes.c_void_p), ("partials", ctypes.c_void_p),
                ("emu_blocks", ctypes.c_void_p), ("emu_rows", ctypes.c_void_p),
                ("emu_rel", ctypes.c_void_p), ("emu_meta", ctypes.c_void_p),
                ("emu_stage", ctypes.c_void_p),
                ("threshold", ctypes.c_int32), ("n_items", ctypes.c_int32),
                ("n_rows", ctypes.c_int32), ("n_pre", ctypes.c_int32),
                ("n_emu_blocks", ctypes.c_int32), ("n_emu_rows", ctypes.c_int32),
                ("emu_part_rows", ctypes.c_int32 * 2), ("emu_part_blocks", ctypes.c_int32 * 2),
                ("emu_scratch_blocks", ctypes.c_int32), ("emu_live", ctypes.c_void_p),
                ("emu_part_max_blocks", ctypes.c_int32 * 2), ("emu_out", ctypes.c_void_p)]


class SidesT(ctypes.Structure):
    """lgcn_sides_t"""
    _fields_ = [("n", ctypes.c_int32), ("split", ctypes.c_int32), ("class_end", ctypes.c_int32 * 2),
                ("part_rows", ctypes.c_int32 * 2)]


class LgcnError(RuntimeError):
    pass


_lib = None
_lib_lock = threading.Lock()

# (name, restype, argtypes) — every symbol include/lgcn.h declares
_P, _I32, _I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
ABI = [
    ("lgcn_abi_version", ctypes.c_int, []),
    ("lgcn_error_string", ctypes.c_char_p, [ctypes.c_int]),
    ("lgcn_tune", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("lgcn_device_info", ctypes.c_int, [ctypes.c_int, _P, _P]),
    ("lgcn_stream_create", ctypes.c_int, [_I32, _P]),
    ("lgcn_capture_full_schedule", ctypes.c_int, []),
    ("lgcn_stream_destroy", ctypes.c_int, [_P]),
    ("lgcn_coo_inspect", ctypes.c_int, [_P, _P, _I64, _I32, _I32, _P, _P]),
    ("lgcn_coo_to_csr", ctypes.c_int, [_P, _P, _P, _I64, _I32, _P, _P, _P, _P, _P]),
    ("lgcn_coo_sort_perm", ctypes.c_int, [_P, _I64, _I32, _P, _P, _P, _P, _P,
                                          ctypes.POINTER(ctypes.c_size_t), _P]),
    ("lgcn_csr_check_symmetric", ctypes.c_int, [_P, _P, _I32, _I64, _P, _P]),
    ("lgcn_csr_order_by_degree", ctypes.c_int, [_P, _P, _I32, _I64, _I32, _I32, _P, _P, _P, _P, _P,
                                                _P, _P, _P, _P, ctypes.POINTER(ctypes.c_size_t),
                                                _P]),
    ("lgcn_csr_check_bipartite", ctypes.c_int, [_P, _P, _P, _I32, _I64, _I32, _I32, _P, _P]),
    ("lgcn_csr_relabel_cols", ctypes.c_int, [_P, _I64, _P, _P, _P]),
    ("lgcn_csr_side_classes", ctypes.c_int, [_P, _P, _P, _I32, _I64, _I32, _I32, _I32, _P, _P, _P,
                                             _P, _P, _P, ctypes.POINTER(ctypes.c_size_t), _P]),
    ("lgcn_adj_degree", ctypes.c_int, [_P, _I64, _I32, _P, _P]),  # (sorted keys, ...)
    ("lgcn_adj_sort_unique", ctypes.c_int, [_P, _P, _I64, _I32, _P, _P, _P, _P, _P, _P,
                                            ctypes.POINTER(ctypes.c_size_t), _P]),
    ("lgcn_adj_finish", ctypes.c_int, [_P, _P, _I64, _I32, _P, _P, _P, _P, _P, _P, _P]),
    ("lgcn_bpr_loss", ctypes.c_int, [_P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64,
                                     _I32, _I32, ctypes.c_float, _P, _P, _P, _P]),
    ("lgcn_fusion_prelayer", ctypes.c_int, [_P, _I64, _P, _I64, _I32, _I32, _I32, _P, _P,
                                            ctypes.c_float, _P, _I64, _P]),
    ("lgcn_chain_max_default", ctypes.c_int32, [_I64]),
    ("lgcn_chain_max_backward_default", ctypes.c_int32, [_I64]),
    ("lgcn_plan_exact", ctypes.c_int, [_P, _P, _I32, _I32, _I32, _I32, _P, _P, _P]),
    ("lgcn_emu_min_default", ctypes.c_int32, [_I64]),
    ("lgcn_plan_items", ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P, _P]),
    ("lgcn_plan_scratch_bytes", ctypes.c_int, [_P, _I32, _I32, ctypes.POINTER(ctypes.c_size_t)]),
    ("lgcn_eval_splits", ctypes.c_int, [_I32, _I32, _I32]),
    ("lgcn_score_topk", ctypes.c_int, [_P, _I64, _P, _I32, _P, _I64, _I32, _I32, _P, _P, _I32,
                                       _I32, _P, _P, _P, _P, _P]),
    ("lgcn_spmm_layer", ctypes.c_int, [_P, _P, _P, _I32, _I32, _P, _I32, _P, RowsT, ctypes.c_float,
                                       _P, _P, _I64, _I32, ctypes.POINTER(EpilogueT), _P]),
    ("lgcn_rows_nonzero", ctypes.c_int, [RowsT, _I32, _I32, _P, _P, _P]),
    ("lgcn_add_nonzero", ctypes.c_int, [_P, _P, _I64, _P]),
    ("lgcn_hub_combine", ctypes.c_int, [_P, _I32, _I32, _P, _P, _I64, _I32,
                                        ctypes.POINTER(EpilogueT), _P]),
    ("lgcn_scale_rows", ctypes.c_int, [RowsT, _I32, _I32, ctypes.c_float, _P, _I64, _P]),
    ("lgcn_emu_blocks", ctypes.c_int, [_P, _P, _I32, RowsT, ctypes.c_float, _P, _I32, _P, _P, _P,
                                       _P, _P]),
    ("lgcn_emu_walk", ctypes.c_int, [_P, _P, _P, _I32, _P, _P, _P, RowsT, ctypes.c_float, _P, _P,
                                     _I64, _I32, ctypes.POINTER(EpilogueT), _I32, _P, _P]),
    ("lgcn_chain_supported", ctypes.c_int, [_I32]),
    ("lgcn_emu_epilogue", ctypes.c_int, [_P, _I32, _P, _I64, _P, _I64, _I32,
                                         ctypes.POINTER(EpilogueT), _P]),
    ("lgcn_live_scratch_bytes", ctypes.c_size_t, [_I32, _I32]),
    ("lgcn_live_rows", ctypes.c_int, [_P, _P, _I32, _P, _I32, RowsT, ctypes.c_float, _P, _P, _I64,
                                      _I32, ctypes.POINTER(EpilogueT), _I32, _I32, _P, _P]),
    ("lgcn_live_flags", ctypes.c_void_p, [_P, _I32, _I32]),
    ("lgcn_chain_rows", ctypes.c_int, [_P, _P, _P, _I32, RowsT, ctypes.c_float, _P, _I64, _I32,
                                       ctypes.POINTER(EpilogueT), _P]),
    ("lgcn_sched_create", ctypes.c_int, [_P, _I32, ctypes.POINTER(ctypes.c_void_p)]),
    ("lgcn_sched_destroy", ctypes.c_int, [_P]),
    ("lgcn_sched_set", ctypes.c_int, [_P, _I32, _I64]),
    ("lgcn_sched_state", ctypes.c_int64, [_P, _I32]),
    ("lgcn_layer", ctypes.c_int, [_P, _P, _P, _I32, ctypes.POINTER(PlanT), RowsT, ctypes.c_float, _P,
                                  _P, _I64, _I32, ctypes.POINTER(EpilogueT), _P, _P]),
    ("lgcn_propagate_forward", ctypes.c_int, [_P, _P, _P, _I32, ctypes.POINTER(PlanT), RowsT, _I32,
                                              _I32, _P, _P, _P, _P, _P]),
    ("lgcn_propagate_backward", ctypes.c_int, [_P, _P, _P, _I32, ctypes.POINTER(PlanT), RowsT, _P,
                                               _I32, _I32, _P, _P, _P, _P]),
    ("lgcn_propagate_forward_sides", ctypes.c_int, [_P, _P, _P, ctypes.POINTER(SidesT),
                                                    ctypes.POINTER(PlanT), RowsT, _I32, _I32, _P,
                                                    _P, _P, _P]),
    ("lgcn_propagate_backward_sides", ctypes.c_int, [_P, _P, _P, ctypes.POINTER(SidesT),
                                                     ctypes.POINTER(PlanT), RowsT, _P, _I32, _I32,
                                                     _P, _P, _P, _P]),
]


def load_library(path=None):
    """Load liblgcn_engine.so (built by __graft_entry__.build()). Raises if absent."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        # LGCN_LIB: an alternative build of the same ABI (A/B timing of kernel variants)
        p = path or os.environ.get("LGCN_LIB") or LIB_PATH
        if not os.path.exists(p):
            raise LgcnError(f"liblgcn_engine.so not found at {p}: run `python -c \"import "
                            f"__graft_entry__ as g; g.build()\"` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(p)
        for name, res, args in ABI:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.lgcn_abi_version() != ABI_VERSION:
            raise LgcnError("liblgcn_engine.so ABI version mismatch")
        _lib = lib
        return lib


def _check(rc, what):
    if rc != 0:
        msg = _lib.lgcn_error_string(rc).decode() if _lib is not None else str(rc)
        raise LgcnError(f"{what} failed: {msg} (code {rc})")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def rows_desc(segments, ld):
    """lgcn_rows_t over 1..3 row segments (each [rows x d] with leading dim ld)."""
    if len(segments) == 1:
        t = segments[0]
        return RowsT(t.data_ptr(), t.data_ptr(), t.data_ptr(), t.shape[0], t.shape[0], ld)
    ps, ends, acc = [], [], 0
    for t in segments:
        ps.append(t.data_ptr())
        acc += t.shape[0]
        ends.append(acc)
    while len(ps) < 3:
        ps.append(ps[-1])
        ends.append(ends[-1])
    return RowsT(ps[0], ps[1], ps[2], ends[0], ends[1], ld)


def rows_desc_from(segments, start, ld):
    """lgcn_rows_t whose row 0 is global row `start` of the concatenation of `segments`
    (a rank's local rows reading E0 in place: segment bases shifted, ends rebased)."""
    ps, ends, acc = [], [], 0
    for t in segments:
        # the kernel addresses local row i of segment s as p_s + (i - end_{s-1}) * ld, and
        # local row end_{s-1} is this segment's row max(start - acc, 0)
        ps.append(t.data_ptr() + max(start - acc, 0) * ld * t.element_size())
        acc += t.shape[0]
        ends.append(max(acc - start, 0))
    while len(ps) < 3:
        ps.append(ps[-1])
        ends.append(ends[-1])
    return RowsT(ps[0], ps[1], ps[2], ends[0], ends[1], ld)


def pack_edges(cols, vals):
    """Host {int32 col, fp32 val} edge records (lgcn_edge_t) from numpy arrays."""
    c = np.asarray(cols, dtype=np.int64).astype(np.uint32).astype(np.uint64)
    v = np.asarray(vals, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return ((v << np.uint64(32)) | c).view(np.int64)


def graph_from_host_csr(rowptr, cols, vals, n_cols, device, order=None, sides=None):
    """Device CSR (possibly rectangular: a rank's row block with global columns) from host
    arrays already in the engine's order. Forward-only: no transpose is attached. sides=(lo, hi)
    (square operators, degree order): side-major slots when the operator is bipartite across
    [lo, hi) and large enough (sides_min_nnz), as graph_from_coo does."""
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int32)
    n_rows = rowptr.size - 1
    nnz = int(rowptr[-1])
    edges = pack_edges(cols, vals) if nnz else np.zeros(1, np.int64)
    g = Graph(n_rows, n_cols, torch.from_numpy(rowptr).to(device),
              torch.from_numpy(edges).to(device), nnz, device)
    g._rowptr_host = rowptr
    if row_order(order) == "degree":
        with torch.cuda.device(device):
            lib, st = load_library(), _stream(device)
            mn = sides_min_nnz()
            if sides is not None and (mn is None or nnz < mn or sides[0] >= sides[1] or
                                      n_rows != n_cols or not is_bipartite(lib, g, sides, st)):
                sides = None
            g = order_by_degree(lib, g, st, sides)
    return g


def row_order(order=None):
    """Processing order of CSR rows: "degree" (default: slots sorted by degree, descending) or
    "stored" (row id order). Env LGCN_ROW_ORDER overrides the default. Results are identical
    either way; only the kernels' load balance changes."""
    o = (order or os.environ.get("LGCN_ROW_ORDER", "degree")).lower()
    if o not in ("degree", "stored"):
        raise LgcnError(f"unknown row order {o!r} (degree | stored)")
    return o


def hub_threshold_from_env(default=DEFAULT_HUB_THRESHOLD):
    v = os.environ.get("LGCN_HUB_THRESHOLD", "")
    if v.lower() in ("exact", "inf", "none", "off"):
        return INT32_MAX
    return int(v) if v else default


# ----------------------------------------------------------------------------------------------
# graph plan: CSR + hub chunks, built once per adjacency tensor and cached on it
# ----------------------------------------------------------------------------------------------
class HubPlan:
    """How one operator's rows above the bundle threshold are summed (lgcn_hub_plan_t).

    chunk mode: `items` are chunks (slot >= 0) and `rows` the combine entries (n_pre
    pre-reductions first). exact mode: `items` are whole long rows (slot = -1: one exact chain,
    epilogue in place) and rows above emu_min are emulated (`emu_blocks` / `emu_rows`)."""

    def __init__(self, threshold, mode="exact", chunk=None, items=None, rows=None, n_slots=0,
                 n_hub_rows=0, n_pre=0, emu_blocks=None, emu_rows=None, emu_min=None,
                 emu_nb=None):
        self.threshold = threshold
        self.mode = mode
        self.chunk = chunk
        self.emu_min = emu_min
        self.items = items      # int32 [n_items, 4] device (lgcn_hub_item_t)
        self.rows = rows        # int32 [n_pre + n_rows, 4] device (lgcn_hub_row_t)
        self.n_items = 0 if items is None else items.shape[0]
        self.n_rows = n_hub_rows  # chunked hub rows (final entries, after the n_pre pre-reductions)
        self.n_pre = n_pre
        self.n_entries = n_pre + n_hub_rows
        self.n_slots = n_slots  # partial rows: chunk slots + pre-reduction slots
        self.emu_blocks = emu_blocks  # int32 [n_emu_blocks, 4] (lgcn_emu_block_t)
        self.emu_rows = emu_rows      # int32 [n_emu_rows, 4] (lgcn_emu_row_t)
        self.n_emu_blocks = 0 if emu_blocks is None else emu_blocks.shape[0]
        self.n_emu_rows = 0 if emu_rows is None else emu_rows.shape[0]
        # host copy of the emulated rows' block counts (longest first): no device read-back
        self.emu_nb = np.zeros(0, np.int64) if emu_nb is None else np.asarray(emu_nb, np.int64)
        self._scratch = {}
        self._live = None
        self._split = None
        self._split_bounds = None

    def emu_parts(self, bounds=(4096, 512)):
        """The emulated rows cut by length into consecutive (row0, row1, block0, block1, short)
        groups: rows of more than bounds[0] blocks, then more than bounds[1], then the rest
        (rows are stored longest first, plan_emulation; short = the last group, whose rows — at
        most bounds[1] * 256 edges — may run as plain sequential chains, lgcn_chain_rows). The
        longest walks are the critical path of a layer. Host data only (graph-capture safe)."""
        if self._split is None or self._split_bounds != bounds:
            nb = self.emu_nb
            cuts = [0] + [int((nb > b).sum()) for b in bounds] + [int(nb.size)]
            firsts = np.concatenate([[0], np.cumsum(nb)])
            self._split = [(r0, r1, int(firsts[r0]), int(firsts[r1]), i == len(bounds))
                           for i, (r0, r1) in enumerate(zip(cuts[:-1], cuts[1:])) if r1 > r0]
            self._split_bounds = bounds
        return self._split

    @property
    def n_long(self):
        return self.n_items if self.mode == "exact" else 0

    def walk_parts(self, nnz, backward=False, part0=None):
        """(part_rows, part_blocks): the emulated rows cut into part 0 (rows of more than
        walk_cut_blocks' b0 blocks, the longest walks: the layer's critical path), part 1 (more
        than chain_max_degree blocks) and the chain rows (lgcn_hub_plan_t emu_part_*)."""
        b0, b1 = walk_cut_blocks(nnz, backward, part0)
        nb = self.emu_nb
        cum = np.concatenate([[0], np.cumsum(nb)])
        r0, r1 = int((nb > b0).sum()), int((nb > b1).sum())
        return [r0, r1], [int(cum[r0]), int(cum[r1])]

    def scratch(self, d, device, n_blocks=None, scratch_set=0):
        """(partials, emu_rel, emu_meta, emu_stage, emu_out) for width d, covering the first n_blocks
        emulated blocks (the walked ones; default all), allocated once per width and set and
        grown on demand (the layers of one operator run in stream order; the bipartite lanes run
        a side's consecutive layers concurrently, on sets 0 and 1). release_scratch() drops it."""
        n_blocks = self.n_emu_blocks if n_blocks is None else n_blocks
        key = (d, scratch_set)
        have = self._scratch.get(key)
        if have is None or have[5] < n_blocks:
            f32 = dict(dtype=torch.float32, device=device)
            part = have[0] if have is not None else (
                torch.empty(self.n_slots * d, **f32) if self.n_slots else None)
            rel = meta = stage = None
            if n_blocks:
                rel = torch.empty(n_blocks * d * LGCN_EMU_CANDS, **f32)
                meta = torch.empty(n_blocks * d * LGCN_EMU_META_BYTES, dtype=torch.uint8,
                                   device=device)
                # the staged X elements of emulated blocks (always: without them re-run blocks
                # gather X one 4-B element per row, forward 19.9 -> 36.8 ms in round 3)
                stage = torch.empty(n_blocks * (d + 1) * LGCN_EMU_BLOCK, **f32)
            # the emulated rows' sums of a deferred mean epilogue (LGCN_EPI_ROWS)
            out = torch.empty(self.n_emu_rows * d, **f32) if self.n_emu_rows and \
                emu_defer_enabled() else None
            self._scratch[key] = (part, rel, meta, stage, out, n_blocks)
        return self._scratch[key][:5]

    def live_scratch(self, device):
        """Scratch of lgcn_live_rows (row-sparse X: the emulated rows as chains over their live
        edges), allocated once per plan: n_emu_blocks x 2 KB of compacted edges + descriptors."""
        if self._live is None and self.n_emu_rows:
            nb = int(load_library().lgcn_live_scratch_bytes(self.n_emu_rows, self.n_emu_blocks))
            self._live = torch.empty(nb, dtype=torch.uint8, device=device)
        return self._live

    def release_scratch(self, d=None):
        """Drop the cached scratch of width d (all widths: None); torch.cuda.empty_cache() can
        then return it."""
        for key in list(self._scratch):
            if d is None or key[0] == d:
                del self._scratch[key]
        if d is None:
            self._live = None

    def struct(self, d, device, nnz=None, walk_all=False, scratch_set=0, live=False,
               backward=False, part0=None):
        """lgcn_hub_plan_t for width d. nnz: the operator's nonzeros (sets the chain/walk cut;
        None = every emulated row walked). walk_all: the chain rows are walked too (no chain
        kernel for this d / alignment, or LGCN_CHAIN=0), so the scratch covers every block.
        scratch_set: which of the plan's scratch sets (0, 1) the layer uses. live: attach the
        live-edge scratch (a layer with a row-sparse X then runs lgcn_live_rows)."""
        if nnz is None or walk_all:
            rows = [self.n_emu_rows, self.n_emu_rows] if nnz is None else None
            blocks = [self.n_emu_blocks, self.n_emu_blocks] if nnz is None else None
        if nnz is not None:
            rows, blocks = self.walk_parts(nnz, backward, part0)
        need = self.n_emu_blocks if (walk_all or nnz is None) else blocks[1]
        part, rel, meta, stage, eout = self.scratch(d, device, need, scratch_set)
        p = PlanT()
        p.items, p.n_items = (self.items.data_ptr() if self.n_items else None), self.n_items
        p.rows, p.n_rows, p.n_pre = (self.rows.data_ptr() if self.n_entries else None), \
            self.n_entries, self.n_pre
        p.partials = part.data_ptr() if part is not None else None
        p.emu_blocks = self.emu_blocks.data_ptr() if self.n_emu_blocks else None
        p.emu_rows = self.emu_rows.data_ptr() if self.n_emu_rows else None
        p.n_emu_blocks, p.n_emu_rows = self.n_emu_blocks, self.n_emu_rows
        p.emu_rel = rel.data_ptr() if rel is not None else None
        p.emu_meta = meta.data_ptr() if meta is not None else None
        p.emu_stage = stage.data_ptr() if stage is not None else None
        p.emu_out = eout.data_ptr() if eout is not None else None
        p.threshold = min(self.threshold, INT32_MAX)
        p.emu_part_rows[0], p.emu_part_rows[1] = rows
        p.emu_part_blocks[0], p.emu_part_blocks[1] = blocks
        p.emu_scratch_blocks = need
        # the longest row of each walked part (emu_nb: longest first)
        nb = self.emu_nb
        p.emu_part_max_blocks[0] = int(nb[0]) if rows[0] > 0 else 0
        p.emu_part_max_blocks[1] = int(nb[rows[0]]) if rows[1] > rows[0] else 0
        lv = self.live_scratch(device) if live and self.mode == "exact" else None
        p.emu_live = lv.data_ptr() if lv is not None else None
        return p


def plan_emulation(rowptr_host, min_degree, device, row_ids_host=None):
    """Every row of degree > min_degree as an emulated row, in blocks of LGCN_EMU_BLOCK edges,
    longest row first whatever the slot order (the walks of the longest rows are a layer's
    critical path; walk_parts cuts the rows by length): the C planner lgcn_plan_exact. Returns
    (blocks, rows) on the device and the host block counts per row."""
    lib = load_library()
    rp = np.ascontiguousarray(rowptr_host, dtype=np.int32)
    n = rp.size - 1
    ids = None if row_ids_host is None else np.ascontiguousarray(row_ids_host, dtype=np.int32)
    ids_p = None if ids is None else ids.ctypes.data
    plan = PlanT()
    _check(lib.lgcn_plan_exact(rp.ctypes.data, ids_p, n, int(min_degree), 0, 0, None, None,
                               ctypes.byref(plan)), "lgcn_plan_exact(size)")
    if plan.n_emu_rows == 0:
        return None, None, np.zeros(0, np.int64)
    rows = np.empty((plan.n_emu_rows, 4), np.int32)
    blocks = np.empty((plan.n_emu_blocks, 4), np.int32)
    _check(lib.lgcn_plan_exact(rp.ctypes.data, ids_p, n, int(min_degree), 0, 0, rows.ctypes.data,
                               blocks.ctypes.data, ctypes.byref(plan)), "lgcn_plan_exact")
    return (torch.from_numpy(blocks).to(device), torch.from_numpy(rows).to(device),
            rows[:, 2].astype(np.int64))


def plan_items(rowptr_host, threshold, emu_min, row_ids_host=None):
    """Whole-row items (int32 [n, 4], lgcn_hub_item_t) of the rows of threshold < degree <=
    emu_min: the C planner lgcn_plan_items."""
    lib = load_library()
    rp = np.ascontiguousarray(rowptr_host, dtype=np.int32)
    n = rp.size - 1
    ids = None if row_ids_host is None else np.ascontiguousarray(row_ids_host, dtype=np.int32)
    ids_p = None if ids is None else ids.ctypes.data
    m = ctypes.c_int32(0)
    _check(lib.lgcn_plan_items(rp.ctypes.data, ids_p, n, int(min(threshold, INT32_MAX)),
                               int(emu_min), None, ctypes.byref(m)), "lgcn_plan_items(size)")
    items = np.empty((m.value, 4), np.int32)
    if m.value:
        _check(lib.lgcn_plan_items(rp.ctypes.data, ids_p, n, int(min(threshold, INT32_MAX)),
                                   int(emu_min), items.ctypes.data, ctypes.byref(m)),
               "lgcn_plan_items")
    return items


def plan_hubs(rowptr_host, threshold, chunk, device, row_ids_host=None, pre_group=None,
              mode="exact", emu_min=None):
    """Plan the rows with degree > threshold (host planner, numpy). rowptr_host is in storage
    (slot) order; row_ids_host maps a slot to its output row.

    exact: rows up to emu_min become whole-row items (one exact chain each), longer rows are
    emulated in blocks (plan_emulation). chunk: rows are cut into `chunk`-edge pieces; a hub row
    with more than pre_group chunks is combined in two levels: pre-reduction entries (leading the
    row list) sum runs of pre_group consecutive chunk partials into extra partial slots, and the
    row's final entry sums those. Without it the combine of a 2.77M-edge row (10.8k partials) is
    one block's 85-step latency chain, longer than all other rows together."""
    if pre_group is None:
        pre_group = DEFAULT_HUB_PRE_GROUP
    if emu_min is None:
        emu_min = emu_min_degree_from_env()
    deg = np.diff(rowptr_host.astype(np.int64))
    hub = np.nonzero(deg > threshold)[0]
    if threshold >= INT32_MAX or hub.size == 0:
        return HubPlan(threshold, mode, chunk, emu_min=emu_min)
    out_row = hub if row_ids_host is None else row_ids_host[hub]
    if mode == "exact":
        items = plan_items(rowptr_host, threshold, emu_min, row_ids_host)
        eb, er, enb = plan_emulation(rowptr_host, max(threshold, emu_min), device,
                                     row_ids_host)
        return HubPlan(threshold, mode, None,
                       torch.from_numpy(items).to(device) if items.shape[0] else None,
                       emu_blocks=eb, emu_rows=er, emu_min=emu_min, emu_nb=enb)
    nch = (deg[hub] + chunk - 1) // chunk
    first = np.concatenate([[0], np.cumsum(nch)[:-1]])
    n_chunks = int(nch.sum())
    row_of = np.repeat(hub, nch)
    k = np.arange(n_chunks) - np.repeat(first, nch)
    beg = rowptr_host[row_of].astype(np.int64) + k * chunk
    end = np.minimum(beg + chunk, rowptr_host[row_of + 1])
    # longest rows first so their combine inputs are ready early; items in slot order
    items = np.stack([np.repeat(out_row, nch), beg, end, np.arange(n_chunks)], 1).astype(np.int32)
    rows = np.stack([out_row, first, nch, np.zeros_like(hub)], 1).astype(np.int64)
    pre = np.zeros((0, 4), np.int64)
    if pre_group > 0:
        big = np.nonzero(nch > pre_group)[0]
        ng = (nch[big] + pre_group - 1) // pre_group           # pre-reductions per big row
        gfirst = np.cumsum(ng) - ng
        n_pre = int(ng.sum())
        j = np.arange(n_pre) - np.repeat(gfirst, ng)
        src0 = np.repeat(first[big], ng) + j * pre_group
        cnt = np.minimum(pre_group, np.repeat(first[big] + nch[big], ng) - src0)
        pre = np.stack([n_chunks + np.arange(n_pre), src0, cnt, np.ones(n_pre, np.int64)], 1)
        rows[big, 1] = n_chunks + gfirst
        rows[big, 2] = ng
    n_slots = n_chunks + pre.shape[0]
    table = np.concatenate([pre, rows]).astype(np.int32)
    return HubPlan(threshold, mode, chunk, torch.from_numpy(items).to(device),
                   torch.from_numpy(table).to(device), n_slots, hub.size, pre.shape[0])


class Graph:
    """Device CSR of a square Â plus its backward operator (Âᵀ, == Â when bitwise symmetric).

    rowptr/edges are in storage order: row id order, or — when row_ids is set — degree-ordered
    slots (slot s holds the edges of row row_ids[s], lgcn_csr_order_by_degree)."""

    def __init__(self, n_rows, n_cols, rowptr, edges, nnz, device, row_ids=None):
        self.n_rows, self.n_cols, self.nnz = n_rows, n_cols, nnz
        self.rowptr, self.edges, self.device = rowptr, edges, device
        self.row_ids = row_ids
        self.transpose = None
        self.symmetric = None
        # bipartite slot order (order_by_degree with sides): rows of [sides[0], sides[1]) in
        # slots [split, n), every other row in [0, split) — the two half-layers of a layer
        self.sides = None
        self.split = None
        # side-0 classes (lgcn_csr_side_classes): class ends and the side-1 part rows they were
        # built from; (split, split) and (0, 0) without classes
        self.class_end = None
        self.class_parts = (0, 0)
        self._plans = {}
        self._rowptr_host = None
        self._row_ids_host = None

    def rowptr_host(self):
        """Row pointers in storage order (slots when degree-ordered)."""
        if self._rowptr_host is None:
            self._rowptr_host = self.rowptr.cpu().numpy()
        return self._rowptr_host

    def row_ids_host(self):
        if self.row_ids is None:
            return None
        if self._row_ids_host is None:
            self._row_ids_host = self.row_ids.cpu().numpy()
        return self._row_ids_host

    def hubs(self, threshold, chunk=None, mode=None, emu_min=None):
        """The hub plan for `threshold` (cached): mode / emu_min default to LGCN_HUB_MODE /
        LGCN_EMU_MIN_DEGREE."""
        mode = mode or hub_mode_from_env()
        if mode not in HUB_MODES:
            raise LgcnError(f"unknown hub mode {mode!r}")
        emu_min = emu_min_degree_from_env(self.nnz) if emu_min is None else emu_min
        chunk = chunk or hub_chunk_for(self.nnz)
        key = (threshold, mode) + ((chunk, DEFAULT_HUB_PRE_GROUP) if mode == "chunk" else (emu_min,))
        if key not in self._plans:
            self._plans[key] = plan_hubs(self.rowptr_host(), threshold, chunk, self.device,
                                         self.row_ids_host(), mode=mode, emu_min=emu_min)
        return self._plans[key]

    def segments(self):
        """Slot ranges of the sided propagation's segments: side 0's three classes, side 1."""
        ce = self.class_end or (self.split, self.split)
        return [(0, ce[0]), (ce[0], ce[1]), (ce[1], self.split), (self.split, self.n_rows)]

    def sides_struct(self):
        """lgcn_sides_t of this side-major graph."""
        ce = self.class_end or (self.split, self.split)
        st = SidesT()
        st.n, st.split = self.n_rows, self.split
        st.class_end[0], st.class_end[1] = ce
        st.part_rows[0], st.part_rows[1] = self.class_parts
        return st

    def side_hubs(self, threshold, chunk=None, mode=None, emu_min=None):
        """The hub plans (cached) of the segments of a side-major graph (segments(): side 0's
        classes, then side 1) — each over its slot range, row ids and edge offsets absolute, as
        lgcn_propagate_*_sides takes them."""
        if self.split is None:
            raise LgcnError("side_hubs needs a side-ordered graph (graph_from_coo(adj, sides=...))")
        mode = mode or hub_mode_from_env()
        if mode not in HUB_MODES:
            raise LgcnError(f"unknown hub mode {mode!r}")
        emu_min = emu_min_degree_from_env(self.nnz) if emu_min is None else emu_min
        chunk = chunk or hub_chunk_for(self.nnz)
        key = ("sides", threshold, mode) + \
            ((chunk, DEFAULT_HUB_PRE_GROUP) if mode == "chunk" else (emu_min,))
        if key not in self._plans:
            rp, ids = self.rowptr_host(), self.row_ids_host()
            self._plans[key] = [
                plan_hubs(rp[a:b + 1], threshold, chunk, self.device, ids[a:b], mode=mode,
                          emu_min=emu_min)
                for a, b in self.segments()]
        return self._plans[key]

    def degrees(self):
        """Degree of every row, indexed by row id."""
        deg = np.diff(self.rowptr_host().astype(np.int64))
        ids = self.row_ids_host()
        if ids is None:
            return deg
        out = np.empty_like(deg)
        out[ids] = deg
        return out


def slot_key_enabled(g):
    """Neighbour-key tie-break of the slot order (square operators; env LGCN_SLOT_KEY=0 turns it
    off): rows of equal degree grouped by their least popular neighbour."""
    return g.n_rows == g.n_cols and os.environ.get("LGCN_SLOT_KEY", "1") != "0"


def order_by_degree(lib, g, stream, sides=None):
    """The same operator with its rows stored in degree-descending slots (lgcn_csr_order_by_degree):
    lane groups of a wave then stream rows of equal length; ties grouped by neighbour key
    (slot_key_enabled). sides=(lo, hi): rows of [lo, hi) after all others (each side
    degree-descending), the bipartite schedule's slot order. Bitwise-neutral."""
    n, nnz, dev = g.n_rows, g.nnz, g.device
    lo, hi = sides if sides is not None else (0, 0)
    i32 = dict(dtype=torch.int32, device=dev)
    deg_tmp, deg_sorted, iota = (torch.empty(max(n, 1), **i32) for _ in range(3))
    row_ids = torch.empty(max(n, 1), **i32)
    rowptr = torch.empty(n + 1, **i32)
    edges = torch.empty(max(nnz, 1), dtype=torch.int64, device=dev)
    keys = (torch.empty(max(n, 1), dtype=torch.int64, device=dev) for _ in range(2)) \
        if slot_key_enabled(g) else (None, None)
    key_tmp, key_sorted = keys
    nbytes = ctypes.c_size_t(0)
    args = (_ptr(g.rowptr), _ptr(g.edges), n, nnz, lo, hi, _ptr(deg_tmp), _ptr(deg_sorted),
            _ptr(iota),
            _ptr(row_ids), _ptr(rowptr), _ptr(edges),
            _ptr(key_tmp) if key_tmp is not None else None,
            _ptr(key_sorted) if key_sorted is not None else None)
    _check(lib.lgcn_csr_order_by_degree(*args, None, ctypes.byref(nbytes), stream),
           "lgcn_csr_order_by_degree(size)")
    temp = torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=dev)
    _check(lib.lgcn_csr_order_by_degree(*args, _ptr(temp), ctypes.byref(nbytes), stream),
           "lgcn_csr_order_by_degree")
    del deg_tmp, deg_sorted, iota, temp, key_tmp, key_sorted
    o = Graph(n, g.n_cols, rowptr, edges, nnz, dev, row_ids=row_ids[:n])
    o.symmetric = g.symmetric
    if lo < hi:
        o.sides, o.split = (lo, hi), n - (hi - lo)
        if classes_enabled():
            o = side_classes(lib, o, stream)
    return o


def classes_enabled():
    """Side-0 classes of a side-major slot order (LGCN_CLASSES=1; off by default: side 0 is then
    one class and every walked part of side 1 waits for all of it; same bits). Measured at C3
    (round 5): forward 14.4 ms with the classes vs 13.1-13.2 ms without — the users' first layer
    as three launches ran 6.9 ms instead of 3.7 under the concurrent item work, which delayed
    the items' layer 2 more than the early start of its longest walk gained."""
    return os.environ.get("LGCN_CLASSES", "0") == "1"


# Part-0 cut of the row-sparse (BPR-batch) backward: its first layer runs live-edge chains, and
# its later layers gain from walking more of the longest rows with part 0's many slots on their
# own stream (C3, A/B on one box, interleaved twice: BPR backward 9.35 / 9.73 -> 8.81 / 9.30 ms
# at 2048 blocks; the forward and the dense-G backward lose at 2048: 11.32 / 11.97 -> 11.71 /
# 12.33 and 13.55 / 13.93 -> 15.80 / 14.39 ms, so they keep 8192; profiles/r06_ab_part0_slots.log).
# Not with side-0 classes (LGCN_CLASSES=1): those were cut with the forward's part 0, and the
# schedule's class waits name the parts by that cut.
PART0_SPARSE_BACKWARD = 2048


def walk_cut_blocks(nnz, backward=False, part0=None):
    """(b0, b1): the emulated rows of more than b0 blocks are part 0 (LGCN_EMU_PART0, else
    part0, else 8192), of more than b1 = chain cut / LGCN_EMU_BLOCK part 1 (walked); the rest
    run as chains."""
    b1 = -(-chain_max_degree(nnz, backward) // LGCN_EMU_BLOCK)
    b0 = int(os.environ.get("LGCN_EMU_PART0", "") or part0 or 8192)
    return max(b0, b1), b1


def side_classes(lib, g, stream):
    """The side-major graph g with side 0's slots re-sorted by class (lgcn_csr_side_classes):
    class 0 = rows linked to side 1's walked part 0 (its longest rows), 1 = to part 1 only, 2 =
    the rest, each class in its degree order. The sided propagation then lets a walked part start
    as soon as the classes it reads are done. Bitwise-neutral."""
    n, nnz, dev, sp = g.n_rows, g.nnz, g.device, g.split
    b0, b1 = walk_cut_blocks(nnz)
    deg1 = np.diff(g.rowptr_host()[sp:].astype(np.int64))     # side 1, degree-descending
    nb = -(-deg1 // LGCN_EMU_BLOCK)
    p0, p01 = int((nb > b0).sum()), int((nb > b1).sum())
    if p01 == 0 or sp == 0:
        g.class_end, g.class_parts = (sp, sp), (0, 0)
        return g
    i32 = dict(dtype=torch.int32, device=dev)
    work = torch.empty(5 * n, **i32)
    row_ids = torch.empty(n, **i32)
    rowptr = torch.empty(n + 1, **i32)
    edges = torch.empty(max(nnz, 1), dtype=torch.int64, device=dev)
    ce = torch.empty(2, **i32)
    nbytes = ctypes.c_size_t(0)
    args = (_ptr(g.rowptr), _ptr(g.edges), _ptr(g.row_ids), n, nnz, sp, p0, p01, _ptr(work),
            _ptr(row_ids), _ptr(rowptr), _ptr(edges), _ptr(ce))
    _check(lib.lgcn_csr_side_classes(*args, None, ctypes.byref(nbytes), stream),
           "lgcn_csr_side_classes(size)")
    temp = torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=dev)
    _check(lib.lgcn_csr_side_classes(*args, _ptr(temp), ctypes.byref(nbytes), stream),
           "lgcn_csr_side_classes")
    del work, temp
    o = Graph(n, g.n_cols, rowptr, edges, nnz, dev, row_ids=row_ids)
    o.symmetric = g.symmetric
    o.sides, o.split = g.sides, sp
    o.class_end = tuple(int(x) for x in ce.cpu().tolist())
    o.class_parts = (p0, p01)
    return o


def sides_min_nnz():
    """Graphs from this many nonzeros run the bipartite schedule when the caller names the sides
    (LGCN_SIDES_MIN_NNZ, default 2^23): below it a layer is a few short launches and splitting
    them into half-layers on 8 streams only adds latency (C2, 1.6M nonzeros: forward 1.54 ms
    with the two lanes, 1.10 ms without)."""
    return int(os.environ.get("LGCN_SIDES_MIN_NNZ", str(1 << 23)))


def is_bipartite(lib, g, sides, stream):
    """lgcn_csr_check_bipartite: every edge joins a row inside [lo, hi) to one outside."""
    bad = torch.zeros(1, dtype=torch.int32, device=g.device)
    _check(lib.lgcn_csr_check_bipartite(_ptr(g.rowptr), _ptr(g.edges), _ptr(g.row_ids), g.n_rows,
                                        g.nnz, sides[0], sides[1], _ptr(bad), stream),
           "lgcn_csr_check_bipartite")
    return int(bad.item()) == 0


def _coo_to_csr(lib, key, other, vals, nnz, n_keys, device, stream, sort):
    rowptr = torch.empty(n_keys + 1, dtype=torch.int32, device=device)
    edges = torch.empty(max(nnz, 1), dtype=torch.int64, device=device)
    perm = keys_sorted = None
    if sort and nnz > 0:
        keys_tmp = torch.empty(nnz, dtype=torch.int32, device=device)
        keys_sorted = torch.empty(nnz, dtype=torch.int32, device=device)
        perm_tmp = torch.empty(nnz, dtype=torch.int32, device=device)
        perm = torch.empty(nnz, dtype=torch.int32, device=device)
        nbytes = ctypes.c_size_t(0)
        _check(lib.lgcn_coo_sort_perm(None, nnz, n_keys, _ptr(keys_tmp), _ptr(keys_sorted),
                                      _ptr(perm_tmp), _ptr(perm), None, ctypes.byref(nbytes),
                                      stream), "lgcn_coo_sort_perm(size)")
        temp = torch.empty(max(nbytes.value, 1), dtype=torch.uint8, device=device)
        _check(lib.lgcn_coo_sort_perm(_ptr(key), nnz, n_keys, _ptr(keys_tmp), _ptr(keys_sorted),
                                      _ptr(perm_tmp), _ptr(perm), _ptr(temp), ctypes.byref(nbytes),
                                      stream), "lgcn_coo_sort_perm")
    _check(lib.lgcn_coo_to_csr(_ptr(key), _ptr(other), _ptr(vals), nnz, n_keys, _ptr(perm),
                               _ptr(keys_sorted), _ptr(rowptr), _ptr(edges), stream),
           "lgcn_coo_to_csr")
    return rowptr, edges


def relabel_slots(g):
    """P·Â·Pᵀ of a degree-ordered graph: rows AND columns in slot space (slot s = row
    row_ids[s]), so X, Y and every layer buffer are indexed by slot and the kernels write
    sequentially. Returns (graph_in_slot_space, perm) with perm[s] = original row (int64).
    Each row keeps its edge order: Y_slot[s] == Y[perm[s]] bitwise."""
    if g.row_ids is None:
        raise LgcnError("relabel_slots needs a degree-ordered graph (order_by_degree)")
    lib = load_library()
    dev = g.device
    perm = g.row_ids.long()
    inv = torch.empty(g.n_rows, dtype=torch.int32, device=dev)
    inv[perm] = torch.arange(g.n_rows, dtype=torch.int32, device=dev)
    edges = torch.empty_like(g.edges)
    with torch.cuda.device(dev):
        _check(lib.lgcn_csr_relabel_cols(_ptr(g.edges), g.nnz, _ptr(inv), _ptr(edges),
                                         _stream(dev)), "lgcn_csr_relabel_cols")
    o = Graph(g.n_rows, g.n_cols, g.rowptr, edges, g.nnz, dev)
    o._rowptr_host = g._rowptr_host
    o.symmetric = g.symmetric
    if g.split is not None:  # side-major slots stay side-major: the sided schedule needs row ids
        o.sides, o.split = g.sides, g.split
        o.class_end, o.class_parts = g.class_end, g.class_parts
        o.row_ids = torch.arange(g.n_rows, dtype=torch.int32, device=dev)
        o._row_ids_host = np.arange(g.n_rows, dtype=np.int32)
    return o, perm


def _finish_graph(lib, rows, cols, vals, rowptr, edges, n, nnz, device, stream, cols_sorted,
                  order=None, sides=None):
    """Attach the backward operator: Â itself if bitwise symmetric, else a stably sorted Âᵀ;
    then store both in the processing order (row_order()) — side-major when `sides` = (lo, hi)
    is given, Â is bipartite across it and large enough (sides_min_nnz)."""
    g = Graph(n, n, rowptr, edges, nnz, device)
    symmetric = False
    if cols_sorted:
        asym = torch.zeros(1, dtype=torch.int32, device=device)
        _check(lib.lgcn_csr_check_symmetric(_ptr(rowptr), _ptr(edges), n, nnz, _ptr(asym),
                                            stream), "lgcn_csr_check_symmetric")
        symmetric = int(asym.item()) == 0
    g.symmetric = symmetric
    t = None
    if not symmetric:
        # Âᵀ with each row's entries in Â's stored order (torch's sparse t() + addmm loop)
        t_rowptr, t_edges = _coo_to_csr(lib, cols, rows, vals, nnz, n, device, stream, sort=True)
        t = Graph(n, n, t_rowptr, t_edges, nnz, device)
        t.symmetric = False
    if row_order(order) == "degree":
        mn = sides_min_nnz()
        if sides is not None and (mn is None or nnz < mn or sides[0] >= sides[1] or
                                  not is_bipartite(lib, g, sides, stream)):
            sides = None  # (Âᵀ is bipartite across the same cut when Â is)
        g = order_by_degree(lib, g, stream, sides)
        t = order_by_degree(lib, t, stream, sides) if t is not None else None
    if t is None:
        g.transpose = g
    else:
        g.transpose, t.transpose = t, g
    return g


def _cache_key(adj):
    idx, vals = adj._indices(), adj._values()
    return (idx.data_ptr(), vals.data_ptr(), idx._version, vals._version, adj._nnz(),
            tuple(adj.shape), str(adj.device))


def attach_graph(adj, g, sides=None):
    """Cache a prepared Graph on the adjacency tensor it was built from."""
    try:
        adj._lgcn_graph = (_cache_key(adj) + (tuple(sides) if sides is not None else None,), g)
    except (AttributeError, RuntimeError):
        pass
    return adj


def graph_from_coo(adj, sides=None):
    """Convert the caller-owned sparse COO Â (main.py:334-336) into the engine's CSR, once.

    The plan is cached on the tensor object and re-validated by storage pointers and version
    counters, so the per-batch call `model(norm_adj_tensor)` (main.py:495) costs nothing extra.
    sides: optional (lo, hi) — the item rows [U, U+I) of main.py:283-287: when Â is bipartite
    across them (users and brands link only to items) the graph is stored side-major and the
    propagation runs the bipartite two-lane schedule (lgcn_propagate_*_sides).
    """
    if not adj.is_sparse or adj.layout != torch.sparse_coo:
        raise LgcnError("adj_mat must be a torch.sparse_coo_tensor")
    if adj.dim() != 2 or adj.shape[0] != adj.shape[1]:
        raise LgcnError(f"adj_mat must be square 2-D, got {tuple(adj.shape)}")
    if adj.dtype != torch.float32:
        raise LgcnError(f"adj_mat must be float32, got {adj.dtype}")
    idx = adj._indices()
    vals = adj._values()
    key = _cache_key(adj) + (tuple(sides) if sides is not None else None,)
    cached = getattr(adj, "_lgcn_graph", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    lib = load_library()
    device = adj.device
    n = int(adj.shape[0])
    nnz = int(adj._nnz())
    if n > INT32_MAX - 1 or nnz > INT32_MAX:
        raise LgcnError("graph too large for int32 CSR")
    with torch.cuda.device(device):
        stream = _stream(device)
        idx = idx.contiguous()
        vals = vals.contiguous()
        rows, cols = idx[0].contiguous(), idx[1].contiguous()
        flags = torch.zeros(1, dtype=torch.int32, device=device)
        _check(lib.lgcn_coo_inspect(_ptr(rows), _ptr(cols), nnz, n, n, _ptr(flags), stream),
               "lgcn_coo_inspect")
        f = int(flags.item())
        if f & COO_OUT_OF_RANGE:
            raise LgcnError("adj_mat has indices out of range")
        rowptr, edges = _coo_to_csr(lib, rows, cols, vals, nnz, n, device, stream,
                                    sort=bool(f & COO_ROWS_UNSORTED))
        g = _finish_graph(lib, rows, cols, vals, rowptr, edges, n, nnz, device, stream,
                          cols_sorted=not (f & (COO_ROWS_UNSORTED | COO_COLS_UNSORTED)),
                          sides=tuple(sides) if sides is not None else None)
    try:
        adj._lgcn_graph = (key, g)
    except (AttributeError, RuntimeError):
        pass
    return g


# ----------------------------------------------------------------------------------------------
# propagation
# ----------------------------------------------------------------------------------------------
def _epilogue(mode, prev0=None, prev_dense=(), ld_prev=0, div=1.0, addend=None):
    """addend: an lgcn_rows_t (segments) for LGCN_EPI_ADD, added as addend / div."""
    ep = EpilogueT()
    ep.mode = mode
    ep.div = div
    if prev0 is not None:
        ep.prev0 = prev0
        ep.n_prev = 1 + len(prev_dense)
        for i, t in enumerate(prev_dense):
            ep.prev_dense[i] = t.data_ptr()
        ep.ld_prev = ld_prev
    if addend is not None:
        ep.addend = addend
    return ep


def _check_emb(segments, d, device):
    for t in segments:
        if t.device != device:
            raise LgcnError(f"embedding on {t.device}, adjacency on {device}")
        if t.dtype != torch.float32:
            raise LgcnError("embeddings must be float32")
        if t.dim() != 2 or t.shape[1] != d:
            raise LgcnError("embedding blocks must be [rows x d]")
        if t.shape[0] > 0 and (t.stride(1) != 1 or t.stride(0) != d):
            raise LgcnError("embedding blocks must be contiguous [rows x d]")


_scheds = {}


def _side_stream(device, i=0, high=False):
    """Per-device side streams the emulated and chain rows run on beside the layer kernel
    (lgcn_sched), one per (index, priority); high = created at high priority, so their waves are
    dispatched first. Created by the library (lgcn_stream_create) and wrapped as
    torch.cuda.ExternalStream: torch.cuda.Stream() hands out streams from a round-robin pool of
    32 per priority, so a pooled side stream could be the very stream some caller (or a graph
    capture) is using."""
    sc = _scheds.setdefault(("streams", str(device)), {})
    if (i, high) not in sc and i >= 3 and not high:
        # the row-sparse backward's lane 1 (role "backward"): four of torch's pooled
        # normal-priority streams, as round 5 — HIP maps them onto the normal-priority hardware
        # queues lane 0's streams hold, pairwise, which serialises the two lanes' half-layers in
        # issue order: the fastest BPR-batch backward measured (8.4-9.3 ms against
        # 9.4-9.5 with lane 0's streams shared outright and 11 ms with library-created streams,
        # which HIP paired differently)
        sc[(i, high)] = torch.cuda.Stream(device)
    if (i, high) not in sc:
        lib = load_library()
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            _check(lib.lgcn_stream_create(1 if high else 0, ctypes.byref(h)),
                   "lgcn_stream_create")
        sc[(i, high)] = torch.cuda.ExternalStream(h.value, device=device)
    return sc[(i, high)]


def _stream_priorities(n_aux, role="forward"):
    """Which auxiliary streams run at high priority. One lane (n_aux <= 3): aux 0, the longest
    rows' walks (a layer's critical path). Two lanes: all of lane 1 (aux 3 = its main stream and
    aux 4..6) — 4 + 4 streams: one hardware queue each under HIP's default 4 per priority.
    Measured at C3 against: no priorities, lane 0's aux streams, both
    lanes' part-0 streams, lane 1's layer kernels or its chains at normal priority (with 8
    queues per priority) — none faster, most slower."""
    if role == "backward":  # (sched_for: the backward's lanes share lane 0's normal streams)
        return [False] * n_aux
    if n_aux <= 3:
        return [i == 0 for i in range(n_aux)]
    return [i >= 3 for i in range(n_aux)]


def hw_queues():
    """Hardware queues HIP gives this process (GPU_MAX_HW_QUEUES, HIP's default 4)."""
    try:
        return int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        return 4


def n_aux_streams():
    """Auxiliary streams of the exact layers (LGCN_AUX_STREAMS, 1..7; default 7: parts 0 and 1
    and the chain rows beside the caller's stream, plus a second lane of half-layers — its main
    stream and its own 3, lgcn_sched_create). HIP keeps a pool of hardware queues per stream
    priority (GPU_MAX_HW_QUEUES each, default 4): the caller's stream and aux 0..2 take the
    normal-priority queues, the second lane's four high-priority streams their own — measured
    at C3, the two lanes run as fast under HIP's default 4 queues as under 8 (17.08 vs 17.17 ms,
    round 4), so the default needs no environment change and main.py gets the two lanes."""
    v = os.environ.get("LGCN_AUX_STREAMS", "")
    n = int(v) if v else 7
    return max(1, min(7, n))


class Sched:
    """lgcn_sched_t over this device's side streams (created once per device and stream count;
    the C library owns the fork/join events). n_aux >= 4: two lanes (lgcn_propagate_*_sides)."""

    def __init__(self, device, n_aux, role="forward", lane1_shared=False):
        lib = load_library()
        self.lib, self.device, self.n_aux = lib, device, n_aux
        self.streams = [_side_stream(device, i, hi)
                        for i, hi in enumerate(_stream_priorities(n_aux, role))]
        arr = (ctypes.c_void_p * n_aux)(*[st.cuda_stream for st in self.streams])
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            _check(lib.lgcn_sched_create(arr, n_aux, ctypes.byref(h)), "lgcn_sched_create")
        self.handle = h
        slots = emu_slots()
        self.set(SCHED_SLOTS0, slots[0])
        self.set(SCHED_SLOTS1, slots[min(1, len(slots) - 1)])
        self.set(SCHED_CHAIN, 1 if chain_enabled() else 0)
        # LGCN_SCHED_CLASSES=0: the walked parts of side 1 wait for the whole side-0 half-layer
        # (A/B; same bits)
        self.set(SCHED_CLASSES, 0 if os.environ.get("LGCN_SCHED_CLASSES", "1") == "0" else 1)
        if lane1_shared:
            self.set(SCHED_LANE1_SHARED, 1)

    def state(self, what):
        """lgcn_sched_state: what the latest sided call on this schedule ran."""
        return int(self.lib.lgcn_sched_state(self.handle, what))

    def set(self, knob, value):
        _check(self.lib.lgcn_sched_set(self.handle, knob, int(value)), "lgcn_sched_set")

    def __del__(self):
        try:
            if self.handle:
                self.lib.lgcn_sched_destroy(self.handle)
        except Exception:
            pass


def sched_for(device, n_aux=None, role="forward"):
    """The device's Sched (None with LGCN_EMU_OVERLAP=0: every part in order on the caller's
    stream). n_aux: default n_aux_streams(). Made outside any capture on first use (the C
    library creates its events there; a captured call reuses them).

    role "backward" (a row-sparse G, _backward_role): both lanes at normal priority, lane 1 on
    four of torch's pooled streams (_side_stream), which HIP pairs with lane 0's hardware queues
    (DESIGN §4e)."""
    if not emu_overlap_enabled():
        return None
    n = n_aux or n_aux_streams()
    key = (str(device), n, chain_enabled(), os.environ.get("LGCN_SCHED_CLASSES", ""), role)
    if key not in _scheds:
        _scheds[key] = Sched(device, n, role)
    return _scheds[key]


def chain_enabled():
    """Rows of the emulated-row list below the chain cut run as plain sequential chains
    (lgcn_chain_rows) instead of block pass + walk; LGCN_CHAIN=0 walks them too."""
    return os.environ.get("LGCN_CHAIN", "1") != "0"


def _aligned16(segments):
    return all(t.data_ptr() % 16 == 0 and (t.dim() < 2 or t.stride(0) % 4 == 0)
               for t in segments)


def emu_slots():
    """LDS slots of the walk (part 0, part 1): 20, 8 — the longest rows run few waves and take
    many slots; part 1's rows are more waves, and fewer slots fit more of them per CU (C3
    forward 20.0 ms at 28,12 -> 19.2 ms at 20,8; 20,4 / 16,6 the same or worse, round 4)."""
    return [20, 8]


def emu_overlap_enabled():
    """LGCN_EMU_OVERLAP=0 runs the emulated rows on the caller's stream, after the layer kernel
    (no lgcn_sched) instead of beside it on side streams."""
    return os.environ.get("LGCN_EMU_OVERLAP", "1") != "0"


emu_trace = None  # a list: spmm_layer appends (phase, torch.cuda.Event) of the layer (SCHED_TRACE)


def spmm_layer(graph, x_segments, y, d, epi, hub_threshold, hubs=None, stream=None, x_div=1.0,
               x_nz=None, kernel_events=None, backward=False):
    """One layer Y = epilogue(Â·(X / x_div)) under the operator's hub plan — lgcn_layer: the layer
    kernel (bundles, chunks, whole long rows) + chunk combine, the block pass + walk of the
    emulated parts and the chain rows, concurrently on the device's side streams (lgcn_sched,
    forked from and joined back into the caller's stream: graph-capture safe).
    x_nz: optional row bitmask of X (rows_nonzero; ADD epilogue only). kernel_events: optional
    (start, end) torch.cuda.Event pair recorded on the caller's stream around the layer kernel
    (bench.py's live timing of that kernel). backward: the operator is the backward's Âᵀ (its
    own chain cut, lgcn_chain_max_backward_default)."""
    lib = load_library()
    hp = hubs or graph.hubs(hub_threshold)
    stream = stream or _stream(graph.device)
    main = torch.cuda.current_stream(graph.device)
    if main.cuda_stream != (stream.value or 0):
        raise LgcnError("spmm_layer: stream must be the device's current stream")
    chains = chain_enabled() and bool(lib.lgcn_chain_supported(d)) and _aligned16(x_segments)
    plan = hp.struct(d, graph.device, nnz=graph.nnz, walk_all=not chains,
                     live=x_nz is not None and live_enabled(), backward=backward)
    x = rows_desc(x_segments, d)
    sc = sched_for(graph.device) if hp.n_emu_rows else None
    args = (_ptr(graph.rowptr), _ptr(graph.edges), _ptr(graph.row_ids), graph.n_rows)
    trace = None
    if sc is not None and (kernel_events is not None or emu_trace is not None):
        if kernel_events is not None:
            for ev in kernel_events:  # materialise the hipEvent_t handles
                ev.record()
            sc.set(SCHED_TIMING_START, kernel_events[0].cuda_event)
            sc.set(SCHED_TIMING_END, kernel_events[1].cuda_event)
        if emu_trace is not None:
            evs = [torch.cuda.Event(enable_timing=True) for _ in TRACE_PHASES]
            for ev in evs:
                ev.record()
            trace = (ctypes.c_void_p * len(evs))(*[ev.cuda_event for ev in evs])
            sc.set(SCHED_TRACE, ctypes.addressof(trace))
    elif kernel_events is not None:
        kernel_events[0].record()
    try:
        _check(lib.lgcn_layer(*args, ctypes.byref(plan), x, x_div, _ptr(x_nz), _ptr(y),
                              y.stride(0), d, ctypes.byref(epi),
                              sc.handle if sc is not None else None, stream), "lgcn_layer")
    finally:
        if sc is not None:
            sc.set(SCHED_TIMING_START, 0)
            sc.set(SCHED_TIMING_END, 0)
            sc.set(SCHED_TRACE, 0)
    if sc is None and kernel_events is not None:
        kernel_events[1].record()  # (no schedule: the whole layer)
    if trace is not None:
        emu_trace[:] = list(zip(TRACE_PHASES, evs))
    return y


def live_enabled():
    """LGCN_LIVE=0 turns off the live-edge chains of a row-sparse X (lgcn_live_rows): the
    emulated rows are then block-passed and walked over all their edges (same bits)."""
    return os.environ.get("LGCN_LIVE", "1") != "0"


def _side_plans(graph, d, hub_threshold, hub_mode, emu_min, xs_aligned, live=False,
                backward=False, part0=None):
    """The 8 lgcn_hub_plan_t of lgcn_propagate_*_sides: plans[2 * segment + set] (segments: the
    side-0 classes, side 1). live: attach the live-edge scratch (the backward of a row-sparse
    G). part0: the part-0 cut in blocks (walk_cut_blocks)."""
    lib = load_library()
    hps = graph.side_hubs(hub_threshold, mode=hub_mode, emu_min=emu_min)
    chains = chain_enabled() and bool(lib.lgcn_chain_supported(d)) and xs_aligned
    arr = (PlanT * (2 * N_SEGS))()
    for g in range(N_SEGS):
        for j in (0, 1):
            arr[2 * g + j] = hps[g].struct(d, graph.device, nnz=graph.nnz, walk_all=not chains,
                                           scratch_set=j, live=live and live_enabled(),
                                           backward=backward, part0=part0)
    return arr, hps


class _SideEvents:
    """Timing / trace events of the sided entry points (SCHED_TIMING_SIDES / SCHED_TRACE_SIDES),
    set on the schedule for one call and cleared after it."""

    def __init__(self, sc, K, timing, trace):
        self.sc = sc
        self.timing = self.trace = None
        self._arrs = []
        if sc is None:
            return
        if timing:
            self.timing = [torch.cuda.Event(enable_timing=True) for _ in range(2 * N_SEGS * K)]
            self._set(SCHED_TIMING_SIDES, self.timing)
        if trace:
            self.trace = [torch.cuda.Event(enable_timing=True) for _ in range(8 * N_SEGS * K)]
            self._set(SCHED_TRACE_SIDES, self.trace)

    def _set(self, knob, evs):
        for ev in evs:  # materialise the hipEvent_t handles
            ev.record()
        arr = (ctypes.c_void_p * len(evs))(*[ev.cuda_event for ev in evs])
        self._arrs.append(arr)
        self.sc.set(knob, ctypes.addressof(arr))

    def clear(self):
        if self.sc is not None:
            self.sc.set(SCHED_TIMING_SIDES, 0)
            self.sc.set(SCHED_TRACE_SIDES, 0)


side_trace = None   # a list: the sided entry points append {(k, g): [(phase, event)]} per call
side_timing = None  # a list: ... append {(k, g): (start, end)} around each segment's layer kernel
# (g: segment — 0..2 the side-0 classes, 3 side 1; empty segments are left out)


last_schedule = None  # the schedule of the latest propagation call (diagnostics, tests)


def _note_schedule(sc, graph):
    """last_schedule from what the C library ran (lgcn_sched_state)."""
    global last_schedule
    if sc is None:
        last_schedule = {"sided": True, "aux_streams": 0, "lanes": 1, "lane1_aux": 0,
                         "captured": torch.cuda.is_current_stream_capturing(), "classes": False}
        return
    last_schedule = {"sided": True, "aux_streams": sc.n_aux,
                     "lanes": sc.state(SCHED_STATE_LANES),
                     "lane1_aux": sc.state(SCHED_STATE_L1_AUX),
                     "captured": bool(sc.state(SCHED_STATE_CAPTURING)),
                     "capture_full": bool(sc.state(SCHED_STATE_CAPTURE_FULL)),
                     "classes": bool(sc.state(SCHED_STATE_CLASSES))}


def use_sides(graph, layer_events=None, kernel_events=None):
    """The bipartite schedule runs when the graph is side-ordered (graph_from_coo with sides)
    and no per-layer events are asked for (a layer has no single boundary in it)."""
    return graph.split is not None and layer_events is None and kernel_events is None


def _collect_sides(ev, K, graph):
    segs = [g for g, (a, b) in enumerate(graph.segments()) if b > a]
    if ev.timing is not None and side_timing is not None:
        side_timing.append({(k, g): (ev.timing[((k - 1) * N_SEGS + g) * 2],
                                     ev.timing[((k - 1) * N_SEGS + g) * 2 + 1])
                            for k in range(1, K + 1) for g in segs})
    if ev.trace is not None and side_trace is not None:
        side_trace.append({(k, g): list(zip(TRACE_PHASES,
                                            ev.trace[((k - 1) * N_SEGS + g) * 8:
                                                     ((k - 1) * N_SEGS + g + 1) * 8]))
                           for k in range(1, K + 1) for g in segs})


def propagate_forward(graph, segments, K, hub_threshold=None, layer_events=None,
                      return_layers=False, hub_mode=None, emu_min=None, kernel_events=None):
    """final = mean(E0, Â E0, ..., Â^K E0) with E0 = cat(segments) (never materialised).

    layer_events: optional list of (start, end) torch.cuda.Event pairs recorded on the current
    stream around each whole layer (every stream of it joined); kernel_events: the same around
    each layer's layer-kernel launch alone (spmm_layer) — bench.py's live timing. A side-ordered
    graph runs the bipartite two-lane schedule (lgcn_propagate_forward_sides) unless per-layer
    events are asked for.
    """
    if hub_threshold is None:
        hub_threshold = hub_threshold_from_env()
    d = segments[0].shape[1]
    n = sum(int(t.shape[0]) for t in segments)
    if n != graph.n_rows:
        raise LgcnError(f"embedding rows {n} != adjacency size {graph.n_rows}")
    _check_emb(segments, d, graph.device)
    if K > LGCN_MAX_LAYERS + 1 or K < 0:
        raise LgcnError(f"n_layers={K} unsupported (0..{LGCN_MAX_LAYERS + 1})")
    lib = load_library()
    dev = graph.device
    with torch.cuda.device(dev):
        stream = _stream(dev)
        e0 = rows_desc(segments, d)
        out = torch.empty((n, d), dtype=torch.float32, device=dev)
        if K == 0:
            _check(lib.lgcn_scale_rows(e0, n, d, 1.0, _ptr(out), d, stream), "lgcn_scale_rows")
            return (out, []) if return_layers else out
        layers = [torch.empty((n, d), dtype=torch.float32, device=dev) for _ in range(K - 1)]
        if use_sides(graph, layer_events, kernel_events):
            plans, _ = _side_plans(graph, d, hub_threshold, hub_mode, emu_min,
                                   _aligned16(segments))
            sc = sched_for(dev)
            ev = _SideEvents(sc, K, side_timing is not None, side_trace is not None)
            bufs = (ctypes.c_void_p * max(K - 1, 1))(*[t.data_ptr() for t in layers])
            sides = graph.sides_struct()
            try:
                _check(lib.lgcn_propagate_forward_sides(
                    _ptr(graph.rowptr), _ptr(graph.edges), _ptr(graph.row_ids),
                    ctypes.byref(sides), plans, e0, d, K, bufs, _ptr(out),
                    sc.handle if sc is not None else None, stream), "lgcn_propagate_forward_sides")
            finally:
                ev.clear()
            _note_schedule(sc, graph)
            _collect_sides(ev, K, graph)
            return (out, layers) if return_layers else out
        hp = graph.hubs(hub_threshold, mode=hub_mode, emu_min=emu_min)
        for k in range(1, K + 1):
            xs = segments if k == 1 else [layers[k - 2]]
            if k < K:
                y, ep = layers[k - 1], _epilogue(LGCN_EPI_STORE)
            else:
                y = out
                ep = _epilogue(LGCN_EPI_MEAN, prev0=e0, prev_dense=layers, ld_prev=d,
                               div=float(K + 1))
            if layer_events is not None:
                layer_events[k - 1][0].record()
            spmm_layer(graph, xs, y, d, ep, hub_threshold, hp, stream,
                       kernel_events=None if kernel_events is None else kernel_events[k - 1])
            if layer_events is not None:
                layer_events[k - 1][1].record()
        return (out, layers) if return_layers else out


def rows_nonzero(segments, d, device):
    """(bitmask of rows holding a nonzero, device int32 count of such rows): lgcn_rows_nonzero.
    Nothing is read back."""
    lib = load_library()
    n = sum(int(t.shape[0]) for t in segments)
    mask = torch.empty(max((n + 31) // 32, 1), dtype=torch.int32, device=device)
    count = torch.empty(1, dtype=torch.int32, device=device)
    with torch.cuda.device(device):
        _check(lib.lgcn_rows_nonzero(rows_desc(segments, d), n, d, _ptr(mask), _ptr(count),
                                     _stream(device)), "lgcn_rows_nonzero")
    return mask, count


# Row-sparse backward: the upstream gradient of a BPR batch (main.py:496-497 gathers, then
# IndexBackward scatters into zeros) has a few thousand live rows out of millions. The backward
# builds G's row mask on the device (lgcn_rows_nonzero) and skips G's zero rows (bitwise-neutral)
# — decided without reading anything back, so a training step stays capturable in a HIP graph.
# env LGCN_SPARSE_GRAD = auto (default: the mask path) | off (dense path) | on (= auto).


def _sparse_grad_mode():
    m = os.environ.get("LGCN_SPARSE_GRAD", "auto").lower()
    if m not in ("auto", "off", "on"):
        raise LgcnError(f"LGCN_SPARSE_GRAD={m!r} (auto | off | on)")
    return m


_live_hint = {}  # device -> [slots, events, scales, next slot, last role, last dense]: recent
#                 live-row counts
_HINT_SLOTS = 8
_HINT_SAMPLE = 64  # a dense-path call counts the live rows of every 64th row of G (an estimate)


def _hint_entry(dev):
    key = str(dev)
    h = _live_hint.get(key)
    if h is None:
        h = [torch.empty(_HINT_SLOTS, dtype=torch.int32, pin_memory=True),
             [None] * _HINT_SLOTS, [1] * _HINT_SLOTS, 0, "forward", False]
        _live_hint[key] = h
    return h


def _hint_latest(dev):
    """The newest landed live-row count of G (scaled up when sampled), or None."""
    slots, evs, scales, nxt = _hint_entry(dev)[:4]
    for k in range(1, _HINT_SLOTS + 1):   # newest first
        i = (nxt - k) % _HINT_SLOTS
        if evs[i] is not None and evs[i].query():
            return int(slots[i]) * scales[i]
    return None


def _hint_push(dev, cnt, scale=1):
    """Copy the device count `cnt` into the next pinned slot, asynchronously."""
    h = _hint_entry(dev)
    slots, evs, scales, nxt = h[:4]
    slot = nxt % _HINT_SLOTS
    slots[slot:slot + 1].copy_(cnt.view(-1)[:1], non_blocking=True)
    if evs[slot] is None:
        evs[slot] = torch.cuda.Event()
    evs[slot].record()
    scales[slot] = scale
    h[3] = nxt + 1


def _hint_dense(dev, n):
    """True when the newest landed count says G was dense (>= n/8 live rows) — the mask would
    mark every row, so the backward skips it and runs the dense kernels. With no
    count landed (the host more than the ring's 8 calls ahead of the device) the previous
    decision stays; False before any count has landed and under a capture."""
    if torch.cuda.is_current_stream_capturing():
        return False
    h = _hint_entry(dev)
    c = _hint_latest(dev)
    if c is not None:
        h[5] = c * 8 >= n
    return h[5]


def _sampled_live_count(segs, d, dev):
    """Device count of the live rows among every _HINT_SAMPLE-th row of G (lgcn_rows_nonzero over
    strided views of the blocks: ~1/64 of G's bytes), for the next call's choice."""
    S = _HINT_SAMPLE
    views = [t[::S] for t in segs if t.shape[0] > 0]
    if not views:
        return None
    lib = load_library()
    n = sum(int(v.shape[0]) for v in views)
    mask = torch.empty(max((n + 31) // 32, 1), dtype=torch.int32, device=dev)
    count = torch.empty(1, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        _check(lib.lgcn_rows_nonzero(rows_desc(views, S * d), n, d, _ptr(mask), _ptr(count),
                                     _stream(dev)), "lgcn_rows_nonzero")
    return count


def _backward_role(dev, n, cnt, scale=1):
    """Which schedule a sided backward runs on. A row-sparse G (a BPR batch: live-edge chains
    instead of walks) runs fastest with both lanes at normal priority, a dense G (walks of the
    hub rows) with lane 1 high as the forward (round 5: BPR-batch backward 9.7 -> 9.0 ms, dense
    17.9 vs 19.9 ms). The device's live-row count is not read back (no sync): each call copies
    it asynchronously into a ring of pinned slots, and the choice uses the newest slot whose copy
    has landed (a training loop's gradients keep their sparsity from step to step); with none
    landed the previous choice stays (the forward's schedule at first and under a HIP-graph
    capture). Same bits either way."""
    if cnt is None:
        return "forward"
    if torch.cuda.is_current_stream_capturing():
        return "forward"
    h = _hint_entry(dev)
    latest = _hint_latest(dev)
    role = h[4] if latest is None else ("backward" if latest * 8 < n else "forward")
    _hint_push(dev, cnt, scale)
    h[4] = role
    return role


def propagate_backward(graph, grad_out, K, hub_threshold=None, sparse=None, hub_mode=None,
                       emu_min=None):
    """dE0 = Σ_k (Âᵀ)^k G/(K+1), Horner order h = G/(K+1) + Âᵀ h (autograd's accumulation).

    grad_out: the [n x d] upstream gradient, or a list of row blocks (the user / item / brand
    output gradients, read in place). c = G/(K+1) is never materialised: layer 1 divides on
    load and every epilogue adds G[row]/(K+1) — the same rounding as a stored c.
    sparse: "auto" | "off" | "on" (default: env LGCN_SPARSE_GRAD): auto/on build G's row mask on
    the device, layer 1 gathers only G's live rows and the epilogues skip its zero rows — same
    bits, fewer bytes for a BPR batch's G; off runs the dense kernels. Nothing is read back."""
    if hub_threshold is None:
        hub_threshold = hub_threshold_from_env()
    gt = graph.transpose
    segs = [t.contiguous() for t in grad_out] if isinstance(grad_out, (list, tuple)) \
        else [grad_out.contiguous()]
    d = segs[0].shape[1]
    n = sum(int(t.shape[0]) for t in segs)
    _check_emb(segs, d, graph.device)
    lib = load_library()
    dev = graph.device
    with torch.cuda.device(dev):
        stream = _stream(dev)
        g = rows_desc(segs, d)
        out = torch.empty((n, d), dtype=torch.float32, device=dev)
        if K == 0:
            _check(lib.lgcn_scale_rows(g, n, d, 1.0, _ptr(out), d, stream), "lgcn_scale_rows")
            return out
        mode = sparse or _sparse_grad_mode()
        nz = cnt = None
        scale = 1
        if mode in ("auto", "on") and n > 0:
            # no host read-back (it would sync every step): the mask costs one pass over G (0.7 ms
            # at C3). When the previous calls' counts say G is dense, the mask would mark every
            # row: skip it (and the live-edge path it gates) and only sample G's rows for the
            # next call's choice
            if mode == "auto" and _hint_dense(dev, n):
                cnt, scale = _sampled_live_count(segs, d, dev), _HINT_SAMPLE
            else:
                nz, cnt = rows_nonzero(segs, d, dev)
        work = torch.empty((n, d), dtype=torch.float32, device=dev) if K > 1 else None
        if use_sides(gt):
            role = _backward_role(dev, n, cnt, scale)
            plans, _ = _side_plans(gt, d, hub_threshold, hub_mode, emu_min, _aligned16(segs),
                                   live=nz is not None, backward=True,
                                   part0=PART0_SPARSE_BACKWARD
                                   if role == "backward" and not any(gt.class_parts) else None)
            sc = sched_for(dev, role=role)
            ev = _SideEvents(sc, K, side_timing is not None, side_trace is not None)
            sides = gt.sides_struct()
            try:
                _check(lib.lgcn_propagate_backward_sides(
                    _ptr(gt.rowptr), _ptr(gt.edges), _ptr(gt.row_ids), ctypes.byref(sides),
                    plans, g, _ptr(nz), d, K, _ptr(work), _ptr(out),
                    sc.handle if sc is not None else None, stream),
                    "lgcn_propagate_backward_sides")
            finally:
                ev.clear()
            _note_schedule(sc, gt)
            _collect_sides(ev, K, gt)
            return out
        if cnt is not None and not torch.cuda.is_current_stream_capturing():
            _hint_push(dev, cnt, scale)
        hp = gt.hubs(hub_threshold, mode=hub_mode, emu_min=emu_min)
        ep = _epilogue(LGCN_EPI_ADD, addend=g, div=float(K + 1))
        ep.addend_nz = None if nz is None else nz.data_ptr()
        h = segs
        for k in range(1, K + 1):
            y = out if (K - k) % 2 == 0 else work
            spmm_layer(gt, h, y, d, ep, hub_threshold, hp, stream,
                       x_div=float(K + 1) if k == 1 else 1.0, x_nz=nz if k == 1 else None,
                       backward=True)
            h = [y]
        return out


class CapturedForward:
    """propagate_forward recorded once into a HIP graph (torch.cuda.CUDAGraph is a hipGraph on
    ROCm) for fixed input buffers: replay() relaunches the K layers and hub combines with one
    graph launch — the launch-bound case is a small graph (C2: 6 launches in 0.3 ms). The
    inputs are read at replay time, so updating `segments` in place (an optimizer step) is
    seen; replay returns the same output buffer every time."""

    def __init__(self, graph, segments, K, hub_threshold=None):
        dev = graph.device
        if hub_threshold is None:
            hub_threshold = hub_threshold_from_env()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # plans, allocator pools and code objects warm
            propagate_forward(graph, segments, K, hub_threshold)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph_exec = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_exec):
            self.out = propagate_forward(graph, segments, K, hub_threshold)
        self.segments = segments  # keep the captured input buffers alive

    def replay(self):
        self.graph_exec.replay()
        return self.out


class PropagateFunction(torch.autograd.Function):
    """(user, item, brand) weights -> the (user, item, brand) blocks of the mean of K propagated
    layers (views of one buffer: no torch.cat / torch.split copies either way); backward by the
    same kernel, reading the three output gradients in place.

    n_e0 > 0 also returns the first n_e0 weights themselves (storage-sharing aliases, not views:
    an optimizer's in-place update shows through them) as further outputs — the ego tables the
    model hands back (lightgcn.py:81) for main.py's regulariser gather (main.py:497). Their
    gradients then reach this backward instead of the weights, and it adds them into the engine's
    dE0 blocks at their nonzero entries only (lgcn_add_nonzero): the sum autograd would form, to
    the bit (dE0 is never -0), without its dense read-read-write of the whole table."""

    @staticmethod
    def forward(ctx, graph, K, hub_threshold, n_e0, *segments):
        ctx.graph, ctx.K, ctx.hub_threshold = graph, K, hub_threshold
        ctx.sizes = [int(t.shape[0]) for t in segments]
        segs = [t.detach() for t in segments]
        out = propagate_forward(graph, segs, K, hub_threshold)
        return tuple(torch.split(out, ctx.sizes, 0)) + tuple(segs[:n_e0])

    @staticmethod
    def backward(ctx, *grads):
        nseg = len(ctx.sizes)
        head = (None, None, None, None)
        gout, ge0 = grads[:nseg], grads[nseg:]
        d = next((g.shape[1] for g in grads if g is not None), None)
        if d is None:
            return head + (None,) * nseg
        if all(g is None for g in gout):  # only the ego aliases were used
            return head + tuple(ge0) + (None,) * (nseg - len(ge0))
        gs = [g if g is not None else
              torch.zeros((sz, d), dtype=torch.float32, device=ctx.graph.device)
              for g, sz in zip(gout, ctx.sizes)]
        g0 = propagate_backward(ctx.graph, gs, ctx.K, ctx.hub_threshold)
        blocks = torch.split(g0, ctx.sizes, 0)
        lib = load_library()
        dev = ctx.graph.device
        for g, blk in zip(ge0, blocks):
            if g is None:
                continue
            g = g.contiguous()
            if g.dtype != torch.float32 or g.shape != blk.shape or g.device != blk.device:
                raise LgcnError(f"ego gradient {tuple(g.shape)} {g.dtype} does not match its "
                                f"block {tuple(blk.shape)}")
            if ctx.K == 0:
                # dE0 is G itself here and may hold -0, where autograd's dense sum with the
                # alias gradient's +0 gives +0: the plain add
                blk.add_(g)
                continue
            with torch.cuda.device(dev):
                _check(lib.lgcn_add_nonzero(_ptr(g), _ptr(blk), g.numel(), _stream(dev)),
                       "lgcn_add_nonzero")
        return head + tuple(blocks)


def segment_sides(segments):
    """(lo, hi) of the second segment's rows — the items of cat(user, item, brand)
    (main.py:283-287) — or None for fewer than two segments."""
    if len(segments) < 2:
        return None
    lo = int(segments[0].shape[0])
    return (lo, lo + int(segments[1].shape[0]))


def propagate_blocks(adj, segments, K, hub_threshold=None, e0_outputs=0):
    """Autograd-aware engine entry used by models.LightGCN / LightGCN_Fusion on a HIP device:
    returns the final embeddings as one block per input segment (user, item, brand). The item
    rows are offered as the bipartite sides (graph_from_coo). e0_outputs = n appends aliases of
    the first n segments whose gradients the backward folds into its own (PropagateFunction)."""
    if not 0 <= e0_outputs <= len(segments):
        raise LgcnError(f"e0_outputs={e0_outputs} for {len(segments)} segments")
    graph = graph_from_coo(adj, sides=segment_sides(segments))
    if hub_threshold is None:
        hub_threshold = hub_threshold_from_env()
    return PropagateFunction.apply(graph, K, hub_threshold, e0_outputs, *segments)


def propagate(adj, segments, K, hub_threshold=None):
    """Like propagate_blocks, as one [n x d] tensor (a concatenating copy: prefer the blocks)."""
    return torch.cat(propagate_blocks(adj, segments, K, hub_threshold), 0)
