"""ctypes binding of libmbx.so (include/mbx.h) -- the GPU executor's C-ABI.

This is how Python callers (tests, bench.py) drive the HIP path; it is a thin
marshalling layer with no compute of its own.  If libmbx.so is missing, or no
MI355X is visible, the calls raise: there is no CPU fallback anywhere.

CNF spec accepted by Context.compile (the flattened CondExpr[] of the reference):
    cnf = [conjunct, ...]                      # AND (CondExpr[] array)
    conjunct = [term, ...]                     # OR (.next chain)
    term = (op, operand1, operand2[, index_type])
    operand = ('sym', fld) | ('int', v) | ('real', v) | ('str', text_or_mutf8_bytes)
"""
import atexit
import ctypes
import os
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmbx.so")

# include/mbx.h constants
STRING, INTEGER, REAL, SYMBOL = 0, 1, 2, 3
EQ, LT, GT, NE, LE, GE, NOT, NOP, RANGE = range(9)
IDX_NONE, IDX_BTREE, IDX_HASH, IDX_BITMAP = range(4)
BM_AND, BM_OR, BM_ANDNOT = range(3)
E_INVALID, E_TYPE, E_RANGE, E_DEVICE, E_NOMEM, E_UNSUPPORTED = -1, -2, -3, -4, -5, -6


class MbxError(RuntimeError):
    """A negative status from the C-ABI; .code is the MBX_E_* value."""

    def __init__(self, code, msg):
        super().__init__(f"mbx error {code}: {msg}")
        self.code = code


class ColDesc(ctypes.Structure):
    _fields_ = [("attr_type", ctypes.c_int32), ("size", ctypes.c_int32)]


class Operand(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("fld", ctypes.c_int32), ("integer", ctypes.c_int32),
                ("real", ctypes.c_float), ("string", ctypes.c_char_p), ("string_len", ctypes.c_int32)]


class CondExprC(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("operand1", Operand), ("operand2", Operand),
                ("index_type", ctypes.c_int32)]


class Cnf(ctypes.Structure):
    _fields_ = [("conds", ctypes.POINTER(CondExprC)), ("conj_offsets", ctypes.POINTER(ctypes.c_int32)),
                ("nconj", ctypes.c_int32)]


class Agg(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int64), ("agg_type", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("isum", ctypes.c_int64), ("imin", ctypes.c_int32), ("imax", ctypes.c_int32),
                ("fsum", ctypes.c_double), ("fmin", ctypes.c_float), ("fmax", ctypes.c_float)]


def java_mutf8(s):
    """DataOutputStream.writeUTF payload bytes of a str (modified UTF-8)."""
    if isinstance(s, (bytes, bytearray)):
        return bytes(s)
    units = s.encode("utf-16-be", "surrogatepass")
    out = bytearray()
    for i in range(0, len(units), 2):
        cu = (units[i] << 8) | units[i + 1]
        if 0 < cu < 0x80:
            out.append(cu)
        elif cu < 0x800:
            out += bytes([0xC0 | (cu >> 6), 0x80 | (cu & 0x3F)])
        else:
            out += bytes([0xE0 | (cu >> 12), 0x80 | ((cu >> 6) & 0x3F), 0x80 | (cu & 0x3F)])
    return bytes(out)


EXPORTS = [
    "mbx_abi_version", "mbx_last_error", "mbx_device_count", "mbx_init", "mbx_free", "mbx_sync", "mbx_stream",
    "mbx_table_stage", "mbx_table_wrap", "mbx_table_free", "mbx_table_info", "mbx_table_group", "mbx_plan_compile", "mbx_plan_free",
    "mbx_scan_count", "mbx_scan_count_async", "mbx_scan_count_frame_async", "mbx_count_frame_decode",
    "mbx_count_frame_fits",
    "mbx_scan_blocks", "mbx_scan_bitmap", "mbx_scan_bitmap_async", "mbx_scan_select",
    "mbx_scan_select_async", "mbx_scan_aggregate",
    "mbx_scan_aggregate_async", "mbx_bitmap_alloc", "mbx_bitmap_upload", "mbx_bitmap_download", "mbx_bitmap_info",
    "mbx_bitmap_free", "mbx_bitmap_combine", "mbx_bitmap_cnf", "mbx_bitmap_cnf_async", "mbx_cnf_materialize_async", "mbx_bitmap_index_build",
    "mbx_bitmap_select", "mbx_materialize", "mbx_materialize_async", "mbx_cursor_open", "mbx_cursor_count",
    "mbx_cursor_next", "mbx_cursor_next_view", "mbx_cursor_restart", "mbx_cursor_close", "mbx_cursor_stats", "mbx_cnf_cursor_open", "mbx_cnf_cursor_launch",
    "mbx_probe_read", "mbx_set_tuning",
    "mbx_diag_select_stamps", "mbx_diag_lookback_epoch", "mbx_dev_alloc", "mbx_dev_free", "mbx_dev_download", "mbx_shard_bounds", "mbx_comm_unique_id", "mbx_comm_init_rank", "mbx_comm_init_all", "mbx_comm_free",
    "mbx_comm_info", "mbx_comm_wait", "mbx_comm_allreduce_count_async", "mbx_comm_scan_count_async",
    "mbx_comm_allreduce_agg_async", "mbx_agg_fold_async",
    "mbx_comm_allgather_count_async", "mbx_comm_allreduce_count_all", "mbx_comm_allreduce_agg_all",
    "mbx_comm_allgather_count_all",
    "mbx_graph_begin", "mbx_graph_end", "mbx_graph_launch", "mbx_graph_free",
    # include/mbx_db.h
    "mbx_db_create", "mbx_db_open", "mbx_db_close", "mbx_db_info", "mbx_db_file_entry", "mbx_db_columnar_create",
    "mbx_db_columnar_insert", "mbx_db_columnar_info", "mbx_db_mark_deleted", "mbx_db_bitmap_write",
    "mbx_db_bitmap_read", "mbx_db_stage", "mbx_db_allocate_pages", "mbx_db_add_file_entry",
    "mbx_db_create_bitmap_index", "mbx_db_bitmap_values", "mbx_db_bitmap_stage", "mbx_db_mark_deleted_many",
    "mbx_db_purge", "mbx_db_stage_range", "mbx_db_bitmap_stage_range",
    # include/mbx_join.h
    "mbx_join", "mbx_join_info", "mbx_join_fetch", "mbx_join_free", "mbx_gather",
]
JOIN_BMJ, JOIN_NLJ = 0, 1


class JoinTerm(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("outer_col", ctypes.c_int32), ("inner_col", ctypes.c_int32),
                ("pad_", ctypes.c_int32)]


class JoinCnf(ctypes.Structure):
    _fields_ = [("terms", ctypes.POINTER(JoinTerm)), ("conj_offsets", ctypes.POINTER(ctypes.c_int32)),
                ("nconj", ctypes.c_int32)]

_lib = None


def lib():
    """Load libmbx.so (built by `make -C minibase-columnar-database_amd/csrc`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MbxError(E_DEVICE, f"{LIB_PATH} missing: build it with __graft_entry__.build() "
                                 "(the executor has no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    P, V, I32, I64 = ctypes.POINTER, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sig = {
        "mbx_abi_version": ([], ctypes.c_int),
        "mbx_last_error": ([], ctypes.c_char_p),
        "mbx_device_count": ([P(I32)], ctypes.c_int),
        "mbx_init": ([I32, P(V)], ctypes.c_int),
        "mbx_free": ([V], ctypes.c_int),
        "mbx_sync": ([V], ctypes.c_int),
        "mbx_stream": ([V], V),
        "mbx_table_stage": ([V, P(ColDesc), I32, I64, P(V), V, I64, P(V)], ctypes.c_int),
        "mbx_table_wrap": ([V, P(ColDesc), I32, I64, P(V), V, I64, P(V)], ctypes.c_int),
        "mbx_table_free": ([V], ctypes.c_int),
        "mbx_table_info": ([V, P(I64), P(I64), P(I32)], ctypes.c_int),
        "mbx_table_group": ([V, V, P(I32), I32], ctypes.c_int),
        "mbx_plan_compile": ([V, V, P(Cnf), P(V)], ctypes.c_int),
        "mbx_plan_free": ([V], ctypes.c_int),
        "mbx_scan_count": ([V, V, P(I64)], ctypes.c_int),
        "mbx_scan_count_async": ([V, V, V], ctypes.c_int),
        "mbx_scan_count_frame_async": ([V, V, V], ctypes.c_int),
        "mbx_count_frame_decode": ([V, P(I64), P(I64), P(I64)], ctypes.c_int),
        "mbx_count_frame_fits": ([I64, ctypes.c_int32], ctypes.c_int),
        "mbx_scan_blocks": ([V, V, P(I64)], ctypes.c_int),
        "mbx_scan_bitmap": ([V, V, P(V), P(I64)], ctypes.c_int),
        "mbx_scan_bitmap_async": ([V, V, V], ctypes.c_int),
        "mbx_scan_select": ([V, V, V, I64, P(I64)], ctypes.c_int),
        "mbx_scan_select_async": ([V, V, V, V, V], ctypes.c_int),
        "mbx_scan_aggregate": ([V, V, I32, P(Agg)], ctypes.c_int),
        "mbx_scan_aggregate_async": ([V, V, I32, V], ctypes.c_int),
        "mbx_bitmap_alloc": ([V, I64, P(V)], ctypes.c_int),
        "mbx_bitmap_upload": ([V, I64, V, P(V)], ctypes.c_int),
        "mbx_bitmap_download": ([V, V, V, I64], ctypes.c_int),
        "mbx_bitmap_info": ([V, P(I64), P(I64), P(I64)], ctypes.c_int),
        "mbx_bitmap_free": ([V], ctypes.c_int),
        "mbx_bitmap_combine": ([V, I32, V, V, P(V), P(I64)], ctypes.c_int),
        "mbx_bitmap_cnf": ([V, I64, P(V), P(I32), I32, V, P(V), P(I64)], ctypes.c_int),
        "mbx_bitmap_cnf_async": ([V, P(V), P(I32), I32, V, V], ctypes.c_int),
        "mbx_bitmap_index_build": ([V, V, I32, P(Operand), I32, P(V)], ctypes.c_int),
        "mbx_bitmap_select": ([V, V, I64, V, I64, P(I64)], ctypes.c_int),
        "mbx_materialize": ([V, V, V, P(I32), I32, V, P(V), I64, P(I64)], ctypes.c_int),
        "mbx_materialize_async": ([V, V, V, P(I32), I32, V, P(V), V], ctypes.c_int),
        "mbx_cnf_materialize_async": ([V, V, P(V), P(I32), I32, V, P(I32), I32, V, P(V), V], ctypes.c_int),
        "mbx_cursor_open": ([V, V, V, P(I32), I32, P(V)], ctypes.c_int),
        "mbx_cursor_count": ([V, P(I64)], ctypes.c_int),
        "mbx_cursor_next": ([V, I64, V, P(V), P(I64)], ctypes.c_int),
        "mbx_cursor_next_view": ([V, I64, P(V), P(V), P(I64)], ctypes.c_int),
        "mbx_cursor_restart": ([V], ctypes.c_int),
        "mbx_cursor_close": ([V], ctypes.c_int),
        "mbx_cursor_stats": ([V, P(I64), P(I64)], ctypes.c_int),
        "mbx_cnf_cursor_open": ([V, V, P(V), P(I32), I32, V, P(I32), I32, P(V)], ctypes.c_int),
        "mbx_cnf_cursor_launch": ([V, V, P(V), P(I32), I32, V, P(I32), I32, P(V), P(V)], ctypes.c_int),
        "mbx_probe_read": ([V, V, P(I32), I32, I64, I32, I64], ctypes.c_int),
        "mbx_set_tuning": ([V, ctypes.c_char_p, I64], ctypes.c_int),
        "mbx_diag_select_stamps": ([V, V, I64], ctypes.c_int),
        "mbx_diag_lookback_epoch": ([V, I64], ctypes.c_int),
        "mbx_dev_alloc": ([V, I64, P(V)], ctypes.c_int),
        "mbx_dev_free": ([V, V], ctypes.c_int),
        "mbx_dev_download": ([V, V, V, I64], ctypes.c_int),
        "mbx_shard_bounds": ([I64, I32, I32, P(I64), P(I64)], ctypes.c_int),
        "mbx_comm_unique_id": ([V], ctypes.c_int),
        "mbx_comm_init_rank": ([V, I32, I32, V, P(V)], ctypes.c_int),
        "mbx_comm_init_all": ([P(V), I32, P(V)], ctypes.c_int),
        "mbx_comm_free": ([V], ctypes.c_int),
        "mbx_comm_info": ([V, P(I32), P(I32)], ctypes.c_int),
        "mbx_comm_wait": ([V], ctypes.c_int),
        "mbx_comm_allreduce_count_async": ([V, V, I64], ctypes.c_int),
        "mbx_comm_scan_count_async": ([V, V, V, I64, V], ctypes.c_int),
        "mbx_comm_allreduce_agg_async": ([V, V], ctypes.c_int),
        "mbx_agg_fold_async": ([V, V, I32, V], ctypes.c_int),
        "mbx_comm_allgather_count_async": ([V, V, V], ctypes.c_int),
        "mbx_comm_allreduce_count_all": ([P(V), I32, P(V), I64], ctypes.c_int),
        "mbx_comm_allreduce_agg_all": ([P(V), I32, P(V)], ctypes.c_int),
        "mbx_comm_allgather_count_all": ([P(V), I32, P(V), P(V)], ctypes.c_int),
        "mbx_graph_begin": ([V], ctypes.c_int),
        "mbx_graph_end": ([V, P(V)], ctypes.c_int),
        "mbx_graph_launch": ([V], ctypes.c_int),
        "mbx_graph_free": ([V], ctypes.c_int),
        "mbx_db_create": ([ctypes.c_char_p, I32, P(V)], ctypes.c_int),
        "mbx_db_open": ([ctypes.c_char_p, P(V)], ctypes.c_int),
        "mbx_db_close": ([V], ctypes.c_int),
        "mbx_db_info": ([V, P(I32), P(I32)], ctypes.c_int),
        "mbx_db_file_entry": ([V, ctypes.c_char_p, P(I32)], ctypes.c_int),
        "mbx_db_columnar_create": ([V, ctypes.c_char_p, I32, P(ColDesc), P(ctypes.c_char_p)], ctypes.c_int),
        "mbx_db_columnar_insert": ([V, ctypes.c_char_p, I64, P(V)], ctypes.c_int),
        "mbx_db_columnar_info": ([V, ctypes.c_char_p, I32, P(I32), P(ColDesc), V, P(I64), P(I64)], ctypes.c_int),
        "mbx_db_mark_deleted": ([V, ctypes.c_char_p, I64], ctypes.c_int),
        "mbx_db_bitmap_write": ([V, ctypes.c_char_p, V, I64], ctypes.c_int),
        "mbx_db_bitmap_read": ([V, ctypes.c_char_p, V, I64, P(I64)], ctypes.c_int),
        "mbx_db_stage": ([V, V, ctypes.c_char_p, P(V)], ctypes.c_int),
        "mbx_db_allocate_pages": ([V, I32, P(I32)], ctypes.c_int),
        "mbx_db_add_file_entry": ([V, ctypes.c_char_p, I32], ctypes.c_int),
        "mbx_db_create_bitmap_index": ([V, V, ctypes.c_char_p, V, I32, P(I32)], ctypes.c_int),
        "mbx_db_bitmap_values": ([V, ctypes.c_char_p, I32, V, I64, P(I32), P(I64)], ctypes.c_int),
        "mbx_db_bitmap_stage": ([V, V, ctypes.c_char_p, I64, P(V)], ctypes.c_int),
        "mbx_db_mark_deleted_many": ([V, ctypes.c_char_p, V, I64], ctypes.c_int),
        "mbx_db_purge": ([V, ctypes.c_char_p], ctypes.c_int),
        "mbx_db_stage_range": ([V, V, ctypes.c_char_p, I64, I64, P(V)], ctypes.c_int),
        "mbx_db_bitmap_stage_range": ([V, V, ctypes.c_char_p, I64, I64, P(V)], ctypes.c_int),
        "mbx_join": ([V, V, V, V, V, P(JoinCnf), I32, I64, P(V)], ctypes.c_int),
        "mbx_join_info": ([V, P(I64), P(I64)], ctypes.c_int),
        "mbx_join_fetch": ([V, V, I64, I64, V, V, V], ctypes.c_int),
        "mbx_join_free": ([V], ctypes.c_int),
        "mbx_gather": ([V, V, V, I64, P(I32), I32, P(V)], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _chk(rc):
    if rc < 0:
        raise MbxError(rc, lib().mbx_last_error().decode(errors="replace"))
    return rc


def device_count():
    n = ctypes.c_int32(0)
    rc = lib().mbx_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def _operand(spec, keep):
    o = Operand()
    kind, v = spec
    if kind == "sym":
        o.type, o.fld = SYMBOL, int(v)
    elif kind == "int":
        o.type, o.integer = INTEGER, int(v)
    elif kind == "real":
        o.type, o.real = REAL, float(v)
    elif kind == "str":
        b = java_mutf8(v)
        keep.append(b)
        o.type, o.string, o.string_len = STRING, b, len(b)
    else:
        raise ValueError(kind)
    return o


def make_cnf(cnf, keep):
    c = Cnf()
    if cnf is None:
        c.nconj = 0
        return c
    terms = [t for conj in cnf for t in conj]
    conds = (CondExprC * max(1, len(terms)))()
    for i, term in enumerate(terms):
        op, a, b = term[:3]
        conds[i].op = op
        conds[i].operand1 = _operand(a, keep)
        conds[i].operand2 = _operand(b, keep)
        conds[i].index_type = term[3] if len(term) > 3 else IDX_BITMAP
    offs = (ctypes.c_int32 * (len(cnf) + 1))()
    k = 0
    for i, conj in enumerate(cnf):
        offs[i] = k
        k += len(conj)
    offs[len(cnf)] = k
    keep += [conds, offs]
    c.conds = conds
    c.conj_offsets = offs
    c.nconj = len(cnf)
    return c


_live_contexts = weakref.WeakSet()


@atexit.register
def _close_all():
    """Free every library object before the HIP runtime tears down."""
    for c in list(_live_contexts):
        c.close()


class Context:
    """mbx_ctx: one GPU, one HIP stream.  Objects created through a context
    (tables, plans, bitmaps, cursors) are freed before it (C-ABI rule)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        _chk(lib().mbx_init(device, ctypes.byref(h)))
        self.h = h
        self.device = device
        self._children = weakref.WeakSet()
        _live_contexts.add(self)

    def _own(self, obj):
        self._children.add(obj)
        return obj

    def close(self):
        if self.h:
            # cursors and bitmaps first, then plans, then tables
            order = {"mbx_graph_free": -2, "mbx_comm_free": -1, "mbx_cursor_close": 0, "mbx_bitmap_free": 1,
                     "mbx_plan_free": 2, "mbx_table_free": 3}
            for ch in sorted(list(self._children), key=lambda o: order.get(o._free, 9)):
                ch.close()
            lib().mbx_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return lib().mbx_stream(self.h)

    def sync(self):
        _chk(lib().mbx_sync(self.h))

    def set_tuning(self, knob, value=0):
        """mbx_set_tuning: one A/B knob of this context ("reset" restores the
        production defaults; the default library reads no environment)."""
        _chk(lib().mbx_set_tuning(self.h, knob.encode(), int(value)))

    def probe_read(self, table, cols, tiles_per_block=0, interleave=False, grid=0):
        """Enqueue the read-bandwidth probe (mbx_probe_read) on self.stream."""
        c = (ctypes.c_int32 * len(cols))(*cols)
        _chk(lib().mbx_probe_read(self.h, table.h, c, len(cols), tiles_per_block, 1 if interleave else 0, grid))

    # -- tables ---------------------------------------------------------
    def stage(self, columns, deleted_words=None, row_offset=0):
        """columns: list of (attr_type, size, ndarray); strings as uint8 [n, size]."""
        arrs, descs = [], (ColDesc * len(columns))()
        nrows = None
        for j, (t, size, a) in enumerate(columns):
            if t == INTEGER:
                a = np.ascontiguousarray(a, dtype=np.int32)
                size = 4
            elif t == REAL:
                a = np.ascontiguousarray(a, dtype=np.float32)
                size = 4
            else:
                a = np.ascontiguousarray(a, dtype=np.uint8).reshape(-1, size)
            descs[j].attr_type, descs[j].size = t, size
            arrs.append(a)
            nrows = a.shape[0] if nrows is None else nrows
        ptrs = (ctypes.c_void_p * len(columns))(*[a.ctypes.data for a in arrs])
        dw = None if deleted_words is None else np.ascontiguousarray(deleted_words, dtype=np.uint64)
        h = ctypes.c_void_p()
        _chk(lib().mbx_table_stage(self.h, descs, len(columns), nrows, ptrs,
                                   None if dw is None else dw.ctypes.data, row_offset, ctypes.byref(h)))
        return Table(self, h, nrows, [(t, s) for t, s, _ in columns], row_offset)

    def wrap(self, col_descs, dev_ptrs, nrows, dev_deleted=None, row_offset=0):
        """Zero-copy table over device buffers (e.g. torch tensors' data_ptr())."""
        descs = (ColDesc * len(col_descs))()
        for j, (t, s) in enumerate(col_descs):
            descs[j].attr_type, descs[j].size = t, s
        ptrs = (ctypes.c_void_p * len(col_descs))(*dev_ptrs)
        h = ctypes.c_void_p()
        _chk(lib().mbx_table_wrap(self.h, descs, len(col_descs), nrows, ptrs, dev_deleted, row_offset,
                                  ctypes.byref(h)))
        return Table(self, h, nrows, list(col_descs), row_offset, keep=[descs, ptrs])

    def group(self, table, cols):
        """mbx_table_group: a row-interleaved copy of 2..4 four-byte columns the
        narrow gathers read (same results, fewer HBM lines when sparse); cols = []: drop
        the table's groups (a snapshot: rebuild after rewriting wrapped
        columns)."""
        arr = (ctypes.c_int32 * len(cols))(*cols) if cols else None
        _chk(lib().mbx_table_group(self.h, table.h, arr, len(cols)))

    def join(self, outer, outer_sel, inner, inner_sel, cnf, order, outer_block=0):
        """mbx_join: cnf = [[(op, outer_col, inner_col), ...], ...] (0-based
        columns); returns (outer positions, inner positions, passes) in the
        reference's order."""
        terms = [t for conj in cnf for t in conj]
        tarr = (JoinTerm * max(1, len(terms)))()
        for k, (op, a, b) in enumerate(terms):
            tarr[k].op, tarr[k].outer_col, tarr[k].inner_col = op, a, b
        offs, o = [0], 0
        for conj in cnf:
            o += len(conj)
            offs.append(o)
        oarr = (ctypes.c_int32 * len(offs))(*offs)
        c = JoinCnf(tarr, oarr, len(cnf))
        h = ctypes.c_void_p()
        _chk(lib().mbx_join(self.h, outer.h, outer_sel.h, inner.h, inner_sel.h, ctypes.byref(c), order, outer_block,
                            ctypes.byref(h)))
        try:
            n, p = ctypes.c_int64(), ctypes.c_int64()
            _chk(lib().mbx_join_info(h, ctypes.byref(n), ctypes.byref(p)))
            op_ = np.zeros(max(1, n.value), dtype=np.int64)
            ip_ = np.zeros(max(1, n.value), dtype=np.int64)
            ps = np.zeros(max(1, n.value), dtype=np.int32)
            _chk(lib().mbx_join_fetch(self.h, h, 0, n.value, op_.ctypes.data, ip_.ctypes.data, ps.ctypes.data))
            return op_[:n.value], ip_[:n.value], ps[:n.value], p.value
        finally:
            lib().mbx_join_free(h)

    def gather(self, table, positions, proj):
        pos = np.ascontiguousarray(positions, dtype=np.int64)
        outs = [table.empty_column(j, len(pos)) for j in proj]
        ptrs = (ctypes.c_void_p * max(1, len(outs)))(*[o.ctypes.data for o in outs])
        pj = (ctypes.c_int32 * max(1, len(proj)))(*proj)
        _chk(lib().mbx_gather(self.h, table.h, pos.ctypes.data, len(pos), pj, len(proj), ptrs))
        return outs

    def create_bitmap_index(self, db, name, table, col):
        """mbx_db_create_bitmap_index: `index db cf <col> bitmap` on the GPU."""
        n = ctypes.c_int32()
        _chk(lib().mbx_db_create_bitmap_index(self.h, db.h, name.encode(), table.h, col, ctypes.byref(n)))
        return n.value

    def stage_db_bitmap(self, db, filename, nbits):
        h = ctypes.c_void_p()
        _chk(lib().mbx_db_bitmap_stage(self.h, db.h, filename.encode(), nbits, ctypes.byref(h)))
        return Bitmap(self, h, nbits)

    def stage_db(self, db, name):
        """mbx_db_stage: a Columnarfile of a Minibase DB file -> HBM table
        (records decoded on the GPU, reference positions kept)."""
        info = db.columnar_info(name)
        h = ctypes.c_void_p()
        _chk(lib().mbx_db_stage(self.h, db.h, name.encode(), ctypes.byref(h)))
        return Table(self, h, info["nrows"], [(t, s) for t, s in info["cols"]], 0)

    def stage_db_range(self, db, name, row_begin, row_end):
        """mbx_db_stage_range: positions [row_begin, row_end) of a Columnarfile
        (one shard; row_offset = row_begin), only that range's pages read."""
        info = db.columnar_info(name)
        h = ctypes.c_void_p()
        _chk(lib().mbx_db_stage_range(self.h, db.h, name.encode(), row_begin, row_end, ctypes.byref(h)))
        n, off, nc = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
        _chk(lib().mbx_table_info(h, ctypes.byref(n), ctypes.byref(off), ctypes.byref(nc)))
        return Table(self, h, n.value, [(t, s) for t, s in info["cols"]], off.value)

    def stage_db_bitmap_range(self, db, filename, bit_begin, nbits):
        h = ctypes.c_void_p()
        _chk(lib().mbx_db_bitmap_stage_range(self.h, db.h, filename.encode(), bit_begin, nbits, ctypes.byref(h)))
        return Bitmap(self, h, nbits)

    # -- plans / scans ---------------------------------------------------
    def compile(self, table, cnf):
        keep = []
        c = make_cnf(cnf, keep)
        h = ctypes.c_void_p()
        _chk(lib().mbx_plan_compile(self.h, table.h, ctypes.byref(c), ctypes.byref(h)))
        return Plan(self, h, table)

    def scan_count(self, plan):
        n = ctypes.c_int64()
        _chk(lib().mbx_scan_count(self.h, plan.h, ctypes.byref(n)))
        return n.value

    def scan_count_async(self, plan, dev_ptr):
        _chk(lib().mbx_scan_count_async(self.h, plan.h, dev_ptr))

    def scan_count_frame_async(self, plan, dev_frame):
        """COUNT added into a zeroed, 128-byte-aligned frame of COUNT_FRAME_WORDS
        int64 words at dev_frame (no in-launch finalize; count_frame_decode)."""
        _chk(lib().mbx_scan_count_frame_async(self.h, plan.h, dev_frame))

    def scan_blocks(self, plan):
        b = ctypes.c_int64()
        _chk(lib().mbx_scan_blocks(self.h, plan.h, ctypes.byref(b)))
        return b.value

    def scan_bitmap(self, plan):
        h = ctypes.c_void_p()
        n = ctypes.c_int64()
        _chk(lib().mbx_scan_bitmap(self.h, plan.h, ctypes.byref(h), ctypes.byref(n)))
        return Bitmap(self, h, plan.table.nrows)

    def scan_bitmap_async(self, plan, bitmap):
        _chk(lib().mbx_scan_bitmap_async(self.h, plan.h, bitmap.h))

    def scan_select(self, plan, cap=None):
        """Ascending global positions of the rows the plan selects (one launch)."""
        cap = plan.table.nrows if cap is None else cap
        ids = np.zeros(max(1, cap), dtype=np.int64)
        n = ctypes.c_int64()
        _chk(lib().mbx_scan_select(self.h, plan.h, ids.ctypes.data, cap, ctypes.byref(n)))
        return ids[:n.value]

    def scan_select_async(self, plan, bitmap, dev_ids, dev_count):
        _chk(lib().mbx_scan_select_async(self.h, plan.h, bitmap.h, dev_ids, dev_count))

    def scan_aggregate(self, plan, col):
        a = Agg()
        _chk(lib().mbx_scan_aggregate(self.h, plan.h, col, ctypes.byref(a)))
        if a.agg_type == INTEGER:
            return dict(count=a.count, sum=a.isum, min=a.imin, max=a.imax)
        return dict(count=a.count, sum=a.fsum, min=a.fmin, max=a.fmax)

    def scan_aggregate_async(self, plan, col, dev_ptr):
        _chk(lib().mbx_scan_aggregate_async(self.h, plan.h, col, dev_ptr))

    # -- bitmaps ---------------------------------------------------------
    def bitmap_alloc(self, nbits):
        h = ctypes.c_void_p()
        _chk(lib().mbx_bitmap_alloc(self.h, nbits, ctypes.byref(h)))
        return Bitmap(self, h, nbits)

    def bitmap_upload(self, nbits, words):
        w = np.ascontiguousarray(words, dtype=np.uint64)
        h = ctypes.c_void_p()
        _chk(lib().mbx_bitmap_upload(self.h, nbits, w.ctypes.data if w.size else None, ctypes.byref(h)))
        return Bitmap(self, h, nbits)

    def bitmap_combine(self, op, a, b):
        h = ctypes.c_void_p()
        n = ctypes.c_int64()
        _chk(lib().mbx_bitmap_combine(self.h, op, a.h, b.h, ctypes.byref(h), ctypes.byref(n)))
        return Bitmap(self, h, a.nbits)

    def bitmap_cnf(self, nbits, conjuncts, deleted=None):
        """conjuncts: list of lists of Bitmap (OR within, AND across)."""
        flat = [b for conj in conjuncts for b in conj]
        bms = (ctypes.c_void_p * max(1, len(flat)))(*[b.h.value for b in flat])
        offs = (ctypes.c_int32 * (len(conjuncts) + 1))()
        k = 0
        for i, conj in enumerate(conjuncts):
            offs[i] = k
            k += len(conj)
        offs[len(conjuncts)] = k
        h = ctypes.c_void_p()
        n = ctypes.c_int64()
        _chk(lib().mbx_bitmap_cnf(self.h, nbits, bms, offs, len(conjuncts), None if deleted is None else deleted.h,
                                  ctypes.byref(h), ctypes.byref(n)))
        return Bitmap(self, h, nbits)

    def bitmap_cnf_async(self, conjuncts, out, deleted=None):
        flat = [b for conj in conjuncts for b in conj]
        bms = (ctypes.c_void_p * max(1, len(flat)))(*[b.h.value for b in flat])
        offs = (ctypes.c_int32 * (len(conjuncts) + 1))()
        k = 0
        for i, conj in enumerate(conjuncts):
            offs[i] = k
            k += len(conj)
        offs[len(conjuncts)] = k
        _chk(lib().mbx_bitmap_cnf_async(self.h, bms, offs, len(conjuncts),
                                        None if deleted is None else deleted.h, out.h))

    @staticmethod
    def _cnf_arrays(conjuncts):
        flat = [b for conj in conjuncts for b in conj]
        bms = (ctypes.c_void_p * max(1, len(flat)))(*[b.h.value for b in flat])
        offs = (ctypes.c_int32 * (len(conjuncts) + 1))()
        k = 0
        for i, conj in enumerate(conjuncts):
            offs[i] = k
            k += len(conj)
        offs[len(conjuncts)] = k
        return bms, offs

    def cnf_cursor(self, table, conjuncts, proj, deleted=None):
        """mbx_cnf_cursor_open: ColumnarIndexScan (CNF of index BitSets) +
        positions + projected rows (any columns) in one launch, as a cursor."""
        bms, offs = self._cnf_arrays(conjuncts)
        pj = (ctypes.c_int32 * max(1, len(proj)))(*proj)
        h = ctypes.c_void_p()
        _chk(lib().mbx_cnf_cursor_open(self.h, table.h, bms, offs, len(conjuncts),
                                       None if deleted is None else deleted.h, pj, len(proj), ctypes.byref(h)))
        return Cursor(self, h, table, list(proj))

    def cnf_cursor_launch(self, table, conjuncts, proj, deleted=None):
        """mbx_cnf_cursor_launch: as cnf_cursor, launch only -> (Cursor, device
        pointer of its count)."""
        bms, offs = self._cnf_arrays(conjuncts)
        pj = (ctypes.c_int32 * max(1, len(proj)))(*proj)
        h, dc = ctypes.c_void_p(), ctypes.c_void_p()
        _chk(lib().mbx_cnf_cursor_launch(self.h, table.h, bms, offs, len(conjuncts),
                                         None if deleted is None else deleted.h, pj, len(proj), ctypes.byref(h),
                                         ctypes.byref(dc)))
        return Cursor(self, h, table, list(proj)), dc.value

    def cnf_materialize_async(self, table, conjuncts, proj, dev_ids, dev_outs, dev_count, deleted=None):
        """mbx_cnf_materialize_async: CNF of index BitSets + positions +
        projected rows in one launch (device pointers as ints; dev_ids may be
        None; dev_outs[j] in the device row layout of column proj[j])."""
        bms, offs = self._cnf_arrays(conjuncts)
        pj = (ctypes.c_int32 * max(1, len(proj)))(*proj)
        outs = (ctypes.c_void_p * max(1, len(proj)))(*dev_outs)
        _chk(lib().mbx_cnf_materialize_async(self.h, table.h, bms, offs, len(conjuncts),
                                             None if deleted is None else deleted.h, pj, len(proj), dev_ids,
                                             outs, dev_count))

    def index_build(self, table, col, values):
        keep = []
        ops = (Operand * len(values))(*[_operand(v, keep) for v in values])
        hs = (ctypes.c_void_p * len(values))()
        _chk(lib().mbx_bitmap_index_build(self.h, table.h, col, ops, len(values), hs))
        return [Bitmap(self, ctypes.c_void_p(hs[i]), table.nrows) for i in range(len(values))]

    def select(self, bitmap, row_offset=0):
        n = ctypes.c_int64()
        known = bitmap.count  # -1 after an async producer: the library counts first
        cap = max(1, known if known >= 0 else bitmap.nbits)
        ids = np.zeros(cap, dtype=np.int64)
        _chk(lib().mbx_bitmap_select(self.h, bitmap.h, row_offset, ids.ctypes.data, cap, ctypes.byref(n)))
        return ids[:n.value]

    def materialize(self, table, bitmap, proj):
        """(ids, [column arrays]) of every selected row, ascending positions."""
        n = ctypes.c_int64()
        cap = max(1, bitmap.count)
        ids = np.zeros(cap, dtype=np.int64)
        outs = [table.empty_column(j, cap) for j in proj]
        ptrs = (ctypes.c_void_p * max(1, len(proj)))(*[o.ctypes.data for o in outs])
        pj = (ctypes.c_int32 * max(1, len(proj)))(*proj)
        _chk(lib().mbx_materialize(self.h, table.h, bitmap.h, pj, len(proj), ids.ctypes.data, ptrs, cap,
                                   ctypes.byref(n)))
        return ids[:n.value], [o[:n.value] for o in outs]

    def cursor(self, table, bitmap, proj):
        h = ctypes.c_void_p()
        pj = (ctypes.c_int32 * max(1, len(proj)))(*proj)
        _chk(lib().mbx_cursor_open(self.h, table.h, bitmap.h, pj, len(proj), ctypes.byref(h)))
        return Cursor(self, h, table, list(proj))

    # -- multi-GPU exchange (RCCL) and graphs ------------------------------
    def comm_init_rank(self, nranks, rank, uid):
        """mbx_comm_init_rank: this context becomes `rank` of an RCCL clique
        (one process per GPU; every rank passes rank 0's comm_unique_id())."""
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        _chk(lib().mbx_comm_init_rank(self.h, nranks, rank, buf, ctypes.byref(h)))
        return Comm(self, h, nranks, rank)

    def agg_fold_async(self, dev_recs, n, dev_out):
        """mbx_agg_fold_async: *dev_out = the rank-ordered fold of n 48-byte
        records at dev_recs (the aggregate exchange's fold, without RCCL)."""
        _chk(lib().mbx_agg_fold_async(self.h, dev_recs, n, dev_out))

    def graph_begin(self):
        _chk(lib().mbx_graph_begin(self.h))

    def graph_end(self):
        h = ctypes.c_void_p()
        _chk(lib().mbx_graph_end(self.h, ctypes.byref(h)))
        return Graph(self, h)


class _Handle:
    _free = None

    def close(self):
        if getattr(self, "h", None):
            getattr(lib(), self._free)(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


COMM_ID_BYTES = 128
COUNT_FRAME_WORDS = 512


def count_frame_decode(frame):
    """(count, nan_blocks, arrivals) of a host copy of a count frame (a numpy
    int64 array of COUNT_FRAME_WORDS words, possibly all-reduced over ranks)."""
    import numpy as np
    f = np.ascontiguousarray(frame, dtype=np.int64)
    assert f.size >= COUNT_FRAME_WORDS, f.size
    n, nan, arr = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    _chk(lib().mbx_count_frame_decode(f.ctypes.data, ctypes.byref(n), ctypes.byref(nan), ctypes.byref(arr)))
    return n.value, nan.value, arr.value


def count_frame_fits(nblocks, nranks):
    """mbx_count_frame_fits: nranks frames of <= nblocks-block scans sum exactly."""
    return bool(lib().mbx_count_frame_fits(int(nblocks), int(nranks)))


def comm_unique_id():
    """mbx_comm_unique_id: rank 0 creates it, the launcher shares it."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    _chk(lib().mbx_comm_unique_id(buf))
    return buf.raw


def shard_bounds(nrows, nshards, shard):
    """mbx_shard_bounds: [begin, end) of one 64-aligned row-range shard."""
    b, e = ctypes.c_int64(), ctypes.c_int64()
    _chk(lib().mbx_shard_bounds(nrows, nshards, shard, ctypes.byref(b), ctypes.byref(e)))
    return b.value, e.value


def comm_init_all(ctxs):
    """mbx_comm_init_all: one process drives every context's GPU; ctxs[i]
    becomes rank i of one clique."""
    n = len(ctxs)
    hs = (ctypes.c_void_p * n)(*[c.h for c in ctxs])
    outs = (ctypes.c_void_p * n)()
    _chk(lib().mbx_comm_init_all(hs, n, outs))
    return [Comm(c, ctypes.c_void_p(outs[i]), n, i) for i, c in enumerate(ctxs)]


def comm_allreduce_count_all(comms, dev_ptrs, count=1):
    n = len(comms)
    _chk(lib().mbx_comm_allreduce_count_all((ctypes.c_void_p * n)(*[c.h for c in comms]), n,
                                            (ctypes.c_void_p * n)(*dev_ptrs), count))


def comm_allreduce_agg_all(comms, dev_ptrs):
    n = len(comms)
    _chk(lib().mbx_comm_allreduce_agg_all((ctypes.c_void_p * n)(*[c.h for c in comms]), n,
                                          (ctypes.c_void_p * n)(*dev_ptrs)))


def comm_allgather_count_all(comms, dev_counts, dev_alls):
    """one grouped all-gather of every rank's device count into every rank's
    dev_alls buffer (nranks int64)"""
    n = len(comms)
    _chk(lib().mbx_comm_allgather_count_all((ctypes.c_void_p * n)(*[c.h for c in comms]), n,
                                            (ctypes.c_void_p * n)(*dev_counts), (ctypes.c_void_p * n)(*dev_alls)))


class Comm:
    """mbx_comm: the exchange step of one context (RCCL over xGMI)."""
    _free = "mbx_comm_free"

    def __init__(self, ctx, h, nranks, rank):
        self.ctx, self.h, self.nranks, self.rank = ctx, h, nranks, rank
        ctx._own(self)

    def close(self):
        if getattr(self, "h", None):
            lib().mbx_comm_free(self.h)
            self.h = None

    def wait(self):
        _chk(lib().mbx_comm_wait(self.h))

    def allreduce_count_async(self, dev_ptr, n=1):
        _chk(lib().mbx_comm_allreduce_count_async(self.h, dev_ptr, n))

    def scan_count_async(self, plan, dev_parts, parts_cap, dev_count):
        """one COUNT query combined over all ranks into *dev_count; the scan's
        per-block counts go to dev_parts (parts_cap int64 device slots), the
        exchange stream sums and all-reduces them"""
        _chk(lib().mbx_comm_scan_count_async(self.h, plan.h, dev_parts, parts_cap, dev_count))

    def allreduce_agg_async(self, dev_ptr):
        _chk(lib().mbx_comm_allreduce_agg_async(self.h, dev_ptr))

    def allgather_count_async(self, dev_count, dev_all):
        _chk(lib().mbx_comm_allgather_count_async(self.h, dev_count, dev_all))


class Graph:
    """mbx_graph: captured *_async calls, replayed with one launch."""
    _free = "mbx_graph_free"

    def __init__(self, ctx, h):
        self.ctx, self.h = ctx, h
        ctx._own(self)

    def launch(self):
        _chk(lib().mbx_graph_launch(self.h))

    def close(self):
        if getattr(self, "h", None):
            lib().mbx_graph_free(self.h)
            self.h = None


class Table(_Handle):
    _free = "mbx_table_free"

    def __init__(self, ctx, h, nrows, descs, row_offset, keep=None):
        self.ctx, self.h, self.nrows, self.descs, self.row_offset = ctx, h, nrows, descs, row_offset
        self._keep = keep
        ctx._own(self)

    def empty_column(self, j, n):
        t, size = self.descs[j]
        if t == STRING:
            return np.zeros((n, size), dtype=np.uint8)
        return np.zeros(n, dtype=np.int32 if t == INTEGER else np.float32)


class Plan(_Handle):
    _free = "mbx_plan_free"

    def __init__(self, ctx, h, table):
        self.ctx, self.h, self.table = ctx, h, table
        ctx._own(self)


class Bitmap(_Handle):
    _free = "mbx_bitmap_free"

    def __init__(self, ctx, h, nbits):
        self.ctx, self.h, self.nbits = ctx, h, nbits
        ctx._own(self)

    @property
    def nwords(self):
        return (self.nbits + 63) // 64

    @property
    def count(self):
        c = ctypes.c_int64()
        _chk(lib().mbx_bitmap_info(self.h, None, None, ctypes.byref(c)))
        return c.value

    def download(self):
        w = np.zeros(max(1, self.nwords), dtype=np.uint64)
        _chk(lib().mbx_bitmap_download(self.ctx.h, self.h, w.ctypes.data, len(w)))
        return w[:self.nwords]


class Cursor(_Handle):
    """iterator.Iterator over a materialised selection: next() hands out batches."""
    _free = "mbx_cursor_close"

    def __init__(self, ctx, h, table, proj):
        self.ctx, self.h, self.table, self.proj = ctx, h, table, proj
        ctx._own(self)

    @property
    def count(self):
        c = ctypes.c_int64()
        _chk(lib().mbx_cursor_count(self.h, ctypes.byref(c)))
        return c.value

    def next(self, max_rows):
        ids = np.zeros(max_rows, dtype=np.int64)
        outs = [self.table.empty_column(j, max_rows) for j in self.proj]
        ptrs = (ctypes.c_void_p * max(1, len(outs)))(*[o.ctypes.data for o in outs])
        n = ctypes.c_int64()
        _chk(lib().mbx_cursor_next(self.h, max_rows, ids.ctypes.data, ptrs, ctypes.byref(n)))
        k = n.value
        return ids[:k], [o[:k] for o in outs]

    def restart(self):
        _chk(lib().mbx_cursor_restart(self.h))

    def stats(self):
        """(rows handed out so far, bytes copied device -> host)"""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        _chk(lib().mbx_cursor_stats(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value


class Db:
    """A Minibase DB file (include/mbx_db.h); host-side page I/O only."""

    def __init__(self, path, num_pages=None):
        h = ctypes.c_void_p()
        if num_pages is None:
            _chk(lib().mbx_db_open(os.fsencode(path), ctypes.byref(h)))
        else:
            _chk(lib().mbx_db_create(os.fsencode(path), num_pages, ctypes.byref(h)))
        self.h, self.path = h, path

    def close(self):
        if getattr(self, "h", None):
            _chk(lib().mbx_db_close(self.h))
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        n, a = ctypes.c_int32(), ctypes.c_int32()
        _chk(lib().mbx_db_info(self.h, ctypes.byref(n), ctypes.byref(a)))
        return n.value, a.value

    def file_entry(self, name):
        p = ctypes.c_int32()
        _chk(lib().mbx_db_file_entry(self.h, name.encode(), ctypes.byref(p)))
        return p.value

    def columnar_create(self, name, cols, attr_names):
        """cols: [(attr_type, size)], size = n for char(n), 4 otherwise."""
        descs = (ColDesc * len(cols))()
        for j, (t, sz) in enumerate(cols):
            descs[j].attr_type, descs[j].size = t, sz
        names = (ctypes.c_char_p * len(cols))(*[n.encode() for n in attr_names])
        _chk(lib().mbx_db_columnar_create(self.h, name.encode(), len(cols), descs, names))

    def columnar_insert(self, name, columns):
        """columns: [(attr_type, size, ndarray)] as for Context.stage."""
        arrs = []
        nrows = None
        for t, size, a in columns:
            if t == INTEGER:
                a = np.ascontiguousarray(a, dtype=np.int32)
            elif t == REAL:
                a = np.ascontiguousarray(a, dtype=np.float32)
            else:
                a = np.ascontiguousarray(a, dtype=np.uint8).reshape(-1, size)
            arrs.append(a)
            nrows = a.shape[0] if nrows is None else nrows
        ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        _chk(lib().mbx_db_columnar_insert(self.h, name.encode(), nrows, ptrs))

    def columnar_info(self, name, max_cols=256):
        n = ctypes.c_int32()
        descs = (ColDesc * max_cols)()
        names = ctypes.create_string_buffer(16 * max_cols)
        nrows, live = ctypes.c_int64(), ctypes.c_int64()
        _chk(lib().mbx_db_columnar_info(self.h, name.encode(), max_cols, ctypes.byref(n), descs, names,
                                        ctypes.byref(nrows), ctypes.byref(live)))
        k = min(n.value, max_cols)
        return {"ncols": n.value, "cols": [(descs[j].attr_type, descs[j].size) for j in range(k)],
                "names": [names.raw[16 * j:16 * j + 16].split(b"\0")[0].decode() for j in range(k)],
                "nrows": nrows.value, "live": live.value}

    def allocate_pages(self, run):
        p = ctypes.c_int32()
        _chk(lib().mbx_db_allocate_pages(self.h, run, ctypes.byref(p)))
        return p.value

    def add_file_entry(self, name, start):
        _chk(lib().mbx_db_add_file_entry(self.h, name.encode(), start))

    def bitmap_values(self, name, col):
        """Registered bitmap-index values of a column (modified UTF-8 bytes)."""
        cnt, nb = ctypes.c_int32(), ctypes.c_int64()
        _chk(lib().mbx_db_bitmap_values(self.h, name.encode(), col, None, 0, ctypes.byref(cnt), ctypes.byref(nb)))
        buf = ctypes.create_string_buffer(max(1, nb.value))
        _chk(lib().mbx_db_bitmap_values(self.h, name.encode(), col, buf, nb.value, ctypes.byref(cnt), ctypes.byref(nb)))
        return buf.raw[:nb.value].split(b"\0")[:cnt.value]

    def mark_deleted(self, name, position):
        _chk(lib().mbx_db_mark_deleted(self.h, name.encode(), position))

    def mark_deleted_many(self, name, positions):
        p = np.ascontiguousarray(positions, dtype=np.int64)
        _chk(lib().mbx_db_mark_deleted_many(self.h, name.encode(), p.ctypes.data if len(p) else None, len(p)))

    def purge(self, name):
        """Columnarfile.purgeAllDeletedTuples."""
        _chk(lib().mbx_db_purge(self.h, name.encode()))

    def bitmap_write(self, filename, words):
        w = np.ascontiguousarray(words, dtype=np.uint64)
        _chk(lib().mbx_db_bitmap_write(self.h, filename.encode(), w.ctypes.data if len(w) else None, len(w)))

    def bitmap_read(self, filename):
        n = ctypes.c_int64()
        _chk(lib().mbx_db_bitmap_read(self.h, filename.encode(), None, 0, ctypes.byref(n)))
        w = np.zeros(max(1, n.value), dtype=np.uint64)
        _chk(lib().mbx_db_bitmap_read(self.h, filename.encode(), w.ctypes.data, len(w), ctypes.byref(n)))
        return w[:n.value]
