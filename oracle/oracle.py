"""ctypes binding of the CPU oracle (oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.

CNF spec used throughout the tests (a flattened ``CondExpr[]``):
    cnf = [conjunct, ...]            # AND of conjuncts (CondExpr[] array)
    conjunct = [term, ...]           # OR of terms (.next linked list)
    term = (op, operand1, operand2[, index_type])  # AttrOperator code, operands
    operand = ('sym', fld)           # FldSpec(outer, fld), 1-based
            | ('int', v) | ('real', v) | ('str', text)
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

STRING, INTEGER, REAL, SYMBOL = 0, 1, 2, 3
EQ, LT, GT, NE, LE, GE, NOT, NOP, RANGE = range(9)
IDX_NONE, IDX_BTREE, IDX_HASH, IDX_BITMAP = range(4)


class _Column(ctypes.Structure):
    _fields_ = [("attr_type", ctypes.c_int32), ("size", ctypes.c_int32), ("data", ctypes.c_void_p)]


class _Operand(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("fld", ctypes.c_int32), ("integer", ctypes.c_int32),
                ("real", ctypes.c_float), ("string", ctypes.c_char_p), ("string_len", ctypes.c_int32)]


class _CondExpr(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("operand1", _Operand), ("operand2", _Operand),
                ("index_type", ctypes.c_int32)]


class _Cnf(ctypes.Structure):
    _fields_ = [("conds", ctypes.POINTER(_CondExpr)), ("conj_offsets", ctypes.POINTER(ctypes.c_int32)),
                ("nconj", ctypes.c_int32)]


class _Agg(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int64), ("agg_type", ctypes.c_int32), ("isum", ctypes.c_int64),
                ("imin", ctypes.c_int32), ("imax", ctypes.c_int32), ("fsum", ctypes.c_double),
                ("fmin", ctypes.c_float), ("fmax", ctypes.c_float)]


def java_mutf8(s):
    """DataOutputStream.writeUTF payload: modified UTF-8 of the UTF-16 units."""
    if isinstance(s, bytes):
        return s
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


def build():
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
                os.path.join(HERE, "oracle.c")):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        L.orc_pred_eval.argtypes = [P(_Cnf), P(_Column), ctypes.c_int32, ctypes.c_int64]
        L.orc_pred_eval.restype = ctypes.c_int
        L.orc_string_compare.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32]
        L.orc_filescan.argtypes = [P(_Column), ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, P(_Cnf),
                                   ctypes.c_void_p, ctypes.c_void_p]
        L.orc_filescan.restype = ctypes.c_int64
        L.orc_aggregate.argtypes = [P(_Column), ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, P(_Cnf),
                                    ctypes.c_int32, P(_Agg)]
        L.orc_bitmap_eq.argtypes = [P(_Column), ctypes.c_int64, ctypes.c_void_p, P(_Operand), ctypes.c_void_p]
        L.orc_bitmap_eq.restype = ctypes.c_int64
        L.orc_column_index_scan.argtypes = [P(_Column), ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                            P(_Operand), ctypes.c_void_p]
        L.orc_column_index_scan.restype = ctypes.c_int64
        L.orc_columnar_index_scan.argtypes = [P(_Column), ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                              P(_Cnf), ctypes.c_void_p]
        L.orc_columnar_index_scan.restype = ctypes.c_int64
        L.orc_filescan_count_mt.argtypes = [P(_Column), ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                            P(_Cnf), ctypes.c_int32]
        L.orc_filescan_count_mt.restype = ctypes.c_int64
        L.orc_gather.argtypes = [P(_Column), ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                 P(ctypes.c_int32), ctypes.c_int32, P(ctypes.c_void_p)]
        _lib = L
    return _lib


class Table:
    """Decoded Columnarfile: columns in position order + deleted BitSet words."""

    def __init__(self, columns, deleted_words=None):
        # columns: list of (attr_type, size, ndarray) ; strings as uint8 [nrows, size]
        self.columns = []
        self.nrows = None
        for t, size, arr in columns:
            if t == INTEGER:
                arr = np.ascontiguousarray(arr, dtype=np.int32)
                size = 4
            elif t == REAL:
                arr = np.ascontiguousarray(arr, dtype=np.float32)
                size = 4
            elif t == STRING:
                arr = np.ascontiguousarray(arr, dtype=np.uint8).reshape(-1, size)
            else:
                raise ValueError(t)
            n = arr.shape[0]
            if self.nrows is None:
                self.nrows = n
            assert n == self.nrows
            self.columns.append((t, size, arr))
        self.deleted = None if deleted_words is None else np.ascontiguousarray(deleted_words, dtype=np.uint64)
        self._c = (_Column * len(self.columns))()
        for i, (t, size, arr) in enumerate(self.columns):
            self._c[i].attr_type = t
            self._c[i].size = size
            self._c[i].data = arr.ctypes.data

    @property
    def nwords(self):
        return (self.nrows + 63) // 64

    def _del_ptr(self):
        return None if self.deleted is None else self.deleted.ctypes.data


def _operand(spec, keep):
    o = _Operand()
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


def _cnf(cnf, keep):
    if cnf is None:
        c = _Cnf()
        c.nconj = 0
        return c
    terms = [t for conj in cnf for t in conj]
    conds = (_CondExpr * max(1, len(terms)))()
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
    c = _Cnf()
    c.conds = conds
    c.conj_offsets = offs
    c.nconj = len(cnf)
    return c


def _check(rc, what):
    if rc < 0:
        raise RuntimeError(f"oracle {what} failed: {rc}")
    return rc


def filescan(table, cnf):
    """ColumnarFileScan selection: (count, words uint64[nwords], ids int64[count])."""
    keep = []
    c = _cnf(cnf, keep)
    words = np.zeros(max(1, table.nwords), dtype=np.uint64)
    ids = np.zeros(max(1, table.nrows), dtype=np.int64)
    n = _check(lib().orc_filescan(table._c, len(table.columns), table.nrows, table._del_ptr(),
                                  ctypes.byref(c), words.ctypes.data, ids.ctypes.data), "filescan")
    return n, words[:table.nwords], ids[:n]


def filescan_count(table, cnf):
    """ColumnarFileScan COUNT only (Query.java:147 resultCount), no outputs."""
    keep = []
    c = _cnf(cnf, keep)
    return _check(lib().orc_filescan(table._c, len(table.columns), table.nrows, table._del_ptr(),
                                     ctypes.byref(c), None, None), "filescan")


def filescan_count_mt(table, cnf, nthreads):
    """filescan_count over nthreads OpenMP threads (the multi-core CPU baseline)."""
    keep = []
    c = _cnf(cnf, keep)
    return _check(lib().orc_filescan_count_mt(table._c, len(table.columns), table.nrows, table._del_ptr(),
                                              ctypes.byref(c), nthreads), "filescan_count_mt")


def pred_eval(table, cnf, row):
    keep = []
    c = _cnf(cnf, keep)
    return lib().orc_pred_eval(ctypes.byref(c), table._c, len(table.columns), row)


def aggregate(table, cnf, agg_col):
    keep = []
    c = _cnf(cnf, keep)
    a = _Agg()
    _check(lib().orc_aggregate(table._c, len(table.columns), table.nrows, table._del_ptr(),
                               ctypes.byref(c), agg_col, ctypes.byref(a)), "aggregate")
    if a.agg_type == INTEGER:
        return dict(count=a.count, sum=a.isum, min=a.imin, max=a.imax)
    return dict(count=a.count, sum=a.fsum, min=a.fmin, max=a.fmax)


def bitmap_eq(table, col, value):
    keep = []
    o = _operand(value, keep)
    words = np.zeros(max(1, table.nwords), dtype=np.uint64)
    n = _check(lib().orc_bitmap_eq(ctypes.byref(table._c[col]), table.nrows, table._del_ptr(), ctypes.byref(o),
                                   words.ctypes.data), "bitmap_eq")
    return n, words[:table.nwords]


def column_index_scan(table, col, op, value):
    keep = []
    o = _operand(value, keep)
    words = np.zeros(max(1, table.nwords), dtype=np.uint64)
    n = _check(lib().orc_column_index_scan(ctypes.byref(table._c[col]), table.nrows, table._del_ptr(), op,
                                           ctypes.byref(o), words.ctypes.data), "column_index_scan")
    return n, words[:table.nwords]


def columnar_index_scan(table, cnf):
    keep = []
    c = _cnf(cnf, keep)
    words = np.zeros(max(1, table.nwords), dtype=np.uint64)
    n = _check(lib().orc_columnar_index_scan(table._c, len(table.columns), table.nrows, table._del_ptr(),
                                             ctypes.byref(c), words.ctypes.data), "columnar_index_scan")
    return n, words[:table.nwords]


def gather(table, ids, proj):
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    outs = []
    for j in proj:
        t, size, _ = table.columns[j]
        if t == STRING:
            outs.append(np.zeros((len(ids), size), dtype=np.uint8))
        else:
            outs.append(np.zeros(len(ids), dtype=np.int32 if t == INTEGER else np.float32))
    ptrs = (ctypes.c_void_p * max(1, len(proj)))(*[o.ctypes.data for o in outs])
    pj = (ctypes.c_int32 * max(1, len(proj)))(*proj)
    _check(lib().orc_gather(table._c, len(table.columns), ids.ctypes.data, len(ids), pj, len(proj), ptrs),
           "gather")
    return outs


def words_to_positions(words):
    """BitSet words -> ascending positions (java.util.BitSet bit order)."""
    w = np.asarray(words, dtype=np.uint64)
    bits = np.unpackbits(w.view(np.uint8), bitorder="little")
    return np.nonzero(bits)[0].astype(np.int64)
