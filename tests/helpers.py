"""Shared test helpers: minidata loading, CNF-string parsing, synthetic tables."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
if os.path.join(ROOT, "oracle") not in sys.path:
    sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402  (test infrastructure)

# AttrOperator.findOperator (R/global/AttrOperator.java:154-172)
OPS = {"=": oracle.EQ, "<": oracle.LT, ">": oracle.GT, "!=": oracle.NE, ">=": oracle.GE, "<=": oracle.LE}
MINI_COLS = ["A", "B", "C", "D"]
MINI_TYPES = [oracle.STRING, oracle.STRING, oracle.INTEGER, oracle.INTEGER]
MINI_SIZES = [25, 25, 4, 4]


def load_golden():
    with open(os.path.join(GOLDEN, "phase3_golden.json")) as f:
        return json.load(f)


def load_minidata():
    """BatchInsert over minidata.txt (R/input/BatchInsert.java:17-137):
    header `A:char(25) B:char(25) C:int D:int`, then one TSV line per row."""
    with open(os.path.join(GOLDEN, "minidata.tsv"), encoding="utf-8") as f:
        lines = [ln.rstrip("\n") for ln in f if ln.strip()]
    rows = []
    for ln in lines[1:]:
        a, b, c, d = ln.split("\t")
        rows.append((a, b, int(c), int(d)))
    return rows


def encode_strings(values, size):
    arr = np.zeros((len(values), size), dtype=np.uint8)
    for i, v in enumerate(values):
        b = oracle.java_mutf8(v)
        assert len(b) <= size
        arr[i, :len(b)] = np.frombuffer(b, dtype=np.uint8)
    return arr


def minidata_columns(rows):
    return [
        (oracle.STRING, 25, encode_strings([r[0] for r in rows], 25)),
        (oracle.STRING, 25, encode_strings([r[1] for r in rows], 25)),
        (oracle.INTEGER, 4, np.array([r[2] for r in rows], dtype=np.int32)),
        (oracle.INTEGER, 4, np.array([r[3] for r in rows], dtype=np.int32)),
    ]


def golden_cnf(cnf, names=MINI_COLS, types=MINI_TYPES):
    """[[['A','=','x'], ...], ...] -> oracle CNF spec, literals typed from the
    column as Query.buildQueryCondExpr / MultiIndexQuery do
    (R/input/Query.java:299-323)."""
    out = []
    for conj in cnf:
        terms = []
        for term in conj:
            col, op, val = term[:3]
            k = names.index(col)
            t = types[k]
            lit = ("int", int(val)) if t == oracle.INTEGER else (("real", float(val)) if t == oracle.REAL
                                                                  else ("str", val))
            idx = {"BT": oracle.IDX_BTREE, "BM": oracle.IDX_BITMAP}.get(term[3] if len(term) > 3 else "BM")
            terms.append((OPS[op], ("sym", k + 1), lit, idx))
        out.append(terms)
    return out


def parse_cnf_string(s, names=MINI_COLS, types=MINI_TYPES):
    """'{(A,=,x)|(B,=,y)}^{(C,=,6)}' (the CLI grammar) -> oracle CNF spec."""
    conjs = []
    for part in s.strip().split("^"):
        part = part.strip()[1:-1]
        conjs.append([[x.strip() for x in t.strip()[1:-1].split(",")] for t in part.split("|")])
    return golden_cnf(conjs, names, types)


def synthetic_int_table(n, ncols=4, hi=1 << 20, seed=42):
    """SURVEY 8(d) generator: int32 columns uniform in [0, hi), seed 42+j."""
    cols = []
    for j in range(ncols):
        rng = np.random.Generator(np.random.PCG64(seed + j))
        cols.append(rng.integers(0, hi, size=n, dtype=np.int32))
    return cols


def random_deleted(n, frac, seed=7):
    rng = np.random.Generator(np.random.PCG64(seed))
    bits = rng.random(n) < frac
    words = np.zeros((n + 63) // 64, dtype=np.uint64)
    idx = np.nonzero(bits)[0]
    np.bitwise_or.at(words, idx // 64, (np.uint64(1) << (idx % 64).astype(np.uint64)))
    return words


def device_dictionary_column(dic, idx, chunk=1 << 23):
    """dic[idx] for a device dictionary `dic` (V, w) and device codes `idx`
    (n,), built chunk by chunk.  One torch advanced-index launch with a large
    output returns wrong rows on this ROCm image (measured: dic.view(int64)[idx]
    over 200M rows left 2^27 rows zero and 67 % of sampled rows wrong), so each
    launch writes at most `chunk` rows and the caller checks the result."""
    import torch
    n = idx.shape[0]
    out = torch.empty((n,) + tuple(dic.shape[1:]), dtype=dic.dtype, device=dic.device)
    for s in range(0, n, chunk):
        out[s:s + chunk].copy_(dic[idx[s:s + chunk].long()])
    return out


def index_registry(ctx, ocols, t, col):
    """`index db cf <col> bitmap`: one BitMapFile per distinct value, built on
    the GPU in one pass; the registry maps value -> device bitmap."""
    typ, size, arr = ocols[col]
    if typ == oracle.STRING:
        vals = sorted({bytes(r).rstrip(b"\0") for r in arr})
        specs = [("str", v) for v in vals]
    else:
        vals = sorted(set(int(x) for x in arr))
        specs = [("int", v) for v in vals]
    bms = ctx.index_build(t, col, specs)
    return dict(zip(vals, bms))


def value_set(reg, typ, op, lit):
    """ColumnIndexScan.getBitSet value selection (R/index/ColumnIndexScan.java:656-740)."""
    if typ == oracle.STRING:
        key = lambda v: oracle.java_mutf8(v).decode("utf-8", "surrogatepass").encode("utf-16-be", "surrogatepass")
        litb = oracle.java_mutf8(lit)
        cmp = lambda other: (key(litb) > key(other)) - (key(litb) < key(other))
        lit_key = litb
    else:
        cmp = lambda other: (lit > other) - (lit < other)
        lit_key = lit
    out = []
    if op in (oracle.EQ, oracle.LE, oracle.GE) and lit_key in reg:
        out.append(reg[lit_key])
    for v, bm in reg.items():
        c = cmp(v)
        if (op in (oracle.LT, oracle.LE) and c > 0) or (op in (oracle.GT, oracle.GE) and c < 0) or \
                (op == oracle.NE and c != 0):
            out.append(bm)
    return out


def index_conjuncts(regs, cnf, types):
    """ColumnarIndexScan's bitmap lists (R/index/ColumnarIndexScan.java:130-181):
    per conjunct the value bitmaps of every term, in term order."""
    out = []
    for conj in cnf:
        lst = []
        for op, (_, fld), (_, lit), *_ in conj:
            lst += value_set(regs[fld - 1], types[fld - 1], op, lit)
        out.append(lst)
    return out
