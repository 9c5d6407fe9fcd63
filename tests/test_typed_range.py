"""Typed range tests (scan_int_range = 2): COUNT and aggregate scans whose
literal terms are int, float or char(16) compares evaluate each term as one
unsigned range test over a signed-ordered key -- the int value, a float's bits
with the low 31 bits flipped when negative (-0.0 and +0.0 adjacent, NaNs
outside [-inf, +inf]), a string's compareTo sign -- built on the host
(mbx_api.cpp float_range_of / str_range_of).  PredEval's float compare
(R/iterator/PredEval.java:131-162, TupleUtils for attrReal) and its NaN rule
(a reached NaN compare raises) are checked against the oracle at the float
literals where a key off-by-one would show (+-0, +-inf, the smallest
subnormals, NaN), every operator, both literal sides, C5-shaped mixed CNFs,
deleted rows, and the PredEval NaN-order cases of tests/test_nan_order.py.
"""
import numpy as np
import pytest

import helpers
import mbx_pkg
import oracle
from test_nan_order import CASES, _check, _table as _nan_table

pytestmark = pytest.mark.gpu

LT, LE, GT, GE, EQ, NE, NOP = oracle.LT, oracle.LE, oracle.GT, oracle.GE, oracle.EQ, oracle.NE, oracle.NOP
F32 = np.float32
SUB = float(np.nextafter(F32(0), F32(1)))
FLITS = [float("-inf"), -1e30, -1.5, -SUB, -0.0, 0.0, SUB, 0.25, 1.0, 3e38, float("inf")]


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


def _mixed(n, seed, deleted_frac=0.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    i0 = rng.integers(0, 1 << 20, n, dtype=np.int32)
    f1 = rng.choice(np.array(FLITS, dtype=F32), n)
    f1[::3] = (rng.random(n, dtype=F32)[::3] - F32(0.5)) * F32(4)
    names = ["Alabama", "Colorado", "M", "Maine", "Ma", "South_Dakota", "Texas", "Zz", "", "Mzzzzzzzzzzzzzzz"]
    s2 = helpers.encode_strings([names[i] for i in rng.integers(0, len(names), n)], 16)
    cols = [(oracle.INTEGER, 4, i0), (oracle.REAL, 4, f1), (oracle.STRING, 16, s2)]
    dele = None
    if deleted_frac:
        bits = rng.random(n) < deleted_frac
        dele = np.frombuffer(np.pad(np.packbits(bits, bitorder="little"), (0, (-((n + 7) // 8)) % 8)).tobytes(),
                             dtype=np.uint64).copy()
    return cols, dele


def _agg_eq(got, want):
    assert got["count"] == want["count"], (got, want)
    if want["count"]:
        assert got["min"] == want["min"] and got["max"] == want["max"], (got, want)
        ws, gs = float(want["sum"]), float(got["sum"])
        if np.isnan(ws) or np.isinf(ws):  # +-inf rows in the selection
            assert (np.isnan(ws) and np.isnan(gs)) or ws == gs, (got, want)
        else:
            assert abs(gs - ws) <= 1e-9 * max(1.0, abs(ws)), (got, want)


def _both(m, ctx, t, ot, cnf, agg_col=1):
    """COUNT and the float aggregate with the typed range body (knob 2) and the
    branchy body (knob 0): both equal to the oracle"""
    want = oracle.filescan_count(ot, cnf)
    want_agg = oracle.aggregate(ot, cnf, agg_col)
    plan = ctx.compile(t, cnf)
    for knob in (2, 0):
        ctx.set_tuning("scan_int_range", knob)
        assert ctx.scan_count(plan) == want, (knob, cnf)
        _agg_eq(ctx.scan_aggregate(plan, agg_col), want_agg)
    ctx.set_tuning("scan_int_range", 2)


@pytest.mark.parametrize("op", [LT, LE, GT, GE, EQ, NE])
def test_float_literals_at_the_edges(m, ctx, op):
    cols, _ = _mixed(50_003, 3)
    t = ctx.stage(cols)
    ot = oracle.Table(cols)
    for lit in FLITS:
        for cnf in ([[(op, ("sym", 2), ("real", lit))]], [[(op, ("real", lit), ("sym", 2))]]):
            _both(m, ctx, t, ot, cnf, agg_col=0)


@pytest.mark.parametrize("op", [LT, LE, GT, GE, EQ, NE])
def test_string_literals(m, ctx, op):
    cols, _ = _mixed(40_001, 4)
    t = ctx.stage(cols)
    ot = oracle.Table(cols)
    for lit in ["M", "Ma", "Maine", "", "Mzzzzzzzzzzzzzzz", "Texas", "A"]:
        for cnf in ([[(op, ("sym", 3), ("str", lit))]], [[(op, ("str", lit), ("sym", 3))]]):
            _both(m, ctx, t, ot, cnf)


LONG_NAMES = ["Abcdefgh", "Abcdefgha", "AbcdefghZ", "Abcdefghé", "Abcdefghéa", "Abcdefghijklmnop",
              "Abcdefghijklmnoo", "Abcdefghijklmnoq", "Abcdefghijklmno", "Abcdefgh\u0000x", "Abcdefg￿",
              "Abcdefgi", "Abcdefg", "ébcdefghijklmno", "zzzzzzzzzzzzzzzz"]


@pytest.mark.parametrize("op", [LT, LE, GT, GE, EQ, NE])
def test_string_literals_past_the_first_eight_bytes(m, ctx, op):
    """Rows and literals that agree on their first 8 bytes and differ after
    them (the scan compares each 16-byte row as two 64-bit big-endian keys),
    including bytes >= 0x80 (UTF-8 / U+FFFF) and an embedded U+0000."""
    rng = np.random.Generator(np.random.PCG64(11))
    n = 30_011
    s = helpers.encode_strings([LONG_NAMES[i] for i in rng.integers(0, len(LONG_NAMES), n)], 16)
    i0 = rng.integers(0, 1 << 20, n, dtype=np.int32)
    cols = [(oracle.INTEGER, 4, i0), (oracle.STRING, 16, s)]
    t = ctx.stage(cols)
    ot = oracle.Table(cols)
    for lit in LONG_NAMES + ["Abcdefghè", "Abcdefghijklmnoa", "Abcdefgh\u0000"]:
        for cnf in ([[(op, ("sym", 2), ("str", lit))]], [[(op, ("str", lit), ("sym", 2))]],
                    [[(op, ("sym", 2), ("str", lit))], [(LT, ("sym", 1), ("int", 1 << 19))]]):
            _both(m, ctx, t, ot, cnf, agg_col=0)


def _random_names(rng, k):
    """k random strings whose modified UTF-8 fits 16 bytes, drawn from ASCII,
    2- and 3-byte characters, U+0000 and supplementary characters (surrogate
    pairs: 6 bytes), many sharing long prefixes."""
    alphabet = ["a", "b", "M", "z", "é", "ÿ", "Ā", "中", "￿", "\u0000", "\U0001F600"]
    prefixes = ["", "Abcdefgh", "Abcdefg", "M", "Maine"]
    out = []
    while len(out) < k:
        s = prefixes[int(rng.integers(0, len(prefixes)))]
        for _ in range(int(rng.integers(0, 12))):
            s += alphabet[int(rng.integers(0, len(alphabet)))]
        if len(oracle.java_mutf8(s)) <= 16:
            out.append(s)
    return out


def test_string_fuzz(m, ctx):
    """Random rows and literals (ragged lengths, bytes >= 0x80, U+0000,
    supplementary characters, shared prefixes): every operator, both literal
    sides, the range body (knob 2) and the branchy body (knob 0) vs the
    oracle."""
    rng = np.random.Generator(np.random.PCG64(13))
    pool = _random_names(rng, 300)
    n = 30_007
    s = helpers.encode_strings([pool[i] for i in rng.integers(0, len(pool), n)], 16)
    cols = [(oracle.INTEGER, 4, rng.integers(0, 1 << 20, n, dtype=np.int32)), (oracle.STRING, 16, s)]
    t = ctx.stage(cols)
    ot = oracle.Table(cols)
    lits = [pool[i] for i in rng.integers(0, len(pool), 10)] + _random_names(rng, 10)
    for k, lit in enumerate(lits):
        for op in [LT, LE, GT, GE, EQ, NE]:
            cnf = [[(op, ("sym", 2), ("str", lit))]] if k % 2 == 0 else [[(op, ("str", lit), ("sym", 2))]]
            _both(m, ctx, t, ot, cnf, agg_col=0)


@pytest.mark.parametrize("with_int", [False, True])
def test_two_string_slots(m, ctx, with_int):
    """Terms on both 16-byte string slots of a plan (the second slot's rows,
    D.s[1]), with and without a 4-byte column: every operator, both literal
    sides, one- and two-term conjuncts."""
    rng = np.random.Generator(np.random.PCG64(12))
    n = 20_011
    a = helpers.encode_strings([LONG_NAMES[i] for i in rng.integers(0, len(LONG_NAMES), n)], 16)
    b = helpers.encode_strings([LONG_NAMES[i] for i in rng.integers(0, len(LONG_NAMES), n)], 16)
    cols = [(oracle.STRING, 16, a), (oracle.STRING, 16, b)]
    if with_int:
        cols.append((oracle.INTEGER, 4, rng.integers(0, 1 << 20, n, dtype=np.int32)))
    t = ctx.stage(cols)
    ot = oracle.Table(cols)
    ops = [LT, LE, GT, GE, EQ, NE]
    for k, op in enumerate(ops):
        la, lb = LONG_NAMES[(3 * k) % len(LONG_NAMES)], LONG_NAMES[(3 * k + 7) % len(LONG_NAMES)]
        cnfs = [[[(op, ("sym", 2), ("str", lb))]],
                [[(op, ("str", la), ("sym", 1))], [(ops[(k + 1) % 6], ("sym", 2), ("str", lb))]],
                [[(op, ("sym", 1), ("str", la)), (ops[(k + 3) % 6], ("str", lb), ("sym", 2))]]]
        if with_int:
            cnfs.append([[(op, ("sym", 2), ("str", lb))], [(LT, ("sym", 3), ("int", 1 << 19))]])
        for cnf in cnfs:
            want = oracle.filescan_count(ot, cnf)
            plan = ctx.compile(t, cnf)
            for knob in (2, 0):
                ctx.set_tuning("scan_int_range", knob)
                assert ctx.scan_count(plan) == want, (knob, cnf)
                if with_int:
                    _agg_eq(ctx.scan_aggregate(plan, 2), oracle.aggregate(ot, cnf, 2))
            ctx.set_tuning("scan_int_range", 2)


def test_c5_shaped_cnfs(m, ctx):
    """(c0 < 2^19) ^ (c1 >= 0.25) ^ (c2 >= "M") and random mixed CNFs of <= 4
    literal terms, with deleted rows"""
    cols, dele = _mixed(400_009, 5, 0.05)
    t = ctx.stage(cols, dele)
    ot = oracle.Table(cols, dele)
    _both(m, ctx, t, ot, [[(LT, ("sym", 1), ("int", 1 << 19))], [(GE, ("sym", 2), ("real", 0.25))],
                          [(GE, ("sym", 3), ("str", "M"))]])
    rng = np.random.Generator(np.random.PCG64(6))
    ops = [LT, LE, GT, GE, EQ, NE]
    for _ in range(30):
        cnf, left = [], 4
        for _c in range(int(rng.integers(1, 4))):
            conj = []
            for _t in range(int(rng.integers(1, 3))):
                if left == 0:
                    break
                left -= 1
                col = int(rng.integers(1, 4))
                lit = [("int", int(rng.integers(0, 1 << 20))), ("real", float(rng.choice(FLITS))),
                       ("str", str(rng.choice(["M", "Maine", "Texas", "", "B"])))][col - 1]
                op = int(rng.choice(ops))
                conj.append((op, ("sym", col), lit) if rng.random() < 0.7 else (op, lit, ("sym", col)))
            if conj:
                cnf.append(conj)
        _both(m, ctx, t, ot, cnf)


@pytest.mark.parametrize("deleted", [False, True])
@pytest.mark.parametrize("name,cnf,raises", CASES, ids=[c[0] for c in CASES])
def test_nan_order_with_typed_ranges(m, ctx, tune, deleted, name, cnf, raises):
    """PredEval's NaN order (raise only where the float compare is reached)
    through the typed range body: COUNT and aggregate scans; the BitSet and
    select scans of the same check keep their own bodies."""
    cols, dele = _nan_table(deleted=deleted)
    t = ctx.stage(cols, dele if deleted else None)
    ot = oracle.Table(cols, dele if deleted else None)
    tune("scan_int_range", 2)
    raised = _check(m, ctx, ot, t, cnf)  # asserts every output against the oracle
    if deleted:  # CASES' expectations are for the table with its deleted rows
        assert raised == raises


def test_nan_fuzz_with_typed_ranges(m, ctx, tune):
    """tests/test_nan_order.py's random CNFs through the typed range body"""
    import test_nan_order
    tune("scan_int_range", 2)
    test_nan_order.test_gpu_nan_fuzz(m, ctx, tune, False)
