"""Branch-free int terms (knob scan_int_range, default on): a scan (COUNT,
BitSet, positions, aggregate) whose terms are all int `column OP literal` compares evaluates each term as one
unsigned range test, ((uint32)(a - rlo) <= rspan) != rneg, built on the host
from the operator and the literal (mbx_api.cpp int_range_of).  PredEval's
integer compare (R/iterator/PredEval.java:131-162, TupleUtils.CompareTupleWithValue
for attrInteger) is a signed 32-bit compare; this checks the range form
against the oracle at the literals where an off-by-one or an overflow would
show (INT_MIN, INT_MAX and their neighbours), for every operator, with the
literal on either side, in multi-term conjunctions and disjunctions, with
deleted rows, and against the same scans with the knob off.
"""
import numpy as np
import pytest

import helpers  # noqa: F401
import mbx_pkg
import oracle

pytestmark = pytest.mark.gpu

LT, LE, GT, GE, EQ, NE, NOP = oracle.LT, oracle.LE, oracle.GT, oracle.GE, oracle.EQ, oracle.NE, oracle.NOP
IMIN, IMAX = -(1 << 31), (1 << 31) - 1
LITS = [IMIN, IMIN + 1, -2, -1, 0, 1, 2, IMAX - 1, IMAX]


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


def _table(n=70_001, seed=17):
    rng = np.random.Generator(np.random.PCG64(seed))
    a = rng.choice(np.array(LITS, dtype=np.int64), n).astype(np.int32)
    a[::7] = rng.integers(IMIN, IMAX, n, dtype=np.int64, endpoint=True)[::7].astype(np.int32)
    b = rng.integers(-5, 5, n, dtype=np.int32)
    c = rng.choice(np.array(LITS, dtype=np.int64), n).astype(np.int32)
    return [(oracle.INTEGER, 4, a), (oracle.INTEGER, 4, b), (oracle.INTEGER, 4, c)]


def _count_both(m, ctx, t, cnf):
    """(range form, branchy form) COUNT of one CNF"""
    plan = ctx.compile(t, cnf)
    ctx.set_tuning("scan_int_range", 2)
    on = ctx.scan_count(plan)
    ctx.set_tuning("scan_int_range", 0)
    off = ctx.scan_count(plan)
    ctx.set_tuning("scan_int_range", 2)
    return on, off


def _all_outputs(m, ctx, t, ot, cnf, agg_col=2):
    """BitSet (k_scan_fast BitSet mode), positions (the one-launch
    k_scan_select) and an int aggregate with the knob on and off, each equal
    to the oracle's"""
    n_o, w_o, ids_o = oracle.filescan(ot, cnf)
    agg_o = oracle.aggregate(ot, cnf, agg_col)
    plan = ctx.compile(t, cnf)
    for ir in (1, 0):
        ctx.set_tuning("scan_int_range", ir)
        bm = ctx.scan_bitmap(plan)
        assert bm.count == n_o and np.array_equal(bm.download(), w_o), (ir, cnf)
        assert np.array_equal(ctx.scan_select(plan), ids_o), (ir, cnf)
        got = ctx.scan_aggregate(plan, agg_col)
        assert got["count"] == agg_o["count"], (ir, cnf)
        if agg_o["count"]:  # empty selections: identities are representation details
            assert got == agg_o, (ir, cnf, got, agg_o)
    ctx.set_tuning("scan_int_range", 2)


@pytest.mark.parametrize("op", [LT, LE, GT, GE, EQ, NE, NOP])
def test_every_operator_at_the_edges(m, ctx, op):
    cols = _table()
    t = ctx.stage(cols)
    ot = oracle.Table(cols)
    for lit in LITS:
        for cnf in ([[(op, ("sym", 1), ("int", lit))]],            # column OP literal
                    [[(op, ("int", lit), ("sym", 3))]]):            # literal OP column (mirrored)
            want = oracle.filescan_count(ot, cnf)
            on, off = _count_both(m, ctx, t, cnf)
            assert on == off == want, (op, lit, cnf, on, off, want)
            if lit in (IMIN, 0, IMAX):
                _all_outputs(m, ctx, t, ot, cnf)


def test_conjunctions_and_disjunctions(m, ctx):
    cols = _table(300_007, 5)
    rng = np.random.Generator(np.random.PCG64(8))
    t = ctx.stage(cols)
    ot = oracle.Table(cols)
    ops = [LT, LE, GT, GE, EQ, NE]
    for _ in range(40):
        cnf = []
        for _c in range(int(rng.integers(1, 4))):
            conj = []
            for _t in range(int(rng.integers(1, 3))):
                col = ("sym", int(rng.integers(1, 4)))
                lit = ("int", int(rng.choice(LITS)) if rng.random() < 0.5 else int(rng.integers(-5, 5)))
                op = int(rng.choice(ops))
                conj.append((op, col, lit) if rng.random() < 0.7 else (op, lit, col))
            cnf.append(conj)
        want = oracle.filescan_count(ot, cnf)
        on, off = _count_both(m, ctx, t, cnf)
        assert on == off == want, (cnf, on, off, want)
        _all_outputs(m, ctx, t, ot, cnf)


def test_deleted_rows_and_ragged_sizes(m, ctx):
    for n in [1, 255, 256, 257, 65_536 + 3]:
        cols = _table(n, n)
        rng = np.random.Generator(np.random.PCG64(n))
        bits = rng.random(n) < 0.2
        dele = np.frombuffer(np.pad(np.packbits(bits, bitorder="little"), (0, (-((n + 7) // 8)) % 8)).tobytes(),
                             dtype=np.uint64).copy()
        t = ctx.stage(cols, dele)
        ot = oracle.Table(cols, dele)
        for cnf in ([[(GE, ("sym", 1), ("int", 0))], [(NE, ("sym", 2), ("int", 0))]],
                    [[(LT, ("sym", 3), ("int", IMIN + 1)), (GT, ("sym", 1), ("int", IMAX - 1))]]):
            want = oracle.filescan_count(ot, cnf)
            on, off = _count_both(m, ctx, t, cnf)
            assert on == off == want, (n, cnf, on, off, want)
            _all_outputs(m, ctx, t, ot, cnf)
