"""Random CNFs through every predicate-scan entry point vs the oracle.

Random tables (1-6 columns of int32 / float32 / char(8|16|25), ragged sizes,
deleted rows or none) and random CNFs in the reference's encoding
(R/iterator/CondExpr.java:12-57: a null-terminated array of conjuncts, each an
OR-list; 0-4 conjuncts of 1-3 terms): every AttrOperator code including NOT,
NOP and RANGE (R/global/AttrOperator.java), the literal on either side,
column-vs-column and literal-vs-literal terms of one type (PredEval's operand-2
aliasing, R/iterator/PredEval.java:170), float literals at +-0 / +-inf /
subnormals (no NaN: tests/test_nan_order.py owns that), string literals that
share prefixes.  Each CNF goes through COUNT (fast and generic kernels), the
BitSet scan, the one-launch positions scan, late materialisation of every
column through a cursor and the aggregate scan of a numeric column -- each
bit-exact vs oracle/oracle.c (PredEval.Eval, TupleUtils.CompareTupleWithTuple,
TupleScan's deleted skip, Projection), SUM within 1e-9 relative."""
import numpy as np
import pytest

import helpers
import mbx_pkg
import oracle

pytestmark = pytest.mark.gpu

OPS = [oracle.EQ, oracle.LT, oracle.GT, oracle.NE, oracle.LE, oracle.GE, oracle.NOT, oracle.NOP, oracle.RANGE]
F32 = np.float32
SUB = float(np.nextafter(F32(0), F32(1)))
FLOATS = [float("-inf"), -1e30, -2.5, -SUB, -0.0, 0.0, SUB, 0.25, 0.5, 1.0, 3e38, float("inf")]
NAMES = ["", "A", "Al", "Alabama", "Alaska", "M", "Ma", "Maine", "Mzzzzzz", "South_Dakota", "Texas", "Zz",
         "Ärger", "日本", "x\u0000y", "\U0001F600"]


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


def random_table(rng, n):
    cols = []
    for _ in range(int(rng.integers(1, 7))):
        kind = int(rng.integers(0, 3))
        if kind == 0:
            hi = int(rng.choice([8, 100, 1 << 20]))
            cols.append((oracle.INTEGER, 4, rng.integers(-hi, hi, n, dtype=np.int32)))
        elif kind == 1:
            v = rng.choice(np.array(FLOATS, dtype=F32), n)
            v[::2] = ((rng.random(n, dtype=F32) - F32(0.5)) * F32(4))[::2]
            cols.append((oracle.REAL, 4, v))
        else:
            size = int(rng.choice([8, 16, 25]))
            pool = [s for s in NAMES if len(oracle.java_mutf8(s)) <= size]
            cols.append((oracle.STRING, size, helpers.encode_strings([pool[i] for i in
                                                                      rng.integers(0, len(pool), n)], size)))
    dele = None
    if n and rng.random() < 0.5:
        bits = rng.random(n) < 0.1
        raw = np.packbits(bits, bitorder="little")
        dele = np.frombuffer(np.pad(raw, (0, (-len(raw)) % 8)).tobytes(), dtype=np.uint64).copy()
    return cols, dele


def literal(rng, typ, col=None):
    if typ == oracle.INTEGER:
        if col is not None and len(col) and rng.random() < 0.6:
            return ("int", int(col[int(rng.integers(0, len(col)))]))
        return ("int", int(rng.integers(-(1 << 20), 1 << 20)))
    if typ == oracle.REAL:
        if col is not None and len(col) and rng.random() < 0.5:
            return ("real", float(col[int(rng.integers(0, len(col)))]))
        return ("real", float(rng.choice(FLOATS)))
    return ("str", str(rng.choice(NAMES)))


def random_cnf(rng, cols):
    k = int(rng.integers(0, 5))
    if k == 0:
        return None
    cnf = []
    for _ in range(k):
        conj = []
        for _ in range(int(rng.integers(1, 4))):
            op = int(rng.choice(OPS))
            j = int(rng.integers(0, len(cols)))
            typ, size, data = cols[j]
            if typ == oracle.STRING and size > 16:
                lit = ("str", str(rng.choice([s for s in NAMES if len(oracle.java_mutf8(s)) <= size])))
            else:
                lit = literal(rng, typ, data if typ != oracle.STRING else None)
            r = rng.random()
            if r < 0.65:
                term = (op, ("sym", j + 1), lit)
            elif r < 0.85:
                term = (op, lit, ("sym", j + 1))
            elif r < 0.95:
                same = [i for i, c in enumerate(cols) if c[0] == typ]
                term = (op, ("sym", j + 1), ("sym", int(rng.choice(same)) + 1))
            else:
                term = (op, lit, literal(rng, typ))
            conj.append(term)
        cnf.append(conj)
    return cnf


def check_all(m, ctx, tune, t, ot, cols, cnf, rng):
    n_o, w_o, ids_o = oracle.filescan(ot, cnf)
    for generic in (0, 1):
        tune("force_generic", generic)
        plan = ctx.compile(t, cnf)
        assert ctx.scan_count(plan) == n_o, (generic, cnf)
        bm = ctx.scan_bitmap(plan)
        assert bm.count == n_o and np.array_equal(bm.download(), w_o), (generic, cnf)
        if not generic:
            assert np.array_equal(ctx.scan_select(plan), ids_o), cnf
            proj = list(range(len(cols)))
            ids, outs = ctx.materialize(t, bm, proj)
            assert np.array_equal(ids, ids_o), cnf
            for j, (got, want) in zip(proj, zip(outs, oracle.gather(ot, ids_o, proj))):
                assert np.array_equal(np.asarray(got).view(np.uint8), np.asarray(want).view(np.uint8)), (j, cnf)
            num = [i for i, c in enumerate(cols) if c[0] != oracle.STRING]
            if num:
                a = int(rng.choice(num))
                got, want = ctx.scan_aggregate(plan, a), oracle.aggregate(ot, cnf, a)
                assert got["count"] == want["count"], (got, want, cnf)
                if want["count"]:
                    assert got["min"] == want["min"] and got["max"] == want["max"], (got, want, cnf)
                    ws, gs = float(want["sum"]), float(got["sum"])
                    if np.isfinite(ws):
                        assert abs(gs - ws) <= 1e-9 * max(1.0, abs(ws)), (got, want, cnf)
                    else:
                        assert (np.isnan(ws) and np.isnan(gs)) or ws == gs, (got, want, cnf)
        plan.close()
    tune("force_generic", 0)


@pytest.mark.parametrize("n", [1, 77, 4099, 100_003, 1_000_003])
@pytest.mark.parametrize("seed", list(range(1, 9)))
def test_random_cnfs_every_entry_point(m, ctx, tune, n, seed):
    rng = np.random.Generator(np.random.PCG64(1000 * seed + n % 997))
    cols, dele = random_table(rng, n)
    t = ctx.stage(cols, dele)
    ot = oracle.Table(cols, dele)
    for _ in range(12 if n < 1_000_000 else 4):
        check_all(m, ctx, tune, t, ot, cols, random_cnf(rng, cols), rng)
    t.close()
