"""NaN follows PredEval's evaluation order.

In the reference a float compare with a NaN operand falls through
TupleUtils.CompareTupleWithTuple's float case into the string case and raises
(R/iterator/TupleUtils.java:61-69).  Whether a row raises therefore depends on
whether PredEval evaluates that compare at all: conjuncts are evaluated in
order and stop at the first false one, the OR list of a conjunct stops at the
first true term (R/iterator/PredEval.java:164-175), and TupleScan never hands
deleted rows to PredEval (R/columnar/TupleScan.java:80-87).  The operator is
applied after the compare, so NOP / RANGE terms raise on a NaN as well, and a
NaN literal raises on every row that reaches its term.

The oracle (oracle/oracle.c) restates exactly that order; the GPU path must
raise (MBX_E_TYPE) for the same queries and return identical results for all
others, in every scan form: COUNT, BitSet, aggregate; the fast kernel
(hoisted terms, plan-read terms, string slots, RI BitSet layout) and the
generic kernel; with and without deleted rows; and through the async entry
points, whose NaN surfaces at mbx_sync.
"""
import numpy as np
import pytest

import helpers
import mbx_pkg
import oracle

NAN = float("nan")


def _table(n=4099, seed=5, deleted=True):
    rng = np.random.Generator(np.random.PCG64(seed))
    c0 = rng.integers(0, 10, n, dtype=np.int32)
    f1 = rng.random(n, dtype=np.float32)
    f2 = rng.random(n, dtype=np.float32)
    # a few NaNs in rows with known c0 values, so short-circuits decide
    for r in (7, 1500, 4000):
        f1[r] = np.nan
    for r in (11, 2222):
        f2[r] = np.nan
    c0[7], c0[1500], c0[4000], c0[11], c0[2222] = 9, 2, 9, 0, 5
    names = ["Alabama", "Colorado", "Maine", "South_Dakota", "Texas", "Zz"]
    s3 = helpers.encode_strings([names[i] for i in rng.integers(0, len(names), n)], 16)
    cols = [(oracle.INTEGER, 4, c0), (oracle.REAL, 4, f1), (oracle.REAL, 4, f2), (oracle.STRING, 16, s3)]
    dele = None
    if deleted:
        bits = rng.random(n) < 0.05
        bits[[7, 11]] = True  # two NaN rows are deleted
        bits[[1500, 2222, 4000]] = False
        dele = np.frombuffer(np.pad(np.packbits(bits, bitorder="little"), (0, (-((n + 7) // 8)) % 8)).tobytes(),
                             dtype=np.uint64).copy()
    return cols, dele


def oracle_count(ot, cnf):
    try:
        return oracle.filescan(ot, cnf)
    except RuntimeError:
        return "raise"


def oracle_agg(ot, cnf, col):
    try:
        return oracle.aggregate(ot, cnf, col)
    except RuntimeError:
        return "raise"


LT, GT, GE, LE, EQ, NE, NOP, RANGE = oracle.LT, oracle.GT, oracle.GE, oracle.LE, oracle.EQ, oracle.NE, oracle.NOP, \
    oracle.RANGE

# (name, cnf, raises?) -- the verdict's four cases and the operator / literal
# variants; expected outcomes are the oracle's and are asserted against it
CASES = [
    # every f1 NaN row (7 and 4000: c0 = 9; 1500: c0 = 2) fails an earlier conjunct
    ("earlier_conjunct_false", [[(LT, ("sym", 1), ("int", 9))], [(NE, ("sym", 1), ("int", 2))],
                                [(LT, ("sym", 2), ("real", 0.5))]], False),
    # f1 NaN at row 1500 (c0 = 2) is reached
    ("reached", [[(LT, ("sym", 1), ("int", 5))], [(GE, ("sym", 2), ("real", 0.25))]], True),
    # an earlier disjunct holds on every NaN row (c0 in {9, 2}; 2 < 5, 9 > 8)
    ("earlier_disjunct_true", [[(LT, ("sym", 1), ("int", 5)), (GT, ("sym", 1), ("int", 8)),
                                (LT, ("sym", 2), ("real", 0.5))]], False),
    # f2 NaN rows: 11 (c0 = 0, deleted) and 2222 (c0 = 5, live)
    ("deleted_nan_row_skipped", [[(EQ, ("sym", 1), ("int", 0))], [(GT, ("sym", 3), ("real", 0.5))]], False),
    ("live_nan_row_reached", [[(EQ, ("sym", 1), ("int", 5))], [(GT, ("sym", 3), ("real", 0.5))]], True),
    # NOP / RANGE compare before they map to false
    ("nop_reached", [[(NOP, ("sym", 2), ("real", 0.5))]], True),
    ("range_short_circuited", [[(GE, ("sym", 1), ("int", 0)), (RANGE, ("sym", 2), ("real", 0.5))]], False),
    # NaN literal: raises only where reached
    ("nan_literal_unreached", [[(GT, ("sym", 1), ("int", 100))], [(LT, ("sym", 2), ("real", NAN))]], False),
    ("nan_literal_reached", [[(LT, ("sym", 1), ("int", 3))], [(LT, ("real", NAN), ("sym", 2))]], True),
    # literal vs literal: operand 2 is compared with itself (PredEval's shared `value` tuple)
    ("lit_lit_nan_reached", [[(EQ, ("sym", 1), ("int", 4))], [(EQ, ("real", 1.0), ("real", NAN))]], True),
    ("lit_lit_nan_unreached", [[(GT, ("sym", 1), ("int", 100))], [(EQ, ("real", 1.0), ("real", NAN))]], False),
    ("lit_lit_nan_operand1_only", [[(EQ, ("real", NAN), ("real", 1.0))], [(LT, ("sym", 1), ("int", 5))]], False),
    # a conjunct folded to true on the host keeps its float terms before the
    # folding term for their reach ...
    ("folded_conjunct_keeps_prefix", [[(LT, ("sym", 2), ("real", 0.5)), (EQ, ("int", 1), ("int", 1))]], True),
    # ... and drops the ones after it
    ("folded_conjunct_drops_suffix", [[(EQ, ("int", 1), ("int", 1)), (LT, ("sym", 2), ("real", 0.5))]], False),
    # strings between the int and the float terms (fast kernel string slot)
    ("string_disjunct_first", [[(GE, ("sym", 4), ("str", "A")), (LT, ("sym", 2), ("real", 0.5))]], False),
    ("string_conjunct_then_float", [[(GE, ("sym", 4), ("str", "A"))], [(LT, ("sym", 2), ("real", 0.5))]], True),
]


@pytest.mark.parametrize("name,cnf,raises", CASES, ids=[c[0] for c in CASES])
def test_oracle_restates_predeval_order(name, cnf, raises):
    """The oracle is the checker: pin its short-circuit / deleted-skip
    behaviour on the cases the GPU tests use (CPU only)."""
    cols, dele = _table()
    got = oracle_count(oracle.Table(cols, dele), cnf)
    assert (got == "raise") == raises, name


def test_verdict_example():
    """(c0 < 5) AND (f < 0.5) with a NaN only in a row where c0 = 9 counts
    that row's conjunct as never reached, deleted or not."""
    c0 = np.array([1, 9, 3], dtype=np.int32)
    f = np.array([0.1, np.nan, 0.9], dtype=np.float32)
    cols = [(oracle.INTEGER, 4, c0), (oracle.REAL, 4, f)]
    cnf = [[(LT, ("sym", 1), ("int", 5))], [(LT, ("sym", 2), ("real", 0.5))]]
    assert oracle.filescan_count(oracle.Table(cols), cnf) == 1
    assert oracle.filescan_count(oracle.Table(cols, np.array([2], dtype=np.uint64)), cnf) == 1


# ---------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


def _gpu_outcomes(m, ctx, t, cnf, agg_col):
    """(count, words) / 'raise' through scan_count, scan_bitmap, the
    aggregate of agg_col and scan_select (positions); all must agree."""
    try:
        plan = ctx.compile(t, cnf)
    except m.MbxError as e:
        assert e.code == m.mbx.E_TYPE
        return "raise", "raise", "raise", "raise"
    out = []
    try:
        out.append(ctx.scan_count(plan))
    except m.MbxError as e:
        assert e.code == m.mbx.E_TYPE
        out.append("raise")
    try:
        bm = ctx.scan_bitmap(plan)
        out.append((bm.count, bm.download()))
    except m.MbxError as e:
        assert e.code == m.mbx.E_TYPE
        out.append("raise")
    try:
        out.append(ctx.scan_aggregate(plan, agg_col))
    except m.MbxError as e:
        assert e.code == m.mbx.E_TYPE
        out.append("raise")
    try:
        out.append(ctx.scan_select(plan))
    except m.MbxError as e:
        assert e.code == m.mbx.E_TYPE
        out.append("raise")
    return out


def _check(m, ctx, ot, t, cnf, agg_col=1):
    want = oracle_count(ot, cnf)
    want_agg = oracle_agg(ot, cnf, agg_col)
    got_count, got_bm, got_agg, got_ids = _gpu_outcomes(m, ctx, t, cnf, agg_col)
    if want == "raise":
        assert isinstance(got_ids, str) and got_ids == "raise", cnf
        assert got_count == got_bm == got_agg == "raise", cnf
        assert want_agg == "raise"
        return True
    n_o, w_o, ids_o = want
    assert got_count == n_o, cnf
    assert not isinstance(got_ids, str) and np.array_equal(got_ids, ids_o), cnf
    assert got_bm != "raise" and got_bm[0] == n_o and np.array_equal(got_bm[1], w_o), cnf
    assert got_agg != "raise" and got_agg["count"] == want_agg["count"], cnf
    if want_agg["count"]:
        assert got_agg["min"] == want_agg["min"] and got_agg["max"] == want_agg["max"]
        if np.isnan(want_agg["sum"]):  # a selected row's aggregated value is NaN (its compare was not reached)
            assert np.isnan(got_agg["sum"])
        else:
            assert abs(got_agg["sum"] - want_agg["sum"]) <= 1e-6 * max(1.0, abs(want_agg["sum"]))
    return False


@pytest.mark.gpu
@pytest.mark.parametrize("generic", [False, True])
@pytest.mark.parametrize("deleted", [False, True])
@pytest.mark.parametrize("name,cnf,raises", CASES, ids=[c[0] for c in CASES])
def test_gpu_nan_follows_predeval_order(m, ctx, tune, generic, deleted, name, cnf, raises):
    if generic:
        tune("force_generic", 1)
    cols, dele = _table(deleted=deleted)
    ot, t = oracle.Table(cols, dele), ctx.stage(cols, dele)
    _check(m, ctx, ot, t, cnf)


@pytest.mark.gpu
@pytest.mark.parametrize("generic", [False, True])
def test_gpu_nan_fuzz(m, ctx, tune, generic):
    """Random CNFs (1-3 conjuncts of 1-4 terms: int, float, string, NOP /
    RANGE, NaN literal, literal-vs-literal, literal on the left, float
    column-vs-column) over a table with a few NaN rows and deleted rows: the
    GPU raises exactly when the oracle does, and otherwise returns identical
    counts, BitSets and aggregates.  > 4 terms use the plan-read term loop."""
    if generic:
        tune("force_generic", 1)
    cols, dele = _table(n=5003, seed=17)
    ot, t = oracle.Table(cols, dele), ctx.stage(cols, dele)
    rng = np.random.Generator(np.random.PCG64(99))
    ops = [EQ, LT, GT, NE, LE, GE, oracle.NOT, NOP, RANGE]

    def term():
        k = rng.integers(0, 10)
        op = int(ops[rng.integers(0, len(ops))]) if rng.random() < 0.3 else int(rng.choice([LT, GT, GE, LE, EQ, NE]))
        if k < 3:
            a, b = ("sym", 1), ("int", int(rng.integers(-1, 11)))
        elif k < 7:
            fcol = int(rng.integers(2, 4))
            lit = NAN if rng.random() < 0.05 else float(np.float32(rng.random()))
            a, b = ("sym", fcol), ("real", lit)
            if k == 6 and rng.random() < 0.3:
                b = ("sym", 5 - fcol)  # float column vs column (generic kernel)
        elif k < 9:
            a, b = ("sym", 4), ("str", str(rng.choice(["", "Colorado", "M", "South_Dakota", "Zz"])))
        else:
            if rng.random() < 0.5:
                a, b = ("int", int(rng.integers(0, 3))), ("int", int(rng.integers(0, 3)))
            else:
                a, b = ("real", 1.0), ("real", NAN if rng.random() < 0.5 else 2.0)
        if a[0] == "sym" and b[0] != "sym" and rng.random() < 0.3:
            a, b = b, a  # literal on the left
        return (op, a, b)

    raised = passed = 0
    for _ in range(150):
        cnf = [[term() for _ in range(int(rng.integers(1, 5)))] for _ in range(int(rng.integers(1, 4)))]
        if _check(m, ctx, ot, t, cnf):
            raised += 1
        else:
            passed += 1
    assert raised > 10 and passed > 10, (raised, passed)


@pytest.mark.gpu
def test_gpu_nan_async_surfaces_at_sync(m, ctx):
    """*_async scans cannot return an error for their data: a NaN they reach
    sets a sticky device word that mbx_sync reports (once) as MBX_E_TYPE."""
    import torch

    cols, dele = _table()
    t = ctx.stage(cols, dele)
    ok = ctx.compile(t, CASES[0][1])
    bad = ctx.compile(t, CASES[1][1])
    out = torch.zeros(8, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # torch's stream is not the library stream
    ctx.sync()
    ctx.scan_count_async(ok, out.data_ptr())
    ctx.sync()  # no NaN reached
    ctx.scan_count_async(bad, out.data_ptr())
    ctx.scan_count_async(ok, out.data_ptr() + 8)  # a later clean scan does not clear it
    with pytest.raises(m.MbxError) as e:
        ctx.sync()
    assert e.value.code == m.mbx.E_TYPE
    ctx.sync()  # reported once
    agg = torch.zeros(8, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.scan_aggregate_async(bad, 1, agg.data_ptr())
    with pytest.raises(m.MbxError):
        ctx.sync()
    bm = ctx.bitmap_alloc(t.nrows)
    ctx.scan_bitmap_async(bad, bm)
    with pytest.raises(m.MbxError):
        ctx.sync()
    ctx.sync()


@pytest.mark.gpu
def test_gpu_nan_every_shard_context_synced_then_clean(m):
    """ADVICE r2 (GpuShardedScan.syncAll): two shard contexts whose async
    scans both reach a NaN each report it once at their own mbx_sync -- the
    caller syncs every context and keeps the first error -- and a clean query
    on either afterwards raises nothing (no sticky word left behind); a
    NaN-free async BitSet scan (no finalize) leaves the word alone too."""
    import torch

    cols, dele = _table()
    ctxs = [m.Context(0), m.Context(0)]
    try:
        tabs = [c.stage(cols, dele) for c in ctxs]
        bad = [c.compile(t, CASES[1][1]) for c, t in zip(ctxs, tabs)]
        ok = [c.compile(t, CASES[0][1]) for c, t in zip(ctxs, tabs)]
        out = torch.zeros(8, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        for i, c in enumerate(ctxs):
            c.scan_count_async(bad[i], out.data_ptr() + 8 * i)
        errors = []
        for c in ctxs:  # every context synced, the first error kept
            try:
                c.sync()
            except m.MbxError as e:
                errors.append(e.code)
        assert errors == [m.mbx.E_TYPE, m.mbx.E_TYPE]
        want = ctxs[0].scan_count(ok[0])
        for i, c in enumerate(ctxs):
            c.scan_count_async(ok[i], out.data_ptr() + 8 * i)
            bm = c.bitmap_alloc(tabs[i].nrows)
            c.scan_bitmap_async(ok[i], bm)
            c.sync()  # clean
            assert int(out[i].item()) == want
            assert c.select(bm).size == want
    finally:
        for c in ctxs:
            c.close()
