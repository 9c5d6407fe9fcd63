"""Pin the CPU oracle against the reference's own recorded outputs.

Every expected value here comes from R/phase3_output (the reference Java engine
run over minidata.txt), extracted by tests/golden/make_golden.py.
"""
import numpy as np
import pytest

import helpers
import oracle

GOLD = helpers.load_golden()


@pytest.mark.parametrize("g", GOLD["bitsets"], ids=lambda g: f"line{g['line']}")
def test_filescan_matches_transcript_bitsets(minidata, g):
    """ColumnarFileScan + PredEval over the CNF selects exactly the positions
    the reference printed for the same CNF (bmj OuterConstraint/InnerConstraint)."""
    _, t = minidata
    n, words, ids = oracle.filescan(t, helpers.golden_cnf(g["cnf"]))
    assert list(ids) == g["positions"]
    assert n == len(g["positions"])
    assert list(oracle.words_to_positions(words)) == g["positions"]


@pytest.mark.parametrize("g", GOLD["bitsets"], ids=lambda g: f"line{g['line']}")
def test_columnar_index_scan_matches_transcript_bitsets(minidata, g):
    """ColumnarIndexScan.getOutputPositions over bitmap indexes (the code path
    that printed these BitSets)."""
    _, t = minidata
    n, words = oracle.columnar_index_scan(t, helpers.golden_cnf(g["cnf"]))
    assert list(oracle.words_to_positions(words)) == g["positions"]
    assert n == len(g["positions"])


@pytest.mark.parametrize("g", GOLD["full_constraint_counts"], ids=lambda g: f"line{g['line']}")
def test_full_constraint_counts(minidata, g):
    _, t = minidata
    n, _, _ = oracle.filescan(t, helpers.golden_cnf(g["cnf"]))
    assert n == g["count"]


@pytest.mark.parametrize("g", GOLD["indexes_query"], ids=lambda g: f"line{g['line']}")
def test_indexes_query_rows(minidata, g):
    """MultiIndexQuery output rows (A, B, C, D) in position order, and the
    'Total Results Count By Query' line."""
    rows, t = minidata
    n, words = oracle.columnar_index_scan(t, helpers.golden_cnf(g["cnf"]))
    pos = oracle.words_to_positions(words)
    got = [[rows[p][0], rows[p][1], rows[p][2], rows[p][3]] for p in pos]
    assert got == g["rows"]
    assert n == g["count"]
    # late materialisation through the oracle's gather gives the same values
    a, b, c, d = oracle.gather(t, pos, [0, 1, 2, 3])
    assert [bytes(x).rstrip(b"\0").decode() for x in a] == [r[0] for r in g["rows"]]
    assert list(c) == [r[2] for r in g["rows"]]


def test_known_answers(minidata):
    """C=6 -> 57 rows, A=South_Dakota -> 22 rows; C!=6 -> 443
    (transcript 'Total Outer Tuples By Iterator: 443', R/phase3_output:3734)."""
    _, t = minidata
    assert oracle.filescan(t, helpers.parse_cnf_string("{(C,=,6)}"))[0] == 57
    assert oracle.filescan(t, helpers.parse_cnf_string("{(A,=,South_Dakota)}"))[0] == 22
    assert oracle.filescan(t, helpers.parse_cnf_string("{(C,!=,6)}"))[0] == 443
    assert oracle.filescan(t, None)[0] == 500


def test_deleted_rows_are_skipped(minidata):
    _, t0 = minidata
    rows = helpers.load_minidata()
    dele = helpers.random_deleted(len(rows), 0.2)
    t = oracle.Table(helpers.minidata_columns(rows), dele)
    cnf = helpers.parse_cnf_string("{(C,!=,6)}")
    _, w_all, _ = oracle.filescan(t0, cnf)
    n, w, _ = oracle.filescan(t, cnf)
    assert np.array_equal(w, w_all & ~dele)
    n2, w2 = oracle.columnar_index_scan(t, cnf)
    assert np.array_equal(w2, w) and n2 == n


def test_predeval_operator_table(minidata):
    """aopNOT == aopNE; aopNOP / opRANGE are never true (PredEval.java:137-162);
    a literal on the left is compared literal-first."""
    _, t = minidata
    ne = oracle.filescan(t, [[(oracle.NE, ("sym", 3), ("int", 6))]])[0]
    assert oracle.filescan(t, [[(oracle.NOT, ("sym", 3), ("int", 6))]])[0] == ne
    assert oracle.filescan(t, [[(oracle.NOP, ("sym", 3), ("int", 6))]])[0] == 0
    assert oracle.filescan(t, [[(oracle.RANGE, ("sym", 3), ("int", 6))]])[0] == 0
    # 6 < C  <=>  C > 6
    a = oracle.filescan(t, [[(oracle.LT, ("int", 6), ("sym", 3))]])[2]
    b = oracle.filescan(t, [[(oracle.GT, ("sym", 3), ("int", 6))]])[2]
    assert list(a) == list(b)
    # column vs column in one tuple: C <= D
    rows = helpers.load_minidata()
    c = oracle.filescan(t, [[(oracle.LE, ("sym", 3), ("sym", 4))]])[2]
    assert list(c) == [i for i, r in enumerate(rows) if r[2] <= r[3]]
    # two literals: the shared `value` tuple compares operand 2 with itself
    assert oracle.filescan(t, [[(oracle.EQ, ("int", 1), ("int", 2))]])[0] == 500
    assert oracle.filescan(t, [[(oracle.LT, ("int", 1), ("int", 2))]])[0] == 0


def test_index_scan_not_operator_selects_nothing(minidata):
    """ColumnIndexScan.getBitSet has no aopNOT branch: the BitSet stays empty
    (R/index/ColumnIndexScan.java:656-740), unlike PredEval where NOT == NE."""
    _, t = minidata
    assert oracle.column_index_scan(t, 2, oracle.NOT, ("int", 6))[0] == 0
    assert oracle.column_index_scan(t, 2, oracle.NE, ("int", 6))[0] == 443


def test_duplicate_constraint_cache_quirk(minidata):
    """ColumnarIndexScan caches the *mutable* conjunct BitSet for a repeated
    constraint (R/index/ColumnarIndexScan.java:147-172): a repeated term ORs
    in the whole earlier (already AND-ed) conjunct."""
    rows, t = minidata
    cnf = helpers.parse_cnf_string("{(A,=,South_Dakota)|(B,=,South_Dakota)}^{(A,=,South_Dakota)|(C,>=,6)}")
    n, w = oracle.columnar_index_scan(t, cnf)
    # the second A=SD ORs in conjunct 0's set (A|B) -> result is A|B
    ab = [i for i, r in enumerate(rows) if r[0] == "South_Dakota" or r[1] == "South_Dakota"]
    assert list(oracle.words_to_positions(w)) == ab
    # while the plain CNF (FileScan) gives the logical answer
    m = oracle.filescan(t, cnf)[0]
    assert m == len([i for i in ab if rows[i][0] == "South_Dakota" or rows[i][2] >= 6])


def test_java_string_compare_order():
    """String.compareTo over UTF-16 units, incl. non-ASCII and supplementary chars."""
    cases = ["", "a", "ab", "b", "South_Dakota", "South", "é", "€", "￿", "\U0001F600", "a\u0000b"]
    for x in cases:
        for y in cases:
            bx, by = oracle.java_mutf8(x), oracle.java_mutf8(y)
            ux, uy = x.encode("utf-16-be", "surrogatepass"), y.encode("utf-16-be", "surrogatepass")
            want = (ux > uy) - (ux < uy)
            assert oracle.lib().orc_string_compare(bx, len(bx), by, len(by)) == want, (x, y)
            # modified UTF-8 byte order agrees except for U+0000 (C0 80); the
            # device image rewrites C0 80 -> 00 01, after which zero-padded
            # byte order agrees everywhere (the GPU compares bytes)
            dx = bx.replace(b"\xc0\x80", b"\x00\x01").ljust(32, b"\0")
            dy = by.replace(b"\xc0\x80", b"\x00\x01").ljust(32, b"\0")
            assert ((dx > dy) - (dx < dy)) == want, (x, y)
            if "\u0000" not in x + y:
                assert ((bx > by) - (bx < by)) == want, (x, y)


def test_aggregate_small(minidata):
    rows, t = minidata
    a = oracle.aggregate(t, helpers.parse_cnf_string("{(A,=,South_Dakota)}"), 2)
    sel = [r[2] for r in rows if r[0] == "South_Dakota"]
    assert a == dict(count=len(sel), sum=sum(sel), min=min(sel), max=max(sel))
