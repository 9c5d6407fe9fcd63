"""ColumnarFileScan's get_next_tid stream as BitSet + ascending positions +
COUNT in ONE launch (k_scan_select, knob scan_select_fused): the fast scan's
tile body forms the words, select_tail turns them into positions with the
chained look-back (R/iterator/ColumnarFileScan.java:174-188,
R/iterator/PredEval.java:25-183).  Checked bit-exact against the oracle:
C2 at full size, ragged sizes, 1..4 int terms over 1..4 columns in
conjunct / disjunct shapes, deleted rows, a shard's row_offset, segment sizes
on both sides of the one-launch envelope (the fallback must agree), launch
after launch, graph replays and interleaving with k_cnf_select (both use the
context's look-back words), and the segment counts it leaves in the BitSet
(a later materialise / count reads them)."""
import numpy as np
import pytest
import torch

import helpers
import mbx_pkg
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    c.set_tuning("scan_select_fused", 1)
    yield c
    c.close()


@pytest.fixture
def tune(ctx):
    yield ctx.set_tuning
    ctx.set_tuning("reset")
    ctx.set_tuning("scan_select_fused", 1)


def run_async(ctx, plan, n):
    bm = ctx.bitmap_alloc(n)
    ids = torch.full((max(1, n),), -3, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.scan_select_async(plan, bm, ids.data_ptr(), cnt.data_ptr())
    ctx.sync()
    k = int(cnt.item())
    return bm, ids[:k].cpu().numpy(), k


def int_cols(n, ncols=4, hi=1000, seed=7):
    return [(oracle.INTEGER, 4, c) for c in helpers.synthetic_int_table(n, ncols, hi, seed)]


CNFS = [
    [[(oracle.LT, ("sym", 1), ("int", 300))]],
    [[(oracle.LT, ("sym", 1), ("int", 500))], [(oracle.GE, ("sym", 2), ("int", 500))]],
    [[(oracle.EQ, ("sym", 3), ("int", 7)), (oracle.GT, ("sym", 1), ("int", 900))],
     [(oracle.NE, ("sym", 2), ("int", 3))]],
    [[(oracle.LE, ("sym", 1), ("int", 600))], [(oracle.GT, ("sym", 2), ("int", 100))],
     [(oracle.LT, ("sym", 3), ("int", 800))], [(oracle.GE, ("sym", 4), ("int", 50))]],
    [[(oracle.GT, (("int", 500)), ("sym", 1))]],   # literal on the left
]


@pytest.mark.parametrize("n", [1, 63, 64, 255, 256, 257, 1000, 4099, 70001, 1_000_003])
@pytest.mark.parametrize("deleted", [None, 0.07])
def test_fused_matches_oracle(ctx, n, deleted):
    cols = int_cols(n, seed=n)
    dele = None if deleted is None else helpers.random_deleted(n, deleted, seed=n + 3)
    ot = oracle.Table(cols, dele)
    t = ctx.stage(cols, dele, row_offset=128)
    for cnf in CNFS:
        n_o, w_o, ids_o = oracle.filescan(ot, cnf)
        plan = ctx.compile(t, cnf)
        bm, ids, k = run_async(ctx, plan, n)
        assert k == n_o, cnf
        assert np.array_equal(ids, ids_o + 128), cnf
        assert np.array_equal(bm.download(), w_o), cnf
        # the segment counts the launch left: a materialise and the count read them
        assert bm.count == -1  # unknown after an async call until something needs it
        assert np.array_equal(ctx.select(bm, row_offset=128), ids_o + 128)
        assert bm.count == n_o


def test_fused_c2_full_size_launch_after_launch(ctx):
    """C2: 10M rows, c0 < 104858 (~10 %), three launches, then a graph of
    three replayed twice: positions + BitSet + COUNT exact every time"""
    n = 10_000_000
    cols = [(oracle.INTEGER, 4, c) for c in helpers.synthetic_int_table(n)]
    ot = oracle.Table(cols)
    t = ctx.stage(cols)
    cnf = [[(oracle.LT, ("sym", 1), ("int", 104858))]]
    n_o, w_o, ids_o = oracle.filescan(ot, cnf)
    plan = ctx.compile(t, cnf)
    for _ in range(3):
        bm, ids, k = run_async(ctx, plan, n)
        assert k == n_o and np.array_equal(ids, ids_o) and np.array_equal(bm.download(), w_o)
    bm = ctx.bitmap_alloc(n)
    ids = torch.zeros(n, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.scan_select_async(plan, bm, ids.data_ptr(), cnt.data_ptr())   # sizes scratch before the capture
    ctx.sync()
    ctx.graph_begin()
    for _ in range(3):
        ctx.scan_select_async(plan, bm, ids.data_ptr(), cnt.data_ptr())
    g = ctx.graph_end()
    for _ in range(2):
        ids.zero_()
        torch.cuda.synchronize()
        g.launch()
        ctx.sync()
        assert int(cnt.item()) == n_o
        assert np.array_equal(ids[:n_o].cpu().numpy(), ids_o)
    g.close()


LOOKBACK = {"poll_spread": (0, 16), "poll": (0, 1), "chained": (128, 1)}


@pytest.mark.parametrize("lookback", list(LOOKBACK))
@pytest.mark.parametrize("tpb", [1, 4, 37, 200, 512, 513, 1000])
def test_fused_segment_sizes_and_fallback(ctx, tune, tpb, lookback):
    """segments of 1..1000 tiles: up to 128 tiles per wave run fused, larger
    ones fall back to the two launches -- both exact, with every look-back
    form (every register count NR: 1, 2, 4, 8 groups of 64 words)"""
    tune("tiles_per_block", tpb)
    tune("select_dbg", LOOKBACK[lookback][0])
    tune("select_flag_stride", LOOKBACK[lookback][1])
    n = 3_000_017
    cols = int_cols(n, hi=1000, seed=5)
    t = ctx.stage(cols)
    plan = ctx.compile(t, [[(oracle.LT, ("sym", 1), ("int", 300))]])
    mask = np.asarray(cols[0][2]) < 300
    bm, ids, k = run_async(ctx, plan, n)
    assert k == int(mask.sum()) and np.array_equal(ids, np.nonzero(mask)[0])
    assert np.array_equal(ctx.select(bm), ids)


@pytest.mark.parametrize("lookback", list(LOOKBACK))
@pytest.mark.parametrize("waves", [4, 16])
@pytest.mark.parametrize("n", [255, 70001, 3_000_017, 10_000_000])
def test_fused_waves_per_block(ctx, tune, waves, n, lookback):
    """one BitSet segment per 4-wave block, or four per 16-wave block (a
    quarter of the blocks in the look-back), with each look-back form (the
    chained walk; every predecessor polled, flags packed or one per 128-byte
    line): the same positions, words and segment counts"""
    tune("scan_select_waves", waves)
    tune("select_dbg", LOOKBACK[lookback][0])
    tune("select_flag_stride", LOOKBACK[lookback][1])
    cols = int_cols(n, ncols=2, hi=1000, seed=n + waves)
    dele = helpers.random_deleted(n, 0.03, seed=n) if n == 70001 else None
    ot = oracle.Table(cols, dele)
    t = ctx.stage(cols, dele, row_offset=64)
    cnf = [[(oracle.LT, ("sym", 1), ("int", 250))], [(oracle.GE, ("sym", 2), ("int", 100))]]
    n_o, w_o, ids_o = oracle.filescan(ot, cnf)
    plan = ctx.compile(t, cnf)
    for _ in range(2):
        bm, ids, k = run_async(ctx, plan, n)
        assert k == n_o and np.array_equal(ids, ids_o + 64)
        assert np.array_equal(bm.download(), w_o)
        assert np.array_equal(ctx.select(bm, row_offset=64), ids_o + 64)
        assert bm.count == n_o


def test_fused_interleaved_with_cnf_select(ctx):
    """k_scan_select and k_cnf_select share the context's look-back words:
    alternating launches of different grid sizes stay exact"""
    rng = np.random.Generator(np.random.PCG64(3))
    runs = []
    for n in (100, 3_000_017, 64, 1_000_003):
        cols = int_cols(n, hi=10, seed=n)
        t = ctx.stage(cols)
        bms = ctx.index_build(t, 2, [("int", v) for v in range(10)])
        runs.append((n, cols, t, bms))
    for _ in range(2):
        for n, cols, t, bms in runs:
            c0 = np.asarray(cols[0][2])
            plan = ctx.compile(t, [[(oracle.LT, ("sym", 1), ("int", 4))]])
            bm, ids, k = run_async(ctx, plan, n)
            assert np.array_equal(ids, np.nonzero(c0 < 4)[0]), n
            cur = ctx.cnf_cursor(t, [[bms[3], bms[5]]], [0])
            want = np.nonzero(np.isin(np.asarray(cols[2][2]), [3, 5]))[0]
            got, (v0,) = cur.next(max(1, n))
            assert np.array_equal(got, want) and np.array_equal(v0, c0[want]), n
            # positions only: the polled look-back whatever the knobs (cnf_lookback auto)
            got2, _ = ctx.cnf_cursor(t, [[bms[3], bms[5]]], []).next(max(1, n))
            assert np.array_equal(got2, want), n
    del rng


def test_fused_100m_rows_large_segments(ctx):
    """100 M rows: 382-tile segments, four per 16-wave block (256 blocks,
    96 tiles per wave, the segment's words staged through 48 KB of LDS):
    positions, count and BitSet equal to the oracle's"""
    n = 100_000_000
    cols = [(oracle.INTEGER, 4, c) for c in helpers.synthetic_int_table(n, 2)]
    ot = oracle.Table(cols)
    t = ctx.stage(cols)
    cnf = [[(oracle.LT, ("sym", 1), ("int", 1 << 19))], [(oracle.GE, ("sym", 2), ("int", 1 << 19))]]
    n_o, w_o, ids_o = oracle.filescan(ot, cnf)
    plan = ctx.compile(t, cnf)
    bm, ids, k = run_async(ctx, plan, n)
    assert k == n_o and np.array_equal(ids, ids_o)
    assert np.array_equal(bm.download(), w_o)


@pytest.mark.parametrize("lookback", list(LOOKBACK))
def test_lookback_epoch_wrap(m, ctx, tune, lookback):
    """Launches across the look-back epoch's wrap (2^31 - 1 -> 1), k_scan_select
    (every look-back form) alternating with k_cnf_select at different grid
    sizes: the words set back to epoch 0 by the last two launches before the
    wrap leave no stale flag that a later launch could take for its own."""
    tune("select_dbg", LOOKBACK[lookback][0])
    tune("select_flag_stride", LOOKBACK[lookback][1])
    runs = []
    for n in (3_000_017, 100_003, 1_000_003):
        cols = int_cols(n, hi=10, seed=n)
        t = ctx.stage(cols)
        bms = ctx.index_build(t, 2, [("int", v) for v in range(10)])
        runs.append((n, cols, t, bms))
    m.mbx._chk(m.lib().mbx_diag_lookback_epoch(ctx.h, 0x7FFFFFFF - 5))
    for _ in range(4):  # 12 launches of each kernel: through the wrap and well past it
        for n, cols, t, bms in runs:
            c0 = np.asarray(cols[0][2])
            plan = ctx.compile(t, [[(oracle.LT, ("sym", 1), ("int", 4))]])
            bm, ids, k = run_async(ctx, plan, n)
            assert np.array_equal(ids, np.nonzero(c0 < 4)[0]), n
            cur = ctx.cnf_cursor(t, [[bms[3], bms[5]]], [0])
            want = np.nonzero(np.isin(np.asarray(cols[2][2]), [3, 5]))[0]
            got, (v0,) = cur.next(max(1, n))
            assert np.array_equal(got, want) and np.array_equal(v0, c0[want]), n
            # positions only: the polled look-back whatever the knobs (cnf_lookback auto)
            got2, _ = ctx.cnf_cursor(t, [[bms[3], bms[5]]], []).next(max(1, n))
            assert np.array_equal(got2, want), n
