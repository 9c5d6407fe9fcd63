"""Column groups (mbx_table_group): a row-interleaved copy of 2..4 four-byte
columns that the narrow gathers of late materialisation read instead of the
columns, so one row's projected values share a line.  A layout choice only:
every result must be identical with and without the group -- the one-launch
ColumnarIndexScan (k_cnf_select: mbx_cnf_cursor_open, mbx_cnf_materialize_async),
the cursor of a predicate scan (k_select_ids<4>: mbx_cursor_open) and the
golden indexes_query rows; wide projections (char(n), > 4 columns) keep
reading the columns.  Checked against numpy and the oracle."""
import numpy as np
import pytest
import torch

import helpers
import mbx_pkg
import oracle

pytestmark = pytest.mark.gpu
GOLD = helpers.load_golden()


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


def table(n, seed=3):
    rng = np.random.Generator(np.random.PCG64(seed))
    return [(oracle.INTEGER, 4, rng.integers(-(1 << 30), 1 << 30, n, dtype=np.int32)),
            (oracle.REAL, 4, rng.random(n, dtype=np.float32)),
            (oracle.INTEGER, 4, rng.integers(0, 10, n, dtype=np.int32)),
            (oracle.INTEGER, 4, rng.integers(0, 10, n, dtype=np.int32)),
            (oracle.STRING, 12, helpers.encode_strings([f"s{i % 97}" for i in range(n)], 12)),
            (oracle.INTEGER, 4, rng.integers(0, 1 << 20, n, dtype=np.int32))]


def value_bitmaps(ctx, cols, t, c):
    reg = helpers.index_registry(ctx, cols, t, c)
    return reg


@pytest.mark.parametrize("n", [1, 63, 64, 4097, 1_000_003])
@pytest.mark.parametrize("group,proj", [([0, 1], [0, 1]), ([0, 1], [1, 0]), ([5, 0, 1], [0, 5]),
                                        ([0, 1, 2, 3], [3, 0, 2]), ([0, 1], [0, 1, 5]), ([0, 1], [4, 0])])
def test_cnf_cursor_equal_with_and_without_group(m, ctx, n, group, proj):
    cols = table(n)
    plain = ctx.stage(cols)
    grouped = ctx.stage(cols)
    ctx.group(grouped, group)
    out = []
    for t in (plain, grouped):
        r2 = helpers.index_registry(ctx, cols, t, 2)
        r3 = helpers.index_registry(ctx, cols, t, 3)
        conj = [[r2[v] for v in (3, 4) if v in r2], [r3[v] for v in (7,) if v in r3]]
        if not all(conj):
            pytest.skip("a value is absent at this size")
        cur = ctx.cnf_cursor(t, conj, proj)
        ids, vals = cur.next(n + 1)
        out.append((ids.copy(), [v.copy() for v in vals]))
    assert np.array_equal(out[0][0], out[1][0])
    for a, b in zip(out[0][1], out[1][1]):
        assert np.array_equal(a, b)
    sel = np.isin(cols[2][2], (3, 4)) & (cols[3][2] == 7)
    assert np.array_equal(out[1][0], np.nonzero(sel)[0])
    for j, c in enumerate(proj):
        want = cols[c][2][sel]
        got = out[1][1][j]
        assert np.array_equal(np.asarray(got).reshape(want.shape).view(np.uint8), want.view(np.uint8))


def test_cnf_materialize_device_rows_use_the_group(m, ctx):
    """the C4 query shape: AND of two value BitSets -> c0, c1 into device
    buffers (mbx_cnf_materialize_async), positions on and off"""
    n = 3_000_017
    cols = table(n, seed=9)
    t = ctx.stage(cols)
    ctx.group(t, [0, 5])
    r2 = helpers.index_registry(ctx, cols, t, 2)
    r3 = helpers.index_registry(ctx, cols, t, 3)
    sel = (cols[2][2] == 3) & (cols[3][2] == 7)
    k = int(sel.sum())
    for with_ids in (False, True):
        ids = torch.full((k + 8,), -1, dtype=torch.int64, device="cuda")
        o0 = torch.zeros(k + 8, dtype=torch.int32, device="cuda")
        o5 = torch.zeros(k + 8, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        ctx.cnf_materialize_async(t, [[r2[3]], [r3[7]]], [5, 0], ids.data_ptr() if with_ids else None,
                                  [o5.data_ptr(), o0.data_ptr()], cnt.data_ptr())
        ctx.sync()
        assert int(cnt.item()) == k
        assert np.array_equal(o5[:k].cpu().numpy(), cols[5][2][sel])
        assert np.array_equal(o0[:k].cpu().numpy(), cols[0][2][sel])
        if with_ids:
            assert np.array_equal(ids[:k].cpu().numpy(), np.nonzero(sel)[0])


def test_predicate_cursor_uses_the_group(m, ctx):
    """ColumnarFileScan's cursor (k_select_ids<4> gathers grouped columns)"""
    n = 2_000_003
    cols = table(n, seed=4)
    t = ctx.stage(cols)
    ctx.group(t, [0, 1, 5])
    cnf = [[(oracle.LT, ("sym", 6), ("int", 50_000))]]
    bm = ctx.scan_bitmap(ctx.compile(t, cnf))
    ids, (a, b, c) = ctx.materialize(t, bm, [5, 1, 0])
    sel = cols[5][2] < 50_000
    assert np.array_equal(ids, np.nonzero(sel)[0])
    assert np.array_equal(a, cols[5][2][sel]) and np.array_equal(b, cols[1][2][sel])
    assert np.array_equal(c, cols[0][2][sel])


def test_golden_rows_with_a_group(m, ctx):
    """minidata's int columns C, D grouped: every golden indexes_query row"""
    rows = helpers.load_minidata()
    cols = helpers.minidata_columns(rows)
    t = ctx.stage(cols)
    ctx.group(t, [2, 3])
    regs = {c: helpers.index_registry(ctx, cols, t, c) for c in range(4)}
    for g in GOLD["indexes_query"]:
        conj = helpers.index_conjuncts(regs, helpers.golden_cnf(g["cnf"]), helpers.MINI_TYPES)
        ids, (c, d) = ctx.cnf_cursor(t, conj, [2, 3]).next(len(rows) + 1)
        assert [[int(x), int(y)] for x, y in zip(c, d)] == [r[2:] for r in g["rows"]], g["line"]


def test_group_errors(m, ctx):
    cols = table(100)
    t = ctx.stage(cols)
    for bad in ([0], [0, 1, 2, 3, 5], [0, 0], [0, 4], [0, 9]):
        with pytest.raises(m.MbxError):
            ctx.group(t, bad)
    ctx.group(t, [0, 1])
    with pytest.raises(m.MbxError):
        ctx.group(t, [1, 2])     # column 1 is already grouped


def test_group_of_wrapped_columns_is_a_snapshot_until_rebuilt(m, ctx):
    """a table over caller memory (mbx_table_wrap): the group copies the
    columns when it is built; after the caller rewrites a column, gathers
    of the grouped columns return the snapshot until the groups are dropped
    (cols = []) and built again"""
    n = 200_003
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    c = [torch.randint(0, 10, (n,), dtype=torch.int32, device="cuda", generator=g) for _ in range(4)]
    t = ctx.wrap([(m.mbx.INTEGER, 4)] * 4, [x.data_ptr() for x in c], n)
    b2 = ctx.index_build(t, 2, [("int", 3)])[0]
    b3 = ctx.index_build(t, 3, [("int", 7)])[0]
    sel = (c[2] == 3) & (c[3] == 7)
    k = int(sel.sum().item())

    def rows():
        o0 = torch.zeros(k + 1, dtype=torch.int32, device="cuda")
        o1 = torch.zeros(k + 1, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        ctx.cnf_materialize_async(t, [[b2], [b3]], [0, 1], None, [o0.data_ptr(), o1.data_ptr()], cnt.data_ptr())
        ctx.sync()
        assert int(cnt.item()) == k
        return o0[:k].clone(), o1[:k].clone()

    ctx.group(t, [0, 1])
    old0 = c[0][sel].clone()
    assert bool((rows()[0] == old0).all())
    c[0].add_(100)                      # the caller rewrites column 0 in place
    torch.cuda.synchronize()
    assert bool((rows()[0] == old0).all())          # the group's snapshot
    ctx.group(t, [])                    # drop ...
    assert bool((rows()[0] == c[0][sel]).all())     # ... the columns again
    ctx.group(t, [0, 1])                # ... and rebuild
    r0, r1 = rows()
    assert bool((r0 == c[0][sel]).all()) and bool((r1 == c[1][sel]).all())


@pytest.mark.parametrize("lookback,store,blocks", [(1, 0, 0), (2, 0, 0), (0, 1, 0), (0, 2, 0), (0, 3, 0),
                                                   (1, 3, 2048), (2, 2, 512), (1, 0, 8192)])
@pytest.mark.parametrize("group", [False, True])
def test_cnf_select_knobs_keep_results(m, ctx, lookback, store, blocks, group):
    """every A/B form of the one-launch ColumnarIndexScan (look-back chained /
    polled, output stores plain / write-through / nontemporal, grids below
    and above the resident one) returns the same positions and rows"""
    n = 1_500_007
    cols = table(n, seed=21)
    t = ctx.stage(cols)
    if group:
        ctx.group(t, [0, 5])
    r2 = helpers.index_registry(ctx, cols, t, 2)
    r3 = helpers.index_registry(ctx, cols, t, 3)
    sel = (cols[2][2] == 3) & (cols[3][2] == 7)
    k = int(sel.sum())
    try:
        ctx.set_tuning("cnf_lookback", lookback)
        ctx.set_tuning("cnf_store", store)
        ctx.set_tuning("cnf_blocks", blocks)
        for proj in ([5, 0], []):
            ids = torch.full((k + 8,), -1, dtype=torch.int64, device="cuda")
            outs = [torch.zeros(k + 8, dtype=torch.int32, device="cuda") for _ in proj]
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            for _ in range(2):  # twice: the second launch reads the first one's look-back words
                ctx.cnf_materialize_async(t, [[r2[3]], [r3[7]]], proj, ids.data_ptr(), [o.data_ptr() for o in outs],
                                          cnt.data_ptr())
            ctx.sync()
            assert int(cnt.item()) == k
            assert np.array_equal(ids[:k].cpu().numpy(), np.nonzero(sel)[0])
            for j, o in zip(proj, outs):
                assert np.array_equal(o[:k].cpu().numpy(), cols[j][2][sel])
    finally:
        ctx.set_tuning("reset")
