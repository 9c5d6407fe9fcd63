"""mbx_cnf_materialize_async: ColumnarIndexScan's CNF of index BitSets
(R/index/ColumnarIndexScan.java:130-181) + positions + projected columns
(:287-308) in one launch with a decoupled look-back.  Checked bit-exact
against numpy's CNF / nonzero / fancy indexing of the same host data and
against the two-call form (mbx_bitmap_cnf_async + mbx_materialize_async):
operand counts on both sides of the batched-load branch (<= 4 / > 4
bitmaps), deleted rows, ragged sizes, densities 0..1, 0-4 int/float
columns (char(n) and wider projections: test_cnf_cursor.py and the limits
test here), positions on or off, a shard's row_offset, a table past the
register-cached range (> 134 M rows: the words are re-formed for the write
pass), many launches in a row (the epoch advances) and graph replays (the
epoch is read from device memory, not baked into the graph)."""
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
    yield c
    c.close()


def words_of(bits):
    n = len(bits)
    w = np.zeros(((n + 63) // 64) * 64, dtype=bool)
    w[:n] = bits
    return np.packbits(w, bitorder="little").view(np.uint64)


def cnf_bits(conj_bits, deleted=None):
    n = len(next(c for c in conj_bits if c)[0])
    r = None
    for conj in conj_bits:
        o = np.zeros(n, dtype=bool)
        for b in conj:
            o = o | b
        r = o if r is None else r & o
    if deleted is not None:
        r = r & ~deleted
    return r


def run(ctx, t, conj, proj, with_ids=True, deleted=None):
    """one fused launch into fresh device buffers -> (ids | None, [columns], count)"""
    n = t.nrows
    cap = max(1, n)
    ids = torch.full((cap,), -7, dtype=torch.int64, device="cuda") if with_ids else None
    outs = [torch.full((cap,), -7, dtype=torch.int32, device="cuda") for _ in proj]
    cnt = torch.full((1,), -7, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.cnf_materialize_async(t, conj, proj, None if ids is None else ids.data_ptr(),
                              [o.data_ptr() for o in outs], cnt.data_ptr(), deleted=deleted)
    ctx.sync()
    k = int(cnt.item())
    return (None if ids is None else ids[:k].cpu().numpy()), [o[:k].cpu().numpy() for o in outs], k


def table(ctx, n, seed, row_offset=0):
    rng = np.random.Generator(np.random.PCG64(seed))
    ints = helpers.synthetic_int_table(n, 2, 1 << 30, seed)
    f0 = rng.random(n, dtype=np.float32)
    f1 = rng.standard_normal(n).astype(np.float32)
    cols = [(oracle.INTEGER, 4, ints[0]), (oracle.REAL, 4, f0), (oracle.INTEGER, 4, ints[1]), (oracle.REAL, 4, f1)]
    return cols, ctx.stage(cols, row_offset=row_offset)


SHAPES = {
    "one": [[0]],
    "and2": [[0], [1]],
    "or2": [[0, 1]],
    "and_or": [[0, 1], [2]],
    "and4": [[0], [1], [2], [3]],
    "wide5": [[0, 1, 2], [3, 4]],        # > 4 operands: the per-word CNF loop
    "empty_conj": [[0], []],            # an empty conjunct is all-zero
}


@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097, 70_001, 700_013])
@pytest.mark.parametrize("shape", list(SHAPES))
def test_cnf_materialize_matches_numpy(ctx, n, shape):
    rng = np.random.Generator(np.random.PCG64(n * 31 + len(shape)))
    dens = [0.5, 0.7, 0.3, 0.9, 0.1]
    bits = [rng.random(n) < d for d in dens]
    bms = [ctx.bitmap_upload(n, words_of(b)) for b in bits]
    cols, t = table(ctx, n, 11, row_offset=6400)
    conj = [[bms[k] for k in c] for c in SHAPES[shape]]
    sel = cnf_bits([[bits[k] for k in c] for c in SHAPES[shape]])
    pos = np.nonzero(sel)[0]
    for proj in ([], [0], [1, 3], [3, 0, 2, 1]):
        ids, outs, k = run(ctx, t, conj, proj)
        assert k == len(pos), (proj, k, len(pos))
        assert np.array_equal(ids, pos + 6400), proj
        for j, o in zip(proj, outs):
            assert np.array_equal(o.view(np.uint32), np.asarray(cols[j][2])[pos].view(np.uint32)), (proj, j)


@pytest.mark.parametrize("density", [0.0, 0.001, 0.01, 0.1, 0.6, 1.0])
def test_cnf_materialize_densities_and_deleted(ctx, density):
    n = 1_000_003
    rng = np.random.Generator(np.random.PCG64(int(density * 1000) + 3))
    a = rng.random(n) < min(1.0, density * 2)
    b = rng.random(n) < 0.5 if density < 1.0 else np.ones(n, dtype=bool)
    dl = rng.random(n) < 0.05
    A, B, D = (ctx.bitmap_upload(n, words_of(x)) for x in (a, b, dl))
    cols, t = table(ctx, n, 5)
    for deleted in (None, D):
        sel = cnf_bits([[a], [b]], dl if deleted is not None else None)
        pos = np.nonzero(sel)[0]
        for with_ids in (True, False):
            ids, (o0, o1), k = run(ctx, t, [[A], [B]], [0, 1], with_ids=with_ids, deleted=deleted)
            assert k == len(pos)
            if with_ids:
                assert np.array_equal(ids, pos)
            assert np.array_equal(o0, np.asarray(cols[0][2])[pos])
            assert np.array_equal(o1.view(np.uint32), np.asarray(cols[1][2])[pos].view(np.uint32))


def test_cnf_materialize_equals_two_call_form(ctx):
    """the fused launch and mbx_bitmap_cnf_async + mbx_materialize_async agree
    on index BitSets built on the device (the C4 shape at 3 M rows)"""
    n = 3_000_017
    rng = np.random.Generator(np.random.PCG64(9))
    c0 = rng.integers(0, 1 << 20, n, dtype=np.int32)
    c1 = rng.integers(0, 1 << 20, n, dtype=np.int32)
    c2 = rng.integers(0, 10, n, dtype=np.int32)
    c3 = rng.integers(0, 10, n, dtype=np.int32)
    t = ctx.stage([(oracle.INTEGER, 4, c) for c in (c0, c1, c2, c3)])
    b2 = ctx.index_build(t, 2, [("int", v) for v in range(10)])
    b3 = ctx.index_build(t, 3, [("int", v) for v in range(10)])
    conj = [[b2[3], b2[4]], [b3[7]]]
    ids, (o0, o1), k = run(ctx, t, conj, [0, 1])
    r = ctx.bitmap_cnf(n, conj)
    ids2, (p0, p1) = ctx.materialize(t, r, [0, 1])
    sel = ((c2 == 3) | (c2 == 4)) & (c3 == 7)
    assert k == len(ids2) == int(sel.sum())
    assert np.array_equal(ids, ids2) and np.array_equal(o0, p0) and np.array_equal(o1, p1)
    assert np.array_equal(o0, c0[sel]) and np.array_equal(o1, c1[sel])


def test_cnf_materialize_repeated_and_graph_replay(ctx):
    """launch after launch (each a new epoch) with different selections, then
    the same launches captured once and replayed: every result exact"""
    n = 2_000_003
    rng = np.random.Generator(np.random.PCG64(21))
    bits = [rng.random(n) < d for d in (0.2, 0.5, 0.05)]
    bms = [ctx.bitmap_upload(n, words_of(b)) for b in bits]
    cols, t = table(ctx, n, 17)
    shapes = [[[0]], [[0], [1]], [[2]], [[1, 2]], [[0], [1]], [[2]]]
    want = [np.nonzero(cnf_bits([[bits[k] for k in c] for c in s]))[0] for s in shapes]
    for _ in range(3):
        for s, w in zip(shapes, want):
            ids, (o0,), k = run(ctx, t, [[bms[k] for k in c] for c in s], [0])
            assert k == len(w) and np.array_equal(ids, w) and np.array_equal(o0, np.asarray(cols[0][2])[w])
    ids = [torch.zeros(n, dtype=torch.int64, device="cuda") for _ in shapes]
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in shapes]
    cnt = torch.zeros(len(shapes), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.graph_begin()
    for i, s in enumerate(shapes):
        ctx.cnf_materialize_async(t, [[bms[k] for k in c] for c in s], [0], ids[i].data_ptr(),
                                  [outs[i].data_ptr()], cnt.data_ptr() + 8 * i)
    g = ctx.graph_end()
    for _ in range(3):
        for x in ids + outs:
            x.zero_()
        cnt.zero_()
        torch.cuda.synchronize()
        g.launch()
        ctx.sync()
        for i, w in enumerate(want):
            k = int(cnt[i].item())
            assert k == len(w)
            assert np.array_equal(ids[i][:k].cpu().numpy(), w)
            assert np.array_equal(outs[i][:k].cpu().numpy(), np.asarray(cols[0][2])[w])
    g.close()


def test_cnf_materialize_past_the_register_range(ctx):
    """> 2048 words per block (150 M rows): the write pass re-forms the words"""
    n = 150_000_007
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    a = torch.rand(n, device="cuda", generator=g) < 0.01
    b = torch.rand(n, device="cuda", generator=g) < 0.5
    col = torch.randint(0, 1 << 30, (n,), dtype=torch.int32, device="cuda", generator=g)

    def pack(x):
        pad = torch.zeros(((n + 63) // 64) * 64, dtype=torch.bool, device="cuda")
        pad[:n] = x
        wts = (1 << torch.arange(8, device="cuda", dtype=torch.int32)).to(torch.uint8)
        by = (pad.view(-1, 8).to(torch.uint8) * wts).sum(1, dtype=torch.int32).to(torch.uint8)
        return by.cpu().numpy().view(np.uint64)

    A, B = ctx.bitmap_upload(n, pack(a)), ctx.bitmap_upload(n, pack(b))
    t = ctx.wrap([(oracle.INTEGER, 4)], [col.data_ptr()], n)
    sel = a & b
    want = torch.nonzero(sel).flatten()
    k_want = int(want.numel())
    ids = torch.zeros(k_want + 64, dtype=torch.int64, device="cuda")
    out = torch.zeros(k_want + 64, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.cnf_materialize_async(t, [[A], [B]], [0], ids.data_ptr(), [out.data_ptr()], cnt.data_ptr())
    ctx.sync()
    assert int(cnt.item()) == k_want
    assert bool((ids[:k_want] == want).all()) and bool((out[:k_want] == col[want]).all())


def test_cnf_materialize_any_projection_and_limits(ctx, m):
    """char(n) rows and more than 4 columns go through the same launch (the
    wide row gather); more than 16 columns, a null output and a bitmap of
    another size are rejected."""
    n = 1000
    words = ["x", "South_Dakota", "", "zzzzzzzzzzzzzzzz"]
    svals = [words[i % 4] for i in range(n)]
    cols = [(oracle.INTEGER, 4, np.arange(n, dtype=np.int32)),
            (oracle.STRING, 16, helpers.encode_strings(svals, 16))]
    t = ctx.stage(cols)
    sel = np.arange(n) % 3 == 1
    A = ctx.bitmap_upload(n, words_of(sel))
    want = np.nonzero(sel)[0]
    torch.cuda.synchronize()
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    srow = torch.zeros(n * 4, dtype=torch.int32, device="cuda")  # 16-byte device rows
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(5)]
    torch.cuda.synchronize()
    ctx.cnf_materialize_async(t, [[A]], [1], None, [srow.data_ptr()], cnt.data_ptr())
    ctx.sync()
    assert int(cnt.item()) == len(want)
    rows = srow.cpu().numpy().view(np.uint8).reshape(n, 16)[:len(want)]
    assert [bytes(r).rstrip(b"\0").decode() for r in rows] == [svals[i] for i in want]
    ctx.cnf_materialize_async(t, [[A]], [0] * 5, None, [o.data_ptr() for o in outs], cnt.data_ptr())
    ctx.sync()
    for o in outs:
        assert np.array_equal(o[:len(want)].cpu().numpy(), want)
    buf = outs[0]
    with pytest.raises(m.MbxError):  # seventeen columns
        ctx.cnf_materialize_async(t, [[A]], [0] * 17, None, [buf.data_ptr()] * 17, cnt.data_ptr())
    with pytest.raises(m.MbxError):  # a null output buffer
        ctx.cnf_materialize_async(t, [[A]], [0, 1], None, [buf.data_ptr(), 0], cnt.data_ptr())
    B = ctx.bitmap_upload(n + 1, words_of(np.ones(n + 1, dtype=bool)))
    with pytest.raises(m.MbxError):  # bitmap / table size mismatch
        ctx.cnf_materialize_async(t, [[B]], [0], None, [buf.data_ptr()], cnt.data_ptr())


def test_cnf_materialize_grid_sizes_alternate(ctx):
    """launches of different grid sizes on one context (small tables use few
    blocks, so flags past their grid must never be mistaken for this
    launch's): every result exact"""
    runs = []
    for n in (100, 3_000_017, 5_000, 3_000_017, 64, 1_000_003, 70_001, 3_000_017):
        rng = np.random.Generator(np.random.PCG64(n))
        a, b = rng.random(n) < 0.3, rng.random(n) < 0.6
        A, B = ctx.bitmap_upload(n, words_of(a)), ctx.bitmap_upload(n, words_of(b))
        cols, t = table(ctx, n, 3)
        runs.append((n, A, B, cols, t, np.nonzero(a & b)[0]))
    for _ in range(2):
        for n, A, B, cols, t, pos in runs:
            ids, (o0,), k = run(ctx, t, [[A], [B]], [0])
            assert k == len(pos), n
            assert np.array_equal(ids, pos) and np.array_equal(o0, np.asarray(cols[0][2])[pos]), n
