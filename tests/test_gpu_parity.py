"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle and
the reference's golden vectors.  Bit-exact for selections, counts, row ids and
integer aggregates; float SUM within 1e-6 relative (BASELINE.json north_star).
"""
import numpy as np
import pytest

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


@pytest.fixture(scope="module")
def mini(ctx):
    rows = helpers.load_minidata()
    cols = helpers.minidata_columns(rows)
    return rows, cols, oracle.Table(cols), ctx.stage(cols)


def gpu_select(ctx, table, cnf):
    plan = ctx.compile(table, cnf)
    bm = ctx.scan_bitmap(plan)
    return bm, bm.download()


# ------------------------------------------------------------------ goldens

@pytest.mark.parametrize("g", GOLD["bitsets"], ids=lambda g: f"line{g['line']}")
def test_golden_bitsets_filescan(ctx, mini, g):
    _, _, _, t = mini
    bm, words = gpu_select(ctx, t, helpers.golden_cnf(g["cnf"]))
    assert list(oracle.words_to_positions(words)) == g["positions"]
    assert bm.count == len(g["positions"])
    assert list(ctx.select(bm)) == g["positions"]


@pytest.mark.parametrize("g", GOLD["full_constraint_counts"], ids=lambda g: f"line{g['line']}")
def test_golden_counts(ctx, mini, g):
    _, _, _, t = mini
    assert ctx.scan_count(ctx.compile(t, helpers.golden_cnf(g["cnf"]))) == g["count"]


index_registry = helpers.index_registry
value_set = helpers.value_set


@pytest.mark.parametrize("g", GOLD["bitsets"] + GOLD["indexes_query"],
                         ids=lambda g: f"line{g['line']}")
def test_golden_index_scan_cnf(ctx, mini, g):
    """ColumnarIndexScan: value-set OR per term, OR within a conjunct, AND
    across conjuncts -- one k_bitmap_cnf launch over the index bitmaps."""
    rows, ocols, _, t = mini
    regs = {c: index_registry(ctx, ocols, t, c) for c in range(4)}
    conjuncts = []
    for conj in helpers.golden_cnf(g["cnf"]):
        lst = []
        for op, (_, fld), (_, lit), *_ in conj:
            lst += value_set(regs[fld - 1], helpers.MINI_TYPES[fld - 1], op, lit)
        conjuncts.append(lst)
    bm = ctx.bitmap_cnf(len(rows), conjuncts)
    pos = list(oracle.words_to_positions(bm.download()))
    if "positions" in g:
        assert pos == g["positions"]
    else:
        ids, (a, b, c, d) = ctx.materialize(t, bm, [0, 1, 2, 3])
        got = [[bytes(x).rstrip(b"\0").decode(), bytes(y).rstrip(b"\0").decode(), int(z), int(w)]
               for x, y, z, w in zip(a, b, c, d)]
        assert got == g["rows"] and bm.count == g["count"]


# ------------------------------------------------------- synthetic parity

def int_table(n, seed=42, hi=1 << 20, ncols=4, deleted_frac=None):
    cols = [(oracle.INTEGER, 4, c) for c in helpers.synthetic_int_table(n, ncols, hi, seed)]
    dele = None if deleted_frac is None else helpers.random_deleted(n, deleted_frac)
    return cols, dele


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 255, 256, 257, 1000, 4099, 70001])
@pytest.mark.parametrize("generic", [False, True])
def test_ragged_sizes(ctx, n, generic, tune):
    if generic:
        tune("force_generic", 1)
    cols, _ = int_table(n, hi=100)
    ot = oracle.Table(cols)
    t = ctx.stage(cols)
    cnf = [[(oracle.LT, ("sym", 1), ("int", 50))], [(oracle.GE, ("sym", 2), ("int", 10)),
                                                      (oracle.EQ, ("sym", 3), ("int", 7))]]
    n_o, w_o, ids_o = oracle.filescan(ot, cnf)
    bm, words = gpu_select(ctx, t, cnf)
    assert bm.count == n_o
    assert np.array_equal(words, w_o)
    assert np.array_equal(ctx.select(bm), ids_o)
    assert ctx.scan_count(ctx.compile(t, cnf)) == n_o


@pytest.mark.parametrize("generic", [False, True])
def test_c2_range_filter_full_size(ctx, generic, tune):
    """C2: 10M rows x 4 int32, `c0 < 104858` -> BitSet + positions + COUNT, bit-exact."""
    if generic:
        tune("force_generic", 1)
    n = 10_000_000
    cols, _ = int_table(n)
    ot = oracle.Table(cols)
    t = ctx.stage(cols)
    cnf = [[(oracle.LT, ("sym", 1), ("int", 104858))]]
    n_o, w_o, ids_o = oracle.filescan(ot, cnf)
    bm, words = gpu_select(ctx, t, cnf)
    assert bm.count == n_o
    assert np.array_equal(words, w_o)
    assert np.array_equal(ctx.select(bm), ids_o)
    # the C2 query proper: mbx_scan_select_async, launch after launch
    import torch
    plan = ctx.compile(t, cnf)
    bm2 = ctx.bitmap_alloc(n)
    dev_ids = torch.zeros(n, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for _ in range(3):
        dev_ids.zero_()
        torch.cuda.synchronize()  # torch's stream is not the library stream
        ctx.scan_select_async(plan, bm2, dev_ids.data_ptr(), cnt.data_ptr())
        ctx.sync()
        assert int(cnt.item()) == n_o
        assert np.array_equal(dev_ids[:n_o].cpu().numpy(), ids_o)
        assert np.array_equal(bm2.download(), w_o)


def test_c3_conjunction_count_full_size(ctx):
    """C3: 100M rows x 4 int32, (c0 < 2^19) AND (c1 >= 2^19) -> COUNT."""
    n = 100_000_000
    cols, _ = int_table(n)
    t = ctx.stage(cols)
    cnf = [[(oracle.LT, ("sym", 1), ("int", 1 << 19))], [(oracle.GE, ("sym", 2), ("int", 1 << 19))]]
    got = ctx.scan_count(ctx.compile(t, cnf))
    ref = int(np.count_nonzero((cols[0][2] < (1 << 19)) & (cols[1][2] >= (1 << 19))))
    assert got == ref
    assert got == oracle.filescan(oracle.Table(cols), cnf)[0]
    # complement identity over the full table (size-independent property)
    neg = [[(oracle.GE, ("sym", 1), ("int", 1 << 19)), (oracle.LT, ("sym", 2), ("int", 1 << 19))]]
    assert got + ctx.scan_count(ctx.compile(t, neg)) == n


@pytest.mark.parametrize("generic", [False, True])
def test_deleted_rows(ctx, generic, tune):
    if generic:
        tune("force_generic", 1)
    n = 1_000_003
    cols, dele = int_table(n, hi=1000, deleted_frac=0.1)
    ot = oracle.Table(cols, dele)
    t = ctx.stage(cols, dele)
    cnf = [[(oracle.NE, ("sym", 4), ("int", 3))], [(oracle.LE, ("sym", 2), ("int", 500))]]
    n_o, w_o, _ = oracle.filescan(ot, cnf)
    bm, words = gpu_select(ctx, t, cnf)
    assert np.array_equal(words, w_o) and bm.count == n_o
    assert ctx.scan_count(ctx.compile(t, None)) == n - int(sum(bin(int(x)).count("1") for x in dele))


def _np_words(mask):
    n = mask.size
    w = np.zeros(((n + 63) // 64) * 64, dtype=bool)
    w[:n] = mask
    return np.packbits(w, bitorder="little").view(np.uint64)


@pytest.mark.parametrize("tpb", [0, 4, 63, 64, 65, 200, 1000])
@pytest.mark.parametrize("ri", ["0", "1"])
@pytest.mark.parametrize("deleted", [False, True])
@pytest.mark.parametrize("sink_lds", ["1", "2"])  # LDS-staged BitSet: default rule / whenever it fits
def test_bitset_segments_and_tile_layouts(ctx, tpb, ri, deleted, sink_lds, tune):
    """BitSet output over segment sizes that give each wave 1..250 tiles (the
    RI layout buffers 16 tiles' words per store) and a ragged tail, both tile
    layouts (MBX_SCAN_RI), with and without deleted rows; numpy is the check
    (the same predicate, bit for bit)."""
    if tpb:
        tune("tiles_per_block", tpb)
    tune("scan_ri", int(ri))
    tune("sink_lds", int(sink_lds))
    n = 2_000_003
    cols, dele = int_table(n, hi=1000, deleted_frac=0.05 if deleted else None)
    t = ctx.stage(cols, dele)
    cnf = [[(oracle.LT, ("sym", 1), ("int", 700))], [(oracle.GE, ("sym", 2), ("int", 100)),
                                                       (oracle.EQ, ("sym", 3), ("int", 7))]]
    c0, c1, c2 = cols[0][2], cols[1][2], cols[2][2]
    mask = (c0 < 700) & ((c1 >= 100) | (c2 == 7))
    want = _np_words(mask)
    if deleted:
        want &= ~dele
    bm, words = gpu_select(ctx, t, cnf)
    assert np.array_equal(words, want)
    assert bm.count == int(np.unpackbits(want.view(np.uint8)).sum())
    ids = ctx.select(bm)
    assert np.array_equal(ids, np.nonzero(np.unpackbits(want.view(np.uint8), bitorder="little"))[0][:bm.count])


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 255, 256, 257, 4099, 70001, 1_000_003])
def test_scan_select_positions(ctx, n):
    """mbx_scan_select gives the oracle's get_next_tid positions (global:
    the shard's row_offset added), launch after launch."""
    cols, dele = int_table(n, hi=100, deleted_frac=0.05)
    ot, t = oracle.Table(cols, dele), ctx.stage(cols, dele, row_offset=640)
    cnf = [[(oracle.LT, ("sym", 1), ("int", 50))], [(oracle.GE, ("sym", 2), ("int", 10)),
                                                      (oracle.EQ, ("sym", 3), ("int", 7))]]
    n_o, w_o, ids_o = oracle.filescan(ot, cnf)
    plan = ctx.compile(t, cnf)
    for _ in range(3):
        assert np.array_equal(ctx.scan_select(plan), ids_o + 640)


@pytest.mark.parametrize("tpb", [1, 4, 37, 200, 512, 513, 1000, 1025])
def test_scan_select_segment_sizes(ctx, tpb, tune):
    """Segments of 4..4100 words; positions and the BitSet left in the
    bitmap both exact, also through the async entry point."""
    tune("tiles_per_block", tpb)
    n = 3_000_017
    cols, _ = int_table(n, hi=1000)
    t = ctx.stage(cols)
    plan = ctx.compile(t, [[(oracle.LT, ("sym", 1), ("int", 300))]])
    mask = cols[0][2] < 300
    ids = ctx.scan_select(plan)
    assert np.array_equal(ids, np.nonzero(mask)[0])
    import torch
    bm = ctx.bitmap_alloc(n)
    dev_ids = torch.zeros(n, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # the zero fills run on torch's stream, not the library's
    ctx.scan_select_async(plan, bm, dev_ids.data_ptr(), cnt.data_ptr())
    ctx.sync()
    k = int(cnt.item())
    assert k == int(mask.sum())
    assert np.array_equal(dev_ids[:k].cpu().numpy(), ids)
    assert np.array_equal(bm.download(), _np_words(mask))
    assert bm.count == -1  # unknown after an async call until something needs it
    assert np.array_equal(ctx.select(bm), ids)  # via the segment counts the scan left
    assert bm.count == k


@pytest.mark.parametrize("generic", [False, True])
def test_scan_select_strings_and_floats(ctx, generic, tune):
    """String-slot (KS > 0) and float plans, fast and generic kernels, with
    and without deleted rows."""
    if generic:
        tune("force_generic", 1)
    cols, _ = mixed_table(200_003, seed=11)
    dm = helpers.random_deleted(200_003, 0.03)
    ot, t = oracle.Table(cols), ctx.stage(cols)
    otd, td = oracle.Table(cols, dm), ctx.stage(cols, dm)
    cnfs = [[[(oracle.GE, ("sym", 3), ("str", "M"))], [(oracle.LT, ("sym", 2), ("real", 0.5)),
                                                       (oracle.LT, ("sym", 1), ("int", 1000))]],
            [[(oracle.GE, ("sym", 3), ("str", "M"))]],                                    # KS=1, K=0
            [[(oracle.LT, ("sym", 3), ("str", "K"))], [(oracle.GT, ("sym", 2), ("real", 0.3))]],  # KS=1, K=1
            [[(oracle.LT, ("sym", 2), ("real", 0.25))]]]                                  # K=1 float
    for cnf in cnfs:
        for o, g in ((ot, t), (otd, td)):
            n_o, w_o, ids_o = oracle.filescan(o, cnf)
            assert np.array_equal(ctx.scan_select(ctx.compile(g, cnf)), ids_o), cnf


def test_scan_select_capacity(ctx, m):
    """host capacity: exactly the count works, one less raises MBX_E_INVALID
    (the device scratch is sized to the count, per call)."""
    cols, _ = int_table(100_000, hi=100)
    t = ctx.stage(cols)
    plan = ctx.compile(t, [[(oracle.LT, ("sym", 1), ("int", 10))]])
    want = np.nonzero(cols[0][2] < 10)[0]
    assert np.array_equal(ctx.scan_select(plan, cap=len(want)), want)
    with pytest.raises(m.MbxError) as e:
        ctx.scan_select(plan, cap=len(want) - 1)
    assert e.value.code == m.mbx.E_INVALID
    assert np.array_equal(ctx.scan_select(plan, cap=len(want) + 5), want)


@pytest.mark.parametrize("op", [oracle.EQ, oracle.LT, oracle.GT, oracle.NE, oracle.LE, oracle.GE, oracle.NOT,
                                oracle.NOP, oracle.RANGE])
@pytest.mark.parametrize("lit_left", [False, True])
def test_operator_table(ctx, op, lit_left):
    cols, _ = int_table(5000, hi=20)
    ot, t = oracle.Table(cols), ctx.stage(cols)
    term = (op, ("int", 9), ("sym", 2)) if lit_left else (op, ("sym", 2), ("int", 9))
    cnf = [[term]]
    n_o, w_o, _ = oracle.filescan(ot, cnf)
    bm, words = gpu_select(ctx, t, cnf)
    assert np.array_equal(words, w_o) and bm.count == n_o


def test_column_vs_column_and_constant_terms(ctx):
    cols, _ = int_table(9999, hi=30)
    ot, t = oracle.Table(cols), ctx.stage(cols)
    for cnf in ([[(oracle.LE, ("sym", 1), ("sym", 2))]],
                [[(oracle.EQ, ("int", 1), ("int", 2))], [(oracle.GT, ("sym", 3), ("int", 20))]],
                [[(oracle.LT, ("int", 1), ("int", 2))]],
                [[(oracle.LT, ("int", 1), ("int", 2)), (oracle.EQ, ("sym", 4), ("int", 5))]]):
        n_o, w_o, _ = oracle.filescan(ot, cnf)
        bm, words = gpu_select(ctx, t, cnf)
        assert np.array_equal(words, w_o) and bm.count == n_o, cnf


def test_errors_follow_the_reference(ctx, m):
    cols, _ = int_table(100)
    t = ctx.stage(cols)
    with pytest.raises(m.MbxError) as e:
        ctx.compile(t, [[(oracle.EQ, ("sym", 9), ("int", 1))]])
    assert e.value.code == m.mbx.E_RANGE           # FieldNumberOutOfBoundException
    with pytest.raises(m.MbxError) as e:
        ctx.compile(t, [[(oracle.EQ, ("sym", 1), ("str", "x"))]])
    assert e.value.code == m.mbx.E_TYPE            # mismatched operand types


def mixed_table(n, seed=5):
    """C5 schema: i32 c0 uniform [0,2^20); f32 c1 uniform [0,1); char(16) c2
    from a 50-name dictionary."""
    rng = np.random.Generator(np.random.PCG64(seed))
    names = [f"{chr(65 + (i * 7) % 26)}{'abcdefghijklmnop'[:(i % 15) + 1]}"[:16] for i in range(50)]
    c0 = rng.integers(0, 1 << 20, size=n, dtype=np.int32)
    c1 = rng.random(n, dtype=np.float32)
    idx = rng.integers(0, 50, size=n)
    dic = helpers.encode_strings(names, 16)
    c2 = dic[idx]
    return [(oracle.INTEGER, 4, c0), (oracle.REAL, 4, c1), (oracle.STRING, 16, c2)], names


C5_CNF = [[(oracle.LT, ("sym", 1), ("int", 1 << 19))], [(oracle.GE, ("sym", 2), ("real", 0.25))],
          [(oracle.GE, ("sym", 3), ("str", "M"))]]


@pytest.mark.parametrize("generic", [False, True])
@pytest.mark.parametrize("deleted", [False, True])
def test_c5_mixed_filter_and_aggregates(ctx, generic, deleted, tune):
    """C5 shape: int32 + float32 + char(16) (16-byte string slot of the fast
    kernel, or the generic kernel), 3 conjuncts + SUM/MIN/MAX."""
    if generic:
        tune("force_generic", 1)
    n = 2_000_003
    cols, _ = mixed_table(n)
    dele = helpers.random_deleted(n, 0.07) if deleted else None
    ot, t = oracle.Table(cols, dele), ctx.stage(cols, dele)
    n_o, w_o, _ = oracle.filescan(ot, C5_CNF)
    bm, words = gpu_select(ctx, t, C5_CNF)
    assert np.array_equal(words, w_o) and bm.count == n_o
    a_o = oracle.aggregate(ot, C5_CNF, 1)
    a_g = ctx.scan_aggregate(ctx.compile(t, C5_CNF), 1)
    assert a_g["count"] == a_o["count"]
    assert a_g["min"] == a_o["min"] and a_g["max"] == a_o["max"]
    assert abs(a_g["sum"] - a_o["sum"]) <= 1e-6 * abs(a_o["sum"])
    i_o = oracle.aggregate(ot, C5_CNF, 0)
    i_g = ctx.scan_aggregate(ctx.compile(t, C5_CNF), 0)
    assert i_g == i_o


@pytest.mark.parametrize("generic", [False, True])
def test_fast_path_aggregates(ctx, generic, tune):
    if generic:
        tune("force_generic", 1)
    n = 3_000_017
    rng = np.random.Generator(np.random.PCG64(11))
    cols = [(oracle.INTEGER, 4, rng.integers(-1000, 1000, n, dtype=np.int32)),
            (oracle.REAL, 4, (rng.random(n, dtype=np.float32) - 0.5) * 100)]
    ot, t = oracle.Table(cols), ctx.stage(cols)
    cnf = [[(oracle.GT, ("sym", 1), ("int", -100))], [(oracle.LT, ("sym", 2), ("real", 10.0))]]
    for col in (0, 1):
        a_o = oracle.aggregate(ot, cnf, col)
        a_g = ctx.scan_aggregate(ctx.compile(t, cnf), col)
        assert a_g["count"] == a_o["count"] and a_g["min"] == a_o["min"] and a_g["max"] == a_o["max"]
        assert abs(a_g["sum"] - a_o["sum"]) <= 1e-6 * max(1.0, abs(a_o["sum"]))
    # empty selection: identities
    empty = ctx.scan_aggregate(ctx.compile(t, [[(oracle.LT, ("sym", 1), ("int", -5000))]]), 0)
    assert empty["count"] == 0 and empty["sum"] == 0


def test_nan_raises_like_the_reference(ctx, m):
    cols = [(oracle.REAL, 4, np.array([1.0, np.nan, 3.0], dtype=np.float32))]
    t = ctx.stage(cols)
    with pytest.raises(m.MbxError) as e:
        ctx.scan_count(ctx.compile(t, [[(oracle.LT, ("sym", 1), ("real", 2.0))]]))
    assert e.value.code == m.mbx.E_TYPE


@pytest.mark.parametrize("generic", [False, True])
def test_strings_java_order(ctx, generic, tune):
    if generic:
        tune("force_generic", 1)
    vals = ["", "a", "ab", "b", "South_Dakota", "South", "é", "€", "\U0001F600", "a\u0000b", "a\u0000",
            "zzzzzzzzzzzzzzzz"]
    arr = helpers.encode_strings(vals, 16)
    cols = [(oracle.STRING, 16, arr)]
    ot, t = oracle.Table(cols), ctx.stage(cols)
    for lit in vals + ["a\u0000a", "zzzzzzzzzzzzzzzzz", "Sout"]:
        for op in (oracle.LT, oracle.EQ, oracle.GE, oracle.NE):
            cnf = [[(op, ("sym", 1), ("str", lit))]]
            n_o, w_o, _ = oracle.filescan(ot, cnf)
            bm, words = gpu_select(ctx, t, cnf)
            assert np.array_equal(words, w_o), (lit, op)
    # materialised strings come back as the caller's modified UTF-8
    bm, _ = gpu_select(ctx, t, None)
    ids, (out,) = ctx.materialize(t, bm, [0])
    assert np.array_equal(out, arr)


def test_bitmap_ops_and_materialize(ctx):
    n = 1_234_567
    rng = np.random.Generator(np.random.PCG64(3))
    a_bits, b_bits = rng.random(n) < 0.3, rng.random(n) < 0.5
    pack = lambda bits: np.packbits(bits, bitorder="little").view(np.uint8)
    words = lambda bits: np.frombuffer(np.pad(pack(bits), (0, (-len(pack(bits))) % 8)).tobytes(), dtype=np.uint64)
    wa, wb = words(a_bits), words(b_bits)
    A, B = ctx.bitmap_upload(n, wa), ctx.bitmap_upload(n, wb)
    assert A.count == int(a_bits.sum())
    m = mbx_pkg.load().mbx
    for op, ref in ((m.BM_AND, wa & wb), (m.BM_OR, wa | wb), (m.BM_ANDNOT, wa & ~wb)):
        r = ctx.bitmap_combine(op, A, B)
        assert np.array_equal(r.download(), ref)
    r = ctx.bitmap_cnf(n, [[A], [B]], deleted=ctx.bitmap_upload(n, words(rng.random(n) < 0.1)))
    cols, _ = int_table(n)
    ot, t = oracle.Table(cols), ctx.stage(cols)
    ids, (c0, c3) = ctx.materialize(t, r, [0, 3])
    assert np.array_equal(ids, oracle.words_to_positions(r.download()))
    g0, g3 = oracle.gather(ot, ids, [0, 3])
    assert np.array_equal(c0, g0) and np.array_equal(c3, g3)
    cur = ctx.cursor(t, r, [0, 3])
    parts = []
    while True:
        i, (x, y) = cur.next(100_000)
        if len(i) == 0:
            break
        parts.append((i, x, y))
    assert np.array_equal(np.concatenate([p[0] for p in parts]), ids)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), c0)


@pytest.mark.parametrize("density", [0.0, 0.001, 0.01, 0.1, 0.6, 1.0])
@pytest.mark.parametrize("fused", [1, 0])
def test_materialize_gather_shapes(ctx, density, fused, tune):
    """The compaction's own gather (<= 4 int / float columns) and the
    two-launch form: sparse, LDS-staged and dense (> 2048 positions per step)
    steps, 1..5 projected columns (5: k_gather), int and float columns, a
    ragged size and a shard's row_offset; numpy gathers are the check."""
    tune("gather_fused", fused)
    n = 700_013
    rng = np.random.Generator(np.random.PCG64(int(density * 1000) + 7))
    bits = rng.random(n) < density
    w = np.zeros(((n + 63) // 64) * 64, dtype=bool)
    w[:n] = bits
    words = np.packbits(w, bitorder="little").view(np.uint64)
    ints = helpers.synthetic_int_table(n, 3, 1 << 30, 5)
    f0 = rng.random(n, dtype=np.float32)
    f1 = rng.standard_normal(n).astype(np.float32)
    cols = [(oracle.INTEGER, 4, ints[0]), (oracle.REAL, 4, f0), (oracle.INTEGER, 4, ints[1]), (oracle.REAL, 4, f1),
            (oracle.INTEGER, 4, ints[2])]
    t = ctx.stage(cols, row_offset=6400)
    bm = ctx.bitmap_upload(n, words)
    pos = np.nonzero(bits)[0]
    for proj in ([0], [1, 3], [3, 0, 2], [4, 3, 2, 1], [0, 1, 2, 3, 4]):
        ids, outs = ctx.materialize(t, bm, proj)
        assert np.array_equal(ids, pos + 6400), proj
        for j, o in zip(proj, outs):
            assert np.array_equal(np.asarray(o).view(np.uint32), np.asarray(cols[j][2])[pos].view(np.uint32)), (proj, j)


def test_index_build_matches_oracle(ctx):
    cols, _ = mixed_table(300_001)
    ot, t = oracle.Table(cols), ctx.stage(cols)
    _, names = mixed_table(1)
    bms = ctx.index_build(t, 2, [("str", s) for s in names[:10]] + [("str", "nope")])
    for s, bm in zip(names[:10] + ["nope"], bms):
        n_o, w_o = oracle.bitmap_eq(ot, 2, ("str", s))
        assert bm.count == n_o and np.array_equal(bm.download(), w_o)
    cols2, _ = int_table(300_001, hi=10)
    ot2, t2 = oracle.Table(cols2), ctx.stage(cols2)
    for v, bm in zip(range(10), ctx.index_build(t2, 2, [("int", v) for v in range(10)])):
        n_o, w_o = oracle.bitmap_eq(ot2, 2, ("int", v))
        assert np.array_equal(bm.download(), w_o)


def test_row_range_shards_concatenate(ctx):
    """Sharding: row ranges on 64-row boundaries; per-shard
    BitSets and global positions concatenate to the unsharded answer."""
    n = 2_000_000
    cols, dele = int_table(n, hi=1000, deleted_frac=0.05)
    cnf = [[(oracle.LT, ("sym", 1), ("int", 300))], [(oracle.GE, ("sym", 2), ("int", 100))]]
    n_o, w_o, ids_o = oracle.filescan(oracle.Table(cols, dele), cnf)
    bounds = [0, 64 * 7001, 64 * 20000, n]
    words, ids = [], []
    for s, e in zip(bounds[:-1], bounds[1:]):
        sh = [(ty, sz, a[s:e]) for ty, sz, a in cols]
        t = ctx.stage(sh, dele[s // 64:(e + 63) // 64].copy(), row_offset=s)
        bm, w = gpu_select(ctx, t, cnf)
        words.append(w)
        ids.append(ctx.select(bm, row_offset=s))
    assert np.array_equal(np.concatenate(words), w_o)
    assert np.array_equal(np.concatenate(ids), ids_o)


@pytest.mark.parametrize("width", [13, 16, 8, 25])
def test_string_slot_shapes(ctx, width):
    """Two string columns + ints: char(13..16) rows take the fast kernel's
    16-byte slots (<= 2 of them), other widths the generic kernel; literals
    longer than 16 bytes also fall back.  All bit-exact vs the oracle."""
    n = 300_007
    rng = np.random.Generator(np.random.PCG64(21))
    words = ["", "a", "ab", "abc", "M", "Mz", "South_Dakota", "Zz", "x" * width, "é€", "a\u0000b"]
    words = [w for w in words if len(oracle.java_mutf8(w)) <= width]
    s1 = helpers.encode_strings([words[i] for i in rng.integers(0, len(words), n)], width)
    s2 = helpers.encode_strings([words[i] for i in rng.integers(0, len(words), n)], width)
    cols = [(oracle.STRING, width, s1), (oracle.INTEGER, 4, rng.integers(0, 100, n, dtype=np.int32)),
            (oracle.STRING, width, s2)]
    ot, t = oracle.Table(cols), ctx.stage(cols)
    for cnf in ([[(oracle.GE, ("sym", 1), ("str", "M"))], [(oracle.LT, ("sym", 3), ("str", "ab")),
                                                            (oracle.GT, ("sym", 2), ("int", 90))]],
                [[(oracle.EQ, ("sym", 3), ("str", "South_Dakota"))]],
                [[(oracle.NE, ("sym", 1), ("str", "x" * width + "y"))]],
                [[(oracle.LE, ("str", "abc"), ("sym", 1))], [(oracle.EQ, ("sym", 2), ("int", 5))]]):
        n_o, w_o, _ = oracle.filescan(ot, cnf)
        bm, words_g = gpu_select(ctx, t, cnf)
        assert np.array_equal(words_g, w_o), cnf
        assert ctx.scan_count(ctx.compile(t, cnf)) == n_o


@pytest.mark.parametrize("n", [1, 63, 257, 4099, 1_000_003])
@pytest.mark.parametrize("deleted", [False, True])
def test_index_build_int_shapes(ctx, n, deleted):
    """k_index_build4 (4-byte columns): ragged tails, deleted rows left clear
    (createBitMapIndex walks a ColumnScan), > 64 values (two launches), the
    per-segment counts it writes (count + positions must agree)."""
    cols, dele = int_table(n, hi=70, deleted_frac=0.1 if deleted else None)
    ot, t = oracle.Table(cols, dele), ctx.stage(cols, dele)
    vals = list(range(72))
    bms = ctx.index_build(t, 1, [("int", v) for v in vals])
    for v, bm in zip(vals, bms):
        n_o, w_o = oracle.bitmap_eq(ot, 1, ("int", v))
        assert bm.count == n_o and np.array_equal(bm.download(), w_o), v
    ids_o = oracle.words_to_positions(oracle.bitmap_eq(ot, 1, ("int", 5))[1])
    assert np.array_equal(ctx.select(bms[5]), ids_o)


def test_index_build_float_column(ctx):
    n = 100_003
    rng = np.random.Generator(np.random.PCG64(9))
    f = rng.integers(0, 5, n).astype(np.float32) * np.float32(0.25)
    cols = [(oracle.INTEGER, 4, rng.integers(0, 9, n, dtype=np.int32)), (oracle.REAL, 4, f)]
    ot, t = oracle.Table(cols), ctx.stage(cols)
    for v, bm in zip([0.0, 0.25, 0.5, 3.0], ctx.index_build(t, 1, [("real", x) for x in [0.0, 0.25, 0.5, 3.0]])):
        n_o, w_o = oracle.bitmap_eq(ot, 1, ("real", v))
        assert bm.count == n_o and np.array_equal(bm.download(), w_o)


def test_c4_full_size_bitmap_and_gather(ctx, m):
    """C4 at BASELINE size: 100M rows, bm(c2=3) AND bm(c3=7) built on the GPU,
    compacted to positions and gathered (c0, c1) -- checked against numpy."""
    n = 100_000_000
    c0, c1 = (np.random.Generator(np.random.PCG64(42 + j)).integers(0, 1 << 20, n, dtype=np.int32) for j in range(2))
    c2, c3 = (np.random.Generator(np.random.PCG64(44 + j)).integers(0, 10, n, dtype=np.int32) for j in range(2))
    t = ctx.stage([(oracle.INTEGER, 4, c) for c in (c0, c1, c2, c3)])
    (b2,) = ctx.index_build(t, 2, [("int", 3)])
    (b3,) = ctx.index_build(t, 3, [("int", 7)])
    sel = ctx.bitmap_combine(m.mbx.BM_AND, b2, b3)
    want = np.nonzero((c2 == 3) & (c3 == 7))[0]
    assert sel.count == len(want)
    ids, (x, y) = ctx.materialize(t, sel, [0, 1])
    assert np.array_equal(ids, want)
    assert np.array_equal(x, c0[want]) and np.array_equal(y, c1[want])


def test_c5_shard_full_size(ctx):
    """One GPU's C5 shard at BASELINE size (125M rows of the 1B-row table over
    8 GPUs): 3-conjunct int/float/char(16) filter + COUNT/SUM/MIN/MAX vs numpy
    (count, min, max exact; SUM within 1e-6 relative), and the complement
    identity count(P) + count(not P) = N."""
    n = 125_000_000
    cols, names = mixed_table(n, seed=77)
    c0, c1, c2 = (a for _, _, a in cols)
    t = ctx.stage(cols)
    plan = ctx.compile(t, C5_CNF)
    agg = ctx.scan_aggregate(plan, 1)
    m_mask = np.array([oracle.java_mutf8(s) >= b"M" for s in names])  # ASCII names: byte order = Java order
    idx = np.frombuffer(c2.tobytes(), dtype="S16")
    keep = (c0 < (1 << 19)) & (c1 >= np.float32(0.25))
    name_ok = np.isin(idx, np.frombuffer(helpers.encode_strings([s for s, ok in zip(names, m_mask) if ok], 16)
                                         .tobytes(), dtype="S16"))
    sel = keep & name_ok
    vals = c1[sel]
    assert agg["count"] == int(sel.sum())
    assert agg["min"] == float(vals.min()) and agg["max"] == float(vals.max())
    assert abs(agg["sum"] - float(vals.astype(np.float64).sum())) <= 1e-6 * abs(float(vals.astype(np.float64).sum()))
    neg = [[(oracle.GE, ("sym", 1), ("int", 1 << 19)), (oracle.LT, ("sym", 2), ("real", 0.25)),
            (oracle.LT, ("sym", 3), ("str", "M"))]]
    assert ctx.scan_count(plan) + ctx.scan_count(ctx.compile(t, neg)) == n


@pytest.mark.gpu
def test_probe_read_runs_and_checks_arguments(m, ctx):
    """mbx_probe_read (bench.py's secondary roofline denominator) launches on
    4-byte columns in every mapping and rejects what it cannot read."""
    n = 1 << 20
    cols = [(oracle.INTEGER, 4, np.arange(n, dtype=np.int32)), (oracle.REAL, 4, np.ones(n, np.float32)),
            (oracle.STRING, 16, helpers.encode_strings(["ab"] * n, 16))]
    t = ctx.stage(cols)
    ctx.probe_read(t, [0, 1])
    ctx.probe_read(t, [0], tiles_per_block=3)
    ctx.probe_read(t, [1, 0, 1, 0], interleave=True, grid=64)
    ctx.sync()
    for bad in ([2], [], [0, 1, 0, 1, 0], [7]):
        with pytest.raises(m.MbxError) as e:
            ctx.probe_read(t, bad)
        assert e.value.code == m.mbx.E_INVALID


def test_c5_full_table_1b_rows(ctx, m):
    """C5 at its full BASELINE size on one GPU: 1,000,000,000 rows of
    i32 / f32 / char(16) (24 GB, generated in HBM), the 3-conjunct filter +
    COUNT/SUM/MIN/MAX.  Checked with size-independent properties against a
    torch reduction of the same device columns (the oracle would need minutes
    here): count, min, max exact; SUM within 1e-6 relative; the complement
    identity count(P) + count(not P) = N; and the 8-way row-range sharding
    (dist.shard_bounds, zero-copy views at row_offset) folded in rank order
    (dist.fold_aggregates) equals the whole-table result -- the 8-GPU C5 flow
    with the exchange replaced by the fold it feeds."""
    import torch
    dist_mod = m.dist
    n = 1_000_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    c0 = torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g)
    c1 = torch.rand(n, dtype=torch.float32, device="cuda", generator=g)
    names = [f"{chr(65 + (i * 7) % 26)}{'abcdefghijklmnop'[:(i % 15) + 1]}"[:16] for i in range(50)]
    dic = torch.from_numpy(helpers.encode_strings(names, 16).reshape(50, 16)).cuda()
    idx = torch.randint(0, 50, (n,), dtype=torch.int32, device="cuda", generator=g)
    c2 = helpers.device_dictionary_column(dic, idx)  # (n, 16) uint8 = the char(16) slot image
    torch.cuda.synchronize()
    descs = [(m.mbx.INTEGER, 4), (m.mbx.REAL, 4), (m.mbx.STRING, 16)]
    t = ctx.wrap(descs, [c0.data_ptr(), c1.data_ptr(), c2.data_ptr()], n)
    plan = ctx.compile(t, C5_CNF)
    agg = ctx.scan_aggregate(plan, 1)

    name_ok = torch.tensor([oracle.java_mutf8(s) >= b"M" for s in names], device="cuda")
    # the checker uses elementwise ops and reductions only (no index or
    # masked-select launch over the full table, see helpers.device_dictionary_column)
    name_sel = helpers.device_dictionary_column(name_ok, idx)
    assert bool((name_sel == (c2[:, 0] >= ord("M"))).all())  # the slot image holds the dictionary rows
    sel = (c0 < (1 << 19)) & (c1 >= 0.25) & name_sel
    del name_sel
    want_sum = float(torch.where(sel, c1.double(), 0.0).sum())
    assert agg["count"] == int(sel.sum())
    assert agg["min"] == float(torch.where(sel, c1, float("inf")).min())
    assert agg["max"] == float(torch.where(sel, c1, float("-inf")).max())
    assert abs(agg["sum"] - want_sum) <= 1e-6 * abs(want_sum)
    del sel
    neg = [[(oracle.GE, ("sym", 1), ("int", 1 << 19)), (oracle.LT, ("sym", 2), ("real", 0.25)),
            (oracle.LT, ("sym", 3), ("str", "M"))]]
    assert ctx.scan_count(plan) + ctx.scan_count(ctx.compile(t, neg)) == n

    recs = []
    for r in range(8):
        s, e = dist_mod.shard_bounds(n, 8, r)
        ts = ctx.wrap(descs, [c0.data_ptr() + 4 * s, c1.data_ptr() + 4 * s, c2.data_ptr() + 16 * s], e - s,
                      None, row_offset=s)
        recs.append(dist_mod.pack_aggregate(ctx.scan_aggregate(ctx.compile(ts, C5_CNF), 1), integer=False))
        ts.close()
    folded = dist_mod.fold_aggregates(np.concatenate(recs))
    assert folded["count"] == agg["count"]
    assert folded["min"] == agg["min"] and folded["max"] == agg["max"]
    assert abs(folded["sum"] - want_sum) <= 1e-6 * abs(want_sum)
    t.close()
    del c0, c1, c2, idx
    torch.cuda.empty_cache()


@pytest.mark.parametrize("knob,value", [
    ("fin_mode", 1),         # plain stores + fences
    ("fin_mode", 4),         # segment words only, forced on a COUNT scan
    ("scan_int_range", 3),   # the removed unsigned range forms
    ("select_dbg", 1),       # compaction A/B bits
    ("select_dbg", 16),
])
def test_ab_only_knob_values_are_compiled_out(m, ctx, knob, value, tune):
    """The A/B-only kernel forms exist in -DMBX_DIAG builds only: the
    production library refuses the knob values that would select them
    (MBX_E_UNSUPPORTED / MBX_E_INVALID) instead of silently running another form."""
    with pytest.raises(m.MbxError) as e:
        tune(knob, value)
    assert e.value.code in (m.mbx.E_UNSUPPORTED, m.mbx.E_INVALID)


@pytest.mark.parametrize("groups,tpb,fin", [
    ("32", "0", None),     # default: 32 group words + the top word
    ("1", "0", None),      # one flat packed word (~1000 arrivals)
    ("1", "4", None),      # flat, > 4095 arrivals: falls back to the write-through partials
    ("64", "4", None),     # 64 groups x ~77 arrivals
    ("5", "7", None),      # groups that do not divide the grid
    ("32", "0", "0"),      # write-through partials (MBX_FIN_MODE=0)
    ("32", "0", "2"),      # separate finalize launch
])
def test_count_and_bitset_finalize_forms(ctx, groups, tpb, fin, tune):
    """COUNT and BitSet scans end in the packed 64-bit ticket words (count |
    NaN blocks | arrivals); every grouping, the > 4095-arrival fallback and
    the other finalize forms give the same count, BitSet and positions
    (numpy check), and back-to-back launches see the words reset."""
    tune("ticket_groups", int(groups))
    if tpb != "0":
        tune("tiles_per_block", int(tpb))
    if fin is not None:
        tune("fin_mode", int(fin))
    n = 5_000_017
    cols, _ = int_table(n, hi=1000)
    t = ctx.stage(cols)
    c0, c1 = cols[0][2], cols[1][2]
    for lim in (700, 3, 1000):  # a different count each launch: a stale ticket word would show
        cnf = [[(oracle.LT, ("sym", 1), ("int", lim))], [(oracle.GE, ("sym", 2), ("int", 100))]]
        mask = (c0 < lim) & (c1 >= 100)
        plan = ctx.compile(t, cnf)
        assert ctx.scan_count(plan) == int(mask.sum())
        bm = ctx.scan_bitmap(plan)
        assert bm.count == int(mask.sum())
        assert np.array_equal(bm.download(), _np_words(mask))
        assert np.array_equal(ctx.select(bm), np.nonzero(mask)[0])
