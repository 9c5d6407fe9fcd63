"""The JNI glue (jni/mbx_jni.c) executed for real: no JDK exists on either
box, so tests/jni_harness/jvm_mock.c implements the JNIEnv table the glue
uses over a minimal object model (the reference classes' public fields with
their JNI signatures, modified-UTF-8 strings, arrays, direct ByteBuffers,
the reference's (Exception, String) exception constructors), and these tests
call the Java_global_Native_* functions through ctypes exactly as
java/global/Native.java declares them.  Every call is checked for
unreleased borrows and JNI-spec violations (tests/jvm.py).

CPU tests: the glue's own argument checks, the CondExpr walk
(R/iterator/CondExpr.java:12-41 read field by field, string operands
borrowed and released) and the status -> exception mapping, with no device.
GPU tests: minidata staged through direct ByteBuffers, `C = 6` -> 57
(R/phase3_output), every golden indexes_query row through the one-launch CNF
cursor, every golden BitSet, a NaN compare -> PredEvalException, modified
UTF-8 literals, and the DB-file staging path equal to the decoded-array one
(the fallback java/columnar/GpuTables takes when a dirty page is pinned)."""
import ctypes

import numpy as np
import pytest

import helpers
import oracle
from jvm import I32, I64, JVM, JavaException, V, mutf8_decode

GOLD = helpers.load_golden()


@pytest.fixture(scope="module")
def jvm():
    j = JVM()
    yield j
    j.L.jh_reset()


def J(x):
    return (I64, x)


# ------------------------------------------------------------------ CPU

def test_device_count_without_a_gpu(jvm):
    import mbx_pkg
    m = mbx_pkg.load()
    if m.device_count() > 0:
        pytest.skip("a GPU is visible")
    assert jvm.call("deviceCount", I32) == 0
    with pytest.raises(JavaException) as e:
        jvm.call("init", I64, (I32, 0))
    assert e.value.cls == "chainexception/ChainException" and "no CPU fallback" in e.value.msg


def test_shard_bounds_long_array(jvm):
    import mbx_pkg
    m = mbx_pkg.load()
    for n, k, r in [(100_000_000, 8, 0), (100_000_000, 8, 7), (1000, 3, 2), (10, 4, 3)]:
        out = jvm.call("shardBounds", V, J(n), (I32, k), (I32, r))
        assert jvm.value(out) == list(m.mbx.shard_bounds(n, k, r))
    with pytest.raises(JavaException) as e:
        jvm.call("shardBounds", V, J(10), (I32, 0), (I32, 0))
    assert e.value.cls == "iterator/FileScanException"


def test_condexpr_walk_releases_every_string(jvm):
    """planCompile walks the CondExpr[] (every field read through its JNI
    signature, string operands borrowed as modified UTF-8 and released)
    before the C-ABI rejects the null context as PredEvalException."""
    cnf = [[(oracle.EQ, ("sym", 1), ("str", "South_Dakota")), (oracle.EQ, ("sym", 2), ("str", "a\u0000b\U0001F600"))],
           [(oracle.LT, ("int", 3), ("sym", 3)), (oracle.GE, ("sym", 4), ("real", 0.25))]]
    with pytest.raises(JavaException) as e:
        jvm.call("planCompile", I64, J(0), J(0), (V, jvm.condexprs(cnf)))
    assert e.value.cls == "iterator/PredEvalException" and "null" in e.value.msg


MBX_MAX_TERMS = 32   # include/mbx.h


def test_condexpr_limits(jvm):
    many = [[(oracle.EQ, ("sym", 1), ("str", f"v{i}")) for i in range(MBX_MAX_TERMS + 1)]]
    with pytest.raises(JavaException) as e:
        jvm.call("planCompile", I64, J(0), J(0), (V, jvm.condexprs(many)))
    assert e.value.cls == "iterator/PredEvalException" and "MBX_MAX_TERMS" in e.value.msg


def test_argument_checks_map_to_the_reference_exceptions(jvm):
    i = lambda v: (V, jvm.array("I", v))
    with pytest.raises(JavaException) as e:                     # conj_offsets empty
        jvm.call("bitmapCnf", I64, J(0), J(64), (V, jvm.array("J", [])), i([]), J(0))
    assert e.value.cls == "index/IndexException"
    with pytest.raises(JavaException) as e:
        jvm.call("cursorNext", V, J(0), (I32, 0), i([]), (V, jvm.array("S", [])))
    assert e.value.cls == "iterator/FileScanException"
    with pytest.raises(JavaException) as e:                     # terms not triples
        jvm.call("join", I64, J(0), J(0), J(0), J(0), J(0), i([1, 2]), i([0, 1]), (I32, 0), J(0))
    assert e.value.cls == "chainexception/ChainException"
    with pytest.raises(JavaException) as e:                     # arrays disagree
        jvm.call("tableStage", I64, J(0), i([1, 1]), (V, jvm.array("S", [4])), J(4),
                 (V, jvm.object_array([None, None])), (V, None), J(0))
    assert e.value.cls == "iterator/FileScanException"
    small = np.zeros(3, dtype=np.int32)                         # 3 values for a 4-row table
    with pytest.raises(JavaException) as e:
        jvm.call("tableStage", I64, J(0), i([1]), (V, jvm.array("S", [4])), J(4),
                 (V, jvm.object_array([jvm.direct_buffer(small)])), (V, None), J(0))
    assert e.value.cls == "iterator/FileScanException" and "direct ByteBuffer" in e.value.msg
    with pytest.raises(JavaException) as e:
        jvm.call("commInitRank", I64, J(0), (I32, 2), (I32, 0), (V, jvm.array("B", [0] * 5)))
    assert e.value.cls == "chainexception/ChainException"
    with pytest.raises(JavaException) as e:
        jvm.call("longsDownload", V, J(0), J(0), (I32, -1))
    assert e.value.cls == "chainexception/ChainException"


def test_table_stage_refuses_a_column_past_2_gib(jvm):
    """a char(16) column of 2^27 rows needs 2^31 bytes -- one past what a Java
    direct ByteBuffer holds: the glue sizes it in jlong (no wrap to a small
    or negative size) and refuses the short buffer with FileScanException,
    before any device call"""
    i = lambda v: (V, jvm.array("I", v))
    buf = np.zeros(1 << 20, dtype=np.uint8)
    for nrows in [(1 << 27), (1 << 27) + 1, (1 << 31) // 16 * 3]:
        with pytest.raises(JavaException) as e:
            jvm.call("tableStage", I64, J(0), i([oracle.STRING]), (V, jvm.array("S", [16])), J(nrows),
                     (V, jvm.object_array([jvm.direct_buffer(buf)])), (V, None), J(0))
        assert e.value.cls == "iterator/FileScanException" and "direct ByteBuffer" in e.value.msg


def test_harness_flags_jni_misuse(jvm):
    """the checker itself: a borrowed array left unreleased and a call made
    with an exception pending are reported"""
    L = jvm.L
    arr = jvm.array("I", [1, 2, 3])
    f = ctypes.CFUNCTYPE(V, V, V, ctypes.c_void_p)
    env = ctypes.cast(jvm.env, ctypes.POINTER(ctypes.c_void_p))[0]
    table = ctypes.cast(env, ctypes.POINTER(ctypes.c_void_p))
    # GetIntArrayElements is slot 25 of jni_min's table (0-based)
    get_elems = f(table[25])
    p = get_elems(jvm.env, arr, None)
    assert p and L.jh_outstanding() == 1
    rel = ctypes.CFUNCTYPE(None, V, V, V, I32)(table[28])
    rel(jvm.env, arr, p, 2)
    assert L.jh_outstanding() == 0
    find = ctypes.CFUNCTYPE(V, V, ctypes.c_char_p)(table[0])
    assert not find(jvm.env, b"no/such/Class") and L.jh_pending()
    before = L.jh_violations()
    find(jvm.env, b"java/lang/Object")
    assert L.jh_violations() == before + 1
    L.jh_reset()


# ------------------------------------------------------------------ GPU

@pytest.fixture(scope="module")
def ctx(jvm):
    import mbx_pkg
    if mbx_pkg.load().device_count() == 0:
        pytest.skip("no GPU")
    c = jvm.call("init", I64, (I32, 0))
    yield c
    jvm.call("free", None, J(c))


def stage(jvm, ctx, cols, deleted_words=None, nrows=None):
    """Native.tableStage: one direct ByteBuffer per column (host order,
    char(n) as n bytes of zero-padded modified UTF-8), cf.md's BitSet as
    toLongArray() (zero tail words dropped, as java.util.BitSet does)"""
    n = nrows if nrows is not None else len(cols[0][2])
    bufs = [jvm.direct_buffer(np.ascontiguousarray(a)) for _, _, a in cols]
    dele = None
    if deleted_words is not None:
        w = np.asarray(deleted_words, dtype=np.uint64)
        nz = np.nonzero(w)[0]
        dele = jvm.array("J", w[:nz[-1] + 1].view(np.int64) if len(nz) else [])
    return jvm.call("tableStage", I64, J(ctx), (V, jvm.array("I", [t for t, _, _ in cols])),
                    (V, jvm.array("S", [s for _, s, _ in cols])), J(n), (V, jvm.object_array(bufs)), (V, dele),
                    J(0))


@pytest.fixture(scope="module")
def mini(jvm, ctx):
    rows = helpers.load_minidata()
    cols = helpers.minidata_columns(rows)
    t = stage(jvm, ctx, cols)
    yield rows, cols, t
    jvm.call("tableFree", None, J(t))


def words_of(jvm, ctx, bm):
    return np.array(jvm.value(jvm.call("bitmapDownload", V, J(ctx), J(bm))), dtype=np.int64).view(np.uint64)


def drain(jvm, cur, types, sizes, batch=64):
    """Native.cursorNext until null: (positions, rows)"""
    ids, rows = [], []
    while True:
        r = jvm.call("cursorNext", V, J(cur), (I32, batch), (V, jvm.array("I", types)), (V, jvm.array("S", sizes)))
        if not r:
            return ids, rows
        p, cols = jvm.value(r)
        ids += p
        rows += [list(x) for x in zip(*cols)] if cols else [[] for _ in p]


@pytest.mark.gpu
def test_query_c_eq_6_counts_57(jvm, ctx, mini):
    """`query db cf [A,B,C,D] {C,=,6} 100 FILESCAN` (R/input/Query.java:121-155):
    Total Results Count 57, the rows in position order."""
    rows, cols, t = mini
    plan = jvm.call("planCompile", I64, J(ctx), J(t), (V, jvm.condexprs(helpers.parse_cnf_string("{(C,=,6)}"))))
    assert jvm.call("scanCount", I64, J(ctx), J(plan)) == 57
    bm = jvm.call("scanBitmap", I64, J(ctx), J(plan))
    n_o, w_o, ids_o = oracle.filescan(oracle.Table(cols), helpers.parse_cnf_string("{(C,=,6)}"))
    assert np.array_equal(words_of(jvm, ctx, bm), w_o)
    assert jvm.call("bitmapCardinality", I64, J(bm)) == 57
    cur = jvm.call("cursorOpen", I64, J(ctx), J(t), J(bm), (V, jvm.array("I", [0, 1, 2, 3])))
    ids, got = drain(jvm, cur, [0, 0, 1, 1], [25, 25, 4, 4], batch=10)
    assert ids == list(ids_o) and got == [list(rows[p]) for p in ids]
    jvm.call("cursorRestart", None, J(cur))
    assert drain(jvm, cur, [0, 0, 1, 1], [25, 25, 4, 4], batch=1000)[0] == ids
    assert jvm.call("cursorCount", I64, J(cur)) == 57
    jvm.call("cursorClose", None, J(cur))
    jvm.call("bitmapFree", None, J(bm))
    # the get_next_tid stream as positions
    assert jvm.value(jvm.call("scanSelect", V, J(ctx), J(plan), J(1000))) == list(ids_o)
    jvm.call("planFree", None, J(plan))


def value_bitmaps(jvm, ctx, cols, nbits):
    """per column: value -> device BitSet uploaded from its long[] image
    (GpuTables.bitmap: Native.bitmapUpload(f.getBitSet().toLongArray()))"""
    regs = {}
    for c, (typ, size, arr) in enumerate(cols):
        keys = [bytes(r).rstrip(b"\0") for r in arr] if typ == oracle.STRING else [int(x) for x in arr]
        reg = {}
        for v in sorted(set(keys)):
            bits = np.array([k == v for k in keys])
            w = np.packbits(np.pad(bits, (0, -len(bits) % 64)), bitorder="little").view(np.int64)
            nz = np.nonzero(w)[0]
            reg[v] = jvm.call("bitmapUpload", I64, J(ctx), J(nbits), (V, jvm.array("J", w[:nz[-1] + 1])))
        regs[c] = reg
    return regs


@pytest.mark.gpu
def test_golden_index_queries_through_the_cnf_cursor(jvm, ctx, mini):
    """every `indexes_query` of R/phase3_output through Native.cnfCursorOpen
    (GpuColumnarIndexScan's one-launch path) and every golden BitSet through
    Native.bitmapCnf + bitmapDownload (getOutputPositions)"""
    rows, cols, t = mini
    regs = value_bitmaps(jvm, ctx, cols, len(rows))
    for g in GOLD["indexes_query"] + GOLD["bitsets"]:
        conj = helpers.index_conjuncts(regs, helpers.golden_cnf(g["cnf"]), helpers.MINI_TYPES)
        bms = [h for c in conj for h in c]
        offs = np.cumsum([0] + [len(c) for c in conj])
        cur = jvm.call("cnfCursorOpen", I64, J(ctx), J(t), (V, jvm.array("J", bms)), (V, jvm.array("I", offs)), J(0),
                       (V, jvm.array("I", [0, 1, 2, 3])))
        ids, got = drain(jvm, cur, [0, 0, 1, 1], [25, 25, 4, 4], batch=16)
        jvm.call("cursorClose", None, J(cur))
        if "positions" in g:
            assert ids == g["positions"], g["line"]
        else:
            assert got == g["rows"] and len(ids) == g["count"], g["line"]
        sel = jvm.call("bitmapCnf", I64, J(ctx), J(len(rows)), (V, jvm.array("J", bms)), (V, jvm.array("I", offs)),
                       J(0))
        assert list(oracle.words_to_positions(words_of(jvm, ctx, sel))) == ids
        jvm.call("bitmapFree", None, J(sel))
    for reg in regs.values():
        for h in reg.values():
            jvm.call("bitmapFree", None, J(h))


@pytest.mark.gpu
def test_table_group_through_the_glue(jvm, ctx):
    """Native.tableGroup (GpuTables.group): C, D grouped, every golden
    indexes_query's C, D rows unchanged; a bad group -> FileScanException"""
    rows = helpers.load_minidata()
    cols = helpers.minidata_columns(rows)
    t = stage(jvm, ctx, cols)
    jvm.call("tableGroup", None, J(ctx), J(t), (V, jvm.array("I", [2, 3])))
    with pytest.raises(JavaException) as e:
        jvm.call("tableGroup", None, J(ctx), J(t), (V, jvm.array("I", [0, 1])))   # char(25) columns
    assert e.value.cls == "iterator/FileScanException"
    regs = value_bitmaps(jvm, ctx, cols, len(rows))
    for g in GOLD["indexes_query"]:
        conj = helpers.index_conjuncts(regs, helpers.golden_cnf(g["cnf"]), helpers.MINI_TYPES)
        bms = [h for c in conj for h in c]
        offs = np.cumsum([0] + [len(c) for c in conj])
        cur = jvm.call("cnfCursorOpen", I64, J(ctx), J(t), (V, jvm.array("J", bms)), (V, jvm.array("I", offs)), J(0),
                       (V, jvm.array("I", [2, 3])))
        _, got = drain(jvm, cur, [1, 1], [4, 4], batch=1000)
        jvm.call("cursorClose", None, J(cur))
        assert got == [r[2:] for r in g["rows"]], g["line"]
    for reg in regs.values():
        for h in reg.values():
            jvm.call("bitmapFree", None, J(h))
    jvm.call("tableFree", None, J(t))


@pytest.mark.gpu
def test_errors_map_to_the_reference_exceptions(jvm, ctx, mini):
    _, _, t = mini
    with pytest.raises(JavaException) as e:
        jvm.call("planCompile", I64, J(ctx), J(t), (V, jvm.condexprs([[(oracle.EQ, ("sym", 9), ("int", 1))]])))
    assert e.value.cls == "heap/FieldNumberOutOfBoundException"
    with pytest.raises(JavaException) as e:
        jvm.call("planCompile", I64, J(ctx), J(t), (V, jvm.condexprs([[(oracle.EQ, ("sym", 3), ("str", "x"))]])))
    assert e.value.cls == "iterator/PredEvalException"


@pytest.mark.gpu
def test_nan_raises_pred_eval_exception(jvm, ctx):
    """a float compare that reaches a NaN (TupleUtils.java:61-69 falls into the
    string branch and raises): PredEvalException from the scan, and from
    Native.sync after an async scan"""
    n = 4099
    rng = np.random.Generator(np.random.PCG64(5))
    c0 = rng.integers(0, 10, n, dtype=np.int32)
    f1 = rng.random(n, dtype=np.float32)
    f1[1500], c0[1500] = np.nan, 2
    cols = [(oracle.INTEGER, 4, c0), (oracle.REAL, 4, f1)]
    t = stage(jvm, ctx, cols)
    reached = [[(oracle.LT, ("sym", 1), ("int", 5))], [(oracle.GE, ("sym", 2), ("real", 0.25))]]
    skipped = [[(oracle.LT, ("sym", 1), ("int", 2))], [(oracle.GE, ("sym", 2), ("real", 0.25))]]
    p = jvm.call("planCompile", I64, J(ctx), J(t), (V, jvm.condexprs(reached)))
    with pytest.raises(JavaException) as e:
        jvm.call("scanCount", I64, J(ctx), J(p))
    assert e.value.cls == "iterator/PredEvalException"
    slot = jvm.call("devAlloc", I64, J(ctx), J(8))
    jvm.call("scanCountAsync", None, J(ctx), J(p), J(slot))
    with pytest.raises(JavaException) as e:
        jvm.call("sync", None, J(ctx))
    assert e.value.cls == "iterator/PredEvalException"
    q = jvm.call("planCompile", I64, J(ctx), J(t), (V, jvm.condexprs(skipped)))
    assert jvm.call("scanCount", I64, J(ctx), J(q)) == oracle.filescan(oracle.Table(cols), skipped)[0]
    agg = jvm.value(jvm.call("scanAggregate", V, J(ctx), J(q), (I32, 1)))
    want = oracle.aggregate(oracle.Table(cols), skipped, 1)
    assert agg[0] == want["count"]
    assert np.float64(np.array([agg[5]], dtype=np.int64).view(np.float64)[0]) == pytest.approx(want["sum"], rel=1e-6)
    jvm.call("devFree", None, J(ctx), J(slot))
    for h in (p, q):
        jvm.call("planFree", None, J(h))
    jvm.call("tableFree", None, J(t))


@pytest.mark.gpu
def test_modified_utf8_literals_and_rows(jvm, ctx):
    """String operands arrive as GetStringUTFChars output (modified UTF-8,
    the bytes writeUTF stores); char(16) rows come back through NewStringUTF:
    U+0000 (C0 80) and supplementary characters (surrogate pairs) included,
    compared in Java's UTF-16 order (String.compareTo)"""
    names = ["Alabama", "a\u0000b", "a", "\U0001F600x", "￿", "Zz", "été", "South_Dakota"]
    rng = np.random.Generator(np.random.PCG64(11))
    n = 3001
    pick = rng.integers(0, len(names), n)
    cols = [(oracle.STRING, 16, helpers.encode_strings([names[i] for i in pick], 16)),
            (oracle.INTEGER, 4, np.arange(n, dtype=np.int32))]
    t = stage(jvm, ctx, cols)
    for lit in ["a\u0000b", "\U0001F600", "￾", "a"]:
        for op in (oracle.LT, oracle.GE, oracle.EQ, oracle.NE):
            cnf = [[(op, ("sym", 1), ("str", lit))]]
            p = jvm.call("planCompile", I64, J(ctx), J(t), (V, jvm.condexprs(cnf)))
            n_o, w_o, ids_o = oracle.filescan(oracle.Table(cols), cnf)
            assert jvm.call("scanCount", I64, J(ctx), J(p)) == n_o, (lit, op)
            if op == oracle.GE:
                bm = jvm.call("scanBitmap", I64, J(ctx), J(p))
                cur = jvm.call("cursorOpen", I64, J(ctx), J(t), J(bm), (V, jvm.array("I", [0, 1])))
                ids, got = drain(jvm, cur, [0, 1], [16, 4], batch=500)
                assert ids == list(ids_o)
                assert [r[0] for r in got] == [names[pick[i]] for i in ids] and [r[1] for r in got] == ids
                jvm.call("cursorClose", None, J(cur))
                jvm.call("bitmapFree", None, J(bm))
            jvm.call("planFree", None, J(p))
    jvm.call("tableFree", None, J(t))
    assert mutf8_decode(oracle.java_mutf8("a\u0000\U0001F600")) == "a\u0000\U0001F600"


@pytest.mark.gpu
def test_db_file_staging_equals_the_decoded_array_path(jvm, ctx, tmp_path):
    """GpuTables stages straight from the DB file after flushing the dirty
    unpinned frames; when a dirty frame is pinned it lifts the columns
    through the buffer pool instead (decoded arrays, Native.tableStage).
    Both must give the same table: minidata with deleted rows, every golden
    BitSet / count, through Native.dbOpen + dbStage vs Native.tableStage."""
    import mbx_pkg
    M = mbx_pkg.load().mbx
    rows = helpers.load_minidata()
    cols = helpers.minidata_columns(rows)
    path = str(tmp_path / "db")
    dead = [3, 48, 64, 65, 200, 499]
    with M.Db(path, 4096) as db:
        db.columnar_create("cf", [(t, s) for t, s, _ in cols], ["A", "B", "C", "D"])
        db.columnar_insert("cf", cols)
        for pos in dead:
            db.mark_deleted("cf", pos)
    words = np.zeros((len(rows) + 63) // 64, dtype=np.uint64)
    for pos in dead:
        words[pos // 64] |= np.uint64(1) << np.uint64(pos % 64)
    dbh = jvm.call("dbOpen", I64, (V, jvm.string(path)))
    assert jvm.call("dbColumnarRows", I64, J(dbh), (V, jvm.string("cf"))) == len(rows)
    t_file = jvm.call("dbStage", I64, J(ctx), J(dbh), (V, jvm.string("cf")))
    t_arr = stage(jvm, ctx, cols, words)
    for g in GOLD["bitsets"][:6] + [{"cnf": [[["C", "=", "6"]]]}, {"cnf": [[["C", "!=", "6"]]]}]:
        cnf = helpers.golden_cnf(g["cnf"])
        res = []
        for t in (t_file, t_arr):
            p = jvm.call("planCompile", I64, J(ctx), J(t), (V, jvm.condexprs(cnf)))
            bm = jvm.call("scanBitmap", I64, J(ctx), J(p))
            res.append((jvm.call("scanCount", I64, J(ctx), J(p)), list(oracle.words_to_positions(words_of(jvm, ctx, bm)))))
            jvm.call("bitmapFree", None, J(bm))
            jvm.call("planFree", None, J(p))
        n_o, _, ids_o = oracle.filescan(oracle.Table(cols, deleted_words=words), cnf)
        assert res[0] == res[1] == (n_o, list(ids_o))
    with pytest.raises(JavaException) as e:
        jvm.call("dbStage", I64, J(ctx), J(dbh), (V, jvm.string("nosuchfile")))
    assert e.value.cls == "iterator/FileScanException"
    for t in (t_file, t_arr):
        jvm.call("tableFree", None, J(t))
    jvm.call("dbClose", None, J(dbh))
