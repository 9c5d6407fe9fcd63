"""Minibase DB files (include/mbx_db.h).

CPU tests: the C++ writer against the page numbers the reference engine
printed for `batchinsert minidata.txt db cf 4` (tests/golden/phase3_golden.json
"db_pages", R/phase3_output:19-22,3172,3228,3246,3264), and against the CPU
restatement of the reader (oracle/minibase_pages.py) for every format detail.
GPU tests: mbx_db_stage (pages -> HBM -> k_page_decode) against the same
restatement, and queries over the staged table against the scan oracle.
"""
import numpy as np
import pytest

import helpers
import mbx_pkg
import minibase_pages as mp
import oracle

GOLD = helpers.load_golden()


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


def minidata_db(m, path, num_pages=1024 * 1024):
    """BatchInsert minidata.txt into a fresh DB (SystemDefs(db, 1024*1024, ...),
    R/input/BatchInsert.java:52-57)."""
    rows = helpers.load_minidata()
    cols = helpers.minidata_columns(rows)
    db = m.mbx.Db(path, num_pages)
    db.columnar_create("cf", [(t, s) for t, s, _ in cols], ["A", "B", "C", "D"])
    db.columnar_insert("cf", cols)
    return db, cols


def test_batchinsert_page_numbers_match_reference(m, tmp_path):
    db, _ = minidata_db(m, str(tmp_path / "db"))
    db.close()
    img = mp.DbImage(str(tmp_path / "db"))
    gp = GOLD["db_pages"]
    # space map: pages 0..128 (first page + 128 map pages of a 1M-page DB)
    # are reserved at creation; the engine wrote 0, 1 and then 129..176
    written = sorted(set(gp["batchinsert_wrote"]))
    assert mp.allocated_pages(img) == list(range(0, 129)) + [p for p in written if p >= 129]
    fe = mp.file_entries(img)
    assert fe == {"cf.hdr": 129, "cf.0": 131, "cf.1": 132, "cf.2": 133, "cf.3": 134, "cf.md": 135, "cf.dtid": 136}
    # the data pages of each column = the pages the engine read when it
    # scanned that column (minus the hdr, .md and directory pages)
    for i, colname in enumerate("ABCD"):
        reads = gp["column_scan_reads"][colname]["pages"]
        assert 131 + i in reads
        want = sorted(p for p in reads if 137 <= p <= 176)
        got = sorted(pid for _, pid, _ in mp.heap_data_pages(img, fe[f"cf.{i}"]))
        assert got == want, colname


def test_minidata_round_trip_through_reader_restatement(m, tmp_path):
    db, cols = minidata_db(m, str(tmp_path / "db"), num_pages=4096)
    info = db.columnar_info("cf")
    assert info["ncols"] == 4 and info["names"] == ["A", "B", "C", "D"]
    assert info["cols"] == [(oracle.STRING, 25), (oracle.STRING, 25), (oracle.INTEGER, 4), (oracle.INTEGER, 4)]
    assert info["nrows"] == 500 and info["live"] == 500
    db.close()
    img = mp.DbImage(str(tmp_path / "db"))
    sc = mp.columnar_schema(img, "cf")
    assert sc["names"] == ["A", "B", "C", "D"] and sc["btree"] == [0] * 4 and sc["bitmap"] == [0] * 4
    n, got, dele = mp.columnar_table(img, "cf")
    assert n == 500 and not dele.any()
    for (t, s, a), (t2, s2, b) in zip(cols, got):
        assert (t, s) == (t2, s2) and np.array_equal(a, b)


def test_page_layouts(m, tmp_path):
    """HFPage fill: 125 int32 / 32 char(25) / 45 char(16) records per data
    page, 83 DataPageInfo per directory page, records packed from the end."""
    n = 125 * 83 + 7   # spills into a second directory page for the int column
    rng = np.random.Generator(np.random.PCG64(3))
    words = ["alpha", "b", "", "é€", "x" * 16]
    cols = [(oracle.INTEGER, 4, rng.integers(-2**31, 2**31 - 1, n, dtype=np.int32)),
            (oracle.STRING, 16, helpers.encode_strings([words[i] for i in rng.integers(0, 5, n)], 16)),
            (oracle.REAL, 4, rng.random(n, dtype=np.float32))]
    path = str(tmp_path / "db")
    with m.mbx.Db(path, 8192) as db:
        db.columnar_create("t", [(t, s) for t, s, _ in cols], ["i", "s", "f"])
        db.columnar_insert("t", cols)
    img = mp.DbImage(path)
    fe = mp.file_entries(img)
    for i, rpp in enumerate([125, 45, 125]):
        pages = mp.heap_data_pages(img, fe[f"t.{i}"])
        assert [pi for pi, _, _ in pages] == list(range(len(pages)))
        assert all(rc == rpp for _, _, rc in pages[:-1])
        pg = img.page(pages[0][1])
        assert mp.be16(pg, 0) == rpp and mp.be16(pg, 2) == 1024 - rpp * (4 if i != 1 else 18)
    nd = sum(1 for _ in iter_dir_pages(img, fe["t.0"]))
    assert nd == 2
    nrows, got, dele = mp.columnar_table(img, "t")
    assert nrows == n and not dele.any()
    for (t, s, a), (_, _, b) in zip(cols, got):
        assert np.array_equal(a, b)


def iter_dir_pages(img, first):
    d = first
    while d != mp.INVALID:
        yield d
        d = mp.be32(img.page(d), 12)


def test_append_and_mark_deleted(m, tmp_path):
    path = str(tmp_path / "db")
    rng = np.random.Generator(np.random.PCG64(5))
    a = [(oracle.INTEGER, 4, rng.integers(0, 50, 1000, dtype=np.int32))]
    b = [(oracle.INTEGER, 4, rng.integers(0, 50, 333, dtype=np.int32))]
    with m.mbx.Db(path, 4096) as db:
        db.columnar_create("cf", [(oracle.INTEGER, 4)], ["x"])
        db.columnar_insert("cf", a)
        db.columnar_insert("cf", b)      # a second batchinsert appends
        for p in (0, 7, 999, 1000, 1332, 64):
            db.mark_deleted("cf", p)
        info = db.columnar_info("cf")
        assert info["nrows"] == 1333 and info["live"] == 1333 - 6
        with pytest.raises(m.MbxError):
            db.mark_deleted("cf", 5000)    # findRID: Invalid Position
    img = mp.DbImage(path)
    n, (col,), dele = mp.columnar_table(img, "cf")
    assert n == 1333 and np.array_equal(col[2], np.concatenate([a[0][2], b[0][2]]))
    assert sorted(oracle.words_to_positions(dele)) == [0, 7, 64, 999, 1000, 1332]
    # cf.dtid holds one TID record (numColumns RIDs: slotNo, pageNo) per delete
    recs = [r for _, _, r in mp.heap_records(img, mp.file_entries(img)["cf.dtid"])]
    assert len(recs) == 6 and all(len(r) == 8 for r in recs)
    data = {pi: pid for pi, pid, _ in mp.heap_data_pages(img, mp.file_entries(img)["cf.0"])}
    assert mp.be32(recs[2], 0) == 999 % 125 and mp.be32(recs[2], 4) == data[999 // 125]


def test_bitmap_files(m, tmp_path):
    path = str(tmp_path / "db")
    rng = np.random.Generator(np.random.PCG64(8))
    big = rng.integers(0, 2**63, 300, dtype=np.uint64)           # 19200 bits -> 3 chunk pages
    small = np.zeros(2, dtype=np.uint64)
    small[1] = np.uint64(1) << np.uint64(40)
    with m.mbx.Db(path, 4096) as db:
        db.bitmap_write("cf.bm.0.7", big)
        db.bitmap_write("cf.bm.0.8", small)
        with pytest.raises(m.MbxError):
            db.bitmap_write("cf.bm.0.9", np.zeros(4, dtype=np.uint64))   # empty BitSet
        with pytest.raises(m.MbxError):
            db.bitmap_write("cf.bm.0.7", big)                           # exists
        assert np.array_equal(db.bitmap_read("cf.bm.0.7")[:300], big)
        assert np.array_equal(db.bitmap_read("cf.bm.0.8")[:2], small)
    img = mp.DbImage(path)
    w = mp.bitmap_words(img, "cf.bm.0.7")
    assert np.array_equal(w[:300], big) and not w[300:].any()
    head = img.page(mp.file_entries(img)["cf.bm.0.7"])
    assert mp.be16(head, 6) == 13                     # NodeType.BMHEAD
    assert mp.hf_slots(head) == [(0, 1000, 24)]       # one 1000-byte record
    assert np.array_equal(mp.bitmap_words(img, "cf.bm.0.8")[:2], small)


def test_many_files_spill_into_directory_pages(m, tmp_path):
    """More than 17 file entries: DB.add_file_entry allocates DBDirectoryPages
    (18 entries each) -- as page 205 in the reference run of `index db cf A bitmap`."""
    path = str(tmp_path / "db")
    with m.mbx.Db(path, 4096) as db:
        for k in range(40):
            w = np.zeros(1, dtype=np.uint64)
            w[0] = np.uint64(1 + k)
            db.bitmap_write(f"f{k}", w)
        for k in range(40):
            assert db.file_entry(f"f{k}") >= 0
        assert db.file_entry("nope") == -1
    img = mp.DbImage(path)
    fe = mp.file_entries(img)
    assert len(fe) == 40 and mp.be32(img.page(0), 4) == 17
    dir1 = mp.be32(img.page(0), 0)
    assert dir1 > 0 and mp.be32(img.page(dir1), 4) == 18
    for k in range(40):
        assert int(mp.bitmap_words(img, f"f{k}")[0]) == 1 + k


def test_errors(m, tmp_path):
    path = str(tmp_path / "db")
    with m.mbx.Db(path, 200) as db:
        db.columnar_create("cf", [(oracle.INTEGER, 4)], ["x"])
        with pytest.raises(m.MbxError):
            db.columnar_create("cf", [(oracle.INTEGER, 4)], ["x"])         # exists
        with pytest.raises(m.MbxError):
            db.columnar_create("a_name_too_long_for_minibase", [(oracle.INTEGER, 4)], ["x"])
        with pytest.raises(m.MbxError):
            db.columnar_info("missing")
        with pytest.raises(m.MbxError) as e:                                # OutOfSpaceException
            db.columnar_insert("cf", [(oracle.INTEGER, 4, np.zeros(200 * 125, dtype=np.int32))])
        assert e.value.code == m.mbx.E_NOMEM
    with pytest.raises(m.MbxError):
        m.mbx.Db(str(tmp_path / "absent"))


# ------------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
def test_stage_minidata_goldens(m, ctx, tmp_path):
    """Golden BitSets of the reference transcript over a table staged from a
    Minibase DB file by the GPU page decoder."""
    db, cols = minidata_db(m, str(tmp_path / "db"), num_pages=4096)
    t = ctx.stage_db(db, "cf")
    for g in GOLD["bitsets"]:
        bm = ctx.scan_bitmap(ctx.compile(t, helpers.golden_cnf(g["cnf"])))
        assert list(oracle.words_to_positions(bm.download())) == g["positions"]
    ids, outs = ctx.materialize(t, ctx.scan_bitmap(ctx.compile(t, None)), [0, 1, 2, 3])
    assert np.array_equal(ids, np.arange(500))
    for (tt, s, a), o in zip(cols, outs):
        assert np.array_equal(a, o)
    db.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 124, 125, 126, 125 * 83, 125 * 83 + 1, 200_003])
def test_stage_matches_reader_restatement(m, ctx, tmp_path, n):
    path = str(tmp_path / "db")
    rng = np.random.Generator(np.random.PCG64(n))
    words = ["", "a", "M", "Mz", "South_Dakota", "é€", "a\u0000b", "zzzzzzzzzzzzzzzz"]
    cols = [(oracle.INTEGER, 4, rng.integers(-1000, 1000, n, dtype=np.int32)),
            (oracle.STRING, 16, helpers.encode_strings([words[i] for i in rng.integers(0, len(words), n)], 16)),
            (oracle.REAL, 4, rng.random(n, dtype=np.float32)),
            (oracle.STRING, 25, helpers.encode_strings([words[i] for i in rng.integers(0, len(words), n)], 25))]
    with m.mbx.Db(path, 1 << 16) as db:
        db.columnar_create("cf", [(t, s) for t, s, _ in cols], ["i", "s", "f", "w"])
        db.columnar_insert("cf", cols)
        for p in range(0, n, 97):
            db.mark_deleted("cf", p)
        t = ctx.stage_db(db, "cf")
    nrows, ocols, dele = mp.columnar_table(mp.DbImage(path), "cf")
    assert nrows == n
    ot = oracle.Table(ocols, dele)
    all_rows = ctx.scan_bitmap(ctx.compile(t, None))
    assert np.array_equal(all_rows.download(), oracle.filescan(ot, None)[1])
    ids, outs = ctx.materialize(t, all_rows, [0, 1, 2, 3])
    live = np.array(oracle.words_to_positions(oracle.filescan(ot, None)[1]), dtype=np.int64)
    assert np.array_equal(ids, live)
    for (tt, s, a), o in zip(cols, outs):
        assert np.array_equal(a[live], o)
    for cnf in ([[(oracle.LT, ("sym", 1), ("int", 0))], [(oracle.GE, ("sym", 2), ("str", "M"))]],
                [[(oracle.EQ, ("sym", 4), ("str", "a\u0000b")), (oracle.GT, ("sym", 3), ("real", 0.5))]]):
        n_o, w_o, _ = oracle.filescan(ot, cnf)
        bm = ctx.scan_bitmap(ctx.compile(t, cnf))
        assert bm.count == n_o and np.array_equal(bm.download(), w_o)


@pytest.mark.gpu
def test_stage_rejects_malformed_pages(m, ctx, tmp_path):
    path = str(tmp_path / "db")
    with m.mbx.Db(path, 1024) as db:
        db.columnar_create("cf", [(oracle.INTEGER, 4)], ["x"])
        db.columnar_insert("cf", [(oracle.INTEGER, 4, np.arange(300, dtype=np.int32))])
    img = mp.DbImage(path)
    pid = mp.heap_data_pages(img, mp.file_entries(img)["cf.0"])[0][1]
    with open(path, "r+b") as f:        # slot 3 claims a 5-byte record
        f.seek(pid * 1024 + 20 + 4 * 3)
        f.write(b"\x00\x05")
    with m.mbx.Db(path) as db:
        with pytest.raises(m.MbxError) as e:
            ctx.stage_db(db, "cf")
        assert "malformed" in str(e.value)


def first_occurrence(values):
    seen, out = set(), []
    for v in values:
        if v not in seen:
            seen.add(v)
            out.append(v)
    return out


@pytest.mark.gpu
def test_bitmap_index_persistence_matches_reference_pages(m, ctx, tmp_path):
    """`index db cf A btree` then `index db cf {A,B,C,D} bitmap` as in the
    reference session (R/phase3_output:3167-3265): the B+-tree file is only
    reserved (18 pages + its file entry -- out of scope), the bitmap indexes
    are built on the GPU and written as BitMapFiles; the pages each command
    allocates equal the ones the reference wrote, the registry holds the
    values in first-occurrence order and every BitMapFile holds the oracle's
    BitSet."""
    path = str(tmp_path / "db")
    db, cols = minidata_db(m, path)
    runs = [r for r in GOLD["db_pages"]["index_runs"] if r["line"] <= 3265]
    assert [r["cmd"] for r in runs] == ["index db cf A btree", "index db cf A bitmap", "index db cf B bitmap",
                                        "index db cf C bitmap", "index db cf D bitmap"]
    head = db.allocate_pages(1)
    db.add_file_entry("cf.btree.0", head)
    assert db.allocate_pages(17) == head + 1
    assert head == 177
    t = ctx.stage_db(db, "cf")
    rows = helpers.load_minidata()
    ot = oracle.Table(cols)
    before = db.info()[1]
    top = 194
    for r in runs[1:]:
        col = "ABCD".index(r["col"])
        n = ctx.create_bitmap_index(db, "cf", t, col)
        want_vals = first_occurrence([row[col] for row in rows])
        assert n == len(want_vals)
        new = [p for p in sorted(set(r["wrote"])) if p > top]
        after = db.info()[1]
        assert after - before == len(new), r["cmd"]
        assert new == list(range(top + 1, top + 1 + len(new)))
        before, top = after, new[-1]
        got_vals = db.bitmap_values("cf", col)
        assert got_vals == [oracle.java_mutf8(str(v)) for v in want_vals]
        for v in want_vals:
            w = db.bitmap_read(f"cf.bm.{col}.{v}")
            spec = ("str", v) if col < 2 else ("int", v)
            n_o, w_o = oracle.bitmap_eq(ot, col, spec)
            assert np.array_equal(w[:len(w_o)], w_o[:len(w)]) and not w[len(w_o):].any()
            bm = ctx.stage_db_bitmap(db, f"cf.bm.{col}.{v}", 500)
            assert bm.count == n_o
        assert ctx.create_bitmap_index(db, "cf", t, col) == 0     # already indexed: no-op
    db.close()
    img = mp.DbImage(path)
    assert mp.columnar_schema(img, "cf")["bitmap"] == [1, 1, 1, 1]


@pytest.mark.gpu
def test_bitmap_index_large_and_deleted(m, ctx, tmp_path):
    """Multi-chunk BitMapFiles (positions past 8000 bits), deleted rows left
    out of every BitSet, value order = first live occurrence."""
    path = str(tmp_path / "db")
    n = 50_000
    rng = np.random.Generator(np.random.PCG64(12))
    vals = rng.integers(-5, 40, n, dtype=np.int32)
    words = ["Ohio", "Iowa", "Utah", "é", "Wyoming_12"]
    svals = [words[i] for i in rng.integers(0, len(words), n)]
    cols = [(oracle.INTEGER, 4, vals), (oracle.STRING, 12, helpers.encode_strings(svals, 12))]
    with m.mbx.Db(path, 1 << 15) as db:
        db.columnar_create("cf", [(oracle.INTEGER, 4), (oracle.STRING, 12)], ["v", "s"])
        db.columnar_insert("cf", cols)
        dead = sorted(set(int(x) for x in rng.integers(0, n, 500)))
        for p in dead:
            db.mark_deleted("cf", p)
        t = ctx.stage_db(db, "cf")
        assert ctx.create_bitmap_index(db, "cf", t, 0) > 0
        assert ctx.create_bitmap_index(db, "cf", t, 1) > 0
        live = np.ones(n, dtype=bool)
        live[dead] = False
        assert db.bitmap_values("cf", 0) == [str(v).encode() for v in first_occurrence(vals[live].tolist())]
        assert db.bitmap_values("cf", 1) == [oracle.java_mutf8(v) for v in
                                             first_occurrence([s for s, l in zip(svals, live) if l])]
    img = mp.DbImage(path)
    _, ocols, dele = mp.columnar_table(img, "cf")
    ot = oracle.Table(ocols, dele)
    for v in set(vals[live].tolist()):
        n_o, w_o = oracle.bitmap_eq(ot, 0, ("int", v))
        w = mp.bitmap_words(img, f"cf.bm.0.{v}")
        k = min(len(w), len(w_o))
        assert np.array_equal(w[:k], w_o[:k]) and not w[k:].any() and not w_o[k:].any()
    for s in set(s for s, l in zip(svals, live) if l):
        n_o, w_o = oracle.bitmap_eq(ot, 1, ("str", s))
        w = mp.bitmap_words(img, "cf.bm.1." + oracle.java_mutf8(s).decode("utf-8", "surrogatepass"))
        k = min(len(w), len(w_o))
        assert np.array_equal(w[:k], w_o[:k]) and not w[k:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("lds_probes", [None, "0", "1"])
def test_bitmap_index_many_values(m, ctx, tmp_path, tune, lds_probes):
    """k_distinct with thousands of distinct values: blocks whose LDS table
    overflows (and, with MBX_DISTINCT_LDS_PROBES=0 / 1, rows sent to the global
    table directly or after one LDS probe) still give every live value once, in
    first-live-occurrence order; BitMapFiles of sampled values equal the
    oracle's.  All values print at one width, so the .hdr registry records are
    equal-sized and Heapfile's first-fit insert keeps them in insertion order
    (with mixed widths a shorter later record can fill an earlier page)."""
    if lds_probes is not None:
        tune("distinct_lds_probes", int(lds_probes))
    path = str(tmp_path / "db")
    n = 40_000
    rng = np.random.Generator(np.random.PCG64(31))
    vals = rng.integers(1000, 4000, n, dtype=np.int32)
    pool = [f"v{k:04d}" for k in range(1200)]
    svals = [pool[i] for i in rng.integers(0, len(pool), n)]
    cols = [(oracle.INTEGER, 4, vals), (oracle.STRING, 8, helpers.encode_strings(svals, 8))]
    with m.mbx.Db(path, 1 << 17) as db:
        db.columnar_create("cf", [(oracle.INTEGER, 4), (oracle.STRING, 8)], ["v", "s"])
        db.columnar_insert("cf", cols)
        dead = sorted(set(int(x) for x in rng.integers(0, n, 300)))
        db.mark_deleted_many("cf", dead)
        t = ctx.stage_db(db, "cf")
        live = np.ones(n, dtype=bool)
        live[dead] = False
        want_i = first_occurrence(vals[live].tolist())
        want_s = first_occurrence([s for s, l in zip(svals, live) if l])
        assert ctx.create_bitmap_index(db, "cf", t, 0) == len(want_i) > 2048
        assert ctx.create_bitmap_index(db, "cf", t, 1) == len(want_s) == 1200
        assert db.bitmap_values("cf", 0) == [str(v).encode() for v in want_i]
        assert db.bitmap_values("cf", 1) == [v.encode() for v in want_s]
        for v in want_i[::97]:
            w = db.bitmap_read(f"cf.bm.0.{v}")
            pos = np.nonzero((vals == v) & live)[0]
            assert list(oracle.words_to_positions(w)) == list(pos), v
        for v in want_s[::53]:
            w = db.bitmap_read(f"cf.bm.1.{v}")
            pos = np.nonzero(np.array([s == v for s in svals]) & live)[0]
            assert list(oracle.words_to_positions(w)) == list(pos), v


def test_purge_all_deleted_tuples(m, tmp_path):
    """Columnarfile.purgeAllDeletedTuples (R/columnar/Columnarfile.java:837-925)
    on a 3 x int32 file spanning 4 directory pages per column: a whole
    directory page of rows, one whole data page and scattered rows deleted.
    After the purge the records are gone, emptied data pages and the emptied
    (non-first) directory page are freed, the positions after the removed
    directory page shift down by 83 * 125, holes stay holes, cf.md is clear and
    cf.dtid empty; a following insert reuses the holes first (HFPage slot
    reuse), then the freed data page's directory slot."""
    path = str(tmp_path / "db")
    per_dir = 83 * 125
    n = 3 * per_dir + 77
    rng = np.random.Generator(np.random.PCG64(17))
    vals = [rng.integers(-1000, 1000, n, dtype=np.int32) for _ in range(3)]
    cols = [(oracle.INTEGER, 4, v) for v in vals]
    scattered = list(range(3, 2000, 7))
    page5 = list(range(5 * 125, 6 * 125))
    dir1 = list(range(per_dir, 2 * per_dir))
    dead = sorted(set(scattered + page5 + dir1))
    with m.mbx.Db(path, 1 << 14) as db:
        db.columnar_create("cf", [(oracle.INTEGER, 4)] * 3, ["a", "b", "c"])
        db.columnar_insert("cf", cols)
        before = db.info()[1]
        db.mark_deleted_many("cf", dead)
        assert db.columnar_info("cf")["live"] == n - len(dead)
        db.purge("cf")
        after = db.info()[1]
        info = db.columnar_info("cf")
    # freed: per column 83 data pages of dir 1 + page 5 + dir page 1; cf.dtid's
    # pages are freed and one new directory page is allocated
    img = mp.DbImage(path)
    assert before - after >= 3 * (83 + 1 + 1) - 1
    fe = mp.file_entries(img)
    assert mp.heap_records(img, fe["cf.dtid"]) == []
    assert not mp.bitmap_words(img, "cf.md").any()
    nrows, got, dele = mp.columnar_table(img, "cf")
    survivors = [p for p in range(n) if p not in set(dead)]

    def shifted(p):
        return p - per_dir if p >= 2 * per_dir else p
    want_pos = [shifted(p) for p in survivors]
    live = [int(x) for x in np.nonzero(~np.unpackbits(dele.view(np.uint8), bitorder="little")[:nrows].astype(bool))[0]]
    assert live == want_pos and nrows == shifted(n - 1) + 1
    for (t, s, a), v in zip(got, vals):
        assert np.array_equal(a[want_pos], v[survivors])
    assert info["live"] == len(survivors) and info["nrows"] == nrows
    # appending refills the holes in position order, then the freed data page's slot
    holes = [p for p in scattered if p not in set(page5)]
    k = len(holes) + 125 + 10
    extra = [rng.integers(5000, 6000, k, dtype=np.int32) for _ in range(3)]
    with m.mbx.Db(path) as db:
        db.columnar_insert("cf", [(oracle.INTEGER, 4, v) for v in extra])
    nrows2, got2, dele2 = mp.columnar_table(mp.DbImage(path), "cf")
    for (t, s, a), v in zip(got2, extra):
        assert np.array_equal(a[holes], v[:len(holes)])
        assert np.array_equal(a[page5], v[len(holes):len(holes) + 125])
    live2 = np.count_nonzero(~np.unpackbits(dele2.view(np.uint8), bitorder="little")[:nrows2].astype(bool))
    assert live2 == len(survivors) + k


@pytest.mark.gpu
def test_purge_updates_bitmap_indexes(m, ctx, tmp_path):
    """Bitmap indexes through a purge (BitMapFile.purgeDelete): deleted
    positions cleared and the removed directory page's position range cut out
    of every BitSet, so each BitMapFile equals the value's positions in the
    purged file; scans of the re-staged table agree with the files."""
    path = str(tmp_path / "db")
    per_dir = 83 * 125
    n = 3 * per_dir + 77
    rng = np.random.Generator(np.random.PCG64(23))
    vals = [rng.integers(0, 10, n, dtype=np.int32) for _ in range(2)]
    dead = sorted(set(list(range(3, 2000, 7)) + list(range(per_dir, 2 * per_dir))))
    with m.mbx.Db(path, 1 << 14) as db:
        db.columnar_create("cf", [(oracle.INTEGER, 4)] * 2, ["a", "b"])
        db.columnar_insert("cf", [(oracle.INTEGER, 4, v) for v in vals])
        t = ctx.stage_db(db, "cf")
        assert ctx.create_bitmap_index(db, "cf", t, 0) == 10
        db.mark_deleted_many("cf", dead)
        db.purge("cf")
        t2 = ctx.stage_db(db, "cf")
        survivors = [p for p in range(n) if p not in set(dead)]
        new_pos = np.array([p - per_dir if p >= 2 * per_dir else p for p in survivors])
        for v in range(10):
            want = new_pos[vals[0][survivors] == v]
            w = db.bitmap_read(f"cf.bm.0.{v}")
            assert list(oracle.words_to_positions(w)) == list(want), v
            plan = ctx.compile(t2, [[(oracle.EQ, ("sym", 1), ("int", v))]])
            assert ctx.scan_count(plan) == len(want)
            bm = ctx.stage_db_bitmap(db, f"cf.bm.0.{v}", t2.nrows)
            assert bm.count == len(want)
