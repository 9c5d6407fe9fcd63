"""ColumnarIndexScan in ONE launch on the drop-in path (k_cnf_select through
mbx_cnf_cursor_open / mbx_cnf_materialize_async, any projection incl.
char(n) rows), pinned to the reference's own vectors and to the oracle:

* every `bmj` selection BitSet and every `indexes_query` result of
  R/phase3_output (positions; rows A, B char(25), C, D in nextSetBit order,
  R/index/ColumnarIndexScan.java:287-308) through the cursor and through the
  device-buffer entry point;
* a synthetic CNF matrix (int / char(n) index columns, every AttrOperator,
  absent literals, deleted rows, ragged sizes, projections of 0..6 columns
  incl. float and wide char(n)) against oracle.columnar_index_scan +
  oracle.gather (R/index/ColumnarIndexScan.java:130-181, ColumnIndexScan
  getBitSet :656-740, Projection.Project);
* the double-buffered cursor: batches of any size, changing sizes, restart
  mid-stream, equal to one materialise;
* the C++ mirror's ColumnarIndexScan (CLI `indexes_query`) takes the
  one-launch path for every transcript query without a repeated constraint.
"""
import os
import subprocess
import tempfile

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


@pytest.fixture(scope="module")
def mini(ctx):
    rows = helpers.load_minidata()
    cols = helpers.minidata_columns(rows)
    t = ctx.stage(cols)
    regs = {c: helpers.index_registry(ctx, cols, t, c) for c in range(4)}
    return rows, cols, t, regs


def as_rows(outs, types):
    cols = []
    for o, typ in zip(outs, types):
        if typ == oracle.STRING:
            cols.append([bytes(x).rstrip(b"\0").decode() for x in o])
        else:
            cols.append([int(x) if typ == oracle.INTEGER else float(x) for x in o])
    return [list(r) for r in zip(*cols)]


# ------------------------------------------------------------------ goldens

@pytest.mark.parametrize("g", GOLD["bitsets"] + GOLD["indexes_query"], ids=lambda g: f"line{g['line']}")
def test_golden_cnf_cursor(ctx, mini, g):
    """phase3 golden positions / rows through mbx_cnf_cursor_open (A, B are
    char(25): the wide row gather inside k_cnf_select)."""
    rows, _, t, regs = mini
    conj = helpers.index_conjuncts(regs, helpers.golden_cnf(g["cnf"]), helpers.MINI_TYPES)
    cur = ctx.cnf_cursor(t, conj, [0, 1, 2, 3])
    ids, outs = cur.next(len(rows) + 1)
    if "positions" in g:
        assert list(ids) == g["positions"]
    else:
        assert as_rows(outs, helpers.MINI_TYPES) == g["rows"] and len(ids) == g["count"]
        # the rows are the ones at those positions (nextSetBit order)
        assert [list(rows[p]) for p in ids] == g["rows"]
    assert cur.count == len(ids)


def device_string_rows(raw_words, n, size):
    """device string image (stride = size rounded up to 4 bytes) -> payloads"""
    stride = (size + 3) // 4 * 4
    b = raw_words.cpu().numpy().view(np.uint8).reshape(-1, stride)[:n]
    return [bytes(x[:size]).rstrip(b"\0").decode() for x in b]


@pytest.mark.parametrize("g", GOLD["indexes_query"], ids=lambda g: f"line{g['line']}")
def test_golden_cnf_materialize_device_rows(ctx, mini, g):
    """the same rows through mbx_cnf_materialize_async into device buffers in
    the table's device row layout (char(25) -> 28-byte rows)."""
    rows, _, t, regs = mini
    conj = helpers.index_conjuncts(regs, helpers.golden_cnf(g["cnf"]), helpers.MINI_TYPES)
    n = len(rows)
    torch.cuda.synchronize()
    ids = torch.full((n,), -1, dtype=torch.int64, device="cuda")
    sa = torch.zeros((n * 7,), dtype=torch.int32, device="cuda")
    sb = torch.zeros((n * 7,), dtype=torch.int32, device="cuda")
    c = torch.zeros((n,), dtype=torch.int32, device="cuda")
    d = torch.zeros((n,), dtype=torch.int32, device="cuda")
    cnt = torch.zeros((1,), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.cnf_materialize_async(t, conj, [0, 1, 2, 3], ids.data_ptr(),
                              [sa.data_ptr(), sb.data_ptr(), c.data_ptr(), d.data_ptr()], cnt.data_ptr())
    ctx.sync()
    k = int(cnt.item())
    assert k == g["count"]
    got = [list(r) for r in zip(device_string_rows(sa, k, 25), device_string_rows(sb, k, 25),
                                 c[:k].cpu().tolist(), d[:k].cpu().tolist())]
    assert got == g["rows"]
    assert [list(rows[p]) for p in ids[:k].cpu().tolist()] == g["rows"]


# -------------------------------------------------------- synthetic matrix

NAMES = [b"Alabama", b"Colorado", b"Iowa", b"Maine", b"Ohio", b"South_Dakota", b"Texas", b"Utah"]
TYPES = [oracle.INTEGER, oracle.STRING, oracle.INTEGER, oracle.REAL, oracle.STRING]


def synth(n, seed):
    """k0 int [0,10), k1 char(12) of 8 names, k2 int [0,5) (index columns);
    f3 float, s4 char(30) (projection only: 32-byte device rows)"""
    rng = np.random.default_rng(seed)
    k0 = rng.integers(0, 10, n, dtype=np.int32)
    k1 = helpers.encode_strings([NAMES[i] for i in rng.integers(0, len(NAMES), n)], 12)
    k2 = rng.integers(0, 5, n, dtype=np.int32)
    f3 = rng.random(n, dtype=np.float32)
    s4 = rng.integers(ord("a"), ord("z") + 1, (n, 30), dtype=np.uint8)
    s4[np.arange(n), rng.integers(1, 31, n) - 1] = 0  # ragged payloads
    s4[np.cumsum(s4 == 0, axis=1) > 0] = 0
    return [(oracle.INTEGER, 4, k0), (oracle.STRING, 12, k1), (oracle.INTEGER, 4, k2), (oracle.REAL, 4, f3),
            (oracle.STRING, 30, s4)]


OPS = [oracle.EQ, oracle.LT, oracle.LE, oracle.GT, oracle.GE, oracle.NE, oracle.NOT]


def random_cnf(rng):
    cnf, seen = [], set()
    for _ in range(int(rng.integers(1, 4))):
        conj = []
        for _ in range(int(rng.integers(1, 4))):
            col = int(rng.choice([0, 1, 2]))
            op = int(rng.choice(OPS))
            if col == 1:
                lit = ("str", (NAMES + [b"Nevada"])[int(rng.integers(0, len(NAMES) + 1))].decode())
            else:
                lit = ("int", int(rng.integers(-1, 11 if col == 0 else 6)))
            key = (col, op, lit)
            if key in seen:  # a repeated constraint takes the reference's step-wise cache instead
                continue
            seen.add(key)
            conj.append((op, ("sym", col + 1), lit))
        if conj:
            cnf.append(conj)
    return cnf


PROJS = [[0, 1, 2, 3, 4], [3], [1, 4], [], [4, 4, 0, 1, 2, 3], [0, 2], [2, 0, 3, 0]]


@pytest.mark.parametrize("n,deleted", [(1, None), (63, None), (64, 0.2), (65, None), (1000, 0.1), (70001, None),
                                       (70001, 0.3), (300_000, 0.05)])
def test_synthetic_cnf_matrix_vs_oracle(ctx, n, deleted):
    cols = synth(n, seed=n)
    dele = None if deleted is None else helpers.random_deleted(n, deleted, seed=n + 1)
    ot = oracle.Table(cols, dele)
    t = ctx.stage(cols, dele)
    dbm = None if dele is None else ctx.bitmap_upload(n, dele)
    regs = {c: helpers.index_registry(ctx, cols, t, c) for c in (0, 1, 2)}
    rng = np.random.default_rng(1000 + n)
    for trial in range(6):
        cnf = random_cnf(rng)
        nw, words = oracle.columnar_index_scan(ot, cnf)
        want_ids = oracle.words_to_positions(words)
        assert len(want_ids) == nw
        conj = helpers.index_conjuncts(regs, cnf, TYPES)
        proj = PROJS[(trial + n) % len(PROJS)]
        cur = ctx.cnf_cursor(t, conj, proj, deleted=dbm)
        ids, outs = cur.next(max(1, n))
        assert np.array_equal(ids, want_ids), (cnf, proj)
        for o, w in zip(outs, oracle.gather(ot, want_ids, proj)):
            assert np.array_equal(np.asarray(o).view(np.uint8), np.asarray(w).view(np.uint8)), (cnf, proj)


def test_synthetic_cnf_large_wide_projection(ctx):
    """2M rows, every column projected incl. the 32-byte string rows, a
    selective and a dense CNF: positions + rows equal to the oracle."""
    n = 2_000_000
    cols = synth(n, seed=5)
    ot = oracle.Table(cols)
    t = ctx.stage(cols)
    regs = {c: helpers.index_registry(ctx, cols, t, c) for c in (0, 1, 2)}
    for cnf in ([[(oracle.EQ, ("sym", 1), ("int", 3))], [(oracle.EQ, ("sym", 3), ("int", 2))]],
                [[(oracle.GE, ("sym", 2), ("str", "Iowa"))], [(oracle.NE, ("sym", 1), ("int", 7)),
                                                               (oracle.LT, ("sym", 3), ("int", 1))]]):
        _, words = oracle.columnar_index_scan(ot, cnf)
        want = oracle.words_to_positions(words)
        cur = ctx.cnf_cursor(t, helpers.index_conjuncts(regs, cnf, TYPES), [0, 1, 2, 3, 4])
        got_ids, got = [], [[] for _ in range(5)]
        while True:
            ids, outs = cur.next(65536)
            if len(ids) == 0:
                break
            got_ids.append(ids)
            for j, o in enumerate(outs):
                got[j].append(o)
        assert np.array_equal(np.concatenate(got_ids), want)
        for j, w in enumerate(oracle.gather(ot, want, [0, 1, 2, 3, 4])):
            assert np.array_equal(np.concatenate(got[j]).view(np.uint8), np.asarray(w).view(np.uint8))


# ------------------------------------------------- double-buffered cursor

@pytest.mark.parametrize("prefetch", [1, 0])
@pytest.mark.parametrize("sizes", [[1], [7], [64], [8192], [3, 100, 3, 100, 5000], [1000, 1, 1, 2000]])
def test_cursor_batches_equal_one_materialise(ctx, sizes, prefetch):
    """double-buffered (prefetch 1) and on-demand (0) delivery: batches of any
    size concatenate to the one-batch read, across a restart"""
    ctx.set_tuning("cursor_prefetch", prefetch)
    try:
        _batches_equal_one_read(ctx, sizes)
    finally:
        ctx.set_tuning("cursor_prefetch", 1)


def _batches_equal_one_read(ctx, sizes):
    n = 100_003
    cols = synth(n, seed=11)
    t = ctx.stage(cols)
    regs = {c: helpers.index_registry(ctx, cols, t, c) for c in (0, 1, 2)}
    cnf = [[(oracle.LT, ("sym", 1), ("int", 6))], [(oracle.NE, ("sym", 2), ("str", "Ohio"))]]
    conj = helpers.index_conjuncts(regs, cnf, TYPES)
    full_ids, full = ctx.cnf_cursor(t, conj, [4, 0, 3]).next(n)
    cur = ctx.cnf_cursor(t, conj, [4, 0, 3])
    for restart_at in (len(full_ids) // 3, None):
        got_ids, got = [], [[], [], []]
        k = 0
        while True:
            ids, outs = cur.next(sizes[k % len(sizes)])
            k += 1
            if len(ids) == 0:
                break
            got_ids.append(ids)
            for j in range(3):
                got[j].append(outs[j])
            if restart_at is not None and sum(len(x) for x in got_ids) >= restart_at:
                cur.restart()
                restart_at = None
                got_ids, got = [], [[], [], []]
        assert np.array_equal(np.concatenate(got_ids), full_ids)
        for j in range(3):
            assert np.array_equal(np.concatenate(got[j]), full[j])
        assert cur.stats()[0] == len(full_ids)
        cur.restart()
    # the bitmap cursor (mbx_cursor_open) delivers through the same buffers
    bm = ctx.bitmap_cnf(n, conj)
    bc = ctx.cursor(t, bm, [4, 0, 3])
    parts = []
    while True:
        ids, _ = bc.next(sizes[0])
        if len(ids) == 0:
            break
        parts.append(ids)
    assert np.array_equal(np.concatenate(parts), full_ids)


def test_empty_and_absent_value_cursor(ctx, mini):
    """a literal with no BitMapFile -> empty BitSet (Columnarfile.java:1124):
    the one-launch cursor is empty and next() returns no rows"""
    rows, _, t, regs = mini
    cnf = [[(oracle.EQ, ("sym", 4), ("int", 50))]]
    cur = ctx.cnf_cursor(t, helpers.index_conjuncts(regs, cnf, helpers.MINI_TYPES), [0, 3])
    assert cur.count == 0
    ids, outs = cur.next(10)
    assert len(ids) == 0 and all(len(o) == 0 for o in outs)


# ------------------------------------------------------- C++ mirror / CLI

BIN = os.path.join(helpers.ROOT, "minibase-columnar-database_amd", "host", "columnar_main")
DATA = os.path.join(helpers.ROOT, "tests", "golden", "minidata.tsv")


def test_cli_indexes_query_takes_the_one_launch_path():
    """host/columnar_main's ColumnarIndexScan (the C++ drop-in) runs every
    transcript indexes_query through mbx_cnf_cursor_open and prints the
    transcript's rows (R/phase3_output:3291-3463)."""
    cmds = [f"batchinsert {DATA} db cf 4"] + [f"index db cf {c} bitmap" for c in "ABCD"]
    cmds += [f"indexes_query db cf [A,B,C,D] {g['raw']} 10" for g in GOLD["indexes_query"]]
    cwd = tempfile.mkdtemp(prefix="mbx_cli_")
    p = subprocess.run([BIN], input="\n".join(cmds + ["exit"]) + "\n", capture_output=True, text=True, timeout=300,
                       cwd=cwd, env=dict(os.environ, MBX_TRACE="1"))
    assert p.returncode == 0, p.stderr[-2000:]
    one = [ln for ln in p.stderr.splitlines() if ln.startswith("trace: ColumnarIndexScan: one launch")]
    step = [ln for ln in p.stderr.splitlines() if ln.startswith("trace: ColumnarIndexScan: step-wise")]
    assert len(one) == len(GOLD["indexes_query"]) and not step, p.stderr[-2000:]
    for line, g in zip(one, GOLD["indexes_query"]):
        assert line.endswith(f"{g['count']} rows")
    for g in GOLD["indexes_query"]:
        for r in g["rows"]:
            assert ", ".join(str(x) for x in r) in p.stdout


def test_wide_rows_are_batched_by_bytes(m, ctx):
    """a cursor batch is capped at 64 MiB of buffer whatever max_rows asks
    (ADVICE r4): two char(256) columns are 8 + 2 x 256 bytes a row, so a
    256 Ki-row request returns 129,055 rows per call; every row arrives once,
    in position order, equal to the table's rows"""
    n = 300_001
    rng = np.random.default_rng(5)
    s0 = rng.integers(ord("a"), ord("z") + 1, (n, 256), dtype=np.uint8)
    s1 = rng.integers(ord("A"), ord("Z") + 1, (n, 256), dtype=np.uint8)
    k = rng.integers(0, 3, n, dtype=np.int32)
    cols = [(oracle.STRING, 256, s0), (oracle.STRING, 256, s1), (oracle.INTEGER, 4, k)]
    t = ctx.stage(cols)
    bms = ctx.index_build(t, 2, [("int", 0), ("int", 1)])
    cur = ctx.cnf_cursor(t, [[bms[0], bms[1]]], [0, 1])
    want = np.nonzero(k <= 1)[0]
    cap = (64 << 20) // (8 + 256 + 256)
    got_ids, got0, got1, sizes = [], [], [], []
    while True:
        ids, (a, b) = cur.next(262144)
        if len(ids) == 0:
            break
        sizes.append(len(ids))
        got_ids.append(ids), got0.append(a), got1.append(b)
    assert sizes[:-1] == [cap] * (len(sizes) - 1) and 0 < sizes[-1] <= cap
    assert np.array_equal(np.concatenate(got_ids), want)
    assert np.array_equal(np.concatenate(got0), s0[want]) and np.array_equal(np.concatenate(got1), s1[want])
    cur.close()
