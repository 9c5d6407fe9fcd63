"""The C++ operator mirror + command driver (host/columnar_main) replays the
reference's recorded session over minidata and prints the same rows and
counts (R/phase3_output).  The driver runs every scan on the GPU."""
import os
import subprocess

import pytest

import helpers
import oracle

pytestmark = pytest.mark.gpu
GOLD = helpers.load_golden()
BIN = os.path.join(helpers.ROOT, "minibase-columnar-database_amd", "host", "columnar_main")
DATA = os.path.join(helpers.ROOT, "tests", "golden", "minidata.tsv")


def run_session(cmds, cwd=None, setup=True):
    """One driver process; DB files ("db") live in cwd (a fresh temp dir by
    default), as the reference keeps its DB file in the working directory."""
    if cwd is None:
        import tempfile
        cwd = tempfile.mkdtemp(prefix="mbx_cli_")
    pre = [f"batchinsert {DATA} db cf 4"] + [f"index db cf {c} bitmap" for c in "ABCD"] if setup else []
    script = "\n".join(pre + cmds + ["exit"]) + "\n"
    p = subprocess.run([BIN], input=script, capture_output=True, text=True, timeout=300, cwd=cwd)
    assert p.returncode == 0, p.stderr[-2000:]
    return p.stdout


def blocks(out):
    """[(header, rows, count)] for every result block the driver printed.
    Each command's output follows its "> " prompt: the column header, the
    rows, a blank line, then the stars / "Total Results Count" footer."""
    res = []
    for chunk in out.split("> ")[1:]:
        if "Total Results Count By Query:" not in chunk:
            continue
        lines = chunk.split("\n")
        end = lines.index("")
        n = int([ln for ln in lines if ln.startswith("Total Results Count By Query:")][0].split(":")[1])
        res.append((lines[0].strip(), lines[1:end], n))
    return res


def test_batchinsert_record_count():
    out = run_session([])
    assert "Record count: 500" in out
    assert "java.lang.Exception" not in out


def test_indexes_query_transcript():
    """indexes_query results at R/phase3_output:3308-3463 (BM and BT terms)."""
    cmds = [f"indexes_query db cf [A,B,C,D] {g['raw']} 10" for g in GOLD["indexes_query"]]
    out = run_session(cmds)
    assert "java.lang.Exception" not in out, out[-3000:]
    got = blocks(out)
    assert len(got) == len(GOLD["indexes_query"])
    for (header, rows, n), g in zip(got, GOLD["indexes_query"]):
        assert header == "A, B, C, D"
        assert n == g["count"]
        assert rows == [", ".join(str(x) for x in r) for r in g["rows"]]


@pytest.mark.parametrize("access", ["FILESCAN", "COLUMNSCAN", "BITMAP"])
def test_query_access_methods(access):
    """`query db cf [A,B,C,D] {C,=,6} 100 <ACCESS>`: 57 rows,
    identical across the three GPU access paths and to the oracle."""
    rows = helpers.load_minidata()
    out = run_session([f"query db cf [A,B,C,D] {{C,=,6}} 100 {access}",
                       f"query db cf [D,A] {{A,>=,South_Dakota}} 100 {access}",
                       f"query db cf [C] {{C,!=,6}} 100 {access}"])
    assert "java.lang.Exception" not in out, out[-3000:]
    (h1, r1, n1), (h2, r2, n2), (h3, r3, n3) = blocks(out)
    assert n1 == 57 and r1 == [f"{a}, {b}, {c}, {d}" for a, b, c, d in rows if c == 6]
    assert h2 == "D, A" and r2 == [f"{d}, {a}" for a, b, c, d in rows if a >= "South_Dakota"]
    assert n3 == 443 and h3 == "C"


def test_duplicate_constraint_quirk_matches_oracle():
    """A repeated identical constraint takes the step-wise path that keeps the
    reference's BitSet aliasing (ColumnarIndexScan.java:147-172)."""
    cnf_s = "{(A,=,South_Dakota,BM)|(B,=,South_Dakota,BM)}^{(A,=,South_Dakota,BM)|(C,>=,6,BM)}"
    out = run_session([f"indexes_query db cf [A,B,C,D] {cnf_s} 10"])
    (_, rows_out, n), = blocks(out)
    rows = helpers.load_minidata()
    t = oracle.Table(helpers.minidata_columns(rows))
    n_o, w = oracle.columnar_index_scan(t, helpers.parse_cnf_string(cnf_s))
    pos = oracle.words_to_positions(w)
    assert n == n_o
    assert rows_out == [", ".join(str(x) for x in rows[p]) for p in pos]


def test_bmj_bitsets_through_indexes_query():
    """The BitSets bmj printed (R/phase3_output:24797-25491) via the driver."""
    rows = helpers.load_minidata()
    cmds, want = [], []
    for g in GOLD["bitsets"]:
        cnf = "^".join("{" + "|".join(f"({c},{o},{v},BM)" for c, o, v, *_ in conj) + "}" for conj in g["cnf"])
        cmds.append(f"indexes_query db cf [A,B,C,D] {cnf} 10")
        want.append([", ".join(str(x) for x in rows[p]) for p in g["positions"]])
    out = run_session(cmds)
    got = blocks(out)
    assert [r for _, r, _ in got] == want


def test_db_file_persists_across_processes(tmp_path):
    """batchinsert + index in one process write the Minibase DB file; a second
    process opens it, stages the Columnarfile with the GPU page decoder, reads
    the BitMapFiles back and answers like the first (the reference's session
    spans separate JVM runs the same way, R/phase3_output:13-22)."""
    q = [f"indexes_query db cf [A,B,C,D] {GOLD['indexes_query'][0]['raw']} 10",
         "query db cf [A,B,C,D] {C,=,6} 100 FILESCAN", "query db cf [A,B,C,D] {C,=,6} 100 BITMAP"]
    first = blocks(run_session(q, cwd=str(tmp_path)))
    assert (tmp_path / "db").exists()
    second = blocks(run_session(q, cwd=str(tmp_path), setup=False))
    assert first == second
    assert second[0][2] == GOLD["indexes_query"][0]["count"] and second[1][2] == 57 and second[2][2] == 57
    out = run_session(["query nodb cf [A] {C,=,6} 100 FILESCAN"], cwd=str(tmp_path), setup=False)
    assert "Database does not exist." in out


def test_join_commands_replay_transcript(tmp_path):
    """Every successful `nlj` / `bmj` run of the reference session
    (R/phase3_output), replayed through the driver over cf, cf1, cf2 (all
    `batchinsert minidata.txt`, bitmap indexes on every column): same rows in
    the same order, same inner-table passes, same statistics (bar the
    "Tuple Size: 10" runs an earlier ColumnarColumnsScan printed), same BitSets."""
    import sys
    sys.path.insert(0, os.path.join(helpers.ROOT, "tests", "golden"))
    import make_golden
    runs = [j for j in GOLD["joins"] if j["error"] is None and j["count"] is not None]
    setup = [f"batchinsert {DATA} db {cf} 4" for cf in ("cf", "cf1", "cf2")]
    setup += [f"index db {cf} {c} bitmap" for cf in ("cf", "cf1", "cf2") for c in "ABCD"]
    out = run_session(setup + [r["raw"] for r in runs], cwd=str(tmp_path), setup=False)
    chunks = out.split("> ")[1:]
    assert len(chunks) >= len(setup) + len(runs)
    for r, chunk in zip(runs, chunks[len(setup):]):
        body = chunk.split("\n")
        got = make_golden.parse_join(r["cmd"], r["raw"], r["raw"].split(), body, r["line"])
        assert got["error"] is None, (r["raw"], chunk[:500])
        assert got["header"] == r["header"], r["raw"]
        assert got["rows"] == r["rows"], r["raw"]
        assert got["count"] == r["count"]
        if r["cmd"] == "nlj":
            assert got["passes"] == r["passes"], r["raw"]
            for k, v in r["stats"].items():
                if r["stats"]["Tuple Size"] == 10 and k in ("Tuple Size", "Number of Tuples Buffer Can Hold"):
                    continue
                assert got["stats"][k] == v, (r["raw"], k)
        else:
            assert got["bitsets"] == r["bitsets"], r["raw"]


def test_delete_query_md_and_pd(tmp_path):
    """delete_query (R/input/DeleteQuery.java): `md` marks the scan's positions
    in cf.md, later queries skip them; `pd` purges (records and BitSets) and
    clears cf.md.  Counts checked against the oracle over minidata."""
    rows = helpers.load_minidata()
    out = run_session(["delete_query db cf {C,=,6} 10 FILESCAN md",
                       "query db cf [A,C] {C,!=,100} 100 FILESCAN",
                       "query db cf [C] {C,=,6} 100 BITMAP",
                       "delete_query db cf {D,=,3} 10 BITMAP pd",
                       "query db cf [A,B,C,D] {D,!=,3} 100 FILESCAN",
                       "indexes_query db cf [A,C,D] {(C,>=,0,BM)} 10"], cwd=str(tmp_path))
    assert "java.lang.Exception" not in out, out[-3000:]
    chunks = out.split("> ")
    md_chunk = [c for c in chunks if "EXTRA METAINFO" in c]
    assert len(md_chunk) == 2
    n6 = sum(1 for r in rows if r[2] == 6)
    six = [i for i, r in enumerate(rows) if r[2] == 6]
    assert md_chunk[0].split("\n")[1].strip() == str(500 - n6)
    assert md_chunk[0].split("\n")[2].strip() == "{" + ", ".join(map(str, six)) + "}"
    (_, r1, n1), (_, r2, n2), (_, r3, n3), (_, r4, n4) = blocks(out)
    assert n1 == 500 - n6 and n2 == 0
    gone = {i for i, r in enumerate(rows) if r[2] == 6 or r[3] == 3}
    assert md_chunk[1].split("\n")[1].strip() == str(500 - len(gone))
    assert md_chunk[1].split("\n")[2].strip() == "{}"
    assert n3 == 500 - len(gone)
    assert r3 == [f"{a}, {b}, {c}, {d}" for i, (a, b, c, d) in enumerate(rows) if i not in gone]
    assert n4 == 500 - len(gone)


def test_columns_scan_mirror_matches_oracle():
    """iterator::ColumnarColumnsScan (R/iterator/ColumnarColumnsScan.java), the
    outer/inner iterator NljQuery builds for COLUMNSCAN (NljQuery.java:269),
    driven directly: rows and positions vs the oracle over minidata, and the
    reference's two quirks -- a string column past the string prefix of
    colNos throws ArrayIndexOutOfBounds (:77-82), get_next_tid over columns
    whose first and last differ throws "Invalid RID" at the first match (:219)."""
    rows = helpers.load_minidata()
    t = oracle.Table(helpers.minidata_columns(rows))
    cnf_s = "{(C,=,6)|(A,>=,South_Dakota)}^{(D,!=,3)}"
    cnf = helpers.parse_cnf_string(cnf_s)
    n_o, _, ids_o = oracle.filescan(t, cnf)
    out = run_session([f"columnsscan db cf [A,C,D] {cnf_s} [A,B,C,D]",
                       f"columnsscan db cf [A,D,C] {cnf_s} [D,A]",
                       "columnsscan db cf [C] {(C,=,6)} [C] tid",
                       f"columnsscan db cf [C,A,D] {cnf_s} [A]",
                       f"columnsscan db cf [A,C,D] {cnf_s} [A] tid"])
    chunks = out.split("> ")[1:][5:]  # after batchinsert + 4 index commands
    (h1, r1, n1), (h2, r2, n2), (h3, r3, n3) = blocks("> " + "> ".join(chunks[:3]))
    assert n1 == n_o and h1 == "A, B, C, D"
    assert r1 == [", ".join(str(x) for x in rows[p]) for p in ids_o]
    assert h2 == "D, A" and r2 == [f"{rows[p][3]}, {rows[p][0]}" for p in ids_o] and n2 == n_o
    six = [i for i, r in enumerate(rows) if r[2] == 6]
    assert n3 == len(six) and r3 == [str(p) for p in six]
    assert "java.lang.Exception" in chunks[3] and "out of bounds" in chunks[3]
    assert "java.lang.Exception: Invalid RID" in chunks[4]
