"""The Java drop-ins resolve against the reference classes (no JDK here or on
the GPU box, so javac cannot check them): every `new C(...)`, method call and
field read they make on a reference class exists there with that arity,
static-ness and visibility, imports name real classes, and every abstract
method of the reference superclass (iterator.Iterator's get_next / close,
R/iterator/Iterator.java) is implemented.  The table is
tests/golden/java_symbols.json, extracted from the reference sources by
tests/golden/make_java_symbols.py (tests/javarefs.py is the reader)."""
import json
import os
import shutil

import pytest

import helpers
import javarefs

JAVA = os.path.join(helpers.ROOT, "java")
REF_SRC = "/root/reference/minijava/src"


@pytest.fixture(scope="module")
def table():
    with open(os.path.join(helpers.GOLDEN, "java_symbols.json")) as f:
        return json.load(f)


def test_every_drop_in_reference_resolves(table):
    refs, bad = javarefs.check(table, JAVA)
    assert not bad, "\n".join(f"{b['file']}:{b['line']}: {b['what']}: {b['why']}" for b in bad)
    seen = {r["what"] for r in refs}
    # the members VERDICT r4 names, among ~400 resolved uses
    for must in ["iterator.TupleUtils.setup_op_tuple(7 args)", "columnar.Columnarfile.getAttributeType(1 args)",
                 "bufmgr.FrameDesc.pin_count(0 args)", "bufmgr.FrameDesc.dirty", "bufmgr.FrameDesc.pageNo",
                 "bufmgr.BufMgr.flushPage(1 args)", "bufmgr.BufMgr.frameTable(0 args)",
                 "bitmap.BitMapFile.getBitSet(0 args)", "columnar.Columnarfile.getMarkedDeleted(0 args)",
                 "global.SystemDefs.JavabaseBM", "implements abstract iterator.Iterator.get_next(0 args)",
                 "implements abstract iterator.Iterator.close(0 args)"]:
        assert must in seen, must
    assert len(refs) >= 400


MUTATIONS = [
    # (drop-in, text, replacement, expected failure)
    ("index/GpuColumnarIndexScan.java", ".getBitSet()", ".getBitset()", "bitmap.BitMapFile.getBitset(0 args)"),
    ("bufmgr/GpuFlush.java", "bm.flushPage(new PageId(f.pageNo.pid))", "bm.flushPage(new PageId(f.pageNo.pid), 1)",
     "bufmgr.BufMgr.flushPage(2 args)"),
    ("bufmgr/GpuFlush.java", "f.pin_count()", "f.pin_cnt()", "bufmgr.FrameDesc.pin_cnt(0 args)"),
    ("bufmgr/GpuFlush.java", "!f.dirty", "!f.isDirty", "bufmgr.FrameDesc.isDirty"),
    ("bufmgr/GpuFlush.java", "bm.frameTable()", "bm.frmeTable", "bufmgr.BufMgr.frmeTable"),  # private field
    ("columnar/GpuTables.java", "import heap.Tuple;", "import heap.Tuples;", "import heap.Tuples"),
    ("columnar/GpuTables.java", "f.getAttributeTypes()", "Columnarfile.getAttributeTypes()",
     "columnar.Columnarfile.getAttributeTypes(0 args)"),  # instance method on the class
    ("columnar/GpuTables.java", "new Columnarfile(name)", "new Columnarfile(name, 3)", "new columnar.Columnarfile(2 args)"),
    ("index/GpuColumnIndexScan.java", "TupleUtils.setup_op_tuple(", "TupleUtils.setupOpTuple(",
     "iterator.TupleUtils.setupOpTuple(7 args)"),
    ("iterator/GpuColumnarFileScan.java", "public Tuple get_next()", "public Tuple getNext()",
     "implements abstract iterator.Iterator.get_next(0 args)"),
    # `f` is a Columnarfile in stageDecoded and a BitMapFile in bitmap(): the use's own method decides
    ("columnar/GpuTables.java", "f.getAttrSizes()", "f.getAttrSize()", "columnar.Columnarfile.getAttrSize(0 args)"),
    ("columnar/GpuTables.java", "f.getBitSet().toLongArray()", "f.getBitset().toLongArray()",
     "bitmap.BitMapFile.getBitset(0 args)"),
]


@pytest.mark.parametrize("path,old,new,expect", MUTATIONS, ids=[m[3] for m in MUTATIONS])
def test_a_misspelled_use_fails(table, tmp_path, path, old, new, expect):
    """each deliberate error in a copy of the tree is reported, and only it"""
    root = tmp_path / "java"
    shutil.copytree(JAVA, root)
    p = root / path
    src = p.read_text()
    assert old in src, (path, old)
    p.write_text(src.replace(old, new, 1))
    _, bad = javarefs.check(table, str(root))
    assert [b["what"] for b in bad] == [expect], bad


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="the reference tree exists only in the build container")
def test_fixture_is_current(table):
    """the committed table equals a fresh extraction from the reference"""
    fresh = javarefs.tree_symbols(REF_SRC)
    for rec in fresh.values():
        rec["source"] = "R/" + rec["source"]
    assert json.loads(json.dumps(fresh)) == table


def test_decoded_staging_sizes_are_long():
    """GpuTables.stageDecoded (the fallback when a dirty frame is pinned)
    sizes and indexes its direct ByteBuffers through long products: no int
    `nrows * width` / `p * width` remains, and a column over
    Integer.MAX_VALUE bytes is refused by columnBytes with
    FileScanException (the JNI side's own check is
    test_jni_harness.test_table_stage_refuses_a_column_past_2_gib)."""
    src = javarefs.strip(open(os.path.join(JAVA, "columnar", "GpuTables.java")).read())
    body = src[src.index("static long stageDecoded"):src.index("static int columnBytes")]
    assert "columnBytes(name, c, nrows, w[c])" in body
    import re
    ints = re.findall(r"(?<!\(long\) )\b(?:nrows|p)\s*\*\s*(?:w\[c\]|4)\b", body)
    assert not ints, ints
    cb = src[src.index("static int columnBytes"):]
    cb = cb[:cb.index("\n  }\n")]
    assert "nrows * (long) width" in cb and "Integer.MAX_VALUE" in cb and "FileScanException" in cb
