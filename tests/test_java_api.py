"""The Java drop-ins declare the whole public API of the reference classes they
replace: every public constructor, method and field of
R/iterator/ColumnarFileScan, ColumnarColumnScan, ColumnarColumnsScan,
ColumnarNestedLoopJoins, R/index/ColumnIndexScan and ColumnarIndexScan, as
extracted into tests/golden/java_api.json by tests/golden/make_java_api.py.
No JDK exists on either box, so this parse is the compile-time guard: a
caller of the reference class (Query, NljQuery, DeleteQuery, MultiIndexQuery,
BitMapQuery) changes only the class name."""
import json
import os
import re

import pytest

import javaapi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with open(os.path.join(ROOT, "tests", "golden", "java_api.json")) as _f:
    REF = json.load(_f)


def dropin_api(rel):
    with open(os.path.join(ROOT, rel)) as f:
        return javaapi.public_api(f.read())


@pytest.mark.parametrize("cls", sorted(REF))
def test_constructors(cls):
    ref = REF[cls]
    got = dropin_api(ref["dropin"])
    assert got["class"] == "Gpu" + cls
    missing = [c for c in ref["ctors"] if c not in got["ctors"]]
    assert not missing, f"{ref['dropin']} lacks constructor(s) {missing} of {ref['source']}"


@pytest.mark.parametrize("cls", sorted(REF))
def test_methods(cls):
    ref = REF[cls]
    got = {(m["name"], tuple(m["params"])): m for m in dropin_api(ref["dropin"])["methods"]}
    for m in ref["methods"]:
        key = (m["name"], tuple(m["params"]))
        assert key in got, f"{ref['dropin']} lacks {m['returns']} {m['name']}({', '.join(m['params'])})"
        assert got[key]["returns"] == m["returns"], (key, got[key]["returns"], m["returns"])
        # a checked exception the reference method does not declare would not
        # compile in its callers
        if not m["throws"]:
            assert not got[key]["throws"], f"{ref['dropin']}: {m['name']}() must not declare checked exceptions"


@pytest.mark.parametrize("cls", sorted(REF))
def test_public_fields(cls):
    ref = REF[cls]
    got = {f["name"]: f["type"] for f in dropin_api(ref["dropin"])["fields"]}
    for f in ref["fields"]:
        assert got.get(f["name"]) == f["type"], f"{ref['dropin']} lacks public {f['type']} {f['name']}"


@pytest.mark.parametrize("cls", sorted(REF))
def test_extends_iterator(cls):
    with open(os.path.join(ROOT, REF[cls]["dropin"])) as f:
        src = f.read()
    assert re.search(r"class\s+Gpu%s\s+extends\s+Iterator\b" % cls, src)


def test_fixture_covers_every_mirrored_class():
    assert sorted(REF) == ["ColumnIndexScan", "ColumnarColumnScan", "ColumnarColumnsScan", "ColumnarFileScan",
                           "ColumnarIndexScan", "ColumnarNestedLoopJoins"]
    # the two bitmap-only constructors BitMapQuery / ColumnarIndexScan call
    assert len(REF["ColumnarIndexScan"]["ctors"]) == 2 and len(REF["ColumnIndexScan"]["ctors"]) == 2


def test_parser_folds_c_style_arrays():
    api = javaapi.public_api("""
        public class X extends Iterator {
          public FldSpec perm_mat[];  // comment (with parens)
          /* public int hidden(int a) */
          public X(final String s, AttrType in1[], short[] b, java.util.List<Map<String, Integer>> m) throws E { if (x) { } }
          public static short[] f(int a) { return null; }
          private int g() { return 0; }
        }""")
    assert api["ctors"] == [["String", "AttrType[]", "short[]", "java.util.List<Map<String,Integer>>"]]
    assert [m["name"] for m in api["methods"]] == ["f"] and api["methods"][0]["returns"] == "short[]"
    assert api["fields"] == [{"name": "perm_mat", "type": "FldSpec[]"}]
