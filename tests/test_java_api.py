"""The Java drop-ins declare the whole public API of the reference classes they
replace: every public constructor, method and field of
R/iterator/ColumnarFileScan, ColumnarColumnScan, ColumnarColumnsScan,
ColumnarNestedLoopJoins, R/index/ColumnIndexScan and ColumnarIndexScan, as
extracted into tests/golden/java_api.json by tests/golden/make_java_api.py,
with every constructor's and method's `throws` list: a drop-in may declare
only checked exceptions the reference declaration covers.
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


with open(os.path.join(ROOT, "tests", "golden", "java_symbols.json")) as _f:
    SYMBOLS = json.load(_f)
# java.lang / java.io exceptions the Minibase classes extend or throw
JDK_SUPER = {"IOException": "Exception", "RuntimeException": "Exception", "Exception": "Throwable",
             "NullPointerException": "RuntimeException", "IllegalArgumentException": "RuntimeException",
             "IllegalStateException": "RuntimeException", "Throwable": None}


def supers(name):
    """name and its superclasses (simple names), from the reference's class
    table (tests/golden/java_symbols.json) and the JDK's few"""
    out, cur = [], name.split(".")[-1]
    while cur and cur not in out:
        out.append(cur)
        if cur in JDK_SUPER:
            cur = JDK_SUPER[cur]
            continue
        cands = [c for c in SYMBOLS.values() if c.get("name") == cur and c.get("kind") == "class"]
        ext = {e for c in cands for e in c.get("extends", [])}
        assert len(ext) <= 1, (cur, ext)
        cur = ext.pop() if ext else None
    return out


def unchecked(name):
    return "RuntimeException" in supers(name)


def undeclared(got, ref):
    """checked exceptions in `got` that no exception of `ref` covers (a caller
    of the reference declaration would not compile against them)"""
    return [t for t in got if not unchecked(t) and not any(r.split(".")[-1] in supers(t) for r in ref)]


def test_exception_hierarchy_resolves():
    assert supers("FileScanException") == ["FileScanException", "ChainException", "Exception", "Throwable"]
    assert supers("heap.InvalidTupleSizeException")[:2] == ["InvalidTupleSizeException", "ChainException"]
    assert undeclared(["Exception"], ["IOException", "FileScanException"]) == ["Exception"]
    assert undeclared(["FileScanException", "NullPointerException"], ["Exception"]) == []


@pytest.mark.parametrize("cls", sorted(REF))
def test_constructor_throws_within_the_reference(cls):
    """each drop-in constructor declares no checked exception outside the
    reference constructor's `throws` list (a `throws Exception`
    constructor breaks a caller that declares only the reference's list)"""
    ref = REF[cls]
    got = dropin_api(ref["dropin"])
    for params, rthrows in zip(ref["ctors"], ref["ctor_throws"]):
        i = got["ctors"].index(params)
        extra = undeclared(got["ctor_throws"][i], rthrows)
        assert not extra, f"{ref['dropin']} ({', '.join(params)}) throws {extra} beyond {ref['source']}'s {rthrows}"


@pytest.mark.parametrize("cls", sorted(REF))
def test_method_throws_within_the_reference(cls):
    ref = REF[cls]
    got = {(m["name"], tuple(m["params"])): m for m in dropin_api(ref["dropin"])["methods"]}
    for m in ref["methods"]:
        g = got[(m["name"], tuple(m["params"]))]
        extra = undeclared(g["throws_list"], m["throws_list"])
        assert not extra, f"{ref['dropin']}: {m['name']}() throws {extra} beyond the reference's {m['throws_list']}"


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
    assert api["ctor_throws"] == [["E"]] and api["methods"][0]["throws_list"] == []
    assert [m["name"] for m in api["methods"]] == ["f"] and api["methods"][0]["returns"] == "short[]"
    assert api["fields"] == [{"name": "perm_mat", "type": "FldSpec[]"}]
