"""The C-ABI boundary: libmbx.so loads and exports every entry point that
include/mbx.h declares; no compute is attempted without a GPU."""
import os
import re

import pytest

import helpers
import mbx_pkg

HEADERS = [os.path.join(helpers.ROOT, "include", h) for h in sorted(os.listdir(os.path.join(helpers.ROOT, "include")))
           if h.endswith(".h")]


def declared_functions():
    out = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        out |= set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(mbx_[a-z_0-9]+)\s*\(", src, flags=re.M))
    return sorted(out)


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ["mbx_init", "mbx_table_stage", "mbx_plan_compile", "mbx_scan_count", "mbx_scan_bitmap",
                 "mbx_bitmap_cnf", "mbx_materialize", "mbx_cursor_next", "mbx_scan_aggregate", "mbx_db_open",
                 "mbx_db_stage", "mbx_db_columnar_insert"]:
        assert must in fns


def test_library_exports_every_declared_symbol():
    m = mbx_pkg.load()
    L = m.lib()
    missing = [f for f in declared_functions() if not hasattr(L, f)]
    assert not missing, missing
    assert sorted(m.mbx.EXPORTS) == declared_functions()
    assert L.mbx_abi_version() == 1


def test_library_is_built_for_gfx950():
    so = os.path.join(mbx_pkg.PKG_DIR, "libmbx.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data


def test_no_gpu_fails_loudly():
    """Without a visible MI355X the executor refuses to run (no CPU fallback)."""
    m = mbx_pkg.load()
    if m.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(m.MbxError) as e:
        m.Context(0)
    assert e.value.code == m.mbx.E_DEVICE
    assert "no CPU fallback" in str(e.value)


def test_null_arguments_are_rejected_without_a_device():
    m = mbx_pkg.load()
    L = m.lib()
    assert L.mbx_sync(None) == m.mbx.E_INVALID
    assert b"null" in L.mbx_last_error()
    assert L.mbx_table_free(None) == 0 and L.mbx_bitmap_free(None) == 0


def test_jni_glue_covers_the_java_side_and_calls_only_the_boundary():
    """jni/mbx_jni.c cannot be compiled here (no JDK): check statically that
    every `native` method of java/global/Native.java has its
    Java_global_Native_<name> implementation, that the glue defines nothing
    else, and that every mbx_* function it calls is declared by include/*.h
    (and so exported by libmbx.so, test above)."""
    root = helpers.ROOT
    java = open(os.path.join(root, "java", "global", "Native.java")).read()
    natives = set(re.findall(r"\bnative\s+[\w\[\]<>]+\s+(\w+)\s*\(", java))
    glue = open(os.path.join(root, "jni", "mbx_jni.c")).read()
    impl = set(re.findall(r"JNICALL\s+Java_global_Native_(\w+)\s*\(", glue))
    assert natives and natives == impl, (sorted(natives - impl), sorted(impl - natives))
    calls = set(re.findall(r"\b(mbx_[a-z_0-9]+)\s*\(", re.sub(r"/\*.*?\*/", "", glue, flags=re.S)))
    undeclared = sorted(calls - set(declared_functions()))
    assert not undeclared, undeclared
    # the drop-ins' constructor / method / field lists: tests/test_java_api.py
    # every native the Java drop-ins call is declared by Native.java
    called = set()
    for d, _, files in os.walk(os.path.join(root, "java")):
        for f in files:
            called |= set(re.findall(r"\bNative\.(\w+)\(", open(os.path.join(d, f)).read()))
    assert called <= natives, sorted(called - natives)
