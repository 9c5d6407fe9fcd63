"""CPU: the C++ mirror's Jtuple accessors (R/heap/Tuple.java:194-343) -- the
all-int bulk copy get_next() uses rejects exactly the fields setIntFld does
(tests/host_unit/tuple_test.cpp, built against host/minibase.o)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "minibase-columnar-database_amd")


def test_tuple_accessors(tmp_path):
    obj = os.path.join(PKG, "host", "minibase.o")
    lib = os.path.join(PKG, "libmbx.so")
    if not (os.path.exists(obj) and os.path.exists(lib)):
        pytest.skip("host mirror not built (__graft_entry__.build())")
    exe = str(tmp_path / "tuple_test")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "host_unit", "tuple_test.cpp"),
                    obj, "-L" + PKG, "-lmbx", "-Wl,-rpath," + PKG], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "TUPLE_TEST_OK" in r.stdout, r.stdout + r.stderr
