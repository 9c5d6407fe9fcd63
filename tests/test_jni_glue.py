"""The JNI glue (jni/mbx_jni.c) through a C compiler, with no JDK in this
image: jni/jni_min/jni.h declares exactly the JNIEnv functions the glue
calls, with the JNI specification's C prototypes, so gcc type-checks every
call (argument counts and types, return types, primitive array element
pointers) and every C-ABI call against include/*.h.  Plus the pairing rules
a compiler cannot see: every Get<T>ArrayElements / GetStringUTFChars is
released in the same function (or, for CondExpr strings, by
strings_release)."""
import os
import re
import shutil
import subprocess

import pytest

import helpers

JNI = os.path.join(helpers.ROOT, "jni")
GLUE = os.path.join(JNI, "mbx_jni.c")
MIN = os.path.join(JNI, "jni_min", "jni.h")


def _gcc():
    g = shutil.which("gcc")
    if not g:
        pytest.skip("no gcc")
    return g


@pytest.mark.parametrize("flags", [["-fsyntax-only"], ["-O2", "-c", "-fPIC", "-o", os.devnull]])
def test_glue_compiles_warning_free(flags):
    p = subprocess.run([_gcc(), "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.dirname(MIN)] + flags +
                       [GLUE], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


def _strip_comments(src):
    return re.sub(r"/\*.*?\*/", "", src, flags=re.S)


def test_min_header_declares_exactly_the_functions_used():
    used = set(re.findall(r"\(\*env\)->(\w+)\(", _strip_comments(open(GLUE).read())))
    hdr = _strip_comments(open(MIN).read())
    body = hdr[hdr.index("struct JNINativeInterface_ {"):]
    declared = set(re.findall(r"\(\*(\w+)\)\(JNIEnv \*env", body))
    assert used == declared, (sorted(used - declared), sorted(declared - used))


def _functions(src):
    """top-level function bodies: name -> text"""
    out, i = {}, 0
    for mt in re.finditer(r"^[A-Za-z].*?\b(\w+)\s*\([^;{]*?\)\s*\{", src, flags=re.M | re.S):
        if mt.start() < i:
            continue
        depth, j = 0, mt.end() - 1
        while True:
            if src[j] == "{":
                depth += 1
            elif src[j] == "}":
                depth -= 1
                if depth == 0:
                    break
            j += 1
        out[mt.group(1)] = src[mt.end():j]
        i = j
    return out


def test_borrowed_arrays_and_strings_are_released():
    fns = _functions(_strip_comments(open(GLUE).read()))
    assert len(fns) > 50
    # helpers that borrow for their caller, and the helper that hands back
    pairs = {"cnf_args_get": "cnf_args_release"}
    for name, body in fns.items():
        for kind in ("Int", "Short", "Long"):
            g = len(re.findall(rf"->Get{kind}ArrayElements\(", body))
            r = len(re.findall(rf"->Release{kind}ArrayElements\(", body))
            if name in pairs:
                rel = fns[pairs[name]]
                assert g == len(re.findall(rf"->Release{kind}ArrayElements\(", rel)), (name, kind)
            elif name not in pairs.values():
                assert g == r, (name, kind, g, r)
        g = len(re.findall(r"->GetStringUTFChars\(", body))
        r = len(re.findall(r"->ReleaseStringUTFChars\(", body))
        if name == "operand_of":    # CondExpr literals: kept until strings_release after the C-ABI call
            assert g == 1 and r == 0 and "ss->js[ss->n] = js" in body
        elif name == "strings_release":
            assert g == 0 and r == 1
        else:
            assert g == r, (name, g, r)
    # every function that borrows through a helper hands back
    for name, body in fns.items():
        if "cnf_of(" in body and name != "cnf_of":
            assert "strings_release(" in body, name
        for get, rel in pairs.items():
            if get + "(" in body and name != get:
                assert body.count(rel + "(") >= body.count(get + "("), name
