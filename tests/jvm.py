"""ctypes side of the JNI harness (tests/jni_harness/): Java objects built as
the reference lays them out, Java_global_Native_* calls through the real glue
(jni/mbx_jni.c) into libmbx.so, pending exceptions surfaced as JavaException,
and every call checked for unreleased borrows and JNI violations."""
import ctypes
import os

import helpers
import oracle

HERE = os.path.join(helpers.ROOT, "tests", "jni_harness")
LIB = os.path.join(HERE, "libmbx_jni_harness.so")
V, I32, I64, F32, C = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_char_p

# R/global/AttrType.java:10-14, R/global/IndexType.java:10-13, R/iterator/RelSpec.java:14
ATTR_STRING, ATTR_INTEGER, ATTR_REAL, ATTR_SYMBOL = 0, 1, 2, 3
INDEX_BITMAP = 3
REL_OUTER = 0


class Ref(int):
    """a Java reference (object handle) as opposed to a Java int"""


class JavaException(Exception):
    def __init__(self, cls, msg):
        super().__init__(f"{cls}: {msg}")
        self.cls, self.msg = cls, msg


def mutf8_decode(b):
    """modified UTF-8 (CESU-8 surrogate pairs, C0 80 for U+0000) -> str"""
    s = bytes(b).replace(b"\xc0\x80", b"\x00").decode("utf-8", "surrogatepass")
    return s.encode("utf-16-le", "surrogatepass").decode("utf-16-le")


class JVM:
    def __init__(self):
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} not built (make -C tests/jni_harness)")
        L = ctypes.CDLL(LIB)
        for name, res, args in [
                ("jh_env", V, []), ("jh_new", V, [C]), ("jh_set_int", I32, [V, C, I32]),
                ("jh_set_float", I32, [V, C, F32]), ("jh_set_obj", I32, [V, C, V]),
                ("jh_string", V, [C, I32]), ("jh_string_utf", V, [V]), ("jh_string_len", I32, [V]),
                ("jh_array", V, [ctypes.c_char, I32, V, C]), ("jh_array_set", I32, [V, I32, V]),
                ("jh_array_get", V, [V, I32]), ("jh_array_type", ctypes.c_char, [V]), ("jh_array_len", I32, [V]),
                ("jh_array_data", V, [V]), ("jh_direct_buffer", V, [V, I64]), ("jh_pending", V, []),
                ("jh_clear", None, []), ("jh_class_name", C, [V]), ("jh_exception_message", V, [V]),
                ("jh_exception_cause", V, [V]), ("jh_outstanding", I32, []), ("jh_violations", I32, []),
                ("jh_last_violation", C, []), ("jh_reset", None, [])]:
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        self.L = L
        self.env = L.jh_env()
        self.keep = []   # host memory behind direct buffers

    # ---- objects -----------------------------------------------------------
    def new(self, cls, **fields):
        o = Ref(self.L.jh_new(cls.encode()))
        assert o, cls
        for k, v in fields.items():
            if v is None or isinstance(v, Ref):
                assert self.L.jh_set_obj(o, k.encode(), v) == 0, k
            elif isinstance(v, float):
                assert self.L.jh_set_float(o, k.encode(), v) == 0, k
            elif isinstance(v, int):
                assert self.L.jh_set_int(o, k.encode(), v) == 0, k
            else:
                raise TypeError(k)
        return o

    def string(self, s):
        b = s if isinstance(s, bytes) else oracle.java_mutf8(s)
        return Ref(self.L.jh_string(b, len(b)))

    def array(self, et, values):
        import numpy as np
        dt = {"I": np.int32, "J": np.int64, "S": np.int16, "B": np.int8, "F": np.float32}[et]
        a = np.ascontiguousarray(values, dtype=dt)
        return Ref(self.L.jh_array(et.encode(), len(a), a.ctypes.data if len(a) else None, None))

    def object_array(self, items, cls="java/lang/Object"):
        a = Ref(self.L.jh_array(b"L", len(items), None, cls.encode()))
        for i, x in enumerate(items):
            self.L.jh_array_set(a, i, x)
        return a

    def direct_buffer(self, arr):
        self.keep.append(arr)
        return Ref(self.L.jh_direct_buffer(arr.ctypes.data, arr.nbytes))

    def attr_type(self, t):
        return self.new("global/AttrType", attrType=t)

    def fldspec(self, k):
        return self.new("iterator/FldSpec", relation=self.new("iterator/RelSpec", key=REL_OUTER), offset=k)

    def condexpr(self, op, a, b, index=None):
        """new CondExpr() (R/iterator/CondExpr.java:45-56) filled the way
        Query.buildQueryCondExpr / MultiIndexQuery do: an operand is
        ("sym", field) | ("int", v) | ("real", f) | ("str", s)"""
        e = self.new("iterator/CondExpr", op=self.new("global/AttrOperator", attrOperator=op),
                     operand1=self.new("iterator/Operand"), operand2=self.new("iterator/Operand"))
        for tname, oname, (kind, v) in (("type1", "operand1", a), ("type2", "operand2", b)):
            od = Ref(self.L.jh_new(b"iterator/Operand"))
            if kind == "sym":
                t = ATTR_SYMBOL
                self.L.jh_set_obj(od, b"symbol", self.fldspec(v))
            elif kind == "int":
                t = ATTR_INTEGER
                self.L.jh_set_int(od, b"integer", int(v))
            elif kind == "real":
                t = ATTR_REAL
                self.L.jh_set_float(od, b"real", float(v))
            else:
                t = ATTR_STRING
                self.L.jh_set_obj(od, b"string", self.string(v))
            self.L.jh_set_obj(e, tname.encode(), self.attr_type(t))
            self.L.jh_set_obj(e, oname.encode(), od)
        if index is not None:
            self.L.jh_set_obj(e, b"indexType", self.new("global/IndexType", indexType=index))
        return e

    def condexprs(self, cnf):
        """CondExpr[] of an oracle CNF spec: one OR-chain (.next) per
        conjunct, null-terminated (R/iterator/PredEval.java:25-183)"""
        heads = []
        for conj in cnf:
            head = prev = None
            for term in conj:
                op, a, b = term[:3]
                e = self.condexpr(op, a, b, INDEX_BITMAP if len(term) > 3 else None)
                if prev is None:
                    head = e
                else:
                    self.L.jh_set_obj(prev, b"next", e)
                prev = e
            heads.append(head)
        return self.object_array(heads + [None], "iterator/CondExpr")

    # ---- results -----------------------------------------------------------
    def value(self, o):
        """int[] / long[] / short[] / float[] -> list, String -> str, Object[] -> list"""
        if not o:
            return None
        et = self.L.jh_array_type(o)
        if et == b"\x00":
            p = self.L.jh_string_utf(o)
            if p is None:
                raise TypeError(self.L.jh_class_name(o))
            return mutf8_decode(ctypes.string_at(p, self.L.jh_string_len(o)))
        n = self.L.jh_array_len(o)
        if et == b"L":
            return [self.value(self.L.jh_array_get(o, i)) for i in range(n)]
        ct = {b"I": ctypes.c_int32, b"J": ctypes.c_int64, b"S": ctypes.c_int16, b"B": ctypes.c_int8,
              b"F": ctypes.c_float}[et]
        return list((ct * n).from_address(self.L.jh_array_data(o))) if n else []

    # ---- natives -----------------------------------------------------------
    def call(self, name, restype, *args):
        """Java_global_Native_<name>(env, Native.class, args...): args are
        (ctype, value) pairs.  A pending exception becomes JavaException;
        unreleased borrows or JNI violations fail the call."""
        f = getattr(self.L, "Java_global_Native_" + name)
        f.restype = restype
        f.argtypes = [V, V] + [t for t, _ in args]
        out = f(self.env, None, *[v for _, v in args])
        assert self.L.jh_outstanding() == 0, f"{name}: {self.L.jh_outstanding()} borrowed arrays/strings not released"
        assert self.L.jh_violations() == 0, f"{name}: JNI violation: {self.L.jh_last_violation().decode()}"
        e = self.L.jh_pending()
        if e:
            self.L.jh_clear()
            m = self.L.jh_exception_message(e)
            raise JavaException(self.L.jh_class_name(e).decode(), self.value(m) if m else None)
        return out
