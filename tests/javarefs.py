"""Symbol resolution of the Java drop-ins against the reference classes, with
no JDK (VERDICT r4 "What's missing" 4): every constructor, method and field
the drop-ins under java/ use on a reference class must exist there with that
arity, static-ness and visibility.

Two halves:
  * symbols(src_text, path) -- the declarations of every class in one Java
    source (top-level and nested): extends / implements, fields (type,
    static, visibility), methods (name, arity, static, return type,
    visibility), constructors (arity, visibility).  Run over the reference
    tree by tests/golden/make_java_symbols.py into the committed fixture
    tests/golden/java_symbols.json (the GPU box has no /root/reference).
  * references(src_text, ...) -- the uses in one drop-in: `new C(...)`,
    `C.m(...)` / `C.F` (static), `v.m(...)` / `v.f` / `a[i].f` with v's
    declared type, chains through return and field types
    (`cf.getMarkedDeleted().getBitSet()`, `SystemDefs.JavabaseBM.flushPage`),
    `super(...)`, and unqualified calls inherited from a reference
    superclass.  check() resolves each against the table and returns the
    failures.

The reader is a declaration scanner over comment- and string-stripped text
(brace depth), not a Java compiler: generic bodies are skipped, overloads are
matched by name and arity, and a chain stops at the first type that is not a
reference class (JDK or drop-in types are not in the table)."""
import os
import re

MODIFIERS = ("public", "private", "protected", "static", "final", "synchronized", "abstract", "native",
             "transient", "volatile", "strictfp")
KEYWORDS = {"if", "for", "while", "switch", "catch", "synchronized", "return", "new", "throw", "else", "do", "try",
            "case", "assert", "super", "this", "instanceof", "finally"}
PRIMITIVES = {"int", "long", "short", "byte", "char", "boolean", "float", "double", "void"}
# java.lang / JDK types the drop-ins use unqualified (not reference classes)
JDK_TYPES = {"String", "Object", "Math", "Integer", "Long", "Short", "Float", "Double", "Boolean", "Byte",
             "Character", "System", "Exception", "RuntimeException", "IllegalStateException",
             "IllegalArgumentException", "UnsupportedOperationException", "Throwable", "StringBuilder", "Class",
             "Iterable", "AutoCloseable", "Override", "SuppressWarnings", "Error", "Runtime", "Thread",
             "IndexOutOfBoundsException", "NullPointerException", "ArithmeticException", "Comparable", "Void"}


def strip(src):
    src = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    src = re.sub(r'"(?:\\.|[^"\\\n])*"', '""', src)
    src = re.sub(r"'(?:\\.|[^'\\\n])+'", "' '", src)
    return src


def split_top(s, sep=","):
    """split at separators outside (), [], {}, <>"""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{<":
            depth += 1
        elif ch in ")]}>":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def base_type(t):
    """'Map<String, Long>' -> 'Map'; keeps array dims: 'AttrType[]'"""
    t = re.sub(r"\s+", "", t)
    dims = t.count("[]")
    t = re.sub(r"<.*>", "", t).replace("[]", "")
    return t + "[]" * dims


def _mods(decl):
    toks = decl.split()
    mods = set()
    while toks and (toks[0] in MODIFIERS or toks[0].startswith("@")):
        mods.add(toks.pop(0))
    return mods, " ".join(toks)


def _vis(mods):
    for v in ("public", "private", "protected"):
        if v in mods:
            return v
    return "package"


# ---------------------------------------------------------------- declarations

def symbols(src, path=""):
    """{qualified class name: {...}} for every class / interface in src."""
    s = strip(src)
    pm = re.search(r"^\s*package\s+([\w.]+)\s*;", s, flags=re.M)
    pkg = pm.group(1) if pm else ""
    out = {}
    # a stack of (class record, body depth)
    stack = []
    depth, stmt, i, n = 0, "", 0, len(s)
    in_init = False  # a field initialiser with braces (array literal) at class depth
    while i < n:
        ch = s[i]
        cls_depth = stack[-1][1] if stack else None
        at_member = stack and depth == cls_depth
        if ch == "{":
            if at_member and in_init:
                depth += 1
                i += 1
                continue
            head = re.sub(r"\s+", " ", stmt).strip()
            cm = re.search(r"\b(class|interface|enum)\s+(\w+)([^{]*)$", head)
            if cm and (not stack or at_member or depth == 0):
                mods, _ = _mods(head[:cm.start()].strip() + " x")
                rest = cm.group(3)
                ext = re.search(r"\bextends\s+([\w.<>,\s]+?)(?:\bimplements\b|$)", rest)
                imp = re.search(r"\bimplements\s+([\w.<>,\s]+)$", rest)
                name = cm.group(2)
                outer = stack[-1][0]["name"] if stack else None
                qual = (outer + "." + name) if outer else name
                rec = {"name": qual, "package": pkg, "kind": cm.group(1), "visibility": _vis(mods),
                       "static": "static" in mods, "abstract": "abstract" in mods,
                       "extends": [base_type(x) for x in split_top(ext.group(1))] if ext else [],
                       "implements": [base_type(x) for x in split_top(imp.group(1))] if imp else [],
                       "fields": {}, "methods": {}, "ctors": [], "source": path}
                out[(pkg + "." if pkg else "") + qual] = rec
                depth += 1
                stack.append((rec, depth))
                stmt = ""
                i += 1
                continue
            if at_member:
                _member(stack[-1][0], head, body=True)
                stmt = ""
            depth += 1
            i += 1
            continue
        if ch == "}":
            if in_init and stack and depth == cls_depth + 1:  # the end of an array initialiser
                depth -= 1
                i += 1
                continue
            depth -= 1
            if stack and depth == stack[-1][1] - 1:
                stack.pop()
            stmt = ""
            i += 1
            continue
        if at_member:
            if ch == ";":
                if in_init:
                    in_init = False
                _member(stack[-1][0], re.sub(r"\s+", " ", stmt).strip(), body=False)
                stmt = ""
            else:
                stmt += ch
                if ch == "=" and "(" not in stmt.split("=")[0]:
                    in_init = True
        elif not stack:  # top level: package / imports / a class header
            stmt = "" if ch == ";" else stmt + ch
        i += 1
    return out


def _member(rec, decl, body):
    if not decl or decl.startswith("static") and decl.strip() == "static":
        return
    if decl in ("static",):
        return
    iface = rec["kind"] == "interface"
    mods, rest = _mods(decl)
    if not rest:
        return
    if "(" in rest and (not ("=" in rest and rest.index("=") < rest.index("("))):
        head, tail = rest.split("(", 1)
        params = tail.rsplit(")", 1)[0]
        head = re.sub(r"<[^<>]*>\s*(?=\w)", "", head).strip()  # generic method type parameters
        toks = head.split()
        arity = len(split_top(params)) if params.strip() else 0
        vis = "public" if iface and _vis(mods) == "package" else _vis(mods)
        simple = rec["name"].split(".")[-1]
        if len(toks) == 1 and toks[0] == simple:
            rec["ctors"].append({"arity": arity, "visibility": vis})
        elif len(toks) >= 2:
            ret = base_type(" ".join(toks[:-1]))
            name = toks[-1]
            dims = 0
            rec["methods"].setdefault(name, []).append({"arity": arity, "static": "static" in mods,
                                                        "returns": ret, "visibility": vis,
                                                        "abstract": "abstract" in mods or (iface and not body)})
        return
    # field(s): Type a [= x], b[] [= y]
    decl_part = rest
    parts = split_top(decl_part)
    first = parts[0].split("=")[0].strip()
    m = re.match(r"^(.*?)\s*\b(\w+)\s*((?:\[\s*\])*)$", first)
    if not m or not m.group(1):
        return
    typ = base_type(m.group(1))
    static = "static" in mods or iface
    vis = "public" if iface else _vis(mods)
    for k, p in enumerate(parts):
        p = p.split("=")[0].strip()
        mm = re.match(r"^(?:.*?\s)?(\w+)\s*((?:\[\s*\])*)$", p) if k else m
        if not mm:
            continue
        name = mm.group(2) if k == 0 else mm.group(1)
        dims = (mm.group(3) if k == 0 else mm.group(2)).count("[")
        rec["fields"][name] = {"type": typ + "[]" * dims, "static": static, "visibility": vis}


def tree_symbols(root):
    """symbols() of every .java under root: {qualified name: record}"""
    out = {}
    for d, _, files in sorted(os.walk(root)):
        for f in sorted(files):
            if f.endswith(".java"):
                p = os.path.join(d, f)
                with open(p, errors="replace") as fh:
                    out.update(symbols(fh.read(), os.path.relpath(p, root)))
    return out


# ---------------------------------------------------------------- references

_TOK = re.compile(r"\s*(?:([A-Za-z_$][\w$]*)|(\d[\w.]*)|(\S))")


def _tokens(s):
    toks, pos = [], 0
    line = 1
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m:
            break
        line += s.count("\n", pos, m.start(0) + len(m.group(0)) - len((m.group(1) or m.group(2) or m.group(3))))
        t = m.group(1) or m.group(2) or m.group(3)
        toks.append((t, line, m.end() - len(t)))
        pos = m.end()
    return toks


def _match_paren(toks, i):
    """index of the token closing toks[i] ('(' or '['), and the arity inside"""
    open_, close = toks[i][0], {"(": ")", "[": "]"}[toks[i][0]]
    depth, j, commas, nonempty = 0, i, 0, False
    while j < len(toks):
        t = toks[j][0]
        if t in "([{":
            depth += 1
        elif t in ")]}":
            depth -= 1
            if depth == 0:
                return j, (commas + 1 if nonempty else 0)
        elif t == "," and depth == 1:
            commas += 1
        if j > i and depth >= 1 and not (depth == 1 and t == ","):
            nonempty = True
        j += 1
    raise ValueError("unbalanced")


_DECL = re.compile(r"(?<![\w.])([A-Za-z_][\w.]*)\s*(<(?:[^<>]|<[^<>]*>)*>)?\s*((?:\[\s*\])*)\s+"
                   r"([A-Za-z_]\w*)\s*((?:\[\s*\])*)\s*(?=[=;,:)])")


def _decls(s):
    """[(position, name, declared base type)] of every field, parameter,
    local and for-each variable in one source"""
    out = []
    for m in _DECL.finditer(s):
        typ, dims1, name, dims2 = m.group(1), m.group(3).count("["), m.group(4), m.group(5).count("[")
        if typ in ("return", "new", "throw", "else", "case", "package", "import") or name in KEYWORDS:
            continue
        out.append((m.start(4), name, typ + "[]" * (dims1 + dims2)))
    return out


def _var_types(s):
    """name -> set of declared (base) types in one source (any scope)"""
    out = {}
    for _, name, typ in _decls(s):
        out.setdefault(name, set()).add(typ)
    return out


def _member_ranges(s):
    """[(start, end)] of each member of the top-level class body: from the end
    of the previous member (its header, parameters included) to its closing
    brace -- the scope of its parameters and locals"""
    out = []
    m = re.search(r"\bclass\s+\w+[^{]*\{", s)
    if not m:
        return out
    depth, start = 1, m.end()
    for i in range(m.end(), len(s)):
        ch = s[i]
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
            if depth == 1:
                out.append((start, i + 1))
                start = i + 1
            elif depth == 0:
                break
        elif ch == ";" and depth == 1:
            start = i + 1
    return out


class Scope:
    """A use's declared type: the nearest declaration before it in the same
    member (parameters and locals), else the class's fields; None when that
    is still ambiguous."""

    def __init__(self, s):
        self.decls = _decls(s)
        self.ranges = _member_ranges(s)

    def _range(self, pos):
        for a, b in self.ranges:
            if a <= pos < b:
                return a, b
        return None

    def type_of(self, name, pos):
        r = self._range(pos)
        if r:
            local = [(p, t) for p, n, t in self.decls if n == name and r[0] <= p < pos]
            if local:
                return max(local)[1]
        fields = {t for p, n, t in self.decls if n == name and self._range(p) is None}
        return next(iter(fields)) if len(fields) == 1 else None


class Resolver:
    def __init__(self, table, dropins=None):
        self.t = table
        self.by_simple = {}
        for q, r in table.items():
            self.by_simple.setdefault(r["name"].split(".")[-1], set()).add(q)
            self.by_simple.setdefault(r["name"], set()).add(q)
        self.dropins = dropins or {}

    def lookup_class(self, name, ctx):
        """qualified reference class for a simple / dotted name in a drop-in's
        context (its package, imports), or None"""
        if name in ctx["imports"]:
            q = ctx["imports"][name]
            return q if q in self.t else None
        cands = self.by_simple.get(name, set())
        for q in cands:
            rec = self.t[q]
            if rec["package"] == ctx["package"] or rec["package"] in ctx["wild"]:
                return q
        if "." in name:
            head = name.split(".")[0]
            hq = self.lookup_class(head, ctx)
            if hq:
                q = hq + name[len(head):]
                return q if q in self.t else None
            if name in self.t:
                return name
        return None

    def supers(self, q):
        """q and its reference superclasses / interfaces, nearest first"""
        seen, order, todo = set(), [], [q]
        while todo:
            c = todo.pop(0)
            if c in seen or c not in self.t:
                continue
            seen.add(c)
            order.append(c)
            rec = self.t[c]
            ctx = {"package": rec["package"], "imports": {}, "wild": set(self.t[c].get("wild", []))}
            for e in rec["extends"] + rec["implements"]:
                sq = self.lookup_class(e.replace("[]", ""), ctx) or self._any(e)
                if sq:
                    todo.append(sq)
        return order

    def _any(self, simple):
        c = self.by_simple.get(simple, set())
        return next(iter(c)) if len(c) == 1 else None

    def accessible(self, member_vis, owner, ctx, subclass=False):
        if member_vis == "public":
            return True
        if member_vis == "private":
            return False
        same_pkg = self.t[owner]["package"] == ctx["package"]
        if member_vis == "protected":
            return same_pkg or subclass
        return same_pkg

    def find_method(self, q, name, arity):
        for c in self.supers(q):
            for mm in self.t[c]["methods"].get(name, []):
                if mm["arity"] == arity:
                    return c, mm
        return None, None

    def find_field(self, q, name):
        for c in self.supers(q):
            f = self.t[c]["fields"].get(name)
            if f:
                return c, f
        return None, None

    def type_of(self, typ, ctx, owner_ctx=None):
        """a declared type string -> (qualified reference class or None, dims)"""
        dims = typ.count("[]")
        q = self.lookup_class(typ.replace("[]", ""), owner_ctx or ctx)
        return q, dims


def file_context(src):
    s = strip(src)
    pm = re.search(r"^\s*package\s+([\w.]+)\s*;", s, flags=re.M)
    ctx = {"package": pm.group(1) if pm else "", "imports": {}, "wild": set(), "bad_imports": []}
    for m in re.finditer(r"^\s*import\s+(static\s+)?([\w.]+?)(\.\*)?\s*;", s, flags=re.M):
        if m.group(1):
            continue
        if m.group(3):
            ctx["wild"].add(m.group(2))
        else:
            ctx["imports"][m.group(2).split(".")[-1]] = m.group(2)
    cm = re.search(r"\bclass\s+(\w+)(?:\s+extends\s+([\w.]+))?", s)
    ctx["class"] = cm.group(1) if cm else None
    ctx["extends"] = cm.group(2) if cm else None
    return ctx


def references(src, resolver, path=""):
    """every use of a reference member in one drop-in source, resolved:
    [{'line', 'what', 'ok', 'why'}] (ok False = the failure to report)"""
    R = resolver
    s = strip(src)
    ctx = file_context(src)
    res = []

    def rep(line, what, ok, why=""):
        res.append({"file": path, "line": line, "what": what, "ok": ok, "why": why})

    # imports of reference packages must name existing classes / packages
    ref_pkgs = {r["package"] for r in R.t.values()}
    for simple, q in ctx["imports"].items():
        pkg = q.rsplit(".", 1)[0]
        if pkg.startswith("java.") or q in R.dropins:
            continue
        if pkg in ref_pkgs or q in R.t:
            rep(0, f"import {q}", q in R.t, "no such reference class")
    for w in ctx["wild"]:
        if not w.startswith("java."):
            rep(0, f"import {w}.*", w in ref_pkgs or any(q.startswith(w + ".") for q in R.dropins),
                "no such package")

    own = symbols(src, path)
    own_rec = next(iter(own.values())) if own else None
    own_methods = set(own_rec["methods"]) if own_rec else set()
    superq = R.lookup_class(ctx["extends"], ctx) if ctx["extends"] else None
    if superq and own_rec and not own_rec["abstract"]:
        # a concrete drop-in implements every abstract method of its
        # reference superclasses, public where they are public
        done = set()
        for c in R.supers(superq):
            for name, ms in R.t[c]["methods"].items():
                for mm in ms:
                    if (name, mm["arity"]) in done:
                        continue
                    done.add((name, mm["arity"]))
                    if not mm.get("abstract"):
                        continue
                    mine = [x for x in own_rec["methods"].get(name, []) if x["arity"] == mm["arity"]]
                    ok = bool(mine) and (mm["visibility"] != "public" or mine[0]["visibility"] == "public")
                    rep(0, f"implements abstract {c}.{name}({mm['arity']} args)", ok,
                        "abstract method not implemented (or with weaker access)")
    vars_ = _var_types(s)
    scope = Scope(s)
    toks = _tokens(s)
    # skip the package / import statements
    k = 0
    while k < len(toks):
        if toks[k][0] in ("package", "import"):
            while toks[k][0] != ";":
                k += 1
        elif toks[k][0] not in ("@",):
            pass
        k += 1
        if k < len(toks) and toks[k][0] not in ("package", "import", ";"):
            break
    i = 0
    while i < len(toks):
        t, line, tpos = toks[i]
        prev = toks[i - 1][0] if i else ""
        if t == "new" and i + 1 < len(toks):
            # new C(...) [.chain]
            j = i + 1
            name = toks[j][0]
            while j + 2 < len(toks) and toks[j + 1][0] == ".":
                j += 2
                name += "." + toks[j][0]
            if j + 1 < len(toks) and toks[j + 1][0] == "<":  # generic arguments
                d = 0
                j += 1
                while j < len(toks):
                    d += toks[j][0] == "<"
                    d -= toks[j][0] == ">"
                    if d == 0:
                        break
                    j += 1
            if j + 1 < len(toks) and toks[j + 1][0] == "(":
                q = R.lookup_class(name, ctx)
                close, arity = _match_paren(toks, j + 1)
                if q:
                    ok = any(c["arity"] == arity and R.accessible(c["visibility"], q, ctx) for c in R.t[q]["ctors"]) \
                        or (arity == 0 and not R.t[q]["ctors"])
                    # an anonymous subclass body may follow (...) { }
                    rep(line, f"new {q}({arity} args)", ok, "no accessible constructor of that arity")
                    i = _chain(R, toks, close + 1, (q, 0), False, ctx, rep)
                    continue
            i += 1
            continue
        if t == "super" and i + 1 < len(toks) and toks[i + 1][0] == "(" and prev in ("{", ";", "}"):
            close, arity = _match_paren(toks, i + 1)
            if superq:
                ok = any(c["arity"] == arity and R.accessible(c["visibility"], superq, ctx, True)
                         for c in R.t[superq]["ctors"]) or (arity == 0 and not R.t[superq]["ctors"])
                rep(line, f"super({arity} args) of {superq}", ok, "no constructor of that arity")
            i = close + 1
            continue
        if re.match(r"[A-Za-z_]", t) and prev != "." and t not in KEYWORDS and t not in PRIMITIVES:
            nxt = toks[i + 1][0] if i + 1 < len(toks) else ""
            if t == "super" and nxt == "." and superq:
                i = _chain(R, toks, i + 1, (superq, 0), False, ctx, rep, subclass=True)
                continue
            if nxt == "(" and superq and t not in own_methods and prev not in ("new",) and \
                    not re.match(r"[A-Z]", t) and (i < 2 or toks[i - 2][0] != "new"):
                # unqualified call: own method, or inherited from the reference superclass
                close, arity = _match_paren(toks, i + 1)
                decl = prev in PRIMITIVES or re.match(r"[A-Z]", prev or "") or prev == "]" or prev == ">"
                if not decl:
                    c, mm = R.find_method(superq, t, arity)
                    rep(line, f"{t}({arity} args) inherited from {superq}", mm is not None,
                        "not declared here nor inherited")
                i += 1
                continue
            if nxt in (".", "["):
                base = None
                if t in vars_:
                    typ = scope.type_of(t, tpos)
                    q = R.type_of(typ, ctx) if typ else (None, 0)
                    if q[0]:
                        base = (q, False)
                elif re.match(r"[A-Z]", t):
                    name, j = t, i
                    q = R.lookup_class(name, ctx)
                    # dotted class names: Outer.Inner
                    while q is None and j + 2 < len(toks) and toks[j + 1][0] == "." and re.match(r"[A-Z]", toks[j + 2][0]):
                        j += 2
                        name += "." + toks[j][0]
                        q = R.lookup_class(name, ctx)
                    if q:
                        i = _chain(R, toks, j + 1, (q, 0), True, ctx, rep)
                        continue
                    elif t not in JDK_TYPES and t not in vars_ and t not in ctx["imports"] and \
                            not _is_dropin(R, t, ctx) and \
                            t != ctx["class"] and nxt == ".":
                        rep(line, f"{t}.…", False, "unknown class (not imported, not in the package, not JDK)")
                if base:
                    i = _chain(R, toks, i + 1, base[0], False, ctx, rep)
                    continue
        i += 1
    return res


def _is_dropin(R, simple, ctx):
    for q in R.dropins:
        pkg, name = q.rsplit(".", 1)
        if name == simple and (pkg == ctx["package"] or ctx["imports"].get(simple) == q or pkg in ctx["wild"]):
            return True
    return False


def _chain(R, toks, i, cur, static_ctx, ctx, rep, subclass=False):
    """walk `.m(...)` / `.f` / `[...]` from toks[i] on a value of type cur =
    (qualified class, array dims); returns the index after the chain"""
    q, dims = cur
    while i < len(toks):
        t = toks[i][0]
        if t == "[":
            close, _ = _match_paren(toks, i)
            if dims == 0:
                return close + 1
            dims -= 1
            i = close + 1
            static_ctx = False
            continue
        if t != "." or i + 1 >= len(toks):
            return i
        name, line, _ = toks[i + 1]
        if q is None:
            return i
        if dims > 0:  # arrays: .length / clone()
            return i + 2
        nxt = toks[i + 2][0] if i + 2 < len(toks) else ""
        rec = R.t[q]
        if nxt == "(":
            close, arity = _match_paren(toks, i + 2)
            owner, mm = R.find_method(q, name, arity)
            if mm is None:
                rep(line, f"{q}.{name}({arity} args)", False, "no method of that name and arity")
                return close + 1
            if static_ctx and not mm["static"]:
                rep(line, f"{q}.{name}({arity} args)", False, "instance method called on the class")
                return close + 1
            ok = R.accessible(mm["visibility"], owner, ctx, subclass)
            rep(line, f"{owner}.{name}({arity} args)", ok, "not accessible from " + ctx["package"])
            q, dims = R.type_of(mm["returns"], ctx, {"package": R.t[owner]["package"], "imports": {},
                                                       "wild": _pkg_imports(R, owner)})
            i = close + 1
        else:
            nested = R.lookup_class(rec["name"] + "." + name, {"package": rec["package"], "imports": {},
                                                                "wild": set()})
            if static_ctx and nested:
                q, dims = nested, 0
                i += 2
                continue
            owner, f = R.find_field(q, name)
            if f is None:
                rep(line, f"{q}.{name}", False, "no field of that name")
                return i + 2
            if static_ctx and not f["static"]:
                rep(line, f"{q}.{name}", False, "instance field read on the class")
                return i + 2
            ok = R.accessible(f["visibility"], owner, ctx, subclass)
            rep(line, f"{owner}.{name}", ok, "not accessible from " + ctx["package"])
            q, dims = R.type_of(f["type"], ctx, {"package": R.t[owner]["package"], "imports": {},
                                                   "wild": _pkg_imports(R, owner)})
            i += 2
        static_ctx = False
    return i


def _pkg_imports(R, owner):
    """a reference class's own import view, approximated: every reference package
    (its return / field types are resolved by simple name)"""
    return {r["package"] for r in R.t.values()}


def check(table, java_root):
    """resolve every drop-in under java_root; returns (all references, failures)"""
    dropins = {}
    srcs = {}
    for d, _, files in sorted(os.walk(java_root)):
        for f in sorted(files):
            if f.endswith(".java"):
                p = os.path.join(d, f)
                src = open(p).read()
                srcs[os.path.relpath(p, java_root)] = src
                for q in symbols(src, p):
                    dropins[q] = True
    R = Resolver(table, dropins)
    refs = []
    for rel, src in srcs.items():
        refs += references(src, R, "java/" + rel)
    return refs, [r for r in refs if not r["ok"]]
