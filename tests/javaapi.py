"""A small Java declaration parser: the public constructors, methods and
fields declared directly in a class body (brace depth 1).  Enough for the
Minibase sources and the drop-ins: comments and string literals stripped,
C-style array declarators (`AttrType in1[]`) folded into the type, `final`
and annotations dropped, generic arguments kept verbatim."""
import re


def _strip(src):
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    src = re.sub(r'"(?:\\.|[^"\\])*"', '""', src)
    src = re.sub(r"'(?:\\.|[^'\\])'", "' '", src)
    return src


def _norm_type(t):
    t = re.sub(r"\s+", "", t)
    return t


def _param(p):
    p = re.sub(r"@\w+", " ", p)
    p = re.sub(r"\bfinal\b", " ", p).strip()
    m = re.match(r"^(.*?)\s*\b(\w+)\s*((?:\[\s*\])*)$", p, flags=re.S)
    if not m:
        raise ValueError(f"cannot parse parameter {p!r}")
    typ, _name, dims = m.groups()
    return _norm_type(typ) + "[]" * dims.count("[")


def _split_params(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [_param(p) for p in out]


def throws_list(tail):
    """the exception types of a declaration's `throws` clause (text after the
    parameter list), in source order, as written (simple or qualified)"""
    m = re.search(r"\bthrows\b(.*)$", tail, flags=re.S)
    if not m:
        return []
    return [re.sub(r"\s+", "", t) for t in m.group(1).split(",") if t.strip()]


def public_api(src):
    """{'class': name, 'ctors': [[types]], 'ctor_throws': [[exception types]] (one
    list per constructor, same order), 'methods': [{'name', 'params', 'returns',
    'throws', 'throws_list'}], 'fields': [{'name','type'}]} of the first
    top-level class in src."""
    s = _strip(src)
    m = re.search(r"\bclass\s+(\w+)", s)
    if not m:
        raise ValueError("no class")
    cls = m.group(1)
    body_start = s.index("{", m.end())
    depth, stmt, decls = 1, "", []
    for ch in s[body_start + 1:]:
        if depth == 1 and ch in "{;":
            decls.append(stmt.strip())
            stmt = ""
        elif depth == 1 and ch == "}":
            stmt = ""
        elif depth == 1 and ch == "=":
            # a field initialiser: keep the declaration part only
            stmt += " = "
        elif depth == 1:
            stmt += ch
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
            if depth == 0:
                break
            if depth == 1:
                stmt = ""
    api = {"class": cls, "ctors": [], "ctor_throws": [], "methods": [], "fields": []}
    for d in decls:
        d = re.sub(r"\s+", " ", d).strip()
        d = d.split(" = ")[0].strip()
        if not re.match(r"^(@\w+ )*public\b", d):
            continue
        d = re.sub(r"\b(public|static|final|synchronized|abstract|native|transient|volatile)\b", " ", d)
        d = re.sub(r"@\w+", " ", d).strip()
        d = re.sub(r"\s+", " ", d)
        if "(" in d:
            head, rest = d.split("(", 1)
            params = rest.rsplit(")", 1)[0]
            throws = rest.rsplit(")", 1)[1]
            ps = _split_params(params) if params.strip() else []
            toks = head.strip().rsplit(" ", 1)
            tl = throws_list(throws)
            if len(toks) == 1:
                api["ctors"].append(ps)
                api["ctor_throws"].append(tl)
            else:
                ret, name = toks
                api["methods"].append({"name": name, "params": ps, "returns": _norm_type(ret),
                                       "throws": bool(tl), "throws_list": tl})
        elif d.startswith("class ") or d.startswith("interface "):
            continue
        else:
            for part in d.split(","):
                mm = re.match(r"^(.*?)\s*\b(\w+)\s*((?:\[\s*\])*)$", part.strip())
                if mm and mm.group(1):
                    api["fields"].append({"name": mm.group(2),
                                          "type": _norm_type(mm.group(1)) + "[]" * mm.group(3).count("[")})
    return api
