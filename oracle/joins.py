"""CPU restatement of the reference's two join operators -- TEST INFRASTRUCTURE.

Used only by tests/ as the checker of the GPU joins (include/mbx.h
mbx_join_pairs, host/ `nlj` / `bmj`).  Restates, on top of the scan oracle
(oracle.py), in the reference's order:

  * `nlj`  R/input/NljQuery.java:30-230 + R/iterator/ColumnarNestedLoopJoins.java:
           block nested loops -- outer blocks of (amt_of_memory - 1) *
           (1024 / outer tuple size) tuples, for each pass the inner relation is
           rescanned and every inner tuple is tried against every outer tuple of
           the block (inner-major order, :160-200); access paths FILESCAN (whole
           CNF in the scan), COLUMNSCAN / BITMAP / BTREE (first conjunct in the
           access path, the others as the pending filter applied while filling
           the buffers, NljQuery.java:356-370).
  * `bmj`  R/input/BitMapQuery.java:187-300: outer / inner CNF BitSets by
           ColumnarIndexScan over bitmap indexes, then per outer position (ascending)
           a ColumnarIndexScan of the inner file with the outer values substituted
           (operators mirrored, AttrOperator.getOppositeOperator), AND the inner
           BitSet, inner positions ascending.

Pinned by the 73 successful `nlj` / `bmj` runs of R/phase3_output
(tests/golden/phase3_golden.json "joins").
"""
import oracle

OPS = {"=": oracle.EQ, "<": oracle.LT, ">": oracle.GT, "!=": oracle.NE, "<=": oracle.LE, ">=": oracle.GE}
OPPOSITE = {"=": "=", "<": ">", ">": "<", "!=": "!=", ">=": "<=", "<=": ">="}
PAGE = 1024


def parse_cnf(s):
    """'{(A,=,x)|(B,=,y)}^{(C,=,6)}' -> [[('A','=','x'), ('B','=','y')], [('C','=','6')]]"""
    out = []
    for part in s.strip().split("^"):
        part = part.strip()
        assert part.startswith("{") and part.endswith("}"), "Invalid query format"
        terms = []
        for t in part[1:-1].split("|"):
            t = t.strip()
            assert t.startswith("(") and t.endswith(")"), "Invalid query format"
            f = [x.strip() for x in t[1:-1].split(",")]
            assert len(f) == 3, "Invalid VALUECONSTRAINT elements"
            terms.append(tuple(f))
        out.append(terms)
    return out


class Rel:
    """A Columnarfile for the join oracle: name, column names, types, sizes, oracle.Table."""

    def __init__(self, name, names, table):
        self.name, self.names, self.table = name, list(names), table
        self.types = [t for t, _, _ in table.columns]
        self.sizes = [s for _, s, _ in table.columns]

    def col(self, cname):
        return self.names.index(cname)

    def value(self, j, pos):
        t, size, a = self.table.columns[j]
        if t == oracle.STRING:
            return bytes(a[pos]).rstrip(b"\0").decode("utf-8", "surrogatepass")
        return int(a[pos]) if t == oracle.INTEGER else float(a[pos])

    def literal(self, j, text):
        t = self.types[j]
        return ("int", int(text)) if t == oracle.INTEGER else ("str", text)


def _cnf_spec(rel, conjuncts, index_type=None):
    out = []
    for conj in conjuncts:
        terms = []
        for c, op, v in conj:
            j = rel.col(c)
            term = (OPS[op], ("sym", j + 1), rel.literal(j, v))
            if index_type is not None:
                term = term + (index_type,)
            terms.append(term)
        out.append(terms)
    return out


def access(rel, conjuncts, kind):
    """(positions the access path's iterator returns, positions that also pass
    the pending filter), both ascending (position order)."""
    kind = kind.upper()
    if kind == "FILESCAN":
        _, _, ids = oracle.filescan(rel.table, _cnf_spec(rel, conjuncts))
        ids = [int(x) for x in ids]
        return ids, ids
    first, rest = conjuncts[:1], conjuncts[1:]
    if kind == "COLUMNSCAN":
        _, _, ids = oracle.filescan(rel.table, _cnf_spec(rel, first))
    else:
        idx = oracle.IDX_BTREE if kind == "BTREE" else oracle.IDX_BITMAP
        _, w = oracle.columnar_index_scan(rel.table, _cnf_spec(rel, first, idx))
        ids = oracle.words_to_positions(w)
    ids = [int(x) for x in ids]
    if not rest:
        return ids, ids
    pend = _cnf_spec(rel, rest)
    return ids, [p for p in ids if oracle.pred_eval(rel.table, pend, p)]


def java_cmp(a, b):
    if isinstance(a, str):
        ka, kb = a.encode("utf-16-be", "surrogatepass"), b.encode("utf-16-be", "surrogatepass")
        return (ka > kb) - (ka < kb)
    return (a > b) - (a < b)


def _op_true(op, c):
    return {"=": c == 0, "<": c < 0, ">": c > 0, "!=": c != 0, "<=": c <= 0, ">=": c >= 0}[op]


def join_ok(outer, inner, jcnf, o, i):
    """PredEval.Eval(JoinFilter, outer tuple, inner tuple): operand 1 from the
    outer tuple, operand 2 from the inner (NljQuery.buildCNFJoinCondExpr)."""
    for conj in jcnf:
        if not any(_op_true(op, java_cmp(outer.value(outer.col(a), o), inner.value(inner.col(b), i)))
                   for a, op, b in conj):
            return False
    return True


def tuple_size(rel, cols):
    """Tuple.setHdr size of a tuple of these columns (R/heap/Tuple.java:369-411)."""
    n = len(cols)
    return (n + 2) * 2 + sum(rel.sizes[j] + 2 if rel.types[j] == oracle.STRING else 4 for j in cols)


def target_cols(rels, targets):
    """[TARGETCOLUMNNAMES] -> (per relation name: sorted column indexes, [(rel, col)] output order)."""
    sets = {r.name: set() for r in rels}
    out = []
    by = {r.name: r for r in rels}
    for t in targets:
        rn, cn = t.split(".")
        rel = by.get(rn, rels[1])
        j = rel.col(cn)
        sets[rel.name].add(j)
        out.append((rel, j))
    return sets, out


def nlj(outer, inner, outer_cons, inner_cons, join_cons, outer_access, inner_access, targets, amt_of_memory):
    """-> dict(header, rows [(pass, outer pos, inner pos)], stats)."""
    oc, ic, jc = parse_cnf(outer_cons), parse_cnf(inner_cons), parse_cnf(join_cons)
    sets, _ = target_cols([outer, inner], targets)
    otargets = set(sets[outer.name])
    # findConsTargetCols: non-FILESCAN access paths project the pending columns too
    if outer_access.upper() != "FILESCAN":
        for conj in oc[1:]:
            otargets |= {outer.col(c) for c, _, _ in conj}
    for conj in jc:
        otargets |= {outer.col(a) for a, _, _ in conj}
    o_iter, o_full = access(outer, oc, outer_access)
    _, i_full = access(inner, ic, inner_access)
    tsize = tuple_size(outer, sorted(otargets))
    cap = (amt_of_memory - 1) * (PAGE // tsize)
    rows = []
    for p in range(0, max(1, (len(o_full) + cap - 1) // cap)):
        block = o_full[p * cap:(p + 1) * cap]
        for i in i_full:
            for o in block:
                if join_ok(outer, inner, jc, o, i):
                    rows.append((p, o, i))
    stats = {"Tuple Size": tsize, "Number of Tuples Buffer Can Hold": cap,
             "Total Outer Tuples By Full Constraint": len(o_full), "Total Outer Tuples By Iterator": len(o_iter)}
    return {"rows": rows, "stats": stats}


def bmj(outer, inner, outer_cons, inner_cons, join_cons):
    """-> dict(outer_bits, inner_bits, rows [(outer pos, inner pos)])."""
    oc, ic, jc = parse_cnf(outer_cons), parse_cnf(inner_cons), parse_cnf(join_cons)
    _, ow = oracle.columnar_index_scan(outer.table, _cnf_spec(outer, oc, oracle.IDX_BITMAP))
    _, iw = oracle.columnar_index_scan(inner.table, _cnf_spec(inner, ic, oracle.IDX_BITMAP))
    obits = [int(x) for x in oracle.words_to_positions(ow)]
    ibits = set(int(x) for x in oracle.words_to_positions(iw))
    rows = []
    for o in obits:
        cnf = []
        for conj in jc:
            terms = []
            for a, op, b in conj:
                jo, ji = outer.col(a), inner.col(b)
                v = outer.value(jo, o)
                terms.append((OPS[OPPOSITE[op]], ("sym", ji + 1), ("int", v) if isinstance(v, int) else ("str", v),
                              oracle.IDX_BITMAP))
            cnf.append(terms)
        _, w = oracle.columnar_index_scan(inner.table, cnf)
        for i in oracle.words_to_positions(w):
            if int(i) in ibits:
                rows.append((o, int(i)))
    return {"outer_bits": obits, "inner_bits": sorted(ibits), "rows": rows}


def render(rels_by_name, targets, o, i, outer, inner):
    vals = []
    for t in targets:
        rn, cn = t.split(".")
        rel = outer if rn == outer.name else inner
        pos = o if rel is outer else i
        vals.append(str(rel.value(rel.col(cn), pos)))
    return ", ".join(vals)
