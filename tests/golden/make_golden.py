"""Extract golden vectors from the reference's recorded CLI session.

Run once in the build container (where /root/reference exists):
    python tests/golden/make_golden.py
It reads /root/reference/phase3_output (the transcript of the reference Java
engine run over minidata.txt) as TEXT and writes tests/golden/phase3_golden.json:

  * "bitsets": the selection BitSets printed by `bmj` (BitMapQuery ->
    ColumnarIndexScan.getOutputPositions), one per distinct CNF, with the
    transcript line they come from;
  * "full_constraint_counts": "Total Outer Tuples By Full Constraint: n"
    printed by `nlj` for its outer CNF (rows of the outer file that satisfy
    the whole CNF);
  * "indexes_query": the rows (A, B, C, D) and the count printed by
    `indexes_query` (MultiIndexQuery -> ColumnarIndexScan.get_next), in the
    engine's position order;
  * "db_pages": the DB pages `batchinsert minidata.txt db cf 4` wrote and the
    pages the first `index db cf <col> ...` of each column read (PCounter sets
    the engine prints) -- they pin the page numbering of the Minibase DB
    writer (include/mbx_db.h) and which data pages hold each column.

All queries run over minidata.txt (500 rows, A:char(25) B:char(25) C:int
D:int), committed as tests/golden/minidata.tsv (a byte copy).  Nothing under
/root/reference is read at test time.
"""
import json
import os
import re
import sys

REF = "/root/reference/phase3_output"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "phase3_golden.json")


def split_cnf(s):
    """'{(A,=,x)|(B,=,y)}^{(C,=,6)}' -> [[('A','=','x'), ...], ...]"""
    s = s.strip()
    conjs = []
    for part in s.split("^"):
        part = part.strip()
        if not (part.startswith("{") and part.endswith("}")):
            return None
        terms = []
        for t in part[1:-1].split("|"):
            t = t.strip()
            if not (t.startswith("(") and t.endswith(")")):
                return None
            f = [x.strip() for x in t[1:-1].split(",")]
            if len(f) not in (3, 4):
                return None
            terms.append(f)
        conjs.append(terms)
    return conjs


STATS = ("Tuple Size: ", "Number of Tuples Buffer Can Hold: ", "Total Outer Tuples By Full Constraint: ",
         "Total Outer Tuples By Iterator: ")


def parse_join(cmd, raw, toks, body, line):
    """One `nlj` / `bmj` run: header, rows (with the inner-table pass each
    nlj row was printed in), count, the nlj statistics, or the error."""
    out = {"cmd": cmd, "raw": raw, "line": line, "rows": [], "passes": [], "stats": {}, "count": None,
           "error": None, "bitsets": {}}
    header, cur_pass, k = None, None, 0
    while k < len(body):
        b = body[k].rstrip()
        k += 1
        if b.startswith("java.lang") or b.startswith("Exception") or "Exception:" in b.split(" ")[0]:
            out["error"] = b
            break
        if not b or b.startswith("****") or b.startswith("Replacer:") or b.startswith("\tat ") or \
                b.startswith("Size while writing") or b.startswith("Read Page") or b.startswith("Write Page") or \
                b.startswith("Read Pages") or b.startswith("Wrote Pages") or b.startswith("Pinned Pages"):
            continue
        m = re.match(r"Next Pass Over Inner Table: (\d+)", b)
        if m:
            cur_pass = int(m.group(1))
            continue
        if any(b.startswith(st) for st in STATS):
            key, val = b.split(": ", 1)
            out["stats"][key] = int(val)
            continue
        m = re.match(r"Total Results Count By Query: (\d+)", b)
        if m:
            out["count"] = int(m.group(1))
            continue
        if b.startswith("OuterConstraint Bitset") or b.startswith("InnerConstraint Bitset"):
            nxt = body[k].strip() if k < len(body) else ""
            out["bitsets"][b.split(" ")[0]] = [int(x) for x in nxt.strip("{}").split(",") if x.strip()]
            k += 1
            continue
        if header is None:
            header = b
            continue
        if out["count"] is None:
            out["rows"].append(b)
            out["passes"].append(cur_pass)
    out["header"] = header
    return out


def main():
    lines = open(REF, encoding="utf-8", errors="replace").read().split("\n")
    bitsets, counts, iq = {}, {}, []
    db_pages = {"column_scan_reads": {}}
    joins = []
    i = 0
    while i < len(lines):
        ln = lines[i]
        if not ln.startswith("> "):
            i += 1
            continue
        toks = ln[2:].split()
        cmd = toks[0] if toks else ""
        j = i + 1
        while j < len(lines) and not lines[j].startswith("> "):
            j += 1
        body = lines[i + 1:j]
        if cmd in ("batchinsert", "index"):
            # PCounter page sets (R/diskmgr/PCounter.java) printed after the command
            sets = {}
            for k, b in enumerate(body):
                m = re.match(r"(Read|Wrote) Pages: \{(.*)\}", b)
                if m:
                    sets[m.group(1)] = ([int(x.split("=")[0]) for x in m.group(2).split(",") if "=" in x], i + k + 2)
            if cmd == "batchinsert" and "Wrote" in sets and "batchinsert_wrote" not in db_pages:
                db_pages["batchinsert_wrote"], db_pages["batchinsert_line"] = sets["Wrote"]
                db_pages["batchinsert_cmd"] = ln[2:].strip()
            elif cmd == "index" and len(toks) >= 5 and "Read" in sets:
                db_pages["column_scan_reads"].setdefault(toks[3], {"pages": sets["Read"][0], "line": sets["Read"][1],
                                                                   "cmd": ln[2:].strip()})
                if "Wrote" in sets:
                    db_pages.setdefault("index_runs", []).append(
                        {"cmd": ln[2:].strip(), "col": toks[3], "kind": toks[4], "wrote": sets["Wrote"][0],
                         "line": sets["Wrote"][1]})
        if cmd in ("nlj", "bmj") and len(toks) >= 7:
            joins.append(parse_join(cmd, ln[2:].strip(), toks, body, i + 1))
        if cmd == "bmj" and len(toks) >= 6 and toks[1] == "db":
            outer, inner = split_cnf(toks[4]), split_cnf(toks[5])
            for k, b in enumerate(body):
                for tag, cnf, raw in (("OuterConstraint", outer, toks[4]), ("InnerConstraint", inner, toks[5])):
                    if b.startswith(tag + " Bitset") and cnf is not None and k + 1 < len(body):
                        m = re.fullmatch(r"\{([0-9, ]*)\}", body[k + 1].strip())
                        if m:
                            pos = [int(x) for x in m.group(1).split(",") if x.strip()]
                            bitsets.setdefault(raw, {"cnf": cnf, "positions": pos, "line": i + k + 3})
        elif cmd == "nlj" and len(toks) >= 6 and toks[1] == "db":
            outer = split_cnf(toks[4])
            for k, b in enumerate(body):
                m = re.match(r"Total Outer Tuples By Full Constraint: (\d+)", b)
                if m and outer is not None:
                    counts.setdefault(toks[4], {"cnf": outer, "count": int(m.group(1)), "line": i + k + 2})
        elif cmd == "indexes_query":
            # rows follow the "A, B, C, D" header until the blank line
            hs = [k for k, b in enumerate(body) if b.strip() == "A, B, C, D"]
            if not hs:
                i = j
                continue
            h = hs[0]
            rows = []
            k = h + 1
            while k < len(body) and body[k].strip():
                a, b, c, d = [x.strip() for x in body[k].split(",")]
                rows.append([a, b, int(c), int(d)])
                k += 1
            cnt = None
            for b in body:
                m = re.match(r"Total Results Count By Query: (\d+)", b)
                if m:
                    cnt = int(m.group(1))
            cnf = split_cnf(toks[4])
            if cnf is not None and cnt is not None:
                iq.append({"cnf": cnf, "raw": toks[4], "rows": rows, "count": cnt, "line": i + 1})
        i = j
    out = {
        "source": "reference phase3_output (Minibase-Columnar CLI transcript over minidata.txt)",
        "schema": {"A": ["string", 25], "B": ["string", 25], "C": ["int", 4], "D": ["int", 4]},
        "bitsets": list(bitsets.values()),
        "full_constraint_counts": list(counts.values()),
        "indexes_query": iq,
        "db_pages": db_pages,
        "joins": joins,
    }
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {OUT}: {len(bitsets)} bitsets, {len(counts)} counts, {len(iq)} indexes_query results")


if __name__ == "__main__":
    sys.exit(main())
