#!/usr/bin/env python3
"""Kernel durations and inter-kernel gaps from a rocprofv3 --kernel-trace CSV
(--output-format csv).  For a query made of a fixed kernel sequence (C2: the
BitSet scan, then the compaction) it pairs consecutive dispatches on one
stream and reports, per sequence position, the kernel time and the gap to
the next dispatch (end -> start): the split DESIGN.md section 5 needs between
kernel time and launch boundary.

  python tools/trace_gaps.py TRACE.csv --seq k_scan_fast,k_select_ids [--json OUT]
"""
import argparse
import csv
import json
import statistics


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            s = int(r.get("Start_Timestamp") or r.get("BeginNs") or 0)
            e = int(r.get("End_Timestamp") or r.get("EndNs") or 0)
            q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
            rows.append((s, e, name, q))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--seq", required=True, help="comma-separated substrings, one per kernel of the query")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    seq = args.seq.split(",")
    rows = load(args.trace)
    by_q = {}
    for r in rows:
        by_q.setdefault(r[3], []).append(r)
    dur = {k: [] for k in range(len(seq))}
    gap = {k: [] for k in range(len(seq))}
    queries = 0
    for q, rs in by_q.items():
        i = 0
        while i + len(seq) <= len(rs):
            if all(seq[k] in rs[i + k][2] for k in range(len(seq))):
                for k in range(len(seq)):
                    s, e = rs[i + k][0], rs[i + k][1]
                    dur[k].append((e - s) / 1e3)
                    nxt = rs[i + k + 1][0] if i + k + 1 < len(rs) else None
                    if nxt is not None:
                        gap[k].append((nxt - e) / 1e3)
                queries += 1
                i += len(seq)
            else:
                i += 1
    out = {"queries": queries, "kernels": []}
    for k, name in enumerate(seq):
        d, g = dur[k], gap[k]
        out["kernels"].append({
            "kernel": name,
            "us_median": statistics.median(d) if d else None,
            "us_mean": statistics.mean(d) if d else None,
            "gap_after_us_median": statistics.median(g) if g else None,
            "gap_after_us_mean": statistics.mean(g) if g else None,
        })
    if dur[0]:
        out["query_us_median"] = sum(x["us_median"] + (x["gap_after_us_median"] or 0) for x in out["kernels"])
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
