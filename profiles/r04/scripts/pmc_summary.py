#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output for one kernel into profiles/*.json.

  kernel trace  (<dir>/**/*kernel_trace.csv): average duration of the kernel
  PMC passes    (<dir>/**/*counter_collection.csv): FETCH_SIZE / WRITE_SIZE per
                dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE
                reports half the bytes of a wide coalesced streaming read, so
                hbm read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE * 1024 as is.

usage: pmc_summary.py --kernel-substr k_scan_fast --rows N --algo-bytes B --out F [--key ROWS:MODE] DIR [DIR...]
  --key merges the summary into F["shards"][key] (bench.py load_traffic) instead of overwriting F.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def rows_of(pattern_dirs, suffix):
    out = []
    for d in pattern_dirs:
        for f in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
            with open(f) as fh:
                out += list(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel-substr", default="k_scan_fast")
    ap.add_argument("--rows", type=int, required=True)
    ap.add_argument("--algo-bytes", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--key", default=None, help="ROWS:MODE entry of the shards map to write")
    args = ap.parse_args()

    kt = [r for r in rows_of(args.dirs, "kernel_trace.csv") if args.kernel_substr in r.get("Kernel_Name", "")]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in kt]
    pmc = [r for r in rows_of(args.dirs, "counter_collection.csv") if args.kernel_substr in r.get("Kernel_Name", "")]
    by = {}
    for r in pmc:
        by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    fetch = statistics.median(by["FETCH_SIZE"]) if "FETCH_SIZE" in by else None
    write = statistics.median(by["WRITE_SIZE"]) if "WRITE_SIZE" in by else None
    hbm = None
    if fetch is not None:
        hbm = 2.0 * fetch * 1024.0 + (write or 0.0) * 1024.0
    summary = {
        "kernel_substr": args.kernel_substr,
        "rows": args.rows,
        "dispatches_traced": len(durs),
        "avg_duration_ns": statistics.mean(durs) if durs else None,
        "median_duration_ns": statistics.median(durs) if durs else None,
        "fetch_size_kb_median": fetch,
        "write_size_kb_median": write,
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": args.algo_bytes,
        "traffic_over_algorithmic": (hbm / args.algo_bytes) if hbm else None,
        "correction": "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 FETCH_SIZE halves wide streaming reads)",
    }
    if args.key:
        try:
            with open(args.out) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            doc = {}
        doc.setdefault("shards", {})[args.key] = summary
        summary_out = doc
    else:
        summary_out = summary
    with open(args.out, "w") as f:
        json.dump(summary_out, f, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
