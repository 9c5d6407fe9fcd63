#!/usr/bin/env python3
"""Per-kernel table from rocprofv3 CSV output: dispatches, average / median
duration (kernel trace), median HBM read / write bytes per dispatch (PMC
FETCH_SIZE x 2 x 1024 and WRITE_SIZE x 1024), plus any other counter.

FETCH_SIZE x 2: MI355X_MICROARCH.md states the gfx950 correction for wide
streaming reads only; round 2 calibrated it for the random 4-byte gathers of
k_gather too (profiles/r02/anatomy/gather_line_calibration.jsonl: BitSets with
one row per 128-B line, per 2nd / 4th line, two per line, and C4's random 1 %):
TCC_EA0_RDREQ = 1.000 x the 128-B lines touched, TCC_EA0_RDREQ_32B = 0, and
FETCH_SIZE x 2 = the touched lines x 128 B within 0.1 % -- every request is one
whole 128-B line tallied as 64 B, whatever the access width.
Since round 6 (profiles/r06/c4_req) a pass with gfx950's read-request size
split (TCC_EA0_RDREQ_32B / _64B / _128B) gives read bytes directly (32 n32 +
64 n64 + 128 n128, `read_basis` "request split"); FETCH_SIZE x 2 is used only
without it.  That split shows the x 2 holds for every kernel measured: C3's
streaming scan, C4's gathers and the probe's 8-byte loads are >= 99.7 %
128-byte requests (FETCH_SIZE's gfx950 formula counts them at 64 B: its
TCC_BUBBLE term is 0).
usage: kernel_pmc_table.py DIR [DIR...]"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def rows_of(dirs, suffix):
    out = []
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
            with open(f) as fh:
                out += list(csv.DictReader(fh))
    return out


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("mbx::", "")[:110]


def main():
    dirs = sys.argv[1:]
    dur = collections.defaultdict(list)
    for r in rows_of(dirs, "kernel_trace.csv"):
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows_of(dirs, "counter_collection.csv"):
        ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(set(dur) | set(ctr), key=lambda k: -sum(dur.get(k, [0]))):
        if not k.startswith(("k_", "k_scan")) and "mbx" not in k and not k.startswith("k"):
            continue
        d = dur.get(k, [])
        c = ctr.get(k, {})
        line = {"kernel": k, "dispatches": len(d)}
        if d:
            line["avg_us"] = round(sum(d) / len(d) / 1e3, 2)
            line["median_us"] = round(statistics.median(d) / 1e3, 2)
        split = [f"TCC_EA0_RDREQ_{w}B_sum" for w in (32, 64, 128)]
        if all(x in c for x in split):
            # gfx950's request-size split (profiles/r06/c4_req): bytes = 32 n32 + 64 n64 + 128 n128
            n32, n64, n128 = (statistics.median(c[x]) for x in split)
            line["read_MB"] = round((32 * n32 + 64 * n64 + 128 * n128) / 1e6, 3)
            line["read_basis"] = "request split"
            line["read_128B_share"] = round(n128 / max(1.0, n32 + n64 + n128), 4)
            if "FETCH_SIZE" in c:
                line["fetch_x2_MB"] = round(2 * statistics.median(c["FETCH_SIZE"]) * 1024 / 1e6, 3)
        elif "FETCH_SIZE" in c:
            line["read_MB"] = round(2 * statistics.median(c["FETCH_SIZE"]) * 1024 / 1e6, 3)
            line["read_basis"] = "FETCH_SIZE x 2"
        if "WRITE_SIZE" in c:
            line["write_MB"] = round(statistics.median(c["WRITE_SIZE"]) * 1024 / 1e6, 3)
        for name, vals in c.items():
            if name not in ("FETCH_SIZE", "WRITE_SIZE"):
                line[name] = statistics.median(vals)
        print(json.dumps(line))


if __name__ == "__main__":
    main()
