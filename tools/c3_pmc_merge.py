#!/usr/bin/env python3
"""Merge a tools/gpu_r6_e.sh session (n{1,2,4,8}_kernels.jsonl: the C3 scan over
rank 0's shard with the COUNT form bench.py uses at that N) into
profiles/c3_scan_pmc.json, keyed ROWS:MODE as bench.py's load_traffic reads it.
Read bytes from gfx950's read-request size split, write = WRITE_SIZE.
    python3 tools/c3_pmc_merge.py profiles/r06/e"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    src = sys.argv[1]
    import mbx_pkg
    mbx = mbx_pkg.load().mbx
    path = os.path.join(ROOT, "profiles", "c3_scan_pmc.json")
    d = json.load(open(path))
    # (file tag, gpus, COUNT form): N = 1's finalize; weak N > 1's 100 M-row frame
    # shard (tools/gpu_r6_e.sh's n1frame pass); strong N = 2, 4, 8's frame shards
    for tag, n, mode in (("n1", 1, "finalize"), ("n1frame", 1, "frame"), ("n2", 2, "frame"), ("n4", 4, "frame"),
                         ("n8", 8, "frame")):
        s, e = mbx.shard_bounds(100_000_000, n, 0)
        rows = e - s
        k = [json.loads(x) for x in open(os.path.join(src, f"{tag}_kernels.jsonl")) if "k_scan_fast" in x]
        assert len(k) == 1, (n, [x["kernel"] for x in k])
        k = k[0]
        assert k.get("read_basis") == "request split", k
        hbm = (k["read_MB"] + k["write_MB"]) * 1e6
        d["shards"][f"{rows}:{mode}"] = {
            "kernel_substr": "k_scan_fast", "kernel": k["kernel"], "rows": rows, "gpus": n,
            "dispatches_traced": k["dispatches"], "avg_duration_ns": k["avg_us"] * 1e3,
            "median_duration_ns": k["median_us"] * 1e3, "read_bytes_per_launch": k["read_MB"] * 1e6,
            "write_bytes_per_launch": k["write_MB"] * 1e6, "hbm_bytes_per_launch": hbm,
            "algorithmic_bytes_per_launch": 8 * rows, "traffic_over_algorithmic": hbm / (8 * rows),
            "read_128B_share": k.get("read_128B_share"),
            "correction": f"round 6: read bytes from gfx950's request-size split, write = WRITE_SIZE x 1024 "
                          f"({os.path.relpath(src, ROOT)})"}
    d["note"] = "round 6: every shard size re-measured by read-request size on the shipped kernel"
    with open(path, "w") as f:
        json.dump(d, f, indent=1)
        f.write("\n")
    print(json.dumps(d["shards"], indent=1))


if __name__ == "__main__":
    main()
