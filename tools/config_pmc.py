#!/usr/bin/env python3
"""profiles/config_pmc.json: HBM bytes per launch of each config record's
kernel (bench.py `configs.*.traffic`), from the per-kernel table of rocprofv3
passes over a short bench.py (tools/kernel_pmc_table.py) and that run's bench
line (the rows per GPU each config ran at).  Read bytes come from gfx950's
read-request size split (TCC_EA0_RDREQ_32B / _64B / _128B: 32 n32 + 64 n64 +
128 n128) when the table has it -- the x 2 correction of FETCH_SIZE is then
not applied anywhere; it is the fallback only for tables without the split
(round 5's).  Write bytes = WRITE_SIZE x 1024 (64-byte write requests,
exact: profiles/r06/c4_req).
    python3 tools/config_pmc.py profiles/r06/b/kernels.jsonl profiles/r06/b/bench_pmc.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"C2": "k_scan_select<", "C4": "k_cnf_select<", "C5": "k_scan_fast<2, 1, 2,"}


def main():
    table = [json.loads(x) for x in open(sys.argv[1]) if x.strip()]
    bench = json.loads(open(sys.argv[2]).read())
    out = {"source": [os.path.relpath(os.path.abspath(p), ROOT) for p in sys.argv[1:3]], "configs": {}}
    for name, sub in KERNELS.items():
        rec = bench["configs"][name]
        k = [t for t in table if t["kernel"].startswith(sub)]
        assert len(k) == 1, (name, [t["kernel"] for t in k])
        k = k[0]
        hbm = (k["read_MB"] + k["write_MB"]) * 1e6
        out["configs"][f"{name}:{rec['rows_per_gpu']}"] = {
            "kernel": k["kernel"], "dispatches": k["dispatches"], "avg_us": k["avg_us"],
            "read_basis": k.get("read_basis"), "read_128B_share": k.get("read_128B_share"),
            "fetch_x2_bytes_per_launch": k["fetch_x2_MB"] * 1e6 if "fetch_x2_MB" in k else None,
            "read_bytes_per_launch": k["read_MB"] * 1e6, "write_bytes_per_launch": k["write_MB"] * 1e6,
            "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": rec["algorithmic_bytes_per_launch"],
            "traffic_over_algorithmic": hbm / rec["algorithmic_bytes_per_launch"]}
    path = os.path.join(ROOT, "profiles", "config_pmc.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
