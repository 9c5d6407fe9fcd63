#!/usr/bin/env python3
"""profiles/config_pmc.json: HBM bytes per launch of each config record's
kernel (bench.py `configs.*.traffic`), from a tools/gpu_r5_e.sh run: the
per-kernel table of rocprofv3 FETCH_SIZE / WRITE_SIZE passes over a short
bench.py (tools/kernel_pmc_table.py: read = FETCH_SIZE x 2 x 1024, the gfx950
correction, write = WRITE_SIZE x 1024) and that run's bench line (the rows
per GPU each config ran at).
    python3 tools/config_pmc.py profiles/r05/e/kernels.jsonl profiles/r05/e/bench_n1.json"""
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
