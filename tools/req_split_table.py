#!/usr/bin/env python3
"""C4 read-request table: per kernel of a tools/gpu_r6_a.sh
session, the L2 -> memory read requests by size (TCC_EA0_RDREQ_32B / _64B /
_128B), their bytes, the byte counter of DRAM-bound requests
(TCC_EA0_RDREQ_DRAM_32B x 32), FETCH_SIZE x 2 (the earlier rounds' read figure),
and for tools/c4_req_probe's kernels the footprint counted on the host (distinct
32 / 64 / 128-byte pieces the loads touch).  Writes table.json + table.md.
    python3 tools/req_split_table.py profiles/r06/c4_req"""
import json
import os
import sys


def main():
    d = sys.argv[1]
    probe = {j["kernel"]: j for j in (json.loads(x) for x in open(os.path.join(d, "probe.jsonl")) if x.strip())}
    rows = []
    for f in ("probe_table.jsonl", "bench_table.jsonl"):
        for line in open(os.path.join(d, f)):
            k = json.loads(line)
            name = k["kernel"]
            if not any(name.startswith(p) for p in ("k_stream", "k_words", "k_pair", "k_col2", "k_scan_fast",
                                                    "k_cnf_select")):
                continue
            n32, n64, n128 = (k.get(f"TCC_EA0_RDREQ_{w}B_sum", 0.0) for w in (32, 64, 128))
            tot = k.get("TCC_EA0_RDREQ_sum", 0.0)
            r = {"kernel": name, "source": f, "avg_us": k.get("avg_us"), "rdreq": tot, "rdreq_32B": n32,
                 "rdreq_64B": n64, "rdreq_128B": n128, "split_read_MB": (32 * n32 + 64 * n64 + 128 * n128) / 1e6,
                 "dram_32B_x32_MB": 32 * k.get("TCC_EA0_RDREQ_DRAM_32B_sum", 0.0) / 1e6,
                 "fetch_x2_MB": k.get("fetch_x2_MB", k.get("read_MB")), "write_MB": k.get("write_MB"),
                 "wrreq_64B": k.get("TCC_EA0_WRREQ_64B_sum"), "wrreq": k.get("TCC_EA0_WRREQ_sum"),
                 "share_128B": n128 / tot if tot else None}
            p = probe.get(name)
            if p:
                if "bytes" in p:
                    r["footprint_MB"] = p["bytes"] / 1e6
                else:  # gathers: touched lines of the values + the streamed positions
                    r["footprint_lines128_MB"] = (p["lines128"] * 128 + p["pos_bytes"]) / 1e6
                    r["footprint_sectors64_MB"] = (p["sectors64"] * 64 + p["pos_bytes"]) / 1e6
                    r["footprint_sectors32_MB"] = (p["sectors32"] * 32 + p["pos_bytes"]) / 1e6
                    r["selected"] = p["selected"]
            rows.append(r)
    with open(os.path.join(d, "table.json"), "w") as f:
        json.dump(rows, f, indent=1)
        f.write("\n")
    hdr = ("| kernel | 32-B req | 64-B req | 128-B req | split bytes (MB) | DRAM 32-B x 32 (MB) | FETCH_SIZE x 2 (MB) |"
           " host footprint (MB): 128-B lines / 64-B / 32-B pieces |\n|---|---|---|---|---|---|---|---|\n")
    out = []
    for r in rows:
        fp = (f"{r['footprint_MB']:.1f} (streamed)" if "footprint_MB" in r else
              f"{r['footprint_lines128_MB']:.1f} / {r['footprint_sectors64_MB']:.1f} / {r['footprint_sectors32_MB']:.1f}"
              if "footprint_lines128_MB" in r else "—")
        out.append(f"| `{r['kernel'][:48]}` | {r['rdreq_32B']:.0f} | {r['rdreq_64B']:.0f} | {r['rdreq_128B']:.0f} | "
                   f"{r['split_read_MB']:.1f} | {r['dram_32B_x32_MB']:.1f} | {r['fetch_x2_MB']:.1f} | {fp} |")
    with open(os.path.join(d, "table.md"), "w") as f:
        f.write(hdr + "\n".join(out) + "\n")
    print(hdr + "\n".join(out))


if __name__ == "__main__":
    main()
