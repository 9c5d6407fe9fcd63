#!/usr/bin/env python3
"""C3 scan timing for an A/B library variant (tools/build_variant.sh):
MBX_LIB=<path of libmbx_NAME.so> selects the library (default: the
production libmbx.so).  One graph of 40 COUNT scans (the bench's
in-launch-finalize form) replayed 5 times between HIP events on the library
stream; every count checked against torch.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

THRESH = 1 << 19


def main():
    import torch
    import mbx_pkg
    m = mbx_pkg.load()
    M = m.mbx
    if os.environ.get("MBX_LIB"):
        M.LIB_PATH = os.environ["MBX_LIB"]
    n, K = 100_000_000, 40
    cols = []
    for j in range(4):
        g = torch.Generator(device="cuda")
        g.manual_seed(42 + j)
        cols.append(torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g))
    want = int(((cols[0] < THRESH) & (cols[1] >= THRESH)).sum().item())
    ctx = m.Context(0)
    ext = torch.cuda.ExternalStream(ctx.stream)
    t = ctx.wrap([(M.INTEGER, 4)] * 4, [x.data_ptr() for x in cols], n)
    plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", THRESH))], [(M.GE, ("sym", 2), ("int", THRESH))]])
    counts = torch.zeros(K, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.graph_begin()
    for k in range(K):
        ctx.scan_count_async(plan, counts.data_ptr() + 8 * k)
    gr = ctx.graph_end()
    gr.launch()
    ctx.sync()
    assert counts.cpu().tolist() == [want] * K
    us = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(ext)
        gr.launch()
        b.record(ext)
        ctx.sync()
        us.append(a.elapsed_time(b) / K * 1e3)
    assert counts.cpu().tolist() == [want] * K
    gr.close()
    ctx.close()
    print(json.dumps({"lib": os.path.basename(M.LIB_PATH), "us_per_scan": sorted(us)[2],
                      "us_all": [round(x, 2) for x in us]}), flush=True)


if __name__ == "__main__":
    main()
