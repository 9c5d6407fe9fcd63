#!/usr/bin/env python3
"""C5 aggregate-scan timing for an A/B library variant (tools/build_variant.sh):
MBX_LIB=<path of libmbx_NAME.so> selects the library (default: the
production libmbx.so).  125M rows of i32 / f32 / char(16),
(c0 < 2^19) ^ (c1 >= 0.25) ^ (c2 >= "M") -> COUNT, SUM / MIN / MAX(c1): one
graph of 20 aggregate scans replayed 5 times between HIP events on the
library stream; the folded record checked against torch.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import mbx_pkg
    m = mbx_pkg.load()
    M, D = m.mbx, m.dist
    if os.environ.get("MBX_LIB"):
        M.LIB_PATH = os.environ["MBX_LIB"]
    n, K = 125_000_000, 20
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    c0 = torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g)
    c1 = torch.rand((n,), dtype=torch.float32, device="cuda", generator=g)
    dic = bench.c5_dictionary(torch)
    c2 = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    for a in range(0, n, 1 << 23):
        idx = torch.randint(0, 50, (min(1 << 23, n - a),), dtype=torch.int64, device="cuda", generator=g)
        c2[a:a + (1 << 23)].copy_(dic[idx])
    sel = (c0 < (1 << 19)) & (c1 >= 0.25) & (c2[:, 0] >= ord("M"))
    want = dict(count=int(sel.sum().item()), sum=float(torch.where(sel, c1.double(), 0.0).sum().item()),
                min=float(torch.where(sel, c1, float("inf")).min().item()),
                max=float(torch.where(sel, c1, float("-inf")).max().item()))
    del sel
    ctx = m.Context(0)
    ext = torch.cuda.ExternalStream(ctx.stream)
    t = ctx.wrap([(M.INTEGER, 4), (M.REAL, 4), (M.STRING, 16)], [c0.data_ptr(), c1.data_ptr(), c2.data_ptr()], n)
    plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", 1 << 19))], [(M.GE, ("sym", 2), ("real", 0.25))],
                           [(M.GE, ("sym", 3), ("str", "M"))]])
    rec = torch.zeros(D.AGG_WORDS, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.scan_aggregate_async(plan, 1, rec.data_ptr())  # uploads the plan and sizes scratch before the capture
    ctx.sync()
    ctx.graph_begin()
    for _ in range(K):
        ctx.scan_aggregate_async(plan, 1, rec.data_ptr())
    gr = ctx.graph_end()
    gr.launch()
    ctx.sync()
    r = bench.check_aggregate("C5", D.fold_aggregates(rec.cpu().numpy()), want)
    assert r is None, r
    us = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(ext)
        gr.launch()
        b.record(ext)
        ctx.sync()
        us.append(a.elapsed_time(b) / K * 1e3)
    r = bench.check_aggregate("C5", D.fold_aggregates(rec.cpu().numpy()), want)
    assert r is None, r
    gr.close()
    ctx.close()
    print(json.dumps({"lib": os.path.basename(M.LIB_PATH), "us_per_scan": sorted(us)[2],
                      "us_all": [round(x, 2) for x in us]}), flush=True)


if __name__ == "__main__":
    main()
