#!/usr/bin/env python3
"""C5 (125 M rows of i32 / f32 / char(16), (c0 < 2^19) ^ (c1 >= 0.25) ^
(c2 >= "M") -> COUNT, SUM / MIN / MAX(c1)) per scan grid (tuning
tiles_per_block; 0 = the default, ~4096 blocks for string-slot plans):
query time from a captured graph of 20 queries (scan + its fold), results
checked against torch for every grid.  One JSON line per grid."""
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
    ctx = m.Context(0)
    ext = torch.cuda.ExternalStream(ctx.stream)
    torch.cuda.set_stream(ext)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    c0 = torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g)
    c1 = torch.rand((n,), dtype=torch.float32, device="cuda", generator=g)
    dic = bench.c5_dictionary(torch)
    c2 = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    for a in range(0, n, 1 << 23):
        idx = torch.randint(0, 50, (min(1 << 23, n - a),), dtype=torch.int64, device="cuda", generator=g)
        c2[a:a + (1 << 23)].copy_(dic[idx])
    t = ctx.wrap([(M.INTEGER, 4), (M.REAL, 4), (M.STRING, 16)], [c0.data_ptr(), c1.data_ptr(), c2.data_ptr()], n)
    plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", 1 << 19))], [(M.GE, ("sym", 2), ("real", 0.25))],
                           [(M.GE, ("sym", 3), ("str", "M"))]])
    sel = (c0 < (1 << 19)) & (c1 >= 0.25) & (c2[:, 0] >= ord("M"))
    want = dict(count=int(sel.sum().item()), sum=float(torch.where(sel, c1.double(), 0.0).sum().item()),
                min=float(torch.where(sel, c1, float("inf")).min().item()),
                max=float(torch.where(sel, c1, float("-inf")).max().item()))
    del sel
    rec = torch.zeros(D.AGG_WORDS, dtype=torch.int64, device="cuda")
    ntiles = -(-n // 256)
    bad = 0
    for blocks in [0, 1024, 2048, 4096, 8192]:
        tpb = 0 if blocks == 0 else -(-ntiles // blocks)
        ctx.set_tuning("tiles_per_block", tpb)
        rec.zero_()
        torch.cuda.synchronize()
        ctx.scan_aggregate_async(plan, 1, rec.data_ptr())
        ctx.sync()
        r = bench.check_aggregate("C5", D.fold_aggregates(rec.cpu().numpy()), want)
        ctx.graph_begin()
        for _ in range(20):
            ctx.scan_aggregate_async(plan, 1, rec.data_ptr())
        gr = ctx.graph_end()
        gr.launch()
        ctx.sync()
        us = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(ext)
            gr.launch()
            e1.record(ext)
            ctx.sync()
            us.append(e0.elapsed_time(e1) / 20 * 1e3)
        gr.close()
        r2 = bench.check_aggregate("C5", D.fold_aggregates(rec.cpu().numpy()), want)
        bad += bool(r or r2)
        print(json.dumps({"rows": n, "blocks": blocks, "tiles_per_block": tpb, "ok": not (r or r2),
                          "us": sorted(us)[2], "us_all": [round(x, 1) for x in us],
                          "gbs": n * 24 / (sorted(us)[2] * 1e-6) / 1e9}), flush=True)
    ctx.set_tuning("tiles_per_block", 0)
    ctx.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
