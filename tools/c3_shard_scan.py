#!/usr/bin/env python3
"""The C3 scan exactly as bench.py launches it on rank 0 of an N-rank run,
for rocprofv3 kernel-trace / PMC passes (profiles/r04/scripts/gpu_r4_shard_pmc.sh): rank 0's
row-range shard of the 100M-row table (mbx_shard_bounds), 4 x int32 columns,
{(c0 < 2^19)} ^ {(c1 >= 2^19)}, COUNT in the same form bench.py picks at that
N (in-launch finalize at N = 1, count frame with an exchange).

    python3 tools/c3_shard_scan.py --gpus N [--launches K] [--count finalize|frame]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--launches", type=int, default=50)
    ap.add_argument("--count", choices=["auto", "finalize", "frame"], default="auto")
    args = ap.parse_args()

    import torch
    import mbx_pkg

    m = mbx_pkg.load()
    ctx = m.Context(0)
    s, e = m.mbx.shard_bounds(args.rows, args.gpus, 0)
    n = e - s
    cols = []
    for j in range(4):
        g = torch.Generator(device="cuda")
        g.manual_seed(42 + j)
        cols.append(torch.randint(0, 1 << 20, (args.rows,), dtype=torch.int32, device="cuda", generator=g)[s:e].clone())
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    t = ctx.wrap([(m.mbx.INTEGER, 4)] * 4, [c.data_ptr() for c in cols], n, None, row_offset=s)
    plan = ctx.compile(t, [[(m.mbx.LT, ("sym", 1), ("int", 1 << 19))], [(m.mbx.GE, ("sym", 2), ("int", 1 << 19))]])
    frame = args.count == "frame" or (args.count == "auto" and args.gpus > 1)
    FW = m.mbx.COUNT_FRAME_WORDS if frame else 1
    buf = torch.zeros((args.launches, FW), dtype=torch.int64, device="cuda")
    for k in range(args.launches):
        if frame:
            ctx.scan_count_frame_async(plan, buf[k].data_ptr())
        else:
            ctx.scan_count_async(plan, buf[k].data_ptr())
    ctx.sync()
    want = int(((cols[0] < (1 << 19)) & (cols[1] >= (1 << 19))).sum().item())
    got = m.mbx.count_frame_decode(buf[-1].cpu().numpy())[0] if frame else int(buf[-1, 0].item())
    assert got == want, (got, want)
    print(f"rows {n} ({s}..{e}) count {'frame' if frame else 'finalize'} x{args.launches}: {got}")
    ctx.close()


if __name__ == "__main__":
    main()
