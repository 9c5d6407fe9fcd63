#!/usr/bin/env python3
"""Where the C3 kernel's time goes, under `rocprofv3 --kernel-trace --stats`:
the read probe (mbx_probe_read: the scan's loads, no predicate, no finalize)
in the scan's segment mapping and grid-stride, and the scan in its variants
with the in-kernel finalize (MBX_FIN_MODE=0) and with a separate finalize
launch (MBX_FIN_MODE=2).  Each configuration runs `--launches` times; the
per-kernel averages come from the trace."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--launches", type=int, default=50)
    ap.add_argument("--variants", default="0,12,16,17")
    args = ap.parse_args()
    import torch
    import mbx_pkg

    m = mbx_pkg.load()
    ctx = m.Context(0)
    n = args.rows
    cols = []
    for j in range(4):
        g = torch.Generator(device="cuda")
        g.manual_seed(42 + j)
        cols.append(torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g))
    torch.cuda.synchronize()
    t = ctx.wrap([(m.mbx.INTEGER, 4)] * 4, [c.data_ptr() for c in cols], n)
    plan = ctx.compile(t, [[(m.mbx.LT, ("sym", 1), ("int", 1 << 19))], [(m.mbx.GE, ("sym", 2), ("int", 1 << 19))]])
    want = int(((cols[0] < (1 << 19)) & (cols[1] >= (1 << 19))).sum().item())
    out = torch.zeros(args.launches, dtype=torch.int64, device="cuda")
    for _ in range(args.launches):
        ctx.probe_read(t, [0, 1])
    for _ in range(args.launches):
        ctx.probe_read(t, [0, 1], interleave=True, grid=1024)
    ctx.sync()
    for fin in ("0", "2"):
        os.environ["MBX_FIN_MODE"] = fin
        for v in args.variants.split(","):
            os.environ["MBX_SCAN_VARIANT"] = v
            for k in range(args.launches):
                ctx.scan_count_async(plan, out.data_ptr() + 8 * k)
            ctx.sync()
            assert bool((out.cpu() == want).all()), (fin, v)
    ctx.close()
    print("ANATOMY_OK")


if __name__ == "__main__":
    main()
