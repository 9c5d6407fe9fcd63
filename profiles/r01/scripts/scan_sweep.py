#!/usr/bin/env python3
"""A/B sweep of the C3 scan kernel variants in ONE process, interleaved
rounds (cdna_hip_programming.md rule 24).  Knobs are the library's tuning
environment variables, read at each launch:
  MBX_SCAN_VARIANT     1..6 = U{1,2,4} x {plain, nontemporal} loads (k_scan_fast<2,COUNT>)
  MBX_TILES_PER_BLOCK  256-row tiles per block (segment size -> grid size)
  MBX_FORCE_GENERIC    1 = one-row-per-lane kernel (read at plan compile)
Prints one JSON line per configuration with median / min kernel time.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="0,1,2,3,4,5,6")
    ap.add_argument("--tpb", default="0,24,48,96,191,382")
    ap.add_argument("--generic", action="store_true")
    ap.add_argument("--fin", default="0", help="MBX_FIN_MODE values: 0 write-through, 2 separate (1 fences: -DMBX_DIAG builds)")
    ap.add_argument("--groups", default="32", help="MBX_TICKET_GROUPS values (0/1: one flat ticket)")
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
    cnf = [[(m.mbx.LT, ("sym", 1), ("int", 1 << 19))], [(m.mbx.GE, ("sym", 2), ("int", 1 << 19))]]
    want = int(((cols[0] < (1 << 19)) & (cols[1] >= (1 << 19))).sum().item())
    plan = ctx.compile(t, cnf)
    os.environ["MBX_FORCE_GENERIC"] = "1"
    gplan = ctx.compile(t, cnf)
    del os.environ["MBX_FORCE_GENERIC"]
    ext = torch.cuda.ExternalStream(ctx.stream)
    out = torch.zeros(args.launches, dtype=torch.int64, device="cuda")

    fins = list(map(int, args.fin.split(",")))
    grps = list(map(int, args.groups.split(",")))
    configs = [(v, tp, False, f, g) for v in map(int, args.variants.split(",")) for tp in map(int, args.tpb.split(","))
               for f in fins for g in grps]
    if args.generic:
        configs += [(0, tp, True, fins[0], grps[0]) for tp in map(int, args.tpb.split(","))]
    res = {c: [] for c in configs}
    for r in range(args.rounds):
        for c in configs:
            v, tp, gen, fin, grp = c
            os.environ["MBX_SCAN_VARIANT"] = str(v)
            os.environ["MBX_TICKET_GROUPS"] = str(grp)
            os.environ["MBX_FIN_MODE"] = str(fin)
            if tp:
                os.environ["MBX_TILES_PER_BLOCK"] = str(tp)
            else:
                os.environ.pop("MBX_TILES_PER_BLOCK", None)
            p = gplan if gen else plan
            for k in range(3):
                ctx.scan_count_async(p, out.data_ptr())
            es = [torch.cuda.Event(enable_timing=True) for _ in range(args.launches + 1)]
            es[0].record(ext)
            for k in range(args.launches):
                ctx.scan_count_async(p, out.data_ptr() + 8 * k)
                es[k + 1].record(ext)
            ctx.sync()
            ts = [es[k].elapsed_time(es[k + 1]) for k in range(args.launches)]
            got = out.cpu()
            assert bool((got == want).all()), (c, got[:4], want)
            res[c].append(statistics.median(ts))
    for c in configs:
        v, tp, gen, fin, grp = c
        med = statistics.median(res[c])
        print(json.dumps({"variant": v, "tiles_per_block": tp or "default", "generic": gen, "fin_mode": fin,
                          "ticket_groups": grp,
                          "median_ms": med, "min_ms": min(res[c]),
                          "gbs": 8 * n / (med * 1e-3) / 1e9, "rows": n}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
