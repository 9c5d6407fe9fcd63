#!/usr/bin/env python3
"""C2 anatomy: k_scan_select's kernel time with parts of its tail removed, so
each part's cost shows in production timing (per-block stamps add stores of
their own and shift the waits they measure).  Needs a -DMBX_DIAG build of
libmbx (tools/build_diag.sh -> minibase-columnar-database_amd/libmbx_diag.so),
loaded with --lib; the variants that skip work give wrong positions by design
and are not checked.  HIP events on the library stream, 3 interleaved rounds.

    python3 tools/c2_anatomy.py --lib minibase-columnar-database_amd/libmbx_diag.so
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    import numpy as np  # noqa: F401
    import torch

    import mbx_pkg
    m = mbx_pkg.load()
    M = m.mbx
    if args.lib:
        M.LIB_PATH = os.path.abspath(args.lib)
    L = M.lib()
    ctx = m.Context(0)
    ext = torch.cuda.ExternalStream(ctx.stream)
    n = 10_000_000
    g = torch.Generator(device="cuda")
    cols = []
    for j in range(4):
        g.manual_seed(42 + j)
        cols.append(torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g))
    t = ctx.wrap([(M.INTEGER, 4)] * 4, [c.data_ptr() for c in cols], n)
    plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", 104858))]])
    bm = ctx.bitmap_alloc(n)
    ids = torch.zeros(n, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    wpos = torch.nonzero(cols[0] < 104858).flatten()

    def step():
        M._chk(L.mbx_scan_select_async(ctx.h, plan.h, bm.h, ids.data_ptr(), cnt.data_ptr()))

    def kernel_ms():
        for _ in range(args.warmup):
            step()
        ctx.sync()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(ext)
        for _ in range(args.steps):
            step()
        b.record(ext)
        ctx.sync()
        return a.elapsed_time(b) / args.steps * 1e3

    # select_dbg values (k_scan_select gets select_dbg >> 4): 0 the default;
    # 32 skips the look-back's wait; 1024 skips the positions; 256 skips the
    # staging (and so the positions); 4096 skips the BitSet words; 2048 ends
    # every block once its count is published; 512 plain (not
    # write-through) positions; 8192 nontemporal positions; 128 the chained walk
    variants = {"default": 0, "no_lookback_wait": 32, "no_positions": 1024, "neither": 32 | 1024,
                "no_staging": 256, "no_words": 4096, "no_staging_no_words": 256 | 4096,
                "count_only": 2048, "plain_stores": 512, "nt_stores": 8192, "chained": 128}
    res = {}
    for rep in range(3):
        for k, v in variants.items():
            ctx.set_tuning("select_dbg", v)
            ids.zero_()
            torch.cuda.synchronize()
            res.setdefault(k, []).append(round(kernel_ms(), 2))
            if v in (0, 512, 8192, 128):
                got = int(cnt.item())
                assert got == wpos.numel() and bool((ids[:got] == wpos).all()), k
    ctx.set_tuning("select_dbg", 0)
    print(json.dumps({"config": "C2 anatomy", "lib": os.path.basename(M.LIB_PATH), "us": res}))


if __name__ == "__main__":
    main()
