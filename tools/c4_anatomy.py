#!/usr/bin/env python3
"""Anatomy of the one-launch C4 query (mbx_cnf_materialize_async, k_cnf_select)
at 100M rows: HIP-event time of the one-launch form beside the two-launch
form (k_bitmap_cnf, then k_select_ids<4>), then per-block wall_clock64 stamps
(100 MHz) of one k_cnf_select launch: start / count published / offset known
(look-back done) / end, as percentiles over blocks and medians by block
decile.  One JSON line per measurement."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--launches", type=int, default=50)
    args = ap.parse_args()
    import numpy as np
    import torch
    import mbx_pkg

    m = mbx_pkg.load()
    M = m.mbx
    L = M.lib()
    ctx = m.Context(0)
    ext = torch.cuda.ExternalStream(ctx.stream)

    def timed(fn):
        for _ in range(3):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(ext)
        for _ in range(args.launches):
            fn()
        b.record(ext)
        ctx.sync()
        return round(a.elapsed_time(b) / args.launches * 1e3, 2)

    def gen_int(n, hi, seed):
        g = torch.Generator(device="cuda")
        g.manual_seed(seed)
        return torch.randint(0, hi, (n,), dtype=torch.int32, device="cuda", generator=g)

    n = args.rows
    c0, c1, c2, c3 = gen_int(n, 1 << 20, 42), gen_int(n, 1 << 20, 43), gen_int(n, 10, 44), gen_int(n, 10, 45)
    t = ctx.wrap([(M.INTEGER, 4)] * 4, [x.data_ptr() for x in (c0, c1, c2, c3)], n)
    a = ctx.index_build(t, 2, [("int", 3)])[0]
    b = ctx.index_build(t, 3, [("int", 7)])[0]
    want = int(((c2 == 3) & (c3 == 7)).sum().item())
    cap = max(1, n // 50)
    ids = torch.zeros(cap, dtype=torch.int64, device="cuda")
    o0 = torch.zeros(cap, dtype=torch.int32, device="cuda")
    o1 = torch.zeros(cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = ctx.bitmap_alloc(n)
    bms = (ctypes.c_void_p * 2)(a.h.value, b.h.value)
    offs = (ctypes.c_int32 * 3)(0, 1, 2)
    proj = (ctypes.c_int32 * 2)(0, 1)
    outs = (ctypes.c_void_p * 2)(o0.data_ptr(), o1.data_ptr())
    torch.cuda.synchronize()

    def fused():
        M._chk(L.mbx_cnf_materialize_async(ctx.h, t.h, bms, offs, 2, None, proj, 2, ids.data_ptr(), outs,
                                           cnt.data_ptr()))

    def two():
        M._chk(L.mbx_bitmap_cnf_async(ctx.h, bms, offs, 2, None, out.h))
        M._chk(L.mbx_materialize_async(ctx.h, t.h, out.h, proj, 2, ids.data_ptr(), outs, cnt.data_ptr()))

    def fused_noids():
        M._chk(L.mbx_cnf_materialize_async(ctx.h, t.h, bms, offs, 2, None, proj, 2, None, outs, cnt.data_ptr()))

    def fused_count_only():
        M._chk(L.mbx_cnf_materialize_async(ctx.h, t.h, bms, offs, 2, None, proj, 0, None, outs, cnt.data_ptr()))

    r = {"one_launch": timed(fused), "two_launch": timed(two), "one_launch_no_ids": timed(fused_noids),
         "one_launch_no_columns_no_ids": timed(fused_count_only)}
    fused()
    ctx.sync()
    assert int(cnt.item()) == want
    print(json.dumps({"part": "c4_times_us", "rows": n, "selected": want, **r}), flush=True)

    # variants (select_dbg >> 4 = the kernel's dbg): 512 = write-through
    # output stores; interleaved with the default so box drift does not pass
    # for a difference.  (Round 3 also measured the operand-word phase at
    # raised wave priority: every block then publishes by 7.9 us instead of
    # the 4th block per CU at ~27 us, but the launch stays 43.0 us -- the
    # gathers are bandwidth-bound either way; profiles/r03/c4.)
    for name, dbg in (("default", 0), ("write_through", 512), ("default", 0)):
        ctx.set_tuning("select_dbg", dbg)
        print(json.dumps({"part": "c4_lookback_variant", "variant": name,
                          "one_launch_projection": timed(lambda: M._chk(L.mbx_cnf_materialize_async(
                              ctx.h, t.h, bms, offs, 2, None, proj, 2, None, outs, cnt.data_ptr()))),
                          "one_launch_no_columns_no_ids": timed(fused_count_only)}), flush=True)
    ctx.set_tuning("reset", 0)
    for _ in range(3):
        fused()
    ctx.sync()
    assert int(cnt.item()) == want

    for label, fn, dbg in (("count_only", fused_count_only, 8), ("positions_and_projection", fused, 8),
                           ):
      ctx.set_tuning("select_dbg", dbg)
      for _ in range(5):
        fn()
      ctx.sync()
      nwords = (n + 63) // 64
      wpb = (nwords + 1023) // 1024
      nb = (nwords + wpb - 1) // wpb
      st = np.zeros(4 * nb, dtype=np.int64)
      M._chk(L.mbx_diag_select_stamps(ctx.h, st.ctypes.data, nb))
      ctx.set_tuning("select_dbg", dbg & ~8)
      ku = timed(fn)
      ctx.set_tuning("reset", 0)
      st = st.reshape(nb, 4).astype(np.float64) * 10.0 / 1e3  # us
      st -= st[:, 0].min()
      q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 100)]
      dec = lambda col: [round(float(np.median(col[i * nb // 10:(i + 1) * nb // 10])), 2) for i in range(10)]
      print(json.dumps({"part": "c4_stamps", "form": label, "blocks": nb, "start": q(st[:, 0]),
                      "published": q(st[:, 1]),
                      "offset_known": q(st[:, 2]), "end": q(st[:, 3]),
                      "words_phase": q(st[:, 1] - st[:, 0]), "lookback": q(st[:, 2] - st[:, 1]),
                      "write_phase": q(st[:, 3] - st[:, 2]),
                      "published_by_decile": dec(st[:, 1]), "offset_by_decile": dec(st[:, 2]),
                      "end_by_decile": dec(st[:, 3]),
                      "kernel_us": ku}), flush=True)
      ctx.set_tuning("reset", 0)


if __name__ == "__main__":
    main()
