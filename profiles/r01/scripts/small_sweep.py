#!/usr/bin/env python3
"""Segment-size sweep for the launch-latency-bound sizes (C2's 10M rows, the
8-GPU C4 shard of 12.5M rows, C4's 100M-row bitmaps): MBX_TILES_PER_BLOCK
(256-row tiles per block; a bitmap's segment = 4 words per tile) is read when
a bitmap is allocated and when a scan is launched, so each setting gets its
own bitmaps.  Per setting, HIP-event times on the library stream of
  scan_count   (c0 < 104858)                      k_scan_fast<1, COUNT>
  scan_bitmap  (c0 < 104858) -> BitSet            k_scan_fast<1, BITMAP>
  select       BitSet -> positions                k_select_ids
  scan_select  BitSet + positions, one launch     k_scan_fast<1, SELECT> (mbx_scan_select_async)
  and          bm_a AND bm_b (random 10 % / 10 %) k_bitmap_cnf
  and_sel_g    AND + positions + gather c0, c1    (C4 query)
Interleaved rounds, median of rounds.  One JSON line per (rows, tpb).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="10000000,12500000,100000000")
    ap.add_argument("--tpb", default="0,2,4,8,12,16,24")
    ap.add_argument("--launches", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ops", default="scan_count,scan_bitmap,select,scan_select,and,and_sel_g")
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
        return a.elapsed_time(b) / args.launches * 1e3  # us

    for n in map(int, args.rows.split(",")):
        cols = []
        for j in range(2):
            g = torch.Generator(device="cuda")
            g.manual_seed(42 + j)
            cols.append(torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g))
        rng = np.random.Generator(np.random.PCG64(7))
        nw = (n + 63) // 64
        wa = np.packbits(rng.random(nw * 64) < 0.1, bitorder="little").view(np.uint64)[:nw].copy()
        wb = np.packbits(rng.random(nw * 64) < 0.1, bitorder="little").view(np.uint64)[:nw].copy()
        t = ctx.wrap([(M.INTEGER, 4)] * 2, [c.data_ptr() for c in cols], n)
        plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", 104858))]])
        want = int((cols[0] < 104858).sum().item())
        want_and = int(np.unpackbits((wa & wb).view(np.uint8)).sum())
        ids = torch.zeros(n, dtype=torch.int64, device="cuda")
        o0 = torch.zeros(n // 20, dtype=torch.int32, device="cuda")
        o1 = torch.zeros(n // 20, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
        proj = (ctypes.c_int32 * 2)(0, 1)
        outs = (ctypes.c_void_p * 2)(o0.data_ptr(), o1.data_ptr())
        res = {}
        tpbs = list(map(int, args.tpb.split(",")))
        for rnd in range(args.rounds):
            for tp in tpbs:
                if tp:
                    os.environ["MBX_TILES_PER_BLOCK"] = str(tp)
                else:
                    os.environ.pop("MBX_TILES_PER_BLOCK", None)
                bm = ctx.bitmap_alloc(n)
                ba = ctx.bitmap_upload(n, wa)
                bb = ctx.bitmap_upload(n, wb)
                out = ctx.bitmap_alloc(n)
                r = {}
                ops = args.ops.split(",")
                if "scan_count" in ops:
                    r["scan_count"] = timed(lambda: ctx.scan_count_async(plan, cnt.data_ptr()))
                    assert int(cnt[0].item()) == want
                r["scan_bitmap"] = timed(lambda: ctx.scan_bitmap_async(plan, bm))
                if "select" in ops:
                    r["select"] = timed(lambda: M._chk(L.mbx_materialize_async(ctx.h, t.h, bm.h, None, 0,
                                                                                ids.data_ptr(), None,
                                                                                cnt.data_ptr() + 8)))
                    assert int(cnt[1].item()) == want
                if "scan_select" in ops:  # BitSet + positions in one launch (C2's query)
                    r["scan_select"] = timed(lambda: M._chk(L.mbx_scan_select_async(ctx.h, plan.h, bm.h, ids.data_ptr(),
                                                                                    cnt.data_ptr() + 24)))
                    if not os.environ.get("SWEEP_NOCHECK"):  # A/B knobs that drop work
                        assert int(cnt[3].item()) == want
                        assert bool((ids[:want] == torch.nonzero(cols[0] < 104858).flatten()).all())
                # ctypes arguments built once: the launch itself is what is timed
                bms = (ctypes.c_void_p * 2)(ba.h.value, bb.h.value)
                offs = (ctypes.c_int32 * 3)(0, 1, 2)
                if "and" in ops:
                    r["and"] = timed(lambda: L.mbx_bitmap_cnf_async(ctx.h, bms, offs, 2, None, out.h))

                def c4():
                    L.mbx_bitmap_cnf_async(ctx.h, bms, offs, 2, None, out.h)
                    M._chk(L.mbx_materialize_async(ctx.h, t.h, out.h, proj, 2, ids.data_ptr(), outs,
                                                   cnt.data_ptr() + 16))

                if "and_sel_g" in ops:
                    r["and_sel_g"] = timed(c4)
                    assert int(cnt[2].item()) == want_and
                for k, v in r.items():
                    res.setdefault((tp, k), []).append(v)
                del bm, ba, bb, out
        os.environ.pop("MBX_TILES_PER_BLOCK", None)
        for tp in tpbs:
            line = {"rows": n, "tpb": tp or "default"}
            for k in ["scan_count", "scan_bitmap", "select", "scan_select", "and", "and_sel_g"]:
                if (tp, k) in res:
                    line[k + "_us"] = round(statistics.median(res[(tp, k)]), 2)
            print(json.dumps(line), flush=True)
        del cols, t, plan, ids, o0, o1
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
