#!/usr/bin/env python3
"""Round-2 anatomy of the two configs furthest below their roofline.

C2 (10M rows x int32, c0 < 104858 -> BitSet + positions + COUNT): HIP-event
times on the library stream, back-to-back launches, of
  boundary     k_read_probe over one 256-row tile (a dependent trivial launch)
  scan_count   k_scan_fast<1, COUNT>
  scan_bitmap  k_scan_fast<1, BITMAP>
  select       k_select_ids alone over the finished BitSet
  scan_select  mbx_scan_select_async (scan + compaction)
Gather calibration (C4 table, 100M rows, 2 int32 projected columns): BitSets
with exactly one selected row every S rows (S = 16, 32, 64, 128: one row per
64-B / 128-B line, every 2nd / 4th 128-B line) and the C4 query's random 1 %
(c2 == 3 AND c3 == 7) -> positions + gather c0, c1 (mbx_materialize_async).
Under rocprofv3 --pmc the per-dispatch FETCH_SIZE of k_gather is set beside
the known number of lines each stride touches (tools/kernel_pmc_table.py).
One JSON line per measurement.  --variants: extra tuning settings to A/B
(knob=value[,knob=value]; "base" = defaults), interleaved over rounds.
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
    ap.add_argument("--launches", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--parts", default="c2,gather")
    ap.add_argument("--variants", default="base")
    ap.add_argument("--gather-rows", type=int, default=100_000_000)
    ap.add_argument("--c2-rows", type=int, default=10_000_000)
    ap.add_argument("--c3-rows", default="12500000,25000000")
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

    def gen_int(n, hi, seed):
        g = torch.Generator(device="cuda")
        g.manual_seed(seed)
        return torch.randint(0, hi, (n,), dtype=torch.int32, device="cuda", generator=g)

    variants = []
    for v in args.variants.split(";"):
        kv = {}
        if v != "base":
            for item in v.split(","):
                k, x = item.split("=")
                kv[k] = int(x)
        variants.append((v, kv))

    def apply(kv):
        ctx.set_tuning("reset", 0)
        for k, x in kv.items():
            ctx.set_tuning(k, x)

    def out(d):
        print(json.dumps(d), flush=True)

    if "c2" in args.parts:
        n = args.c2_rows
        c0 = gen_int(n, 1 << 20, 42)
        tiny = gen_int(256, 1 << 20, 7)
        t = ctx.wrap([(M.INTEGER, 4)], [c0.data_ptr()], n)
        tt = ctx.wrap([(M.INTEGER, 4)], [tiny.data_ptr()], 256)
        plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", 104858))]])
        want = int((c0 < 104858).sum().item())
        ids = torch.zeros(n, dtype=torch.int64, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        ref = torch.nonzero(c0 < 104858).flatten()
        res = {name: [] for name, _ in variants}
        for _ in range(args.rounds):
            for name, kv in variants:
                apply(kv)
                bm = ctx.bitmap_alloc(n)  # segment size read at allocation
                r = {}
                r["boundary"] = timed(lambda: ctx.probe_read(tt, [0]))
                r["probe"] = timed(lambda: ctx.probe_read(t, [0]))
                r["scan_count"] = timed(lambda: ctx.scan_count_async(plan, cnt.data_ptr()))
                r["scan_bitmap"] = timed(lambda: ctx.scan_bitmap_async(plan, bm))
                r["select"] = timed(lambda: M._chk(L.mbx_materialize_async(ctx.h, t.h, bm.h, None, 0, ids.data_ptr(),
                                                                          None, cnt.data_ptr())))
                r["scan_select"] = timed(lambda: ctx.scan_select_async(plan, bm, ids.data_ptr(), cnt.data_ptr()))
                got = int(cnt.item())
                if not (kv.get("select_dbg", 0) & 3):  # bits 0 / 1 make wrong output on purpose
                    assert got == want, (name, got, want)
                    assert bool((ids[:got] == ref).all()), name
                res[name].append(r)
                bm.close()
        for name, _ in variants:
            med = {k: round(statistics.median(r[k] for r in res[name]), 2) for k in res[name][0]}
            out({"part": "c2", "rows": n, "variant": name, "selected": want, "us": med})
        # per-block wall_clock64 stamps (100 MHz) of one compaction after its
        # scan (two launches), and of the one-launch form
        for stamp_cfg in ({"select_dbg": 8, "scan_select_fused": 0}, {"select_dbg": 8, "scan_select_fused": 1},
                          {"select_dbg": 8 | 1024, "scan_select_fused": 1}):
          apply(stamp_cfg)
          bm = ctx.bitmap_alloc(n)
          for _ in range(5):
            ctx.scan_select_async(plan, bm, ids.data_ptr(), cnt.data_ptr())
          ctx.sync()
          nbits, nwords, bcount = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
          M._chk(L.mbx_bitmap_info(bm.h, ctypes.byref(nbits), ctypes.byref(nwords), ctypes.byref(bcount)))
          tpb = max(4, (((n + 255) // 256) + 1023) // 1024)  # choose_tiles_per_block
          nb = (nwords.value + 4 * tpb - 1) // (4 * tpb)
          if stamp_cfg.get("scan_select_fused") and stamp_cfg.get("scan_select_waves", 16) == 16:
              nb = (nb + 3) // 4  # k_scan_select: four BitSet segments per 16-wave block
          st = np.zeros(4 * nb, dtype=np.int64)
          M._chk(L.mbx_diag_select_stamps(ctx.h, st.ctypes.data, nb))
          xcc = None
          st = st.reshape(nb, 4)
          st[:, 0] &= (1 << 60) - 1
          st = st.astype(np.float64) * 10.0 / 1e3  # us
          t0 = st[:, 0].min()
          st -= t0
          q = lambda a: [round(float(np.percentile(a, p)), 2) for p in (0, 10, 50, 90, 100)]
          # k_select_ids: start / words+prefix in / barrier / end
          out({"part": "c2_stamps", "cfg": stamp_cfg, "blocks": nb, "s0_pct": q(st[:, 0]), "s1_pct": q(st[:, 1]),
               "s2_pct": q(st[:, 2]), "s3_pct": q(st[:, 3]),
               "s1_s0_pct": q(st[:, 1] - st[:, 0]), "s2_s1_pct": q(st[:, 2] - st[:, 1]),
               "s3_s2_pct": q(st[:, 3] - st[:, 2]),
               "scan_done_by_xcd": None if xcc is None else
               {int(x): [round(float(np.median(st[xcc == x, 1])), 2), round(float(st[xcc == x, 1].max()), 2)]
                for x in np.unique(xcc)},
               "scan_done_by_block_decile": [round(float(np.median(st[i * nb // 10:(i + 1) * nb // 10, 1])), 2)
                                             for i in range(10)]})
          bm.close()
        apply({})
        del c0, tiny, t, tt, plan, ids, ref
        torch.cuda.empty_cache()

    if "c3small" in args.parts:
        # the strong-scaling shard (12.5M rows = 100M / 8 GPUs) and 25M: C3
        # COUNT scan vs its read probe, finalize / ticket / grid variants
        for n in map(int, args.c3_rows.split(",")):
            cols = [gen_int(n, 1 << 20, 42 + j) for j in range(2)]
            t = ctx.wrap([(M.INTEGER, 4)] * 2, [c.data_ptr() for c in cols], n)
            plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", 1 << 19))], [(M.GE, ("sym", 2), ("int", 1 << 19))]])
            want = int(((cols[0] < (1 << 19)) & (cols[1] >= (1 << 19))).sum().item())
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            res = {}
            for _ in range(args.rounds):
                for name, kv in variants:
                    apply(kv)
                    r = res.setdefault(name, {"scan": [], "probe": []})
                    r["scan"].append(timed(lambda: ctx.scan_count_async(plan, cnt.data_ptr())))
                    r["probe"].append(timed(lambda: ctx.probe_read(t, [0, 1])))
                    if kv.get("fin_mode") != 4:  # the diagnostic form produces no count
                        assert int(cnt.item()) == want, name
            for name, _ in variants:
                out({"part": "c3small", "rows": n, "variant": name,
                     "scan_us": round(statistics.median(res[name]["scan"]), 2),
                     "probe_us": round(statistics.median(res[name]["probe"]), 2),
                     "scan_tbs": round(8 * n / statistics.median(res[name]["scan"]) / 1e6, 3)})
            del cols, t, plan
            torch.cuda.empty_cache()
        apply({})

    if "bitset" in args.parts:
        # BitSet vs COUNT scan of one column at 100M rows
        n = 100_000_000
        c0 = gen_int(n, 1 << 20, 42)
        t = ctx.wrap([(M.INTEGER, 4)], [c0.data_ptr()], n)
        plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", 104858))]])
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        res = {}
        for _ in range(args.rounds):
            for name, kv in variants:
                apply(kv)
                bm = ctx.bitmap_alloc(n)
                r = res.setdefault(name, {"count": [], "bitset": [], "probe": []})
                r["count"].append(timed(lambda: ctx.scan_count_async(plan, cnt.data_ptr())))
                r["bitset"].append(timed(lambda: ctx.scan_bitmap_async(plan, bm)))
                r["probe"].append(timed(lambda: ctx.probe_read(t, [0])))
                bm.close()
        for name, _ in variants:
            out({"part": "bitset", "rows": n, "variant": name,
                 **{k + "_us": round(statistics.median(v), 2) for k, v in res[name].items()}})
        del c0, t, plan
        torch.cuda.empty_cache()
        apply({})

    if "gather" in args.parts:
        n = args.gather_rows
        c0, c1 = gen_int(n, 1 << 20, 42), gen_int(n, 1 << 20, 43)
        c2, c3 = gen_int(n, 10, 44), gen_int(n, 10, 45)
        t = ctx.wrap([(M.INTEGER, 4)] * 4, [x.data_ptr() for x in (c0, c1, c2, c3)], n)
        nw = (n + 63) // 64
        cases = []
        for S in (16, 32, 64, 128):
            assert n % 128 == 0
            w = np.zeros(nw, dtype=np.uint64)
            if S <= 64:
                w[:] = np.uint64(sum(1 << (k * S) for k in range(64 // S)))
            else:
                w[::S // 64] = np.uint64(1)
            pos = np.arange(0, n, S, dtype=np.int64)
            cases.append((f"stride{S}", ctx.bitmap_upload(n, w), len(pos), pos))
        sel = (c2 == 3) & (c3 == 7)
        bms = ctx.index_build(t, 2, [("int", 3)]) + ctx.index_build(t, 3, [("int", 7)])
        rnd = ctx.bitmap_cnf(n, [[bms[0]], [bms[1]]])
        cases.append(("c4_random_1pct", rnd, int(sel.sum().item()), None))
        cap = max(c[2] for c in cases)
        ids = torch.zeros(cap, dtype=torch.int64, device="cuda")
        o0 = torch.zeros(cap, dtype=torch.int32, device="cuda")
        o1 = torch.zeros(cap, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        proj = (ctypes.c_int32 * 2)(0, 1)
        outs = (ctypes.c_void_p * 2)(o0.data_ptr(), o1.data_ptr())
        for name, bm, k, pos in cases:
            for vname, kv in variants:
                apply(kv)
                f_sel = lambda: M._chk(L.mbx_materialize_async(ctx.h, t.h, bm.h, None, 0, ids.data_ptr(), None,
                                                               cnt.data_ptr()))
                f_all = lambda: M._chk(L.mbx_materialize_async(ctx.h, t.h, bm.h, proj, 2, ids.data_ptr(), outs,
                                                               cnt.data_ptr()))
                ts = statistics.median(timed(f_sel) for _ in range(args.rounds))
                ta = statistics.median(timed(f_all) for _ in range(args.rounds))
                got = int(cnt.item())
                assert got == k, (name, got, k)
                if pos is not None:
                    p = torch.from_numpy(pos).cuda()
                    assert bool((ids[:k] == p).all()) and bool((o0[:k] == c0[p]).all()) and bool((o1[:k] == c1[p]).all())
                else:
                    assert bool((o0[:k] == c0[sel]).all()) and bool((o1[:k] == c1[sel]).all())
                # lines the 2 projected columns touch (one 4-byte value per selected row)
                if pos is not None:
                    l128 = 2 * len(np.unique(pos >> 5))
                    l64 = 2 * len(np.unique(pos >> 4))
                else:
                    sp = torch.nonzero(sel).flatten()
                    l128 = 2 * int(torch.unique(sp >> 5).numel())
                    l64 = 2 * int(torch.unique(sp >> 4).numel())
                out({"part": "gather", "case": name, "variant": vname, "rows": n, "selected": k,
                     "select_us": round(ts, 2), "select_gather_us": round(ta, 2), "gather_us": round(ta - ts, 2),
                     "lines128": l128, "lines64": l64, "bytes_line128": l128 * 128, "bytes_line64": l64 * 64,
                     "ids_bytes": 8 * k, "out_bytes": 8 * k})
        apply({})
    ctx.close()


if __name__ == "__main__":
    main()
