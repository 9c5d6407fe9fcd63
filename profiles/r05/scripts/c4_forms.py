#!/usr/bin/env python3
"""C4 (ColumnarIndexScan: bm(c2=3) AND bm(c3=7) -> positions + c0, c1) in
one k_cnf_select launch, with and without the (c0, c1) column group: kernel
time from a captured graph of 20 launches (HIP events on the library stream),
results checked against torch at several table sizes first.  One JSON line
per (rows, layout); the process's kernel form is set by the environment
(MBX_GATHER_PAIR=0: two 4-byte loads per grouped row instead of one 8-byte).
Round 5 also A/B'd a two-rounds-per-block form here (profiles/r05/c)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="100000000")
    ap.add_argument("--check-rows", default="1000,70001,1000003,10000000,33554431")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--blocks", default="0", help="comma list of tuning cnf_blocks values (0: the default grid)")
    ap.add_argument("--positions-only", action="store_true", help="no projection: positions + COUNT only")
    ap.add_argument("--waves", default="4", help="4 (the 16-wave A/B knob cnf_waves was removed after round 5's profiles/r05/p)")
    ap.add_argument("--store", default="0",
                    help="comma list of tuning cnf_store values (0 default, 1 plain, 2 write-through, 3 nontemporal)")
    ap.add_argument("--lookback", default="default",
                    help="comma list: default | chained | poll16 | poll1 (k_cnf_select's look-back form)")
    args = ap.parse_args()
    import torch
    import mbx_pkg
    m = mbx_pkg.load()
    M = m.mbx
    ctx = m.Context(0)
    ext = torch.cuda.ExternalStream(ctx.stream)
    torch.cuda.set_stream(ext)

    def table(n, seed=42):
        g = torch.Generator(device="cuda")
        g.manual_seed(seed)
        c0 = torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g)
        c1 = torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g)
        c2 = torch.randint(0, 10, (n,), dtype=torch.int32, device="cuda", generator=g)
        c3 = torch.randint(0, 10, (n,), dtype=torch.int32, device="cuda", generator=g)
        t = ctx.wrap([(M.INTEGER, 4)] * 4, [x.data_ptr() for x in (c0, c1, c2, c3)], n, row_offset=64 * 3)
        a = ctx.index_build(t, 2, [("int", 3)])[0]
        b = ctx.index_build(t, 3, [("int", 7)])[0]
        return (c0, c1, c2, c3), t, a, b

    LB = {"default": None, "chained": (1, 1), "poll16": (2, 16), "poll1": (2, 1)}  # (cnf_lookback, flag stride)

    def run(n, group, timed, blocks=0, lookback="default", store=0, waves=4):
        cols, t, a, b = table(n)
        if group:
            ctx.group(t, [0, 1])
        c0, c1, c2, c3 = cols
        sel = (c2 == 3) & (c3 == 7)
        want = int(sel.sum().item())
        cap = max(64, want + 64)
        ids = torch.zeros(cap, dtype=torch.int64, device="cuda")
        o0 = torch.zeros(cap, dtype=torch.int32, device="cuda")
        o1 = torch.zeros(cap, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        ctx.set_tuning("cnf_blocks", blocks)
        ctx.set_tuning("cnf_store", store)
        if waves != 4:  # round 5's 16-wave A/B (profiles/r05/p) ran a build with the cnf_waves knob, since removed
            raise SystemExit("c4_forms: the library launches 4-wave blocks only (knob cnf_waves removed)")
        if LB[lookback]:
            ctx.set_tuning("cnf_lookback", LB[lookback][0])
            ctx.set_tuning("cnf_flag_stride", LB[lookback][1])
        proj = [] if args.positions_only else [0, 1]
        outs = [] if args.positions_only else [o0.data_ptr(), o1.data_ptr()]
        f = lambda: ctx.cnf_materialize_async(t, [[a], [b]], proj, ids.data_ptr(), outs, cnt.data_ptr())
        torch.cuda.synchronize()
        f()
        ctx.sync()
        ok = (int(cnt.item()) == want and bool((ids[:want] == torch.nonzero(sel).flatten() + 192).all())
              and (args.positions_only or (bool((o0[:want] == c0[sel]).all()) and bool((o1[:want] == c1[sel]).all()))))
        res = {"rows": n, "group": group, "blocks": blocks, "lookback": lookback, "store": store, "waves": waves, "positions_only": args.positions_only, "gather_pair": os.environ.get("MBX_GATHER_PAIR", "1"),
               "selected": want, "ok": ok}
        if timed:
            ctx.graph_begin()
            for _ in range(20):
                f()
            gr = ctx.graph_end()
            gr.launch()
            ctx.sync()
            ms = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(ext)
                gr.launch()
                e1.record(ext)
                ctx.sync()
                ms.append(e0.elapsed_time(e1) / 20)
            gr.close()
            ok2 = int(cnt.item()) == want and (args.positions_only or bool((o0[:want] == c0[sel]).all()))
            res.update(us=sorted(ms)[len(ms) // 2] * 1e3, us_all=[round(x * 1e3, 2) for x in ms], ok_after=ok2)
        ctx.set_tuning("reset")
        del cols, t, a, b, ids, o0, o1, sel
        torch.cuda.empty_cache()
        return res

    bad = 0
    blocks = [int(x) for x in args.blocks.split(",")]
    lbs = args.lookback.split(",")
    sdbgs = [int(x) for x in args.store.split(",")]
    wavess = [int(x) for x in args.waves.split(",")]
    for n in map(int, args.check_rows.split(",")):
        for group in (True, False):
            for b in blocks:
                for lb in lbs:
                    for sd in sdbgs:
                        for wv in wavess:
                            r = run(n, group, False, b, lb, sd, wv)
                            bad += not r["ok"]
                            print(json.dumps(r), flush=True)
    for n in map(int, args.rows.split(",")):
        for rep in range(2):
            for group in (True, False):
                for b in blocks:
                    for lb in lbs:
                        for sd in sdbgs:
                            for wv in wavess:
                                r = run(n, group, True, b, lb, sd, wv)
                                bad += not (r["ok"] and r["ok_after"])
                                print(json.dumps(r), flush=True)
    ctx.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
