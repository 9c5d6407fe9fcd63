#!/usr/bin/env python3
"""Per-config throughput of the other BASELINE.json workloads, with their A/B
variants (one-launch vs two-launch forms, look-back forms, segment sizes).
Since round 5 the driver's own bench line carries one record per config
(bench.py `configs`: C2, C4 with its column group, C5 per GPU, sharded with
their RCCL exchange at N > 1); this tool keeps the variant sweeps.  Inputs resident in HBM; each query is timed with
HIP events on the library stream over K async steps, and its result checked
against a torch reduction of the same device data.

  C2  10M rows x 4 int32, c0 < 104858 -> BitSet + positions + COUNT (1 GPU)
  C4  100M rows, AND of BitMapFiles bm(c2=3), bm(c3=7) -> positions + c0, c1
  C5  mixed i32 / f32 / char(16), (c0<2^19) ^ (c1>=0.25) ^ (c2>="M") -> COUNT,
      SUM/MIN/MAX(c1)

One process per GPU: launched by torch.distributed.run, C4
and C5 shard the global table by 64-aligned row ranges (dist.shard_bounds,
positions global through row_offset) and run with no data-path collective;
the one exchange step per query is libmbx's RCCL communicator
(mbx_comm_*, on its exchange stream after the query's kernels):
  C4  all-gather of the per-rank selected counts (the concatenation offsets
      of the per-rank outputs, shard order = ascending positions)
  C5  all-gather of every rank's 48-byte aggregate record straight from
      device memory, folded in rank order on the device (in place)
torch.distributed (gloo) only bootstraps the communicator id and runs the
barriers / max-over-ranks clock.
Reported per config (rank 0, one JSON line): max-over-ranks wall time per
query with the exchange included (barrier + synchronize around K queries),
the per-phase kernel times (max over ranks) and global rows/s.

  python tools/bench_configs.py [--configs C2,C4,C5] [--c5-rows 125000000,1000000000]
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_configs.py \\
      --configs C4,C5 --c4-rows 100000000 --c5-rows 1000000000
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--configs", default="C2,C4,C5")
    ap.add_argument("--c2-stamps", action="store_true", help="C2: per-block stamps of each one-launch form")
    ap.add_argument("--c2-tpb", default="", help="C2: comma list of tiles_per_block to sweep (one launch)")
    ap.add_argument("--c2-stamps-out", default="", help="C2: per-block stamps of each form to PREFIX.<form>.csv")
    ap.add_argument("--c4-rows", type=int, default=100_000_000, help="global rows")
    ap.add_argument("--c4-positions", action="store_true",
                    help="C4 query also writes the selected positions (default: the projected rows only)")
    ap.add_argument("--c4-group", action="store_true",
                    help="C4: the projected c0, c1 also staged as a column group (mbx_table_group, 8-byte rows)")
    ap.add_argument("--c4-two-call", action="store_true",
                    help="C4 query as mbx_bitmap_cnf_async + mbx_materialize_async (default: one launch)")
    ap.add_argument("--c5-rows", default="125000000,1000000000", help="global rows, comma separated")
    args = ap.parse_args()
    # JSON lines only on stdout: libraries (RCCL's version banner) write to fd 1
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch
    import torch.distributed as dist

    import mbx_pkg

    # rehearsal knobs, as in bench.py: MBX_BENCH_BACKEND=gloo,
    # MBX_BENCH_SAME_DEVICE=1 run N ranks on one GPU
    backend = os.environ.get("MBX_BENCH_BACKEND", "nccl")
    device = 0 if os.environ.get("MBX_BENCH_SAME_DEVICE") == "1" else local_rank
    torch.cuda.set_device(device)
    if world > 1:  # host bootstrap, barriers and the clock only
        dist.init_process_group("gloo")
    m = mbx_pkg.load()
    M = m.mbx
    D = m.dist
    L = M.lib()
    ctx = m.Context(device)
    ext = torch.cuda.ExternalStream(ctx.stream)
    xs = torch.cuda.Stream() if world > 1 else None
    comm = None
    if world > 1 and backend == "nccl":  # libmbx's RCCL communicator carries the exchange
        box = [M.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        comm = ctx.comm_init_rank(world, rank, box[0])

    def rmax(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def kernel_ms(fn, steps, warmup):
        """HIP events on the library stream around `steps` calls, max over ranks."""
        for _ in range(warmup):
            fn()
        ctx.sync()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(ext)
        for _ in range(steps):
            fn()
        b.record(ext)
        ctx.sync()
        return rmax(a.elapsed_time(b) / steps)

    def wall_ms(step, steps, warmup):
        """Whole queries incl. the exchange: barrier + synchronize on both sides."""
        for k in range(warmup):
            step(k)
        ctx.sync()
        barrier()
        t0 = time.perf_counter()
        for k in range(steps):
            step(warmup + k)
        ctx.sync()
        barrier()
        return rmax((time.perf_counter() - t0) * 1e3 / steps)

    def exchange(k, src_words, out_rows):
        """The one collective of a query (gloo rehearsal only; with RCCL the
        queries call the communicator): all_gather of `src_words` (int64) into
        out_rows[k] on a side stream after the library stream's work."""
        if world == 1:
            return
        ev = torch.cuda.Event()
        ev.record(ext)
        xs.wait_event(ev)
        with torch.cuda.stream(xs):
            if backend == "nccl":
                dist.all_gather_into_tensor(out_rows[k], src_words)
            else:  # gloo rehearsal: host copies
                parts = [torch.empty_like(src_words, device="cpu") for _ in range(world)]
                dist.all_gather(parts, src_words.cpu())
                out_rows[k].copy_(torch.cat(parts))

    def gen_int(n, hi, seed):
        g = torch.Generator(device="cuda")
        g.manual_seed(seed)
        return torch.randint(0, hi, (n,), dtype=torch.int32, device="cuda", generator=g)

    def emit(d):
        if rank == 0:
            os.write(out_fd, (json.dumps(d) + "\n").encode())

    if "C2" in args.configs and world == 1:
        n = 10_000_000
        cols = [gen_int(n, 1 << 20, 42 + j) for j in range(4)]
        t = ctx.wrap([(M.INTEGER, 4)] * 4, [c.data_ptr() for c in cols], n)
        plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", 104858))]])
        bm = ctx.bitmap_alloc(n)
        ids = torch.zeros(n, dtype=torch.int64, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")

        def step(k=0):  # BitSet + positions + COUNT: mbx_scan_select_async (BitSet scan, then the compaction)
            M._chk(L.mbx_scan_select_async(ctx.h, plan.h, bm.h, ids.data_ptr(), cnt.data_ptr()))

        want = int((cols[0] < 104858).sum().item())
        wpos = torch.nonzero(cols[0] < 104858).flatten()
        # both forms, interleaved: the BitSet scan + compaction (two launches)
        # and k_scan_select (one launch, knob scan_select_fused)
        # (its default look-back: every predecessor polled, one flag per
        # 128-byte line), with the flags packed (select_flag_stride 1) and
        # with the chained walk (select_dbg 128)
        forms = {}
        variants = {0: (0, 0, 16), 1: (1, 0, 16), "poll_packed": (1, 0, 1), "chained": (1, 128, 1)}
        for rep in range(3):
            for key, (fused, dbg, fs) in variants.items():
                ctx.set_tuning("scan_select_fused", fused)
                ctx.set_tuning("select_dbg", dbg)
                ctx.set_tuning("select_flag_stride", fs)
                ids.zero_()
                torch.cuda.synchronize()
                forms.setdefault(key, []).append(kernel_ms(step, args.steps, args.warmup))
                got = int(cnt.item())
                assert got == want, (key, got, want)
                assert bool((ids[:got] == wpos).all()), key
        stamps = {}
        if args.c2_stamps:
            # per-block wall_clock64() stamps (start / count published / offset
            # known / end, select_dbg bit 3) of one launch of each one-launch form
            ntiles = -(-n // 256)
            tpb = max(4, -(-ntiles // 1024))
            nb = -(-(-(-ntiles // tpb)) // 4)  # 16-wave blocks of 4 BitSet segments
            for key in (1, "poll_packed", "chained"):
                ctx.set_tuning("scan_select_fused", 1)
                ctx.set_tuning("select_flag_stride", variants[key][2])
                ctx.set_tuning("select_dbg", 8 | variants[key][1])
                step()
                ctx.sync()
                st = np.zeros(4 * nb, dtype=np.int64)
                M._chk(L.mbx_diag_select_stamps(ctx.h, st.ctypes.data, nb))
                st = st.reshape(nb, 4).astype(np.float64) / 100.0  # 100 MHz wall clock -> us
                st -= st[:, 0].min()
                pct = lambda x: [round(float(v), 2) for v in np.percentile(x, [0, 10, 50, 90, 100])]
                if args.c2_stamps_out:
                    with open(f"{args.c2_stamps_out}.{key}.csv", "w") as fh:
                        fh.write("block,start_us,staged_us,offset_known_us,end_us\n")
                        for b in range(nb):
                            fh.write(f"{b},{st[b, 0]:.2f},{st[b, 1]:.2f},{st[b, 2]:.2f},{st[b, 3]:.2f}\n")
                stamps[str(key)] = {"blocks": nb, "s1_pct": pct(st[:, 1]), "s2_pct": pct(st[:, 2]),
                                    "s3_pct": pct(st[:, 3]), "s2_s1_pct": pct(st[:, 2] - st[:, 1]),
                                    "s3_s2_pct": pct(st[:, 3] - st[:, 2])}
                ctx.set_tuning("select_dbg", 0)
        fused_default = int(os.environ.get("MBX_SCAN_SELECT_FUSED", "1") or 0)
        ctx.set_tuning("reset")
        ctx.set_tuning("scan_select_fused", fused_default)
        ms = sorted(forms[fused_default])[1]  # the median of the three interleaved rounds
        # the same queries replayed from a HIP graph of 10 (mbx_graph_*: no host launches between them)
        ctx.sync()
        ctx.graph_begin()
        for _ in range(10):
            step()
        gr = ctx.graph_end()
        graph_ms = kernel_ms(gr.launch, max(1, args.steps // 10), 2) / 10
        gr.close()
        assert int(cnt.item()) == want
        scan_ms = kernel_ms(lambda: ctx.scan_bitmap_async(plan, bm), args.steps, args.warmup)
        byts = n * 4 + n / 8 + got * 8
        emit({"config": "C2", "rows": n, "gpus": 1, "selected": got, "ms_per_query": ms, "rows_per_s": n / ms * 1e3,
              "form": "one launch (k_scan_select)" if fused_default else "two launches (BitSet scan + k_select_ids)",
              "ms_per_query_two_launch": forms[0], "ms_per_query_one_launch": forms[1],
              "ms_per_query_one_launch_flags_packed": forms["poll_packed"],
              "ms_per_query_one_launch_chained": forms["chained"],
              "stamps_us": stamps,
              "graph_replay_ms_per_query": graph_ms,
              "algorithmic_gbs": byts / ms / 1e6, "scan_bitmap_ms": scan_ms,
              "scan_gbs": (n * 4 + n / 8) / scan_ms / 1e6})
        # segment size sweep (knob tiles_per_block, read by the BitSet's
        # allocation): smaller segments = more waves per CU and more blocks
        # in the look-back
        for tpb in [int(x) for x in args.c2_tpb.split(",") if x]:
            ctx.set_tuning("tiles_per_block", tpb)
            bmt = ctx.bitmap_alloc(n)
            res = {}
            for rep in range(3):
                for key in (1, "chained"):
                    ctx.set_tuning("scan_select_fused", 1)
                    ctx.set_tuning("select_dbg", variants[key][1])
                    ctx.set_tuning("select_flag_stride", variants[key][2])
                    ids.zero_()
                    torch.cuda.synchronize()
                    f = lambda: M._chk(L.mbx_scan_select_async(ctx.h, plan.h, bmt.h, ids.data_ptr(), cnt.data_ptr()))
                    res.setdefault(str(key), []).append(kernel_ms(f, args.steps, args.warmup))
                    got = int(cnt.item())
                    assert got == want and bool((ids[:got] == wpos).all()), (tpb, key)
            emit({"config": "C2-tpb", "tiles_per_block": tpb, "ms_one_launch": res})
            del bmt
            ctx.set_tuning("tiles_per_block", 0)
        ctx.set_tuning("reset")
        ctx.set_tuning("scan_select_fused", fused_default)
        del cols, t, plan, bm, ids
        torch.cuda.empty_cache()

    if "C4" in args.configs:
        N = args.c4_rows
        s, e = D.shard_bounds(N, world, rank)
        n = e - s
        seed = 42 + 1000 * rank
        c0, c1 = gen_int(n, 1 << 20, seed), gen_int(n, 1 << 20, seed + 1)
        c2, c3 = gen_int(n, 10, seed + 2), gen_int(n, 10, seed + 3)
        t = ctx.wrap([(M.INTEGER, 4)] * 4, [x.data_ptr() for x in (c0, c1, c2, c3)], n, row_offset=s)
        bm2 = ctx.index_build(t, 2, [("int", v) for v in range(10)])
        bm3 = ctx.index_build(t, 3, [("int", v) for v in range(10)])
        a, b = bm2[3], bm3[7]
        if args.c4_group:
            ctx.group(t, [0, 1])
        out = ctx.bitmap_alloc(n)
        cap = max(1, n // 50)
        ids = torch.zeros(cap, dtype=torch.int64, device="cuda")
        o0 = torch.zeros(cap, dtype=torch.int32, device="cuda")
        o1 = torch.zeros(cap, dtype=torch.int32, device="cuda")
        steps, warmup = args.steps, args.warmup
        cnts = torch.zeros(steps + warmup, dtype=torch.int64, device="cuda")
        counts_all = torch.zeros(steps + warmup, world, dtype=torch.int64, device="cuda")
        proj = (ctypes.c_int32 * 2)(0, 1)
        outs = (ctypes.c_void_p * 2)(o0.data_ptr(), o1.data_ptr())
        bms = (ctypes.c_void_p * 2)(a.h.value, b.h.value)
        offs = (ctypes.c_int32 * 3)(0, 1, 2)

        def and_():
            M._chk(L.mbx_bitmap_cnf_async(ctx.h, bms, offs, 2, None, out.h))

        def query_two_call(k):
            and_()
            M._chk(L.mbx_materialize_async(ctx.h, t.h, out.h, proj, 2, ids.data_ptr(), outs, cnts.data_ptr() + 8 * k))

        def query_fused(k, with_ids=False):  # one launch: CNF words + look-back + gather (+ positions)
            M._chk(L.mbx_cnf_materialize_async(ctx.h, t.h, bms, offs, 2, None, proj, 2,
                                               ids.data_ptr() if with_ids else None, outs, cnts.data_ptr() + 8 * k))

        # the query: ColumnarIndexScan's output, the projected rows (its
        # get_next returns tuples; the positions are an intermediate), in one
        # launch; --c4-positions also writes the positions, --c4-two-call runs
        # the two-launch form (AND BitSet, then positions + gather)
        mode = "two_call" if args.c4_two_call else ("positions" if args.c4_positions else "projection")

        def query(k):
            if mode == "two_call":
                query_two_call(k)
            else:
                query_fused(k, with_ids=mode == "positions")
            if comm is not None:
                comm.allgather_count_async(cnts.data_ptr() + 8 * k, counts_all[k].data_ptr())
            else:
                exchange(k, cnts[k:k + 1], counts_all)

        ms = wall_ms(query, steps, warmup)
        sel = (c2 == 3) & (c3 == 7)
        want = int(sel.sum().item())
        got = int(cnts[-1].item())
        assert got == want and got <= cap, (got, want)
        assert bool((o0[:got] == c0[sel]).all()) and bool((o1[:got] == c1[sel]).all())
        glob = got if world == 1 else int(D.combine_count(want))
        if world > 1:
            assert bool((counts_all[:, rank] == want).all()) and int(counts_all[-1].sum().item()) == glob
        o0.zero_(), o1.zero_(), ids.zero_()
        torch.cuda.synchronize()
        proj_ms = kernel_ms(lambda: query_fused(0), steps, warmup)
        pos_ms = kernel_ms(lambda: query_fused(0, with_ids=True), steps, warmup)
        assert int(cnts[0].item()) == want
        assert bool((o0[:got] == c0[sel]).all()) and bool((o1[:got] == c1[sel]).all())
        assert bool((ids[:got] == torch.nonzero(sel).flatten() + s).all())
        two_ms = kernel_ms(lambda: query_two_call(0), steps, warmup)
        assert bool((ids[:got] == torch.nonzero(sel).flatten() + s).all())
        and_ms = kernel_ms(and_, steps, warmup)
        sel_ms = kernel_ms(lambda: M._chk(L.mbx_materialize_async(ctx.h, t.h, out.h, proj, 2, ids.data_ptr(), outs,
                                                                   cnts.data_ptr())), steps, warmup)
        # algorithmic bytes: the two operand BitSets read once, the projected
        # values (+ positions) written once; the two-call form also writes and
        # re-reads the AND BitSet
        byts = 2 * N / 8 + glob * 8 + (glob * 8 if mode != "projection" else 0) + (2 * N / 8 if mode == "two_call"
                                                                                    else 0)
        emit({"config": "C4", "rows": N, "gpus": world, "rows_per_gpu": n, "selected": glob,
              "layout": "column group (c0, c1) for the gather" if args.c4_group else "columns",
              "ms_per_query": ms, "rows_per_s": N / ms * 1e3, "algorithmic_gbs": byts / ms / 1e6,
              "query": {"projection": "one launch (mbx_cnf_materialize_async): projected rows c0, c1",
                        "positions": "one launch (mbx_cnf_materialize_async): positions + c0, c1",
                        "two_call": "two launches (mbx_bitmap_cnf_async + mbx_materialize_async): positions + c0, c1"
                        }[mode],
              "kernel_ms": {"one_launch_projection": proj_ms, "one_launch_positions_and_projection": pos_ms,
                            "two_launch_positions_and_projection": two_ms},
              "phases_ms": {"bitmap_and": and_ms, "positions_and_gather": sel_ms},
              "bitmap_and_gbs": 3 * n / 8 / and_ms / 1e6,
              "exchange": "none" if world == 1 else ("RCCL all-gather of per-rank counts (libmbx mbx_comm)"
                                                     if comm is not None else "gloo all_gather (rehearsal)"),
              "backend": backend if world > 1 else None})
        del c0, c1, c2, c3, t, bm2, bm3, a, b, out, ids, o0, o1
        torch.cuda.empty_cache()

    if "C5" in args.configs:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import helpers
        names = [f"{chr(65 + (i * 7) % 26)}{'abcdefghijklmnop'[:(i % 15) + 1]}"[:16] for i in range(50)]
        dic = torch.zeros(50, 16, dtype=torch.uint8)
        for i, nm in enumerate(names):
            dic[i, :len(nm)] = torch.tensor(list(nm.encode()), dtype=torch.uint8)
        dic = dic.cuda()
        for N in map(int, args.c5_rows.split(",")):
            s, e = D.shard_bounds(N, world, rank)
            n = e - s
            g = torch.Generator(device="cuda")
            g.manual_seed(5 + 1000 * rank)
            c0 = torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g)
            c1 = torch.rand((n,), dtype=torch.float32, device="cuda", generator=g)
            idx = torch.randint(0, 50, (n,), dtype=torch.int64, device="cuda", generator=g)
            c2 = helpers.device_dictionary_column(dic, idx)
            del idx
            t = ctx.wrap([(M.INTEGER, 4), (M.REAL, 4), (M.STRING, 16)], [c0.data_ptr(), c1.data_ptr(), c2.data_ptr()],
                         n, row_offset=s)
            cnf = [[(M.LT, ("sym", 1), ("int", 1 << 19))], [(M.GE, ("sym", 2), ("real", 0.25))],
                   [(M.GE, ("sym", 3), ("str", "M"))]]
            plan = ctx.compile(t, cnf)
            steps, warmup = max(10, args.steps // 5), 2
            W = D.AGG_WORDS
            recs = torch.zeros(steps + warmup, W, dtype=torch.int64, device="cuda")
            gathered = torch.zeros(steps + warmup, world * W, dtype=torch.int64, device="cuda")

            def query(k):
                ctx.scan_aggregate_async(plan, 1, recs[k].data_ptr())
                if comm is not None:  # all-gather + rank-ordered fold into recs[k], on the device
                    comm.allreduce_agg_async(recs[k].data_ptr())
                else:
                    exchange(k, recs[k], gathered)

            ms = wall_ms(query, steps, warmup)
            glob_rec = recs[-1].cpu().numpy().copy()
            scan_ms = kernel_ms(lambda: ctx.scan_aggregate_async(plan, 1, recs[0].data_ptr()), steps, warmup)
            # check: this rank's record vs torch, the folded global vs torch combined
            sel = (c0 < (1 << 19)) & (c1 >= 0.25) & (c2[:, 0] >= ord("M"))
            want = int(sel.sum().item())
            mine = D.fold_aggregates(recs[0].cpu().numpy())
            assert mine["count"] == want, (mine["count"], want)
            # elementwise + reductions only (no masked-select launch over the table)
            ref_sum = float(torch.where(sel, c1.double(), 0.0).sum().item())
            assert abs(mine["sum"] - ref_sum) <= 1e-6 * abs(ref_sum)
            ref = dict(count=want, sum=ref_sum, min=float(torch.where(sel, c1, float("inf")).min().item()),
                       max=float(torch.where(sel, c1, float("-inf")).max().item()))
            assert mine["min"] == ref["min"] and mine["max"] == ref["max"]
            if world > 1:
                glob = D.fold_aggregates(glob_rec if comm is not None else gathered[-1].cpu().numpy())
                gref = D.combine_aggregate(ref)
                assert glob["count"] == gref["count"] and glob["min"] == gref["min"] and glob["max"] == gref["max"]
                assert abs(glob["sum"] - gref["sum"]) <= 1e-6 * abs(gref["sum"])
            else:
                glob = mine
            byts = N * (4 + 4 + 16)
            emit({"config": "C5", "rows": N, "gpus": world, "rows_per_gpu": n, "selected": glob["count"],
                  "ms_per_query": ms, "rows_per_s": N / ms * 1e3, "algorithmic_gbs": byts / ms / 1e6,
                  "phases_ms": {"scan_aggregate": scan_ms},
                  "scan_gbs_per_gpu": n * 24 / scan_ms / 1e6,
                  "sum": glob["sum"], "min": glob["min"], "max": glob["max"],
                  "exchange": "none" if world == 1 else ("RCCL all-gather of the 48-byte records + device fold (libmbx)"
                                                         if comm is not None else "gloo all_gather (rehearsal)"),
                  "backend": backend if world > 1 else None})
            del c0, c1, c2, t, plan, sel
            torch.cuda.empty_cache()
    if comm is not None:
        comm.close()
    ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
