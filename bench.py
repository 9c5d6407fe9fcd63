#!/usr/bin/env python3
"""bench.py -- BASELINE.json headline: scanned rows/s + HBM GB/s on the C3
workload (100M-row 4 x int32 Columnarfile, 2-predicate conjunction + COUNT),
at 1 / 2 / 4 / 8 GPUs.

One "step" = one ColumnarFileScan COUNT pass over the resident table:
`query ... {(c0 < 2^19)} ^ {(c1 >= 2^19)} FILESCAN` -> Total Results Count,
executed as ONE kernel launch per GPU (k_scan_fast<2, COUNT>; its last block
folds the per-block counts), plus -- on N > 1 GPUs -- the path's one exchange
step: an in-place RCCL all-reduce of the COUNTs over xGMI, issued by libmbx
(mbx_comm_allreduce_count_async) right after the scan on the same stream
(libmbx's default: inside a captured graph a collective forked to a second
stream is not overlapped on this ROCm and costs more, profiles/r03/parts).
Every step (= query) has its own collective
(--exchange-bucket 1, the default: SURVEY 8(e)'s per-query
N_total / (max_k t_kernel,k + t_reduce)); --exchange-bucket B > 1 lets the
COUNTs of B consecutive steps share one all-reduce (a diagnostic: a tiny
all-reduce costs its latency, not its bytes).
Inputs are resident in HBM before the timed region.

Scaling.  The path partitions by row
range with no data-path collective and one exchange per query (the COUNT
reduce north_star names), so the default reports weak scaling:
  --scaling weak (default): per-GPU work fixed at the C3 table -- rank r owns
      rows [r * 100M, (r + 1) * 100M) of an N x 100M-row logical table (its own
      seeds 42 + 1000 r + col; N = 1 is exactly the C3 table); every step's
      global COUNT is checked against the sum of the ranks' torch counts.
  --scaling strong: ONE 100M-row table split into N 64-aligned row-range
      shards (mbx_shard_bounds), generated full size with the same seeds on
      every rank and sliced, the global COUNT checked against a torch
      reduction of the whole table (12.5M rows per GPU at N = 8: launch- and
      exchange-latency bound).
The timed steps replay HIP graphs (mbx_graph_*) of --graph-steps captured
steps (scans + their exchange), so small shards do not wait on the host.
value = global rows scanned by all ranks / max-over-ranks wall time.  stdout
carries only the JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak]

Launch: with WORLD_SIZE unset and --gpus N > 1, this process is only a
launcher: before anything touches a GPU it starts N rank processes of this
same script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT in their env), relays rank 0's JSON line and exits with the
first failing rank's status (the others are then stopped by PID).  Under an
external torch.distributed.run, WORLD_SIZE must equal --gpus.
--dry-launch: the ranks print their rank env as JSON and exit before
importing torch (the launcher's CPU test, tests/test_bench_launch.py).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "scanned rows/sec + HBM GB/s, 100M-row 4×int32 conjunctive filter, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
THRESH = 1 << 19


def cpu_baseline(rows, min_seconds):
    """The oracle (C restatement of ColumnarFileScan + PredEval) timed on the
    same workload definition: a host copy of the C3 table (numpy PCG64, seeds
    42..45), full passes until min_seconds elapsed -- row ranges split over the
    host cores this process may use (OMP_NUM_THREADS, 16 per GPU on the box;
    SURVEY 8(d)(ii)), each range evaluated row by row exactly like the
    single-thread oracle."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import helpers
    import oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    cols = [(oracle.INTEGER, 4, c) for c in helpers.synthetic_int_table(rows, 4, 1 << 20, 42)]
    t = oracle.Table(cols)
    cnf = [[(oracle.LT, ("sym", 1), ("int", THRESH))], [(oracle.GE, ("sym", 2), ("int", THRESH))]]
    t0 = time.perf_counter()
    count1 = oracle.filescan_count(t, cnf)          # one single-thread pass, for the record
    one = time.perf_counter() - t0
    passes, elapsed, count = 0, 0.0, None
    while elapsed < min_seconds and passes < 5000:
        t0 = time.perf_counter()
        count = oracle.filescan_count_mt(t, cnf, threads)
        elapsed += time.perf_counter() - t0
        passes += 1
    assert count == count1
    return {
        "value": rows * passes / elapsed,
        "unit": "rows/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{passes} full pass(es) over a {rows:,}-row 4xint32 host table (same C3 predicate, count {count}); "
                  f"oracle/oracle.c orc_filescan_count_mt, {threads} OpenMP threads, {elapsed:.1f} s total; "
                  f"single thread: {rows / one:.3g} rows/s",
    }


def load_traffic(rows, count_mode):
    """HBM bytes per launch of the C3 scan over a `rows`-row shard with the
    given COUNT form ("finalize" | "frame"), from the committed rocprofv3 PMC
    summary (profiles/c3_scan_pmc.json: one entry per shard size bench.py
    runs at N = 1, 2, 4, 8; written by tools/pmc_summary.py), or None."""
    path = os.path.join(ROOT, "profiles", "c3_scan_pmc.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get("shards", {}).get(f"{rows}:{count_mode}")
        return (e or {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, dry):
    """Start n rank processes of this script (one per GPU; none of this
    process's code has touched a GPU), relay rank 0's stdout (every rank's
    with --dry-launch) and return the exit status: 0, or the first failing
    rank's status, after the remaining ranks were stopped by their PIDs."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = subprocess.PIPE if (r == 0 or dry) else sys.stderr
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env, stdout=out))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"bench launcher: rank {procs.index(p)} exited with {rc}; stopping the others",
                      file=sys.stderr)
                for q in live:
                    q.kill()
        time.sleep(0.05)
    for p in procs:
        if p.stdout is not None:
            data = p.stdout.read()
            if data:
                os.write(1, data)
    return status


def read_probe(ctx, table, ext, torch, reps=30):
    """Best read bandwidth of k_read_probe (mbx_probe_read: the C3 kernel's
    tiles and non-temporal dwordx4 loads over c0, c1 with no predicate) over a
    few block mappings, timed with HIP events on the library stream."""
    n = table.nrows
    nbytes = 2 * 4 * (n // 256 * 256)
    variants = [("segments, scan default", dict()), ("segments, tpb=256", dict(tiles_per_block=256)),
                ("segments, tpb=96", dict(tiles_per_block=96)),
                ("grid-stride 1024 blocks", dict(interleave=True, grid=1024)),
                ("grid-stride 2048 blocks", dict(interleave=True, grid=2048))]
    res = {}
    for name, kw in variants:
        for _ in range(3):
            ctx.probe_read(table, [0, 1], **kw)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(ext)
        for _ in range(reps):
            ctx.probe_read(table, [0, 1], **kw)
        b.record(ext)
        ctx.sync()
        ms = a.elapsed_time(b) / reps
        res[name] = nbytes / (ms * 1e-3) / 1e9
    best = max(res, key=res.get)
    return {"best_gbs": res[best], "best": best, "gbs": res}


def quiet_stdout():
    """The one JSON line is the only thing on stdout: fd 1 is pointed at
    stderr for the libraries (RCCL prints a version banner when it creates
    its first communicator) and the result goes to a duplicate of the
    original fd 1."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return fd


def make_columns(torch, n_global, s, e, seed_base):
    """Columns c0..c3 of rows [s, e) of one logical table: each column is
    generated whole on this GPU from its own seed (torch Philox), so every
    shard count N slices the same table, then the shard is copied out."""
    cols = []
    for j in range(4):
        g = torch.Generator(device="cuda")
        g.manual_seed(seed_base + j)
        full = torch.randint(0, 1 << 20, (n_global,), dtype=torch.int32, device="cuda", generator=g)
        cols.append(full[s:e].clone())
        del full
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return cols


def full_count(torch, n_global, seed_base):
    """The global C3 COUNT of the whole table (torch reduction, chunk-free)."""
    out = []
    for j in range(2):
        g = torch.Generator(device="cuda")
        g.manual_seed(seed_base + j)
        out.append(torch.randint(0, 1 << 20, (n_global,), dtype=torch.int32, device="cuda", generator=g))
    c = int(((out[0] < THRESH) & (out[1] >= THRESH)).sum().item())
    del out
    torch.cuda.empty_cache()
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rows", type=int, default=100_000_000,
                    help="global rows (strong scaling) or rows per GPU (weak)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="weak")
    ap.add_argument("--graph-steps", type=int, default=10, help="steps per captured HIP graph (0: eager launches)")
    ap.add_argument("--exchange-bucket", type=int, default=1,
                    help="steps whose COUNTs share one all-reduce (1, the default: one collective per query)")
    ap.add_argument("--count", choices=["auto", "frame", "finalize"], default="auto",
                    help="frame: each scan adds its COUNT into a 32-slot count frame (no in-launch finalize; the "
                         "exchange all-reduces whole frames); finalize: the scan's last block writes the COUNT; "
                         "auto: frame with an exchange, finalize without")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-launch", action="store_true",
                    help="ranks print their rank env as JSON and exit before importing torch (launcher test)")
    args = ap.parse_args()
    if args.gpus < 1:
        print(f"bench: --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.dry_launch))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_launch:
        env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world, "gpus": args.gpus,
                          "torch_imported": "torch" in sys.modules, "env": env}), flush=True)
        return
    out_fd = quiet_stdout()

    import torch
    import torch.distributed as dist

    import mbx_pkg

    # rehearsal knob (never set by the driver): MBX_BENCH_SAME_DEVICE=1 runs N
    # ranks on one GPU (RCCL refuses two ranks on one device, so the exchange
    # then goes over gloo on the host)
    same_device = os.environ.get("MBX_BENCH_SAME_DEVICE") == "1"
    device = 0 if same_device else local_rank
    torch.cuda.set_device(device)
    # MBX_BENCH_FORCE_EXCHANGE=1 keeps the per-step exchange at N=1 (a one-rank
    # RCCL clique): the N>1 step on one GPU
    exchange = world > 1 or os.environ.get("MBX_BENCH_FORCE_EXCHANGE") == "1"
    if world > 1:
        # host-side bootstrap, barriers and the max-over-ranks clock only: the
        # data-path exchange is libmbx's own RCCL communicator
        dist.init_process_group("gloo")
    m = mbx_pkg.load()
    ctx = m.Context(device)

    n_global = args.rows if args.scaling == "strong" else args.rows * world
    if args.scaling == "strong":
        s, e = m.mbx.shard_bounds(args.rows, world, rank)
        seed_base = 42
    else:
        s, e = rank * args.rows, (rank + 1) * args.rows
        seed_base = 42 + 1000 * rank
    n = e - s

    # synthetic C3 shard, generated in HBM: 4 x int32 uniform [0, 2^20)
    if args.scaling == "strong":
        cols = make_columns(torch, args.rows, s, e, seed_base)
    else:
        cols = make_columns(torch, n, 0, n, seed_base)
    table = ctx.wrap([(m.mbx.INTEGER, 4)] * 4, [col.data_ptr() for col in cols], n, None, row_offset=s)
    cnf = [[(m.mbx.LT, ("sym", 1), ("int", THRESH))], [(m.mbx.GE, ("sym", 2), ("int", THRESH))]]
    plan = ctx.compile(table, cnf)

    comm = None
    torch_pg = None  # fallback exchange: torch.distributed's own RCCL group
    if exchange and not same_device:
        uid = m.mbx.comm_unique_id() if rank == 0 else None
        if world > 1:
            box = [uid]
            dist.broadcast_object_list(box, src=0)
            uid = box[0]
        ok = 1
        try:
            comm = ctx.comm_init_rank(world, rank, uid)
        except m.MbxError as err:
            if world == 1:
                raise
            ok = 0
            print(f"rank {rank}: libmbx RCCL communicator failed ({err})", file=sys.stderr)
        if world > 1:
            # every rank takes the same exchange: libmbx's communicator if it
            # came up everywhere, else torch.distributed's RCCL group (eager)
            flag = torch.tensor([ok], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if int(flag[0]) == 0:
                if comm is not None:
                    comm.close()
                    comm = None
                torch_pg = dist.new_group(backend="nccl")
                print(f"rank {rank}: exchange falls back to torch.distributed (nccl = RCCL)", file=sys.stderr)

    # correctness gate before timing: the kernel's count vs a torch reduction
    # of the same device columns; with the exchange, the global count vs the
    # whole table (strong) (the oracle cross-check lives in tests/)
    got = ctx.scan_count(plan)
    want = int(((cols[0] < THRESH) & (cols[1] >= THRESH)).sum().item())
    assert got == want, f"rank {rank}: scan count {got} != reference {want}"

    steps, warmup = args.steps, args.warmup
    # count frames (mbx_scan_count_frame_async): with an exchange, each step's
    # scan adds its packed per-block counts into its own zeroed 4 KB frame with
    # no-return atomics and the all-reduce sums whole frames -- the launch ends
    # without the finalize's dependent atomic round trips
    frames = args.count == "frame" or (args.count == "auto" and exchange)
    if frames:
        # a frame slot's 12-bit arrival field sums every rank's arrivals: it
        # must stay < 4096 (mbx_count_frame_fits); otherwise the in-launch
        # finalize (one int64 per rank, summed exactly) is used
        nb = ctx.scan_blocks(plan)
        if world > 1:
            tb = torch.tensor([nb], dtype=torch.int64)
            dist.all_reduce(tb, op=dist.ReduceOp.MAX)
            nb = int(tb[0])
        if not m.mbx.count_frame_fits(nb, world):
            if args.count == "frame":
                raise SystemExit(f"bench: {world} ranks x {nb} blocks overflow a count frame")
            frames = False
            print(f"rank {rank}: {world} ranks x {nb} blocks overflow a count frame; in-launch finalize",
                  file=sys.stderr)
    FW = m.mbx.COUNT_FRAME_WORDS if frames else 1
    counts = torch.zeros((steps + warmup, FW), dtype=torch.int64, device="cuda")
    ext = torch.cuda.ExternalStream(ctx.stream)
    torch.cuda.set_stream(ext)
    base = counts.data_ptr()
    gloo_works = []

    B = max(1, args.exchange_bucket)
    # diagnostic (MBX_BENCH_XS_KERNEL=1): one more real kernel per step where
    # the collective runs (an aggregate all-gather + device fold of a dummy
    # record), standing in on one GPU for an N-rank collective's kernel
    xs_kernel = comm is not None and os.environ.get("MBX_BENCH_XS_KERNEL") == "1"
    dummy = torch.zeros(8, dtype=torch.int64, device="cuda") if xs_kernel else None

    def run_steps(k0, k1):
        """steps k0..k1-1: one scan each; the exchange all-reduces the COUNTs
        of every B consecutive steps in one collective (bucketed: each step's
        count is still combined over all ranks, B per collective)"""
        for j in range(k0, k1, B):
            je = min(j + B, k1)
            for k in range(j, je):
                if frames:
                    ctx.scan_count_frame_async(plan, base + 8 * FW * k)
                else:
                    ctx.scan_count_async(plan, base + 8 * k)
            if comm is not None:
                comm.allreduce_count_async(base + 8 * FW * j, FW * (je - j))
                if xs_kernel:
                    comm.allreduce_agg_async(dummy.data_ptr())
            elif torch_pg is not None:
                dist.all_reduce(counts[j:je], group=torch_pg)
            elif exchange:  # same-device rehearsal: gloo over host copies
                gloo_works.extend(range(j, je))

    def drain():
        ctx.sync()
        if gloo_works:
            h = counts[gloo_works].cpu()
            dist.all_reduce(h)
            counts[gloo_works] = h.cuda()
            gloo_works.clear()

    run_steps(0, warmup)
    drain()

    # HIP graphs of G steps each (the timed region replays them); captured
    # after the warm-up, which sized every scratch buffer
    G = args.graph_steps if (args.graph_steps > 0 and not gloo_works and not (exchange and comm is None)) else 0
    if torch_pg is not None:
        G = 0
    graphs = []
    if G:
        try:
            k0 = warmup
            while k0 < warmup + steps:
                g = min(G, warmup + steps - k0)
                ctx.graph_begin()
                try:
                    run_steps(k0, k0 + g)
                finally:
                    graphs.append(ctx.graph_end())
                k0 += g
            for gr in graphs:  # one untimed replay
                gr.launch()
            drain()
        except m.MbxError as err:
            # a capture the runtime refuses (e.g. a collective it cannot
            # capture) is not fatal: the steps run eagerly instead
            print(f"rank {rank}: HIP graph capture failed ({err}); timing eager steps", file=sys.stderr)
            for gr in graphs:
                gr.close()
            graphs, G = [], 0
            ctx.sync()
    counts.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # timed region: exactly `steps` steps, barrier + synchronize on both sides
    t0 = time.perf_counter()
    if G:
        for gr in graphs:
            gr.launch()
    else:
        run_steps(warmup, warmup + steps)
    t_enq = time.perf_counter() - t0  # host enqueue time of the steps (diagnostic, stderr)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    if frames:
        # decode every step's frame (mbx_count_frame_decode's sums, on the
        # device): count = sum of the slots' high bits; every block of every
        # rank must have arrived exactly once
        slots = counts[warmup:].view(steps, 32, 16)[:, :, 0]
        c = (slots >> 24).sum(1).cpu()
        arrivals = (slots & 0xFFF).sum(1).cpu()
        nblocks = ctx.scan_blocks(plan)
        if world > 1:  # shards may differ by a block: the frames hold every rank's
            tb = torch.tensor([nblocks], dtype=torch.int64)
            dist.all_reduce(tb)
            nblocks = int(tb[0])
        assert bool((arrivals == nblocks).all()), f"rank {rank}: frame arrivals {arrivals[:4].tolist()} != {nblocks}"
        assert int(((slots >> 12) & 0xFFF).sum()) == 0, "NaN blocks in an integer plan"
        h0 = counts[warmup].cpu().numpy()
        assert m.mbx.count_frame_decode(h0)[0] == int(c[0])
    else:
        c = counts[warmup:, 0].cpu()

    # kernel duration: the scans alone again, each bracketed by HIP events
    # recorded on the stream the kernel runs on (the library's stream)
    ev_s = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    ev_e = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    for k in range(steps):
        ev_s[k].record(ext)
        if frames:
            ctx.scan_count_frame_async(plan, base + 8 * FW * (warmup + k))
        else:
            ctx.scan_count_async(plan, base + 8 * (warmup + k))
        ev_e[k].record(ext)
    ctx.sync()
    kern_ms = sum(a.elapsed_time(b) for a, b in zip(ev_s, ev_e)) / steps
    print(f"rank {rank}: rows [{s}, {e}), host enqueue {t_enq * 1e6 / steps:.1f} us/step, "
          f"wall {wall * 1e6 / steps:.1f} us/step, scan kernel {kern_ms * 1e3:.1f} us", file=sys.stderr)
    probe = read_probe(ctx, table, ext, torch) if rank == 0 else None

    if exchange:
        if args.scaling == "strong":
            glob = full_count(torch, n_global, seed_base)
        else:  # the sum of every rank's own torch count
            tw = torch.tensor([want], dtype=torch.int64)
            if world > 1:
                dist.all_reduce(tw)
            glob = int(tw[0])
        assert bool((c == glob).all()), f"rank {rank}: per-step global counts {c[:4].tolist()} != {glob}"
    else:
        assert bool((c == got).all()), "per-step counts differ"

    t_max, kern_max = wall, kern_ms
    if world > 1:
        tt = torch.tensor([wall, kern_ms], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max, kern_max = float(tt[0]), float(tt[1])

    if rank == 0:
        total_rows = n_global * steps
        ms_per_step = t_max * 1e3 / steps
        algo_bytes = 2 * 4 * n  # c0 + c1 read once per launch (rank 0's shard)
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        xchg = ((f"RCCL all-reduce of the COUNTs of every {B} steps (libmbx mbx_comm, after the scans)" if B > 1
                 else "RCCL all-reduce of every step's COUNT (one collective per query; libmbx mbx_comm, right "
                      "after the step's scan on the same stream)")
                if comm is not None else None) or (
            "torch.distributed RCCL all-reduce per step (fallback: libmbx's communicator failed)" if torch_pg is not None
            else None) or ("gloo all-reduce (same-device rehearsal)" if exchange else "none")
        out = {
            "metric": METRIC,
            "value": total_rows / t_max,
            "unit": "rows/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: 4 x int32 uniform [0, 2^20) per row, generated in HBM (torch Philox, seed 42+col"
                    + (", one global table sliced into row-range shards)" if args.scaling == "strong"
                       else "+1000*rank: rank r holds rows [r*N_gpu, (r+1)*N_gpu) of the N-GPU table)"),
            "config": {
                "workload": "C3: 100M-row 4xint32 Columnarfile, {(c0 < 2^19)} ^ {(c1 >= 2^19)} + COUNT "
                            "(ColumnarFileScan / PredEval), 1 scan launch per GPU per step"
                            + (" + 1 exchange" if exchange else ""),
                "global_rows": n_global,
                "rows_per_gpu": n,
                "parallelism": f"row-range shards x{world}",
                "exchange": xchg,
                "graph_steps": G,
                "exchange_bucket_steps": B if exchange else None,
                "count": "frame (32 packed slots per query, summed by the all-reduce; mbx_scan_count_frame_async)"
                         if frames else "in-launch finalize (mbx_scan_count_async)",
            },
            "phases_us": {
                "step_wall": ms_per_step * 1e3,
                "scan_kernel_max_over_ranks": kern_max * 1e3,
                "host_enqueue_rank0": t_enq * 1e6 / steps,
                "exchange_and_overlap": max(0.0, ms_per_step * 1e3 - kern_max * 1e3),
            },
            "hbm_gbs": 2 * 4 * n_global / (t_max / steps) / 1e9,
            "roofline": {
                "bound": "hbm",
                "kernel": "mbx::k_scan_fast<2, COUNT, no-deleted>",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": load_traffic(n, "frame" if frames else "finalize"),
                "traffic_unit": "HBM bytes per launch of rank 0's shard scan (rocprofv3 PMC, "
                                "profiles/c3_scan_pmc.json, same rows and COUNT form)",
                "kernel_ms": kern_ms,
                "algorithmic_bytes_per_launch": algo_bytes,
                # secondary denominator: the best read rate of the
                # scan's own load pattern with the predicate removed
                "measured_read_peak": probe["best_gbs"],
                "frac_of_measured_read_peak": achieved / probe["best_gbs"],
                "read_probe": probe,
            },
            "cpu_baseline": None,
        }
        if not args.no_cpu_baseline:
            # rank 0, after the timed region, over rank 0's shard (the other
            # ranks wait at the closing barrier)
            out["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds)
        os.write(out_fd, (json.dumps(out) + "\n").encode())

    for gr in graphs:
        gr.close()
    ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
