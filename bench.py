#!/usr/bin/env python3
"""bench.py -- BASELINE.json headline: scanned rows/s + HBM GB/s on the C3
workload (100M-row 4 x int32 Columnarfile, 2-predicate conjunction + COUNT),
at 1 / 2 / 4 / 8 GPUs, plus one record per other BASELINE config (C2, C4, C5).

One "step" = one ColumnarFileScan COUNT pass over the resident table:
`query ... {(c0 < 2^19)} ^ {(c1 >= 2^19)} FILESCAN` -> Total Results Count
(R/input/Query.java:137-152), executed as ONE kernel launch per GPU
(k_scan_fast<2, COUNT>), plus -- on N > 1 GPUs -- the path's one exchange
step: an in-place RCCL all-reduce of the COUNTs over xGMI, issued by libmbx
(mbx_comm_allreduce_count_async) right after the scan on the same stream.
Every step (= query) has its own collective (--exchange-bucket 1, the
default: SURVEY 8(e)'s per-query N_total / (max_k t_kernel,k + t_reduce)).
Inputs are resident in HBM before the timed region.

Scaling.  The path partitions by row
range with no data-path collective and one exchange per query, so the
headline reports weak scaling:
  --scaling weak (default): per-GPU work fixed at the C3 table -- rank r owns
      rows [r * 100M, (r + 1) * 100M) of an N x 100M-row logical table (its own
      seeds 42 + 1000 r + col; N = 1 is exactly the C3 table).  At N > 1 the
      same run also times the STRONG form and reports it as the `strong`
      sub-record: the metric's ONE 100M-row table in N 64-aligned shards
      (mbx_shard_bounds), with its phases (scan max over ranks, exchange).
      Both forms are also timed with the COUNTs of each captured graph's
      steps in ONE all-reduce (`bucketed`, `strong.bucketed`: the throughput
      form for a stream of queries; --no-bucketed drops them).
  --scaling strong: the headline itself is the strong form.
The timed steps replay HIP graphs (mbx_graph_*) of --graph-steps captured
steps (scans + their exchange), so small shards do not wait on the host.
Before any timing, ONE exchanged step runs eagerly and is verified (global
COUNT, every count-frame arrival): a broken collective or frame decode exits
non-zero with a one-line reason before any timed work (`pre_check`).
value = global rows scanned by all ranks / max-over-ranks wall time.

Kernel time (`roofline.kernel_ms`, every config's `kernel_ms`): one captured
HIP graph of --kernel-graph launches of the query's kernels alone, replayed,
HIP events on the library stream around the replays / launches -- so
kernel_ms <= ms_per_step (no per-launch event pair).

Config records (`configs`, --configs, default C5,C4,C2 -- C5 first, on the
heap C3 leaves, profiles/r05/m):
  C2  10M rows x 4 int32, c0 < 104858 -> BitSet + positions + COUNT, one
      launch (k_scan_select); a 1-GPU config: rank 0 only
  C4  100M rows (global, row-range sharded over the N GPUs), AND of the
      BitMapFiles bm(c2=3), bm(c3=7) -> positions + projected c0, c1 in ONE
      launch (k_cnf_select, (c0, c1) column group); at N > 1 + the RCCL
      all-gather of the per-rank counts (the concatenation offsets)
      (R/index/ColumnarIndexScan.java:130-181,287-308)
  C5  125M rows PER GPU (1B at N = 8) i32 / f32 / char(16),
      (c0 < 2^19) ^ (c1 >= 0.25) ^ (c2 >= "M") -> COUNT, SUM / MIN / MAX(c1);
      at N > 1 + the RCCL all-gather of the 48-byte records + the device
      rank-ordered fold (k_fold_agg)
Each is checked against torch reductions of the same device data before
and after its timing.  stdout carries only the JSON line.  A rank still
running --watchdog seconds (420) after its imports prints its threads'
tracebacks and exits 1 (the backstop behind the per-phase deadlines).
cpu_baseline (N = 1, rank 0): the oracle over the GPU run's own C3 table,
copied to host after timing; its COUNT must equal the GPU's.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak] [--configs C2,C4,C5|none]

Launch: with WORLD_SIZE unset and --gpus N > 1, this process is only a
launcher: before anything touches a GPU it starts N rank ("worker")
processes of this same script (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT in their env); rank 0's stdout is the
JSON line; it exits with the first failing rank's status (the others are
then stopped by PID).  Under an external torch.distributed.run (WORLD_SIZE
set, must equal --gpus) each rank process is a supervisor of ONE worker,
the supervisors sharing exit codes through a TCPStore.  Neither launcher nor
supervisor touches a GPU; workers die with them (PR_SET_PDEATHSIG).

Graph-phase fallback: before timing, the first replay of every set of
captured graphs (scans + their RCCL exchange) is waited for against a 60 s
deadline (a HIP event polled) and its steps verified on every rank; a hang or
a wrong result exits 4 (GRAPH_EXIT) with its reason, and the launcher /
supervisors start fresh workers ONCE with --graph-steps 0 (every step eager);
the line then says `"exchange_form": "eager (graph replay failed: ...)"`.
Each phase (setup, each C3 run, probe, each config, cpu baseline) re-arms a
deadline of its own (PHASE_S).
--dry-launch: the ranks print their rank env as JSON and exit before
importing torch (the launcher's CPU test, tests/test_bench_launch.py).
Rehearsal knobs (never set by the driver): MBX_BENCH_FORCE_GRAPH_FAIL=verify|timeout
(rank 0 reports that graph-phase failure: the fallback must follow),
MBX_BENCH_FAKE=graph:R|fail:R|ok (workers that touch no GPU, for the
launcher tests), MBX_BENCH_SAME_DEVICE=1 (N ranks on
one GPU, gloo exchange), MBX_BENCH_FORCE_EXCHANGE=1 (the exchange at N = 1),
MBX_BENCH_CORRUPT=frame|count (rank 0 damages its pre-check frame: the
pre-check must fire), MBX_BENCH_TORCH_EXCHANGE=1 (the fallback exchange --
torch.distributed's RCCL group, taken when libmbx's communicator fails on any
rank -- on purpose, at N = 1 too).
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
C2_LIT = 104858  # c0 < 104,858 (~10 %)
PRECHECK_EXIT = 3

# the keys every config record carries (tests/test_bench_launch.py)
CONFIG_KEYS = ("workload", "rows", "rows_per_gpu", "gpus", "selected", "ms_per_query", "rows_per_s", "kernel",
               "kernel_ms", "kernel_ms_max_over_ranks", "algorithmic_bytes_per_launch", "achieved_gbs", "frac",
               "exchange", "pre_check", "timing", "traffic")


def cpu_baseline(host_cols, gpu_count, min_seconds):
    """The oracle (C restatement of ColumnarFileScan + PredEval) timed on the
    GPU run's own C3 table: `host_cols` are the 4 device columns copied to
    host memory after the timed regions (the same arrays), full
    passes until min_seconds elapsed -- row ranges split over the host cores
    this process may use (OMP_NUM_THREADS, 16 per GPU on the box; SURVEY
    8(d)(ii)), each range evaluated row by row exactly like the single-thread
    oracle.  Its COUNT must equal the GPU's verified COUNT of that table."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    rows = len(host_cols[0])
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    t = oracle.Table([(oracle.INTEGER, 4, c) for c in host_cols])
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
    if not (count == count1 == gpu_count):
        print(f"bench: cpu_baseline COUNT {count1} / {count} (1 / {threads} threads) != GPU COUNT {gpu_count}",
              file=sys.stderr, flush=True)
        os._exit(5)
    return {
        "value": rows * passes / elapsed,
        "unit": "rows/s",
        "cores": threads,
        "kind": "port",
        "count": count,
        "count_equals_gpu": True,
        "sample": f"{passes} full pass(es) over the GPU run's own {rows:,}-row 4xint32 C3 table, copied from HBM "
                  f"after timing (same predicate; COUNT {count} = the GPU's verified COUNT); oracle/oracle.c "
                  f"orc_filescan_count_mt, {threads} OpenMP threads, {elapsed:.1f} s total; "
                  f"single thread: {rows / one:.3g} rows/s",
    }


def load_traffic(rows, count_mode):
    """HBM bytes per launch of the C3 scan over a `rows`-row shard with the
    given COUNT form ("finalize" | "frame"), from the committed rocprofv3 PMC
    summary (profiles/c3_scan_pmc.json: one entry per shard size bench.py
    runs at N = 1, 2, 4, 8; written by tools/c3_pmc_merge.py from tools/gpu_r6_e.sh), or None."""
    path = os.path.join(ROOT, "profiles", "c3_scan_pmc.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get("shards", {}).get(f"{rows}:{count_mode}")
        return (e or {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def load_config_traffic(name, rows_per_gpu):
    """HBM bytes per launch of a config record's kernel at this shard size
    (rocprofv3 PMC, profiles/config_pmc.json from tools/config_pmc.py), or
    None when that size was not profiled."""
    try:
        with open(os.path.join(ROOT, "profiles", "config_pmc.json")) as f:
            e = json.load(f)["configs"].get(f"{name}:{rows_per_gpu}")
        return (e or {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError, KeyError):
        return None


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# ---------------------------------------------------------------- launchers
# Neither launcher touches a GPU: they only start rank ("worker") processes,
# watch their exit codes and start fresh ones on two failures that another
# exchange form avoids.  The failing worker writes a one-line reason to
# $MBX_BENCH_STATUS and exits with the failure's code:
#   GRAPH_EXIT  the first replay of the captured graphs (the timed steps' form:
#               scans + their RCCL exchange) hung or was wrong -> relaunch with
#               --graph-steps 0 (every step eager, the same collective issued
#               step by step); $MBX_BENCH_FALLBACK carries the reason
#   COMM_EXIT   the RCCL exchange itself failed: its communicators did not come
#               up (in time), or the first exchanged step hung / was wrong ->
#               relaunch with $MBX_BENCH_HOST_EXCHANGE=<reason>: the exchange
#               as a gloo collective over host copies (the GPU work unchanged)
# Each fallback is taken at most once (at most 3 attempts); the line's
# `exchange_form` names what ran and why.  Any other failure is final.

GRAPH_EXIT = 4
COMM_EXIT = 6
KILLED = -9


def read_reason(path):
    try:
        with open(path) as f:
            return f.read().strip().splitlines()[0][:300]
    except (OSError, IndexError):
        return "no reason recorded"


def next_attempt(codes, argv, env, who):
    """The fallback after an attempt whose ranks ended with `codes` [(rank,
    exit code, reason)]: (argv, env) of the next attempt, or None when the
    status is final.  A failure whose fallback was already taken is final."""
    retry = [(r, c, why) for r, c, why in codes
             if (c == GRAPH_EXIT and "MBX_BENCH_FALLBACK" not in env)
             or (c == COMM_EXIT and "MBX_BENCH_HOST_EXCHANGE" not in env)]
    if not retry:
        return None
    own = [x for x in retry if not x[2].startswith("another rank")]
    r, c, why = (own or retry)[0]
    env = dict(env)
    if c == GRAPH_EXIT:
        env["MBX_BENCH_FALLBACK"] = f"rank {r}: {why}"
        argv = list(argv) + ["--graph-steps", "0"]
        what = "fresh ranks, eager steps"
    else:
        env["MBX_BENCH_HOST_EXCHANGE"] = f"rank {r}: {why}"
        what = "fresh ranks, host exchange"
    if who:
        print(f"bench {who}: {'graph replay' if c == GRAPH_EXIT else 'RCCL exchange'} failed on rank {r} ({why}); "
              f"{what}", file=sys.stderr, flush=True)
    return argv, env


def final_status(codes):
    """0, or the exit status of the first rank that failed on its own (not
    killed for a peer's failure)"""
    fails = [c for _, c, _ in codes if c not in (0, KILLED)]
    if fails:
        return fails[0] if fails[0] > 0 else 128 - fails[0]
    return 1 if any(c == KILLED for _, c, _ in codes) else 0


def worker_cmd(argv):
    return [sys.executable, os.path.abspath(__file__)] + list(argv)


def die_with_parent():
    """A worker's first act (long before any GPU call): SIGKILL when its
    launcher / supervisor dies (PR_SET_PDEATHSIG), so a launcher stopped by
    the driver's clock or by torch.distributed.run never leaves a rank holding
    a GPU; a parent already gone by then ends the worker at once.  Set here
    rather than in a Popen preexec_fn, which is unsafe in a launcher with
    threads (torch's TCPStore client)."""
    import ctypes
    import signal
    ctypes.CDLL(None, use_errno=True).prctl(1, int(signal.SIGKILL))  # PR_SET_PDEATHSIG
    parent = os.environ.get("MBX_BENCH_PARENT")
    if parent and os.getppid() != int(parent):
        os._exit(1)


def forward_term(procs):
    """SIGTERM / SIGINT to this launcher stop its workers too, then exit"""
    import signal

    def handler(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.kill()
        os._exit(128 + signum)
    signal.signal(signal.SIGTERM, handler)
    signal.signal(signal.SIGINT, handler)


def run_local_attempt(n, argv, env_extra, status_dir, attempt):
    """n worker processes on this node; returns [(rank, exit code, reason)]
    once all ended: the first failure stops the others by PID (their code is
    then KILLED).  Rank 0's stdout is this process's (the JSON line), the
    others' go to stderr (--dry-launch: every rank's to stdout)."""
    import subprocess
    port = free_port()
    dry = "--dry-launch" in argv
    procs, status = [], []
    for r in range(n):
        st = os.path.join(status_dir, f"a{attempt}_rank{r}.txt")
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MBX_BENCH_WORKER="1",
                   MBX_BENCH_PARENT=str(os.getpid()), MBX_BENCH_STATUS=st, **env_extra)
        out = None if (r == 0 or dry) else sys.stderr
        procs.append(subprocess.Popen(worker_cmd(argv), env=env, stdout=out))
        status.append(st)
    forward_term(procs)
    codes, killed, failed = {}, set(), False
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            r = procs.index(p)
            codes[r] = KILLED if r in killed else rc
            if rc != 0 and not failed and r not in killed:
                failed = True
                print(f"bench launcher: rank {r} exited with {rc}; stopping the others", file=sys.stderr)
                for q in live:
                    killed.add(procs.index(q))
                    q.kill()
        time.sleep(0.05)
    return [(r, codes[r], read_reason(status[r]) if codes[r] in (GRAPH_EXIT, COMM_EXIT) else "")
            for r in range(n)]


def launch_ranks(n, argv):
    """this node's N ranks (WORLD_SIZE unset, --gpus N > 1)"""
    import shutil
    import tempfile
    status_dir = tempfile.mkdtemp(prefix="mbx_bench_")
    try:
        env = {}
        for attempt in range(3):
            codes = run_local_attempt(n, argv, env, status_dir, attempt)
            nxt = next_attempt(codes, argv, env, "launcher")
            if nxt is None:
                return final_status(codes)
            argv, env = nxt
        return final_status(codes)
    finally:
        shutil.rmtree(status_dir, ignore_errors=True)


def supervise_rank(argv):
    """Under an external launcher (torch.distributed.run: WORLD_SIZE, RANK,
    MASTER_* set), this process supervises ONE worker: it starts it, shares
    its exit code with the other ranks' supervisors through a TCPStore (torch
    run's own agent store when TORCHELASTIC_USE_AGENT_STORE, else one hosted by
    rank 0), stops its worker when another rank's worker failed, and after a
    graph-phase or exchange failure anywhere every supervisor starts one fresh
    worker with the same fallback (next_attempt: every supervisor sees the same
    codes, so all decide alike).  Workers rendezvous on a fresh port per
    attempt (rank 0's worker hosts that store).  Returns the exit status."""
    import datetime
    import shutil
    import subprocess
    import tempfile

    import torch.distributed as dist  # host side only: no GPU is touched here
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
    store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]), world,
                          is_master=(rank == 0 and not agent), timeout=datetime.timedelta(seconds=600),
                          wait_for_workers=False)
    run_id = os.environ.get("TORCHELASTIC_RUN_ID", "") + os.environ.get("TORCHELASTIC_RESTART_COUNT", "")
    key = lambda a, r: f"mbx_bench/{run_id}/a{a}/rank{r}"  # noqa: E731
    status_dir = tempfile.mkdtemp(prefix="mbx_bench_")
    extra, args_now = {}, list(argv)
    try:
        for attempt in range(3):
            if rank == 0:
                store.set(f"mbx_bench/{run_id}/a{attempt}/port", str(free_port()))
            port = store.get(f"mbx_bench/{run_id}/a{attempt}/port").decode()
            env = dict(os.environ, MASTER_PORT=port, MBX_BENCH_WORKER="1", MBX_BENCH_PARENT=str(os.getpid()),
                       MBX_BENCH_STATUS=os.path.join(status_dir, f"a{attempt}.txt"), **extra)
            env.pop("TORCHELASTIC_USE_AGENT_STORE", None)  # the workers' store is hosted by rank 0's worker
            p = subprocess.Popen(worker_cmd(args_now), env=env, stdout=None if rank == 0 else sys.stderr)
            forward_term([p])
            peers = [key(attempt, r) for r in range(world) if r != rank]
            killed = False
            while p.poll() is None:
                for k in peers:  # a peer's worker already failed: this one would wait on it
                    if store.check([k]) and not store.get(k).decode().startswith(("0|", f"{KILLED}|")):
                        p.kill()
                        killed = True
                        break
                time.sleep(0.1)
            rc = p.wait()
            rc = KILLED if killed else rc
            reason = read_reason(env["MBX_BENCH_STATUS"]) if rc in (GRAPH_EXIT, COMM_EXIT) else ""
            store.set(key(attempt, rank), f"{rc}|{reason}")
            deadline = time.time() + 600
            while not store.check([key(attempt, r) for r in range(world)]):
                if time.time() > deadline:
                    print(f"bench supervisor {rank}: peers never reported", file=sys.stderr)
                    return 1
                time.sleep(0.1)
            codes = []
            for r in range(world):
                c, _, why = store.get(key(attempt, r)).decode().partition("|")
                codes.append((r, int(c), why))
            nxt = next_attempt(codes, args_now, extra, "supervisor" if rank == 0 else None)
            if nxt is None:
                return final_status(codes)
            args_now, extra = nxt
        return final_status(codes)
    finally:
        shutil.rmtree(status_dir, ignore_errors=True)


def fake_worker(args, world, rank):
    """MBX_BENCH_FAKE=<modes>:R (launcher tests, no GPU).  Modes, '+'-joined:
    graph (rank R's graph phase fails until the eager fallback), comm (its
    exchange fails until the host fallback), fail (it exits 7: final); the
    other ranks wait as if inside a collective.  A rank with nothing left to
    fail prints a line as rank 0 would."""
    modes, _, who = os.environ["MBX_BENCH_FAKE"].partition(":")
    modes = modes.split("+")
    fallback, host = os.environ.get("MBX_BENCH_FALLBACK"), os.environ.get("MBX_BENCH_HOST_EXCHANGE")
    pending = [m for m in modes if (m == "graph" and args.graph_steps and not fallback)
               or (m == "comm" and not host) or m == "fail"]
    if pending:
        time.sleep(0.5)
        if str(rank) == who:
            m = pending[0]
            if m == "graph":
                fail_exit(GRAPH_EXIT, "C3: first replay of the captured graphs did not finish within 60 s (fake)")
            if m == "comm":
                fail_exit(COMM_EXIT, "communicators: ncclCommInitRank did not return within 120 s (fake)")
            sys.exit(7)
        time.sleep(60)
        sys.exit(1)
    if rank == 0:
        print(json.dumps({"fake": True, "n_gpus": world, "graph_steps": args.graph_steps,
                          "exchange_form": exchange_form(args.graph_steps, fallback, host)}), flush=True)


def fail_exit(code, reason):
    """a failure the launcher may answer with a fallback: the reason into
    $MBX_BENCH_STATUS, then exit `code`"""
    path = os.environ.get("MBX_BENCH_STATUS")
    if path:
        try:
            with open(path, "w") as f:
                f.write(reason + "\n")
        except OSError:
            pass
    what = {GRAPH_EXIT: "graph phase", COMM_EXIT: "exchange"}.get(code, "run")
    print(f"bench: {what} failed: {reason}", file=sys.stderr, flush=True)
    sys.stderr.flush()
    os._exit(code)


def graph_failed(reason):
    fail_exit(GRAPH_EXIT, reason)


def exchange_form(graph_steps, fallback, host=None):
    if host:
        form = f"host gloo exchange of the device results, eager (RCCL exchange failed: {host})"
        return form + (f"; earlier, graph replay failed: {fallback}" if fallback else "")
    if fallback:
        return f"eager (graph replay failed: {fallback})"
    return f"HIP graphs of {graph_steps} steps (first replay verified)" if graph_steps else "eager"


class PhaseClock:
    """Per-phase deadlines: a daemon thread that, when the armed phase outlives
    its budget, prints the phase and every thread's traceback and exits with
    the phase's code (GRAPH_EXIT for a graph replay, COMM_EXIT for the
    exchange's setup and first use, 1 otherwise).  Ctypes and
    torch calls release the GIL while they wait, so the thread runs while the
    main thread is stuck in a HIP / RCCL call; faulthandler's --watchdog stays
    as the backstop for a wait that holds the GIL."""

    def __init__(self):
        import threading
        self.phase, self.deadline, self.code = None, None, 1
        self.lock = threading.Lock()
        threading.Thread(target=self._run, daemon=True).start()

    def arm(self, phase, seconds, code=1):
        with self.lock:
            self.phase, self.deadline, self.code = phase, time.monotonic() + seconds, code

    def _run(self):
        import faulthandler
        while True:
            time.sleep(0.25)
            with self.lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                phase, code = self.phase, self.code
            if late:
                print(f"bench: phase `{phase}` outlived its budget", file=sys.stderr, flush=True)
                faulthandler.dump_traceback(all_threads=True)
                if code in (GRAPH_EXIT, COMM_EXIT):
                    fail_exit(code, f"{phase}: did not finish within its budget")
                os._exit(code)


PHASE_S = {"comm": 120, "setup": 180, "c3": 120, "probe": 60, "config": 150, "cpu": 120}
GRAPH_WAIT_S = 60.0
CLOCK = None


def arm(phase, seconds, code=1):
    if CLOCK is not None:
        CLOCK.arm(phase, seconds, code)


def quiet_stdout():
    """The one JSON line is the only thing on stdout: fd 1 is pointed at
    stderr for the libraries (RCCL prints a version banner when it creates
    its first communicator) and the result goes to a duplicate of the
    original fd 1."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return fd


# ---------------------------------------------------------------- checks
# pure functions over host copies (numpy), unit-tested on the CPU

FRAME_SLOTS, FRAME_SLOT_WORDS = 32, 16


def frame_fields(frames):
    """(count, nan_blocks, arrivals) per step of (k, 512) int64 count frames:
    slot i = word 16 i (its own 128-byte line), count in bits 24.., NaN blocks
    in bits 12..23, arrivals in bits 0..11 (mbx_count_frame_decode)."""
    import numpy as np
    f = np.asarray(frames, dtype=np.int64).reshape(-1, FRAME_SLOTS, FRAME_SLOT_WORDS)[:, :, 0]
    return (f >> 24).sum(1), ((f >> 12) & 0xFFF).sum(1), (f & 0xFFF).sum(1)


def check_counts(kind, got, want, frames=None, nblocks=None):
    """None, or the one-line reason the exchanged step(s) are wrong: every
    step's global COUNT must equal `want`; with count frames every block of
    every rank must have arrived exactly once (`nblocks` summed over ranks)
    and no block may report NaN."""
    import numpy as np
    if frames is not None:
        c, nan, arr = frame_fields(frames)
        if not (arr == nblocks).all():
            return f"{kind}: frame arrivals {arr[:4].tolist()} != {nblocks} blocks over all ranks"
        if nan.any():
            return f"{kind}: {int(nan.sum())} NaN blocks in an integer plan"
        got = c
    got = np.asarray(got).reshape(-1)
    if not (got == want).all():
        return f"{kind}: global COUNT {got[:4].tolist()} != {want}"
    return None


def check_aggregate(kind, got, want, rel=1e-6):
    """None, or why dict(count, sum, min, max) `got` differs from `want`:
    COUNT / MIN / MAX exact, SUM within `rel` (north_star: 1e-6 relative)."""
    for k in ("count", "min", "max"):
        if got[k] != want[k]:
            return f"{kind}: {k} {got[k]!r} != {want[k]!r}"
    if abs(got["sum"] - want["sum"]) > rel * abs(want["sum"]):
        return f"{kind}: sum {got['sum']!r} vs {want['sum']!r} beyond {rel} relative"
    return None


def config_record(workload, rows, rows_per_gpu, gpus, selected, ms_per_query, kernel, kernel_ms, kernel_ms_max,
                  algo_bytes, exchange, pre_check, timing, **extra):
    """One `configs` entry: global rows/s of the query with its exchange, the
    dominant kernel's time from graph replay and its fraction of 8 TB/s over
    SURVEY 8(d)'s algorithmic bytes of rank 0's launch."""
    gbs = algo_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    traffic = load_config_traffic(workload.split(":")[0], rows_per_gpu)
    rec = {"workload": workload, "rows": rows, "rows_per_gpu": rows_per_gpu, "gpus": gpus, "selected": selected,
           "ms_per_query": ms_per_query, "rows_per_s": rows / (ms_per_query * 1e-3) if ms_per_query > 0 else 0.0,
           "kernel": kernel, "kernel_ms": kernel_ms, "kernel_ms_max_over_ranks": kernel_ms_max,
           "algorithmic_bytes_per_launch": algo_bytes, "achieved_gbs": gbs, "frac": gbs / HBM_PEAK_GBS,
           "exchange": exchange, "pre_check": pre_check, "timing": timing,
           "traffic": traffic, "traffic_over_algorithmic": traffic / algo_bytes if traffic and algo_bytes else None,
           # the bytes the kernel really moves per launch over its time: for C4's
           # random rows every selected row costs a whole 128-byte line
           # (profiles/r06/c4_req), so its frac of algorithmic bytes is low while
           # this one is not
           "traffic_gbs": traffic / (kernel_ms * 1e-3) / 1e9 if traffic and kernel_ms > 0 else None,
           "traffic_frac": traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic and kernel_ms > 0 else None,
           "traffic_unit": "HBM bytes per launch of rank 0's kernel at this shard size (rocprofv3 PMC, "
                           "profiles/config_pmc.json: read = gfx950's request-size split 32 n32 + 64 n64 + 128 n128, "
                           "write = WRITE_SIZE)"}
    rec.update(extra)
    return rec


def make_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rows", type=int, default=100_000_000,
                    help="global rows (strong scaling) or rows per GPU (weak)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="weak")
    ap.add_argument("--graph-steps", type=int, default=20, help="steps per captured HIP graph (0: eager launches)")
    ap.add_argument("--kernel-graph", type=int, default=20, help="launches per graph timed for kernel_ms")
    ap.add_argument("--exchange-bucket", type=int, default=1,
                    help="steps whose COUNTs share one all-reduce (1, the default: one collective per query)")
    ap.add_argument("--count", choices=["auto", "frame", "finalize"], default="auto",
                    help="frame: each scan adds its COUNT into a 32-slot count frame (no in-launch finalize; the "
                         "exchange all-reduces whole frames); finalize: the scan's last block writes the COUNT; "
                         "auto: frame with an exchange, finalize without")
    # C5 first: its 3 GB per GPU read 3-4 % slower when allocated after C4's
    # tables and groups were freed (a fragmented heap, profiles/r05/m)
    ap.add_argument("--configs", default="C5,C4,C2", help="config records to add, in this order (comma list, or none)")
    ap.add_argument("--c4-rows", type=int, default=100_000_000, help="C4 global rows (sharded)")
    ap.add_argument("--c5-rows", type=int, default=125_000_000, help="C5 rows per GPU")
    ap.add_argument("--no-strong", action="store_true", help="no strong sub-record at N > 1")
    ap.add_argument("--no-bucketed", action="store_true",
                    help="no bucketed sub-records at N > 1 (the COUNTs of each captured graph's steps in one all-reduce)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--watchdog", type=float, default=420.0,
                    help="seconds after which a still-running rank prints every thread's traceback and exits 1 "
                         "(a hung collective fails with its place named, inside the driver's budget); 0: off")
    ap.add_argument("--dry-launch", action="store_true",
                    help="ranks print their rank env as JSON and exit before importing torch (launcher test)")
    return ap


def agree(torch, dist, world, rank, reason, code=PRECHECK_EXIT):
    """A collective verdict: every rank learns whether any rank's check
    failed (reason not None); then each failing rank prints its one-line
    reason, the others a line naming the cause, and ALL exit `code`
    (PRECHECK_EXIT; COMM_EXIT for the first exchanged step, which the
    launcher answers with the host exchange) -- no rank is left waiting in a
    later collective."""
    bad = int(reason is not None)
    if world > 1:
        t = torch.tensor([bad], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        anybad = int(t[0])
    else:
        anybad = bad
    if anybad:
        print(f"bench: pre-check failed on rank {rank}: {reason}" if reason else
              f"bench: rank {rank} stops: another rank's pre-check failed", file=sys.stderr, flush=True)
        sys.stderr.flush()
        if code != PRECHECK_EXIT:
            fail_exit(code, reason or "another rank's pre-check failed")
        os._exit(PRECHECK_EXIT)


# ---------------------------------------------------------------- GPU side

class Harness:
    """One rank's clocks, barriers and collective verdicts."""

    def __init__(self, torch, dist, m, ctx, world, rank, comm, same_device, exchange, torch_pg=None):
        self.torch, self.dist, self.m, self.ctx = torch, dist, m, ctx
        self.world, self.rank, self.comm, self.torch_pg = world, rank, comm, torch_pg
        self.same_device, self.exchange = same_device, exchange
        self.ext = torch.cuda.ExternalStream(ctx.stream)
        torch.cuda.set_stream(self.ext)

    def solo(self):
        """This rank alone (a 1-GPU config inside an N-rank run): the same
        context and stream, no collectives, no exchange."""
        import copy
        h = copy.copy(self)
        h.world, h.comm, h.torch_pg, h.exchange = 1, None, None, False
        return h

    def barrier(self):
        self.ctx.sync()
        self.torch.cuda.synchronize()
        if self.world > 1:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def rmax(self, x):
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

    def rsum(self, x):
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.int64)
        self.dist.all_reduce(t)
        return int(t[0])

    def agree(self, reason, code=PRECHECK_EXIT):
        agree(self.torch, self.dist, self.world, self.rank, reason, code)

    def graphs(self, enqueue, k0, k1, per):
        """HIP graphs of `per` steps each covering steps k0..k1-1 (None when
        the runtime refuses a capture: the steps then run eagerly)."""
        out = []
        try:
            k = k0
            while k < k1:
                g = min(per, k1 - k)
                self.ctx.graph_begin()
                try:
                    enqueue(k, k + g)
                finally:
                    out.append(self.ctx.graph_end())
                k += g
            return out
        except self.m.MbxError as err:
            print(f"rank {self.rank}: HIP graph capture failed ({err}); eager steps", file=sys.stderr)
            for gr in out:
                gr.close()
            self.ctx.sync()
            return None

    def kernel_ms(self, enqueue_one, k, reps=3):
        """Average duration of one launch of the query's kernels: one graph of
        k launches (enqueue_one(i), i < k), one untimed replay, then `reps`
        replays between HIP events on the library stream; (own, max over
        ranks).  Eager launches if the capture is refused."""
        torch = self.torch
        gr = self.graphs(lambda a, b: [enqueue_one(i) for i in range(a, b)], 0, k, k)
        run = (lambda: gr[0].launch()) if gr else (lambda: [enqueue_one(i) for i in range(k)])
        run()
        self.ctx.sync()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(self.ext)
        for _ in range(reps):
            run()
        b.record(self.ext)
        self.ctx.sync()
        ms = a.elapsed_time(b) / (reps * k)
        for g in gr or []:
            g.close()
        return ms, self.rmax(ms)

    def first_replay(self, gr, drain, verify, k0, k1, label):
        """The captured graphs' first replay, before anything is timed: every
        graph launched, then a HIP event on the library stream polled against
        GRAPH_WAIT_S (a collective that never completes inside a replay is
        caught here, not by the timed region), then the replayed steps
        verified (verify(k0, k1, kind) -> None | reason) on every rank.  A
        hang or a wrong result exits GRAPH_EXIT (the launcher then starts fresh
        ranks with eager steps).  MBX_BENCH_FORCE_GRAPH_FAIL=timeout|verify
        (rehearsal) makes rank 0 report that failure."""
        torch = self.torch
        force = os.environ.get("MBX_BENCH_FORCE_GRAPH_FAIL", "") if self.rank == 0 else ""
        phase = f"{label}: first replay of {len(gr)} captured graph(s)"
        arm(phase, GRAPH_WAIT_S + 30, GRAPH_EXIT)
        for g in gr:
            g.launch()
        ev = torch.cuda.Event()
        ev.record(self.ext)
        t0 = time.monotonic()
        while not ev.query():
            if time.monotonic() - t0 > GRAPH_WAIT_S:
                graph_failed(f"{phase} did not finish within {GRAPH_WAIT_S:.0f} s")
            time.sleep(0.0005)
        if force == "timeout":
            graph_failed(f"{phase} did not finish within {GRAPH_WAIT_S:.0f} s (MBX_BENCH_FORCE_GRAPH_FAIL)")
        drain()
        reason = verify(k0, k1, f"{label} first graph replay") if verify else None
        if force == "verify":
            reason = f"{label} first graph replay: forced mismatch (MBX_BENCH_FORCE_GRAPH_FAIL)"
        bad = int(reason is not None)
        if self.world > 1:
            t = torch.tensor([bad], dtype=torch.int32)
            try:
                self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            except Exception as err:  # a peer left the group inside its graph phase
                graph_failed(f"{phase}: verdict all-reduce failed ({type(err).__name__}: {err})")
            bad = int(t[0])
        if bad:
            graph_failed(reason or f"{label}: another rank's first graph replay failed")
        arm(f"{label}: timed steps", PHASE_S["c3"])

    def timed(self, enqueue, drain, steps, warmup, graph_steps, reset=None, verify=None, label=""):
        """warmup steps (eager), graphs of graph_steps captured and replayed
        once untimed (first_replay: bounded wait + verified), reset(), then
        EXACTLY `steps` steps between barrier + synchronize on both sides;
        (max-over-ranks ms per step, host enqueue us per step, graph steps
        used)."""
        enqueue(0, warmup)
        drain()
        gr = None
        if graph_steps and (self.comm is not None or not self.exchange):  # gloo exchanges run eagerly
            gr = self.graphs(enqueue, warmup, warmup + steps, graph_steps)
            if gr:
                self.first_replay(gr, drain, verify, warmup, warmup + steps, label)
        if reset:
            reset()
        self.barrier()
        t0 = time.perf_counter()
        if gr:
            for g in gr:
                g.launch()
        else:
            enqueue(warmup, warmup + steps)
        t_enq = time.perf_counter() - t0
        if self.exchange and self.comm is None:
            drain()  # the same-device rehearsal's host exchange belongs to the steps
        self.torch.cuda.synchronize()  # the whole device: the library stream's steps included
        if self.world > 1:
            self.dist.barrier()
        wall = time.perf_counter() - t0
        for g in gr or []:
            g.close()
        return self.rmax(wall * 1e3 / steps), t_enq * 1e6 / steps, (graph_steps if gr else 0)


def gen_column(torch, n_global, s, e, seed, hi):
    """Rows [s, e) of one int32 column uniform in [0, hi), generated whole
    from its seed (torch Philox on the device), so every shard count slices
    the same table."""
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    full = torch.randint(0, hi, (n_global,), dtype=torch.int32, device="cuda", generator=g)
    if s == 0 and e == n_global:
        return full
    out = full[s:e].clone()
    del full
    return out


def make_columns(torch, n_global, s, e, seed_base, his=(1 << 20,) * 4):
    cols = [gen_column(torch, n_global, s, e, seed_base + j, hi) for j, hi in enumerate(his)]
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return cols


def full_count(torch, n_global, seed_base):
    """The global C3 COUNT of the whole table (torch reduction)."""
    a = gen_column(torch, n_global, 0, n_global, seed_base, 1 << 20)
    b = gen_column(torch, n_global, 0, n_global, seed_base + 1, 1 << 20)
    c = int(((a < THRESH) & (b >= THRESH)).sum().item())
    del a, b
    torch.cuda.empty_cache()
    return c


def read_probe(H, table, reps=20):
    """Best read bandwidth of k_read_probe (mbx_probe_read: the C3 kernel's
    tiles and non-temporal dwordx4 loads over c0, c1 with no predicate) over a
    few block mappings, timed like the scan: one captured graph of `reps`
    launches replayed between HIP events on the library stream."""
    torch, ctx = H.torch, H.ctx
    n = table.nrows
    nbytes = 2 * 4 * (n // 256 * 256)
    variants = [("segments, scan default", dict()), ("segments, tpb=256", dict(tiles_per_block=256)),
                ("segments, tpb=96", dict(tiles_per_block=96)),
                ("grid-stride 1024 blocks", dict(interleave=True, grid=1024)),
                ("grid-stride 2048 blocks", dict(interleave=True, grid=2048))]
    res = {}
    for name, kw in variants:
        ms, _ = H.solo().kernel_ms(lambda i: ctx.probe_read(table, [0, 1], **kw), reps)
        res[name] = nbytes / (ms * 1e-3) / 1e9
    best = max(res, key=res.get)
    return {"best_gbs": res[best], "best": best, "gbs": res}


def run_c3(H, args, cols, n, s, glob, label, bucket=None):
    """The C3 query over one rank's shard (`cols`, rows [s, s + n)), whose
    global COUNT over all ranks is `glob`: pre-check of one exchanged step,
    `args.steps` timed steps (graph replay), kernel time, every step's count
    checked.  Returns the measurements (the table stays open for the probe)."""
    torch, ctx, m, world, rank = H.torch, H.ctx, H.m, H.world, H.rank
    # the first exchanged step of the run is the exchange's first use: a hang or
    # a wrong global result there is an exchange failure (COMM_EXIT: the
    # launcher's host-exchange fallback), later ones are ordinary failures
    rccl = H.comm is not None or H.torch_pg is not None
    first_use = rccl and label == "C3"
    arm(f"{label}: pre-check, graph capture", PHASE_S["c3"], COMM_EXIT if first_use else 1)
    table = ctx.wrap([(m.mbx.INTEGER, 4)] * 4, [col.data_ptr() for col in cols], n, None, row_offset=s)
    cnf = [[(m.mbx.LT, ("sym", 1), ("int", THRESH))], [(m.mbx.GE, ("sym", 2), ("int", THRESH))]]
    plan = ctx.compile(table, cnf)

    # the kernel's count vs a torch reduction of the same device columns
    got = ctx.scan_count(plan)
    want = int(((cols[0] < THRESH) & (cols[1] >= THRESH)).sum().item())
    H.agree(None if got == want else f"{label}: scan count {got} != torch {want}")

    # count frames (mbx_scan_count_frame_async): with an exchange, each step's
    # scan adds its packed per-block counts into its own zeroed 4 KB frame with
    # no-return atomics and the all-reduce sums whole frames -- the launch ends
    # without the finalize's dependent atomic round trips.  A slot's 12-bit
    # arrival field sums every rank's arrivals: it must stay < 4096
    # (mbx_count_frame_fits), else the in-launch finalize is used.
    frames = args.count == "frame" or (args.count == "auto" and H.exchange)
    nb_own = ctx.scan_blocks(plan)
    nb_all = H.rsum(nb_own)
    if frames and not m.mbx.count_frame_fits(int(H.rmax(nb_own)), world):
        if args.count == "frame":
            raise SystemExit(f"bench: {world} ranks x {nb_own} blocks overflow a count frame")
        frames = False
        print(f"rank {rank}: {world} ranks x {nb_own} blocks overflow a count frame; in-launch finalize",
              file=sys.stderr)
    FW = m.mbx.COUNT_FRAME_WORDS if frames else 1
    steps, warmup = args.steps, args.warmup
    counts = torch.zeros((steps + warmup, FW), dtype=torch.int64, device="cuda")
    base = counts.data_ptr()
    B = max(1, bucket if bucket is not None else args.exchange_bucket)
    gloo_works = []

    def scan(k, buf=base):
        if frames:
            ctx.scan_count_frame_async(plan, buf + 8 * FW * k)
        else:
            ctx.scan_count_async(plan, buf + 8 * k)

    def enqueue(k0, k1):
        """steps k0..k1-1: one scan each; the exchange all-reduces the COUNTs
        of every B consecutive steps in one collective"""
        for j in range(k0, k1, B):
            je = min(j + B, k1)
            for k in range(j, je):
                scan(k)
            if H.comm is not None:
                H.comm.allreduce_count_async(base + 8 * FW * j, FW * (je - j))
            elif H.torch_pg is not None:  # on the library stream (torch's current stream)
                H.dist.all_reduce(counts[j:je], group=H.torch_pg)
            elif H.exchange:  # same-device rehearsal: gloo over host copies
                gloo_works.extend(range(j, je))

    def drain():
        ctx.sync()
        if gloo_works:
            h = counts[gloo_works].cpu()
            H.dist.all_reduce(h)
            counts[gloo_works] = h.cuda()
            gloo_works.clear()
        torch.cuda.synchronize()

    def verify(k0, k1, kind):
        c = counts[k0:k1].cpu().numpy()
        if frames:
            return check_counts(kind, None, glob if H.exchange else want, frames=c,
                                nblocks=nb_all if H.exchange else nb_own)
        return check_counts(kind, c[:, 0], glob if H.exchange else want)

    # pre-check: ONE exchanged step, eagerly, verified on every rank before
    # anything is timed
    torch.cuda.synchronize()
    enqueue(0, 1)
    drain()
    corrupt = os.environ.get("MBX_BENCH_CORRUPT", "")
    if corrupt and rank == 0:  # rehearsal: a damaged frame / count must stop the run here
        counts[0, 0] += (1 << 24) if (corrupt == "count" or not frames) else 1
        torch.cuda.synchronize()
    H.agree(verify(0, 1, f"{label} pre-check"), COMM_EXIT if first_use else PRECHECK_EXIT)
    arm(f"{label}: graph capture", PHASE_S["c3"])
    counts.zero_()
    torch.cuda.synchronize()

    ms_step, enq_us, G = H.timed(enqueue, drain, steps, warmup, args.graph_steps,
                                 reset=lambda: (counts.zero_(), torch.cuda.synchronize()), verify=verify, label=label)
    reason = verify(warmup, warmup + steps, f"{label} timed steps")
    H.agree(reason)

    # kernel duration: a graph of --kernel-graph scans alone (own scratch slots)
    KG = max(1, args.kernel_graph)
    scratch = torch.zeros((KG, FW), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    kern_ms, kern_max = H.kernel_ms(lambda i: scan(i, scratch.data_ptr()), KG)
    print(f"rank {rank}: {label} rows [{s}, {s + n}), host enqueue {enq_us:.1f} us/step, "
          f"wall {ms_step * 1e3:.1f} us/step, scan kernel {kern_ms * 1e3:.1f} us (graph of {KG})", file=sys.stderr)
    return dict(table=table, plan=plan, frames=frames, ms_step=ms_step, enq_us=enq_us, G=G, B=B,
                kern_ms=kern_ms, kern_max=kern_max, want=want)


def timing_label(G, steps):
    return f"HIP graphs of {G} queries replayed, {steps} timed" if G else \
        f"{steps} eager queries (host-side or torch.distributed exchange)"


def exchange_name(H, what):
    if H.comm is not None:
        return what
    if H.torch_pg is not None:
        return "torch.distributed RCCL group (fallback: libmbx's communicator failed), eager"
    if H.exchange:
        return (f"gloo over host copies (fallback: the RCCL exchange failed: {H.host_reason})"
                if getattr(H, "host_reason", None) else "gloo (same-device rehearsal)")
    return "none"


def config_c2(H, args):
    """C2 (1 GPU, rank 0): 10M x 4 int32, c0 < 104858 -> BitSet + ascending
    positions + COUNT in one launch (mbx_scan_select_async, k_scan_select);
    ColumnarFileScan's get_next_tid stream (R/iterator/ColumnarFileScan.java:174-188)."""
    torch, ctx, m = H.torch, H.ctx, H.m
    n = 10_000_000
    cols = make_columns(torch, n, 0, n, 42)
    t = ctx.wrap([(m.mbx.INTEGER, 4)] * 4, [c.data_ptr() for c in cols], n)
    plan = ctx.compile(t, [[(m.mbx.LT, ("sym", 1), ("int", C2_LIT))]])
    bm = ctx.bitmap_alloc(n)
    ids = torch.zeros(n, dtype=torch.int64, device="cuda")
    steps, warmup = args.steps, args.warmup
    cnt = torch.zeros(steps + warmup, dtype=torch.int64, device="cuda")
    sel = cols[0] < C2_LIT
    want = int(sel.sum().item())
    wpos = torch.nonzero(sel).flatten()

    def query(k):
        ctx.scan_select_async(plan, bm, ids.data_ptr(), cnt.data_ptr() + 8 * k)

    def verify(k0, k1, kind):
        c = cnt[k0:k1].cpu().numpy()
        r = check_counts(kind, c, want)
        if r is None and not bool((ids[:want] == wpos).all()):
            r = f"{kind}: positions differ from torch.nonzero"
        return r

    torch.cuda.synchronize()
    query(0)
    ctx.sync()
    H.agree(verify(0, 1, "C2 pre-check"))
    ms, _, G = H.timed(lambda a, b: [query(k) for k in range(a, b)], ctx.sync, steps, warmup, args.graph_steps,
                       reset=lambda: (cnt.zero_(), ids.zero_(), torch.cuda.synchronize()), verify=verify, label="C2")
    H.agree(verify(warmup, warmup + steps, "C2 timed steps"))
    kms, kmax = H.kernel_ms(lambda i: query(0), max(1, args.kernel_graph))
    byts = n * 4 + n // 8 + want * 8
    # C2's 40 MB column stays in the 256 MB Infinity Cache across back-to-back
    # queries, so 8 TB/s is a generous denominator: beside it, the
    # predicate-free read of that column with the scan's own tiles and loads
    # (k_read_probe, one launch, timed like the query)
    pms, _ = H.kernel_ms(lambda i: ctx.probe_read(t, [0]), max(1, args.kernel_graph))
    probe_gbs = 4 * (n // 256 * 256) / (pms * 1e-3) / 1e9
    rec = config_record("C2: 10M-row 4xint32, c0 < 104858 -> BitSet + positions + COUNT (one launch)",
                        n, n, 1, want, ms, "mbx::k_scan_select", kms, kmax, byts, "none", "ok",
                        timing_label(G, steps),
                        resident_read_probe={"kernel_ms": pms, "gbs": probe_gbs,
                                             "what": "k_read_probe over c0 (40 MB, cache-resident across launches), "
                                                     "no predicate, no outputs: the launch + read floor"},
                        kernel_over_read_probe=kms / pms)
    del cols, t, plan, bm, ids, sel, wpos
    torch.cuda.empty_cache()
    return rec


def config_c4(H, args):
    """C4: 100M global rows sharded by row range; ColumnarIndexScan over the
    BitMapFiles bm(c2=3) AND bm(c3=7) -> positions + projected c0, c1 in one
    launch (mbx_cnf_materialize_async, (c0, c1) column group), at N > 1 the
    RCCL all-gather of the per-rank counts (the concatenation offsets)."""
    torch, ctx, m, world, rank = H.torch, H.ctx, H.m, H.world, H.rank
    N = args.c4_rows
    s, e = m.mbx.shard_bounds(N, world, rank)
    n = e - s
    c0, c1, c2, c3 = make_columns(torch, N, s, e, 42, his=(1 << 20, 1 << 20, 10, 10))
    t = ctx.wrap([(m.mbx.INTEGER, 4)] * 4, [x.data_ptr() for x in (c0, c1, c2, c3)], n, row_offset=s)
    bm2 = ctx.index_build(t, 2, [("int", v) for v in range(10)])
    bm3 = ctx.index_build(t, 3, [("int", v) for v in range(10)])
    a, b = bm2[3], bm3[7]
    ctx.group(t, [0, 1])
    sel = (c2 == 3) & (c3 == 7)
    want = int(sel.sum().item())
    cap = max(1, n // 50)
    ids = torch.zeros(cap, dtype=torch.int64, device="cuda")
    o0 = torch.zeros(cap, dtype=torch.int32, device="cuda")
    o1 = torch.zeros(cap, dtype=torch.int32, device="cuda")
    steps, warmup = args.steps, args.warmup
    cnts = torch.zeros(steps + warmup, dtype=torch.int64, device="cuda")
    alls = torch.zeros(steps + warmup, world, dtype=torch.int64, device="cuda")
    conj = [[a], [b]]
    glob = H.rsum(want)
    gloo = []

    def launch(k):
        ctx.cnf_materialize_async(t, conj, [0, 1], ids.data_ptr(), [o0.data_ptr(), o1.data_ptr()],
                                  cnts.data_ptr() + 8 * k)

    def enqueue(k0, k1):
        for k in range(k0, k1):
            launch(k)
            if H.comm is not None:
                H.comm.allgather_count_async(cnts.data_ptr() + 8 * k, alls[k].data_ptr())
            elif H.torch_pg is not None:
                H.dist.all_gather_into_tensor(alls[k], cnts[k:k + 1], group=H.torch_pg)
            elif world > 1:
                gloo.append(k)

    def drain():
        ctx.sync()
        if gloo:
            parts = [torch.empty(len(gloo), dtype=torch.int64) for _ in range(world)]
            H.dist.all_gather(parts, cnts[gloo].cpu())
            alls[gloo] = torch.stack(parts, 1).cuda()
            gloo.clear()
        torch.cuda.synchronize()

    def verify(k0, k1, kind):
        r = check_counts(kind + " (own)", cnts[k0:k1].cpu().numpy(), want)
        al = alls[k0:k1] if (H.comm is not None or world > 1) else cnts[k0:k1].unsqueeze(1)  # no exchange at N = 1
        if r is None:
            r = check_counts(kind + " (all-gathered)", al.sum(1).cpu().numpy(), glob)
        if r is None and not bool((al[:, rank] == want).all()):
            r = f"{kind}: all-gathered slot {rank} != own count {want}"
        if r is None and want > cap:
            r = f"{kind}: {want} rows exceed the output capacity {cap}"
        if r is None and not (bool((o0[:want] == c0[sel]).all()) and bool((o1[:want] == c1[sel]).all())
                              and bool((ids[:want] == torch.nonzero(sel).flatten() + s).all())):
            r = f"{kind}: positions / projected rows differ from torch"
        return r

    torch.cuda.synchronize()
    enqueue(0, 1)
    drain()
    H.agree(verify(0, 1, "C4 pre-check"))

    def reset():
        cnts.zero_(), alls.zero_(), o0.zero_(), o1.zero_(), ids.zero_()
        torch.cuda.synchronize()

    ms, _, G = H.timed(enqueue, drain, steps, warmup, args.graph_steps, reset=reset, verify=verify, label="C4")
    H.agree(verify(warmup, warmup + steps, "C4 timed steps"))
    kms, kmax = H.kernel_ms(lambda i: launch(0), max(1, args.kernel_graph))
    byts = 2 * ((n + 63) // 64) * 8 + want * (8 + 8)
    rec = config_record(
        "C4: 100M-row BitMapFile AND bm(c2=3) ^ bm(c3=7) -> positions + c0, c1 (one launch, column group), "
        "row-range sharded", N, n, world, glob, ms, "mbx::k_cnf_select", kms, kmax, byts,
        exchange_name(H, "RCCL all-gather of the per-rank counts (libmbx mbx_comm, after each query)"), "ok",
        timing_label(G, steps),
        algorithmic_bytes_global=2 * N // 8 + glob * 16)
    del c0, c1, c2, c3, t, bm2, bm3, a, b, ids, o0, o1, sel, conj
    torch.cuda.empty_cache()
    return rec


def c5_dictionary(torch):
    """50 ASCII names of <= 16 characters, zero padded."""
    names = [f"{chr(65 + (i * 7) % 26)}{'abcdefghijklmnop'[:(i % 15) + 1]}"[:16] for i in range(50)]
    dic = torch.zeros(50, 16, dtype=torch.uint8)
    for i, nm in enumerate(names):
        dic[i, :len(nm)] = torch.tensor(list(nm.encode()), dtype=torch.uint8)
    return dic.cuda()


def config_c5(H, args):
    """C5: 125M rows per GPU (1B over 8) of i32 / f32 / char(16),
    (c0 < 2^19) ^ (c1 >= 0.25) ^ (c2 >= "M") -> COUNT, SUM / MIN / MAX(c1) in
    one scan; at N > 1 the RCCL all-gather of the 48-byte records + the
    device rank-ordered fold (mbx_comm_allreduce_agg_async)."""
    torch, ctx, m, world, rank = H.torch, H.ctx, H.m, H.world, H.rank
    D = m.dist
    n = args.c5_rows
    N, s = n * world, n * rank
    g = torch.Generator(device="cuda")
    g.manual_seed(5 + 1000 * rank)
    c0 = torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g)
    c1 = torch.rand((n,), dtype=torch.float32, device="cuda", generator=g)
    dic = c5_dictionary(torch)
    c2 = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    chunk = 1 << 23  # one advanced-index launch per chunk (tests/helpers.device_dictionary_column)
    for a in range(0, n, chunk):
        idx = torch.randint(0, 50, (min(chunk, n - a),), dtype=torch.int64, device="cuda", generator=g)
        c2[a:a + chunk].copy_(dic[idx])
    t = ctx.wrap([(m.mbx.INTEGER, 4), (m.mbx.REAL, 4), (m.mbx.STRING, 16)],
                 [c0.data_ptr(), c1.data_ptr(), c2.data_ptr()], n, row_offset=s)
    cnf = [[(m.mbx.LT, ("sym", 1), ("int", 1 << 19))], [(m.mbx.GE, ("sym", 2), ("real", 0.25))],
           [(m.mbx.GE, ("sym", 3), ("str", "M"))]]
    plan = ctx.compile(t, cnf)
    sel = (c0 < (1 << 19)) & (c1 >= 0.25) & (c2[:, 0] >= ord("M"))
    want = dict(count=int(sel.sum().item()), sum=float(torch.where(sel, c1.double(), 0.0).sum().item()),
                min=float(torch.where(sel, c1, float("inf")).min().item()),
                max=float(torch.where(sel, c1, float("-inf")).max().item()))
    del sel
    gwant = D.combine_aggregate(want) if world > 1 else want
    W = D.AGG_WORDS
    steps, warmup = args.steps, args.warmup
    recs = torch.zeros(steps + warmup, W, dtype=torch.int64, device="cuda")
    gathered = torch.zeros(world, W, dtype=torch.int64, device="cuda")
    gloo = []

    def scan(k):
        ctx.scan_aggregate_async(plan, 1, recs[k].data_ptr())

    def enqueue(k0, k1):
        for k in range(k0, k1):
            scan(k)
            if H.comm is not None:  # all-gather + rank-ordered fold into recs[k], on the device
                H.comm.allreduce_agg_async(recs[k].data_ptr())
            elif H.torch_pg is not None:  # the same all-gather + the same device fold
                H.dist.all_gather_into_tensor(gathered.view(-1), recs[k], group=H.torch_pg)
                ctx.agg_fold_async(gathered.data_ptr(), world, recs[k].data_ptr())
            elif world > 1:
                gloo.append(k)

    def drain():
        ctx.sync()
        for k in gloo:  # rehearsal: gloo all-gather of the records, then the same device fold
            parts = [torch.empty(W, dtype=torch.int64) for _ in range(world)]
            H.dist.all_gather(parts, recs[k].cpu())
            gathered.copy_(torch.stack(parts))
            torch.cuda.synchronize()
            ctx.agg_fold_async(gathered.data_ptr(), world, recs[k].data_ptr())
            ctx.sync()
        gloo.clear()
        torch.cuda.synchronize()

    def verify(k0, k1, kind):
        h = recs[k0:k1].cpu().numpy()
        for k in range(h.shape[0]):
            r = check_aggregate(kind, D.fold_aggregates(h[k]), gwant)
            if r:
                return r
        return None

    # own record first (no exchange), then one exchanged step
    torch.cuda.synchronize()
    scan(0)
    ctx.sync()
    H.agree(check_aggregate("C5 pre-check (own shard)", D.fold_aggregates(recs[0].cpu().numpy()), want))
    recs.zero_()
    torch.cuda.synchronize()
    enqueue(0, 1)
    drain()
    H.agree(verify(0, 1, "C5 pre-check"))
    ms, _, G = H.timed(enqueue, drain, steps, warmup, args.graph_steps,
                       reset=lambda: (recs.zero_(), torch.cuda.synchronize()), verify=verify, label="C5")
    H.agree(verify(warmup, warmup + steps, "C5 timed steps"))
    kms, kmax = H.kernel_ms(lambda i: scan(0), max(1, args.kernel_graph))
    glob = D.fold_aggregates(recs[-1].cpu().numpy())
    rec = config_record(
        "C5: mixed int32 / float32 / char(16), (c0 < 2^19) ^ (c1 >= 0.25) ^ (c2 >= \"M\") -> COUNT, SUM / MIN / "
        "MAX(c1), 125M rows per GPU", N, n, world, glob["count"], ms, "mbx::k_scan_fast<aggregate>", kms, kmax,
        n * 24, exchange_name(H, "RCCL all-gather of the 48-byte records + device rank-ordered fold (libmbx)"), "ok",
        timing_label(G, steps),
        sum=glob["sum"], min=glob["min"], max=glob["max"])
    del c0, c1, c2, t, plan, recs
    torch.cuda.empty_cache()
    return rec


def bucketed_form(args, world, exchange):
    """The bucketed sub-records: only at N > 1 (the exchange is real), only
    when the headline itself keeps one collective per query and graphs of
    several steps are captured."""
    return world > 1 and exchange and args.exchange_bucket == 1 and args.graph_steps > 1 and not args.no_bucketed


def bucketed_record(r, rows, exchange="one RCCL all-reduce of the COUNT frames of every bucket_steps queries"):
    """value / step / phases of a run_c3 result whose COUNTs of every
    captured graph share one all-reduce (bucket_steps = graph steps)."""
    return {"bucket_steps": r["B"], "value": rows / (r["ms_step"] * 1e-3), "unit": "rows/s",
            "ms_per_step": r["ms_step"], "graph_steps": r["G"],
            "phases_us": {"step_wall": r["ms_step"] * 1e3, "scan_kernel_max_over_ranks": r["kern_max"] * 1e3,
                          "exchange_and_overlap": max(0.0, (r["ms_step"] - r["kern_max"]) * 1e3)},
            "exchange": exchange}


def main():
    args = make_parser().parse_args()
    if args.gpus < 1:
        print(f"bench: --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)

    configs = [c.strip().upper() for c in args.configs.split(",") if c.strip() and c.strip().lower() != "none"]
    bad = [c for c in configs if c not in ("C2", "C4", "C5")]
    if bad:
        print(f"bench: unknown config(s) {bad}", file=sys.stderr)
        sys.exit(2)
    worker = os.environ.get("MBX_BENCH_WORKER") == "1"
    if worker:
        die_with_parent()
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    elif not worker and not args.dry_launch:
        sys.exit(supervise_rank(sys.argv[1:]))  # under torch.distributed.run

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_launch:
        env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
        print(json.dumps({"rank": rank, "local_rank": local_rank, "world": world, "gpus": args.gpus,
                          "torch_imported": "torch" in sys.modules, "env": env}), flush=True)
        return
    if os.environ.get("MBX_BENCH_FAKE"):
        fake_worker(args, world, rank)
        return
    fallback = os.environ.get("MBX_BENCH_FALLBACK")
    host_reason = os.environ.get("MBX_BENCH_HOST_EXCHANGE")
    out_fd = quiet_stdout()

    import torch
    import torch.distributed as dist

    import mbx_pkg

    global CLOCK
    if args.watchdog > 0:  # armed after the imports (a cold box's first `import torch` takes minutes)
        import faulthandler
        faulthandler.dump_traceback_later(args.watchdog, exit=True)
        CLOCK = PhaseClock()
    arm("setup: process group, context", PHASE_S["setup"])

    same_device = os.environ.get("MBX_BENCH_SAME_DEVICE") == "1"
    host_xchg = same_device or bool(host_reason)  # the exchange as gloo over host copies
    device = 0 if same_device else local_rank
    torch.cuda.set_device(device)
    # MBX_BENCH_TORCH_EXCHANGE=1 (rehearsal): the fallback exchange
    # (torch.distributed's RCCL group) even where libmbx's communicator works;
    # at N = 1 over a one-rank group
    torch_exchange = os.environ.get("MBX_BENCH_TORCH_EXCHANGE") == "1"
    exchange = world > 1 or os.environ.get("MBX_BENCH_FORCE_EXCHANGE") == "1" or torch_exchange
    if world > 1:
        # host-side bootstrap, barriers, verdicts and the max-over-ranks clock
        # only: the data-path exchange is libmbx's own RCCL communicator
        dist.init_process_group("gloo")
    elif torch_exchange or (exchange and host_xchg):  # a one-rank group for the rehearsals' exchange at N = 1
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1)
    m = mbx_pkg.load()
    ctx = m.Context(device)

    comm = None
    torch_pg = None  # fallback exchange: torch.distributed's own RCCL group (eager)
    reason = None
    if exchange and not host_xchg:
        # the RCCL exchange's setup: a hang or an error here is COMM_EXIT (the
        # launcher's host-exchange fallback), as is MBX_BENCH_FORCE_COMM_FAIL=1
        # on rank 0 (rehearsal)
        arm("communicators: RCCL clique", PHASE_S["comm"], COMM_EXIT)
        if os.environ.get("MBX_BENCH_FORCE_COMM_FAIL") == "1" and rank == 0:
            fail_exit(COMM_EXIT, "communicators: forced failure (MBX_BENCH_FORCE_COMM_FAIL)")
        uid = m.mbx.comm_unique_id() if rank == 0 else None
        if world > 1:
            box = [uid]
            dist.broadcast_object_list(box, src=0)
            uid = box[0]
        try:
            if torch_exchange:
                raise m.MbxError(m.mbx.E_INVALID, "MBX_BENCH_TORCH_EXCHANGE=1")
            comm = ctx.comm_init_rank(world, rank, uid)
        except m.MbxError as err:
            reason = f"libmbx RCCL communicator failed ({err})"
            print(f"rank {rank}: {reason}", file=sys.stderr)
        if world > 1 or torch_exchange:
            # every rank takes the same exchange: libmbx's communicator if it
            # came up everywhere, else torch.distributed's RCCL group
            flag = torch.tensor([int(comm is not None)], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if int(flag[0]) == 0:
                if comm is not None:
                    comm.close()
                    comm = None
                try:
                    torch_pg = dist.new_group(backend="nccl")
                except Exception as err:  # neither RCCL form came up
                    fail_exit(COMM_EXIT, f"communicators: libmbx ({reason or 'peer failed'}) and torch.distributed "
                                         f"nccl ({type(err).__name__}: {err}) both failed")
                reason = None
                print(f"rank {rank}: exchange falls back to torch.distributed (nccl = RCCL)", file=sys.stderr)
    H = Harness(torch, dist, m, ctx, world, rank, comm, same_device, exchange, torch_pg)
    H.host_reason = host_reason
    H.agree(reason, COMM_EXIT)
    arm("setup: tables", PHASE_S["setup"])

    # ---- headline: C3 ------------------------------------------------------
    if args.scaling == "strong":
        n_global = args.rows
        s, e = m.mbx.shard_bounds(args.rows, world, rank)
        cols = make_columns(torch, args.rows, s, e, 42)
        glob = full_count(torch, n_global, 42) if exchange else None
    else:
        n_global = args.rows * world
        s, e = rank * args.rows, (rank + 1) * args.rows
        cols = make_columns(torch, args.rows, 0, args.rows, 42 + 1000 * rank)
        glob = None
    n = e - s
    if glob is None and exchange:  # weak: the sum of every rank's own torch count
        glob = H.rsum(int(((cols[0] < THRESH) & (cols[1] >= THRESH)).sum().item()))
    r3 = run_c3(H, args, cols, n, s, glob, "C3")
    arm("read probe", PHASE_S["probe"])
    probe = read_probe(H, r3["table"]) if rank == 0 else None
    # the CPU baseline scans THIS table (the GPU run's arrays): one
    # device -> host copy of the 4 columns, outside every timed region
    host_cols = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host_cols = [c.cpu().numpy() for c in cols]
    r3["table"].close()
    r3["plan"].close()
    # at N > 1 with one collective per query (the headline, SURVEY 8(e)'s
    # per-query t_reduce), the same steps again with the COUNTs of each
    # captured graph's steps sharing ONE all-reduce: the throughput form for a
    # stream of queries (xGMI collectives cost their latency, not their bytes)
    bucketed = None
    if bucketed_form(args, world, exchange):
        rb = run_c3(H, args, cols, n, s, glob, "C3 bucketed", bucket=args.graph_steps)
        rb["table"].close()
        rb["plan"].close()
        bucketed = bucketed_record(rb, n_global, exchange_name(
            H, "one RCCL all-reduce of the COUNT frames of every bucket_steps queries (libmbx mbx_comm)"))
    del cols
    torch.cuda.empty_cache()

    # ---- strong sub-record at N > 1: the metric's ONE 100M-row table ----------
    strong = None
    if world > 1 and args.scaling == "weak" and not args.no_strong:
        ss, se = m.mbx.shard_bounds(args.rows, world, rank)
        scols = make_columns(torch, args.rows, ss, se, 42)
        sglob = full_count(torch, args.rows, 42)
        rs = run_c3(H, args, scols, se - ss, ss, sglob, "C3 strong")
        rs["table"].close()
        rs["plan"].close()
        sb = None
        if bucketed_form(args, world, exchange):
            rsb = run_c3(H, args, scols, se - ss, ss, sglob, "C3 strong bucketed", bucket=args.graph_steps)
            rsb["table"].close()
            rsb["plan"].close()
            sb = bucketed_record(rsb, args.rows, exchange_name(
                H, "one RCCL all-reduce of the COUNT frames of every bucket_steps queries (libmbx mbx_comm)"))
        del scols
        torch.cuda.empty_cache()
        strong = {"rows": args.rows, "rows_per_gpu_rank0": se - ss if rank == 0 else None,
                  "value": args.rows / (rs["ms_step"] * 1e-3), "unit": "rows/s", "ms_per_step": rs["ms_step"],
                  "phases_us": {"step_wall": rs["ms_step"] * 1e3, "scan_kernel_max_over_ranks": rs["kern_max"] * 1e3,
                                "exchange_and_overlap": max(0.0, (rs["ms_step"] - rs["kern_max"]) * 1e3)},
                  "count": "frame" if rs["frames"] else "finalize", "graph_steps": rs["G"], "pre_check": "ok",
                  "bucketed": sb}
        if rank == 0:
            strong["rows_per_gpu_rank0"] = se - ss

    # ---- the other BASELINE configs ------------------------------------------
    crecs = {}
    for name in configs:
        arm(f"config {name}", PHASE_S["config"])
        if name == "C2":
            if rank == 0:
                crecs["C2"] = config_c2(H.solo(), args)
            H.barrier()
        elif name == "C4":
            crecs["C4"] = config_c4(H, args)
        elif name == "C5":
            crecs["C5"] = config_c5(H, args)

    if rank == 0:
        steps = args.steps
        ms_per_step = r3["ms_step"]
        kern_ms, kern_max, frames = r3["kern_ms"], r3["kern_max"], r3["frames"]
        algo_bytes = 2 * 4 * n  # c0 + c1 read once per launch (rank 0's shard)
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        B = r3["B"]
        xchg = ((f"RCCL all-reduce of the COUNTs of every {B} steps (libmbx mbx_comm, after the scans)" if B > 1
                 else "RCCL all-reduce of every step's COUNT (one collective per query; libmbx mbx_comm, right "
                      "after the step's scan on the same stream)")
                if comm is not None else None) or (
            "torch.distributed RCCL all-reduce per step (fallback: libmbx's communicator failed), eager"
            if torch_pg is not None else None) or (
            (f"gloo all-reduce over host copies (fallback: the RCCL exchange failed: {host_reason})" if host_reason
             else "gloo all-reduce (same-device rehearsal)") if exchange else "none")
        out = {
            "metric": METRIC,
            "value": n_global * steps / (ms_per_step * 1e-3 * steps),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
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
                "graph_steps": r3["G"],
                "exchange_bucket_steps": B if exchange else None,
                "count": "frame (32 packed slots per query, summed by the all-reduce; mbx_scan_count_frame_async)"
                         if frames else "in-launch finalize (mbx_scan_count_async)",
            },
            "pre_check": "ok: one exchanged step verified on every rank before timing" if exchange else
                         "ok: one step verified before timing",
            "exchange_form": exchange_form(r3["G"], fallback, host_reason),
            "phases_us": {
                "step_wall": ms_per_step * 1e3,
                "scan_kernel_max_over_ranks": kern_max * 1e3,
                "host_enqueue_rank0": r3["enq_us"],
                "exchange_and_overlap": max(0.0, ms_per_step * 1e3 - kern_max * 1e3),
            },
            "hbm_gbs": 2 * 4 * n_global / (ms_per_step * 1e-3) / 1e9,
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
                "kernel_timing": f"one HIP graph of {max(1, args.kernel_graph)} scans replayed 3 times, HIP events "
                                 "on the library stream / launches",
                "algorithmic_bytes_per_launch": algo_bytes,
                # secondary denominator: the best read rate of the
                # scan's own load pattern with the predicate removed
                "measured_read_peak": probe["best_gbs"],
                "frac_of_measured_read_peak": achieved / probe["best_gbs"],
                "read_probe": probe,
            },
            "bucketed": bucketed,
            "strong": strong,
            "configs": crecs,
            "cpu_baseline": None,
        }
        if host_cols is not None:
            # rank 0 at N = 1 only, after the timed regions (at N > 1 the
            # line carries null: the baseline is the single-GPU comparison)
            arm("cpu baseline", PHASE_S["cpu"])
            out["cpu_baseline"] = cpu_baseline(host_cols, r3["want"], args.cpu_seconds)
        os.write(out_fd, (json.dumps(out) + "\n").encode())

    arm("teardown", 60)
    ctx.close()
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
