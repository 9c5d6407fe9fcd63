"""bench.py's own N-rank launcher (no GPU): with WORLD_SIZE unset, --gpus N
starts N rank processes with the rank env torch.distributed.run would give
them (one process per GPU, row-range shards), before any GPU
call; under an external launcher WORLD_SIZE must equal --gpus."""
import json
import time
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run_bench(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_launcher_hands_each_rank_its_env(n):
    r = run_bench(["--gpus", str(n), "--dry-launch", "--steps", "3"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.strip()]
    assert sorted(x["rank"] for x in lines) == list(range(n))
    ports = {x["env"]["MASTER_PORT"] for x in lines}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for x in lines:
        assert x["world"] == n and x["gpus"] == n
        assert x["local_rank"] == x["rank"]
        assert x["env"]["MASTER_ADDR"] == "127.0.0.1"
        assert x["env"]["WORLD_SIZE"] == str(n)
        assert not x["torch_imported"], "a rank imported torch before its env was checked"


def test_single_gpu_runs_in_process():
    r = run_bench(["--gpus", "1", "--dry-launch"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1 and lines[0]["world"] == 1 and lines[0]["env"]["WORLD_SIZE"] is None


def test_world_size_mismatch_exits_nonzero():
    r = run_bench(["--gpus", "4", "--dry-launch"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and not r.stdout.strip()


def test_external_launcher_matching_world_size():
    r = run_bench(["--gpus", "2", "--dry-launch"], {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"})
    assert r.returncode == 0, r.stderr
    x = json.loads(r.stdout)
    assert x["rank"] == 1 and x["world"] == 2


def test_bad_gpu_count():
    assert run_bench(["--gpus", "0", "--dry-launch"]).returncode != 0


def test_failing_rank_fails_the_launch():
    """A rank that dies makes the launcher exit non-zero (and stops the rest):
    an unparsable option fails every rank the same way."""
    r = run_bench(["--gpus", "2", "--dry-launch", "--scaling", "sideways"])
    assert r.returncode != 0


def test_count_frame_fits():
    """The frame exchange's exactness bound: nranks x ceil(blocks
    / 32) summed arrivals per 12-bit slot field must stay below 4096."""
    sys.path.insert(0, ROOT)
    import mbx_pkg
    m = mbx_pkg.load().mbx
    assert m.count_frame_fits(32 * 255, 16)          # 255 per slot x 16 ranks = 4080
    assert not m.count_frame_fits(32 * 256, 1)       # one rank past its slot bound
    assert not m.count_frame_fits(32 * 255, 17)      # 4335 arrivals: would carry into the NaN bits
    assert m.count_frame_fits(32 * 127, 32) and not m.count_frame_fits(32 * 128, 32)
    assert not m.count_frame_fits(10, 0)


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


def test_default_run_adds_every_config_record():
    """The driver's plain `bench.py --gpus N` measures C2, C4 and C5 beside
    the C3 headline, and every record carries CONFIG_KEYS
    with kernel time from graph replay."""
    b = _bench_module()
    a = b.make_parser().parse_args([])
    assert sorted(a.configs.split(",")) == ["C2", "C4", "C5"] and a.scaling == "weak" and not a.no_strong
    assert a.c4_rows == 100_000_000 and a.c5_rows == 125_000_000 and a.kernel_graph >= 10
    rec = b.config_record("C4", 100_000_000, 50_000_000, 2, 1_000_000, 0.040, "k", 0.030, 0.031, 33_000_000,
                          "RCCL", "ok", "graph replay")
    assert set(b.CONFIG_KEYS) <= set(rec)
    assert abs(rec["achieved_gbs"] - 1100.0) < 1e-6 and abs(rec["frac"] - 1100.0 / 8000.0) < 1e-12
    assert abs(rec["rows_per_s"] - 100_000_000 / 40e-6) < 1
    # PMC traffic of the profiled shard sizes (profiles/config_pmc.json)
    assert rec["traffic"] is None
    for name, rows in (("C2", 10_000_000), ("C4", 100_000_000), ("C5", 125_000_000)):
        t = b.load_config_traffic(name, rows)
        assert t and t > 0, name
        r = b.config_record(f"{name}: x", rows, rows, 1, 1, 1.0, "k", 0.5, 0.5, 1000, "none", "ok", "g")
        assert r["traffic"] == t and r["traffic_over_algorithmic"] == t / 1000


def test_watchdog_names_a_hang_and_exits():
    """A rank still running after --watchdog seconds prints every thread's
    traceback and exits 1 (faulthandler), so a hung collective at N > 1 fails
    inside the driver's budget with its place named."""
    b = _bench_module()
    assert 0 < b.make_parser().parse_args([]).watchdog < 600
    code = ("import faulthandler, time; faulthandler.dump_traceback_later(0.5, exit=True); "
            "time.sleep(30)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and ("sleep" in r.stderr or "Thread" in r.stderr), r.stderr


def test_bucketed_sub_records_only_beside_a_per_query_headline():
    """At N > 1 the line adds `bucketed` (and strong.bucketed): the same steps
    with each captured graph's COUNTs in one all-reduce; never at N = 1, never
    when the headline is bucketed itself, and --no-bucketed turns it off."""
    b = _bench_module()
    p = b.make_parser()
    a = p.parse_args([])
    assert a.exchange_bucket == 1 and a.graph_steps > 1
    assert b.bucketed_form(a, 2, True) and b.bucketed_form(a, 8, True)
    assert not b.bucketed_form(a, 1, False) and not b.bucketed_form(a, 1, True)
    assert not b.bucketed_form(p.parse_args(["--exchange-bucket", "20"]), 8, True)
    assert not b.bucketed_form(p.parse_args(["--graph-steps", "0"]), 8, True)
    assert not b.bucketed_form(p.parse_args(["--no-bucketed"]), 8, True)
    r = b.bucketed_record(dict(B=20, ms_step=0.125, kern_max=0.118, G=20), 800_000_000)
    assert r["bucket_steps"] == 20 and abs(r["value"] - 800_000_000 / 125e-6) < 1
    assert abs(r["phases_us"]["exchange_and_overlap"] - 7.0) < 1e-9


def _frame(count, arrivals, nan=0, slots=32):
    import numpy as np
    f = np.zeros(512, dtype=np.int64)
    for i in range(slots):  # spread over the slots like blockIdx % 32
        c = count // slots + (1 if i < count % slots else 0)
        a = arrivals // slots + (1 if i < arrivals % slots else 0)
        f[16 * i] = (c << 24) | ((nan if i == 0 else 0) << 12) | a
    return f


def test_precheck_fires_on_a_wrong_frame_or_count():
    """bench.py's pre-check (one exchanged step, verified before timing):
    exact frames pass; a missing / duplicated block arrival, a NaN block or
    a wrong global COUNT each give a one-line reason."""
    import numpy as np
    b = _bench_module()
    nb = 2 * 1000  # two ranks x 1000 blocks
    good = np.stack([_frame(12_345_678, nb), _frame(12_345_678, nb)])
    assert b.check_counts("C3", None, 12_345_678, frames=good, nblocks=nb) is None
    c, nan, arr = b.frame_fields(good)
    assert c.tolist() == [12_345_678] * 2 and arr.tolist() == [nb] * 2 and nan.tolist() == [0, 0]
    late = good.copy()
    late[1, 16 * 5] -= 1                                      # one block of step 1 never arrived
    assert "arrivals" in b.check_counts("C3", None, 12_345_678, frames=late, nblocks=nb)
    dup = good.copy()
    dup[0, 0] += 1                                            # MBX_BENCH_CORRUPT=frame
    assert "arrivals" in b.check_counts("C3", None, 12_345_678, frames=dup, nblocks=nb)
    wrong = good.copy()
    wrong[0, 0] += 1 << 24                                    # MBX_BENCH_CORRUPT=count
    assert "COUNT" in b.check_counts("C3", None, 12_345_678, frames=wrong, nblocks=nb)
    nanf = np.stack([_frame(5, nb, nan=1)])
    assert "NaN" in b.check_counts("C3", None, 5, frames=nanf, nblocks=nb)
    assert b.check_counts("C3", [7, 7, 7], 7) is None
    assert "COUNT" in b.check_counts("C3", [7, 8, 7], 7)


def test_aggregate_check_tolerances():
    b = _bench_module()
    want = dict(count=10, sum=1.0e6, min=0.25, max=0.99)
    assert b.check_aggregate("C5", dict(want, sum=1.0e6 * (1 + 5e-7)), want) is None
    assert "sum" in b.check_aggregate("C5", dict(want, sum=1.0e6 * (1 + 2e-6)), want)
    assert "count" in b.check_aggregate("C5", dict(want, count=11), want)
    assert "min" in b.check_aggregate("C5", dict(want, min=0.2500001), want)


AGREE = """
import os, sys
sys.path.insert(0, {root!r})
import torch, torch.distributed as dist
import bench
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
bad = os.environ.get("BAD_RANK")
bench.agree(torch, dist, world, rank, "C3 pre-check: frame arrivals [2047] != 2046" if bad == str(rank) else None)
print("passed", rank, flush=True)
dist.destroy_process_group()
"""


@pytest.mark.parametrize("bad_rank", [None, "0", "1"])
def test_precheck_verdict_is_collective(bad_rank):
    """gloo world 2 (the bench's host-side group): a pre-check failure on ANY
    rank makes every rank exit 3 before timing -- the failing rank with its
    one-line reason, the other naming the cause -- and no failure lets both
    go on"""
    port = free_port_local()
    procs = []
    for r in range(2):
        env = {k: v for k, v in os.environ.items() if k not in ("BAD_RANK",)}
        env.update(RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if bad_rank is not None:
            env["BAD_RANK"] = bad_rank
        procs.append(subprocess.Popen([sys.executable, "-c", AGREE.format(root=ROOT)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    for r, (p, (out, err)) in enumerate(zip(procs, outs)):
        if bad_rank is None:
            assert p.returncode == 0 and f"passed {r}" in out, err
        else:
            assert p.returncode == 3 and "passed" not in out, (r, err)
            if str(r) == bad_rank:
                assert f"pre-check failed on rank {r}: C3 pre-check: frame arrivals" in err
            else:
                assert "another rank's pre-check failed" in err


def free_port_local():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_unknown_config_exits_before_any_gpu_work():
    r = run_bench(["--configs", "C2,C9"])
    assert r.returncode == 2 and "C9" in r.stderr and not r.stdout.strip()


# ---- graph-phase fallback: fake workers, no GPU --------

def _line(stdout):
    lines = [json.loads(x) for x in stdout.splitlines() if x.strip().startswith("{")]
    assert len(lines) == 1, stdout
    return lines[0]


def test_local_launcher_relaunches_eager_after_a_graph_phase_failure():
    """rank 1's first attempt exits GRAPH_EXIT (its graph replay 'hung'), rank
    0 waits as if inside a collective: the launcher stops it, starts fresh
    ranks once with --graph-steps 0 and relays their line, marked"""
    t0 = time.time()
    r = run_bench(["--gpus", "2"], {"MBX_BENCH_FAKE": "graph:1"})
    assert r.returncode == 0, r.stderr
    x = _line(r.stdout)
    assert x["graph_steps"] == 0 and x["n_gpus"] == 2
    assert x["exchange_form"].startswith("eager (graph replay failed: rank 1: C3: first replay"), x
    assert "fresh ranks, eager steps" in r.stderr
    assert time.time() - t0 < 50  # rank 0 was stopped, not waited for


def test_local_launcher_without_failure_keeps_graphs():
    r = run_bench(["--gpus", "4"], {"MBX_BENCH_FAKE": "ok"})
    assert r.returncode == 0, r.stderr
    x = _line(r.stdout)
    assert x["graph_steps"] == 20 and x["exchange_form"].startswith("HIP graphs of 20 steps")


def test_other_failures_are_not_retried():
    r = run_bench(["--gpus", "2"], {"MBX_BENCH_FAKE": "fail:1"})
    assert r.returncode == 7 and not r.stdout.strip()
    assert "fresh ranks" not in r.stderr


def _torchrun(n, env_extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port_local()), BENCH, "--gpus", str(n)]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("bad", ["0", "1"])
def test_torchrun_supervisors_relaunch_eager_after_a_graph_phase_failure(bad):
    """the driver's N > 1 form (python -m torch.distributed.run ... bench.py
    --gpus N): each rank process supervises one worker; a graph-phase failure
    on any rank gives one eager relaunch on every rank and one line"""
    r = _torchrun(2, {"MBX_BENCH_FAKE": f"graph:{bad}"})
    assert r.returncode == 0, r.stderr[-3000:]
    x = _line(r.stdout)
    assert x["graph_steps"] == 0 and x["n_gpus"] == 2
    assert x["exchange_form"].startswith(f"eager (graph replay failed: rank {bad}: C3"), x


def test_torchrun_supervisors_pass_through_success_and_failure():
    r = _torchrun(2, {"MBX_BENCH_FAKE": "ok"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert _line(r.stdout)["graph_steps"] == 20
    r = _torchrun(2, {"MBX_BENCH_FAKE": "fail:1"})
    assert r.returncode != 0 and not r.stdout.strip()


def test_phase_clock_exits_with_the_phase_code():
    """PhaseClock: a phase that outlives its budget prints its name and every
    thread's traceback and exits with the phase's code (GRAPH_EXIT for a
    graph replay, after writing its reason to $MBX_BENCH_STATUS)"""
    import tempfile
    status = os.path.join(tempfile.mkdtemp(), "s.txt")
    code = (f"import sys, time; sys.path.insert(0, {ROOT!r}); import bench; c = bench.PhaseClock(); "
            "c.arm('C3: first replay of 1 captured graph(s)', 0.3, bench.GRAPH_EXIT); time.sleep(30)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, MBX_BENCH_STATUS=status))
    assert r.returncode == 4 and "outlived its budget" in r.stderr and "Thread" in r.stderr, r.stderr
    with open(status) as f:
        assert f.read().startswith("C3: first replay of 1 captured graph(s): did not finish")
    b = _bench_module()
    assert b.GRAPH_WAIT_S <= 60 and sum(b.PHASE_S.values()) < 1000


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGKILL"])
def test_workers_die_with_their_launcher(sig):
    """a launcher stopped from outside (the driver's clock, torch.distributed.run
    tearing a failed group down) leaves no rank behind: SIGTERM is forwarded and
    every worker carries PR_SET_PDEATHSIG"""
    import signal
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MBX_BENCH_FAKE"] = "fail:9"  # no rank fails: every rank waits 60 s
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2"], env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    time.sleep(3)
    kids = subprocess.run(["pgrep", "-P", str(p.pid)], capture_output=True, text=True).stdout.split()
    assert len(kids) == 2, kids
    p.send_signal(getattr(signal, sig))
    p.wait(timeout=30)
    time.sleep(1)
    for k in kids:
        assert not os.path.exists(f"/proc/{k}") or open(f"/proc/{k}/stat").read().split()[2] == "Z", k


@pytest.mark.parametrize("launch", ["local", "torchrun"])
def test_exchange_failure_falls_back_to_the_host_exchange(launch):
    """an RCCL exchange that does not come up (COMM_EXIT) -> fresh ranks with
    the exchange as a gloo collective over host copies, marked in the line"""
    env = {"MBX_BENCH_FAKE": "comm:1"}
    r = run_bench(["--gpus", "2"], env) if launch == "local" else _torchrun(2, env)
    assert r.returncode == 0, r.stderr[-3000:]
    x = _line(r.stdout)
    assert x["graph_steps"] == 20  # the graph form is kept: only the exchange changed
    assert x["exchange_form"].startswith("host gloo exchange of the device results, eager (RCCL exchange failed: "
                                         "rank 1: communicators: ncclCommInitRank"), x


@pytest.mark.parametrize("launch", ["local", "torchrun"])
def test_both_fallbacks_in_turn(launch):
    """graph replay fails first (eager relaunch), then the exchange itself
    (host relaunch): three attempts, one line naming both"""
    env = {"MBX_BENCH_FAKE": "graph+comm:0"}
    r = run_bench(["--gpus", "2"], env) if launch == "local" else _torchrun(2, env)
    assert r.returncode == 0, r.stderr[-3000:]
    x = _line(r.stdout)
    assert x["graph_steps"] == 0
    assert "RCCL exchange failed: rank 0: communicators" in x["exchange_form"]
    assert "earlier, graph replay failed: rank 0: C3" in x["exchange_form"]


def test_a_fallback_is_taken_once():
    b = _bench_module()
    codes = [(0, b.COMM_EXIT, "communicators: x"), (1, b.KILLED, "")]
    argv, env = b.next_attempt(codes, ["--gpus", "2"], {}, None)
    assert env["MBX_BENCH_HOST_EXCHANGE"] == "rank 0: communicators: x" and argv == ["--gpus", "2"]
    assert b.next_attempt(codes, argv, env, None) is None            # the same failure again: final
    assert b.final_status(codes) == b.COMM_EXIT
    g = [(0, b.KILLED, ""), (1, b.GRAPH_EXIT, "another rank's first graph replay failed"),
         (2, b.GRAPH_EXIT, "C4 first graph replay: x")]
    argv2, env2 = b.next_attempt(g, argv, env, None)
    assert argv2[-2:] == ["--graph-steps", "0"] and env2["MBX_BENCH_FALLBACK"] == "rank 2: C4 first graph replay: x"
    assert b.next_attempt([(0, 7, ""), (1, b.KILLED, "")], argv, {}, None) is None
    assert b.final_status([(0, 0, ""), (1, 0, "")]) == 0


def test_every_shard_size_has_request_split_traffic():
    """roofline.traffic at every N the driver runs (C3 shard of rank 0, its
    COUNT form) and every config record's traffic come from rocprofv3 passes
    with gfx950's read-request size split (profiles/r06/e, profiles/r06/final)"""
    b = _bench_module()
    sys.path.insert(0, ROOT)
    import mbx_pkg
    m = mbx_pkg.load().mbx
    with open(os.path.join(ROOT, "profiles", "c3_scan_pmc.json")) as f:
        shards = json.load(f)["shards"]
    for n in (1, 2, 4, 8):
        s, e = m.shard_bounds(100_000_000, n, 0)
        mode = "finalize" if n == 1 else "frame"
        key = f"{e - s}:{mode}"
        assert b.load_traffic(e - s, mode) and "request-size split" in shards[key]["correction"], key
        assert abs(shards[key]["traffic_over_algorithmic"] - 1) < 0.002, key
    assert "request-size split" in shards["100000000:frame"]["correction"]  # weak N > 1
    with open(os.path.join(ROOT, "profiles", "config_pmc.json")) as f:
        cfg = json.load(f)["configs"]
    for key in ("C2:10000000", "C4:100000000", "C5:125000000"):
        assert cfg[key]["read_basis"] == "request split", key
