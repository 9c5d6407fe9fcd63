"""bench.py's own N-rank launcher (no GPU): with WORLD_SIZE unset, --gpus N
starts N rank processes with the rank env torch.distributed.run would give
them (one process per GPU, row-range shards), before any GPU
call; under an external launcher WORLD_SIZE must equal --gpus."""
import json
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
