# Round 3: count frames (mbx_scan_count_frame_async) -- GPU tests, then the
# 12.5M-row shard with a per-query exchange, frame vs in-launch finalize,
# interleaved, and the full 100M-row table -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_frame}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_count_frame.py tests/test_comm.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for cnt in frame finalize; do
    MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python3 bench.py --rows 12500000 --steps 200 --warmup 20 --count $cnt --no-cpu-baseline > $OUT/shard_$cnt.$r.json 2> $OUT/shard_$cnt.$r.err || { echo SHARD_FAIL; tail -20 $OUT/shard_$cnt.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/shard_$cnt.$r.json')); print('$cnt', $r, round(d['phases_us']['step_wall'],2), round(d['phases_us']['scan_kernel_max_over_ranks'],2))"
  done
done
for cnt in frame finalize; do
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --count $cnt --no-cpu-baseline > $OUT/full_$cnt.json 2> $OUT/full_$cnt.err || { echo FULL_FAIL; tail -20 $OUT/full_$cnt.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/full_$cnt.json')); print('full $cnt', round(d['phases_us']['step_wall'],2), round(d['phases_us']['scan_kernel_max_over_ranks'],2))"
done
echo FRAME_OK
