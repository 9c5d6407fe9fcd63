# Round 3: branch-free int terms in every fast-scan mode + k_scan_select -- GPU tests, then the C3
# bench and the 12.5M-row shard with the knob on / off, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_ir2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_int_range.py tests/test_scan_select_fused.py tests/test_gpu_parity.py tests/test_nan_order.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for ir in 1 0; do
    MBX_SCAN_INT_RANGE=$ir timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/full_ir$ir.$r.json 2> $OUT/full_ir$ir.$r.err || { echo FULL_FAIL; tail -20 $OUT/full_ir$ir.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/full_ir$ir.$r.json')); print('full ir=$ir', $r, round(d['phases_us']['step_wall'],2), round(d['roofline']['kernel_ms']*1e3,2), round(d['roofline']['measured_read_peak']))"
    MBX_SCAN_INT_RANGE=$ir MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python3 bench.py --rows 12500000 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/shard_ir$ir.$r.json 2> $OUT/shard_ir$ir.$r.err || { echo SHARD_FAIL; tail -20 $OUT/shard_ir$ir.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/shard_ir$ir.$r.json')); print('shard ir=$ir', $r, round(d['phases_us']['step_wall'],2), round(d['roofline']['kernel_ms']*1e3,2))"
  done
done
for r in 1 2; do
  for ir in 1 0; do
    MBX_SCAN_INT_RANGE=$ir timeout -k 10 300 python3 tools/bench_configs.py --configs C2 > $OUT/c2_ir$ir.$r.jsonl 2> $OUT/c2_ir$ir.$r.err || { echo C2_FAIL; tail -20 $OUT/c2_ir$ir.$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c2_ir$ir.$r.jsonl').readline()); print('C2 ir=$ir', $r, round(d['ms_per_query']*1e3,2), round(d['scan_bitmap_ms']*1e3,2))"
  done
done
echo IR_OK
