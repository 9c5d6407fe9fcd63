# round 3: mbx_comm_scan_count_async (the scan's per-block counts summed and
# all-reduced on the exchange stream) -- tests, and the 12.5M-row shard step
# with a per-query exchange (bucket 1: the new path; bucket 10: the old one)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_parts}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_comm.py tests/test_nan_order.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 1 10 1; do
  MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python3 bench.py --rows 12500000 --steps 200 --warmup 20 --exchange-bucket $b --no-cpu-baseline > $OUT/shard_12m5_bucket$b.json 2> $OUT/shard_12m5_bucket$b.err || { echo SHARD_FAIL; tail -20 $OUT/shard_12m5_bucket$b.err; exit 1; }
  cat $OUT/shard_12m5_bucket$b.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('bucket', $b, d['ms_per_step'] * 1e3, d['phases_us'])"
done
echo PARTS_OK
