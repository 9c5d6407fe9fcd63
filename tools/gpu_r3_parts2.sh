# round 3: the 12.5M-row shard with a per-query exchange, HIP graphs vs eager,
# the scan's own finalize + all-reduce (MBX_BENCH_PARTS=0) vs the per-block
# counts summed on the exchange stream (mbx_comm_scan_count_async)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_parts2}
mkdir -p $OUT
for cfg in "0 10" "1 10" "0 0" "1 0" "0 10" "1 0"; do
  set -- $cfg
  MBX_BENCH_PARTS=$1 MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python3 bench.py --rows 12500000 --steps 200 --warmup 20 --exchange-bucket 1 --graph-steps $2 --no-cpu-baseline > $OUT/shard_p$1_g$2.json 2> $OUT/shard_p$1_g$2.err || { echo SHARD_FAIL; tail -20 $OUT/shard_p$1_g$2.err; exit 1; }
  cat $OUT/shard_p$1_g$2.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('parts', $1, 'graph', $2, round(d['ms_per_step'] * 1e3, 2), d['phases_us'])"
done
echo PARTS2_OK
