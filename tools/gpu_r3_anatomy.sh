# round 3 anatomy: C2 / C4 kernel traces (kernel time vs inter-kernel gap),
# the 12.5M-row shard step with a per-query exchange (bucket 1) and bucketed
# (bucket 10), the full bench line -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_anatomy}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c2 -o c2 --output-format csv -- python3 tools/bench_configs.py --configs C2 > $OUT/c2.jsonl 2> $OUT/c2.err || { echo KT_C2_FAIL; tail -20 $OUT/c2.err; exit 1; }
find $OUT/kt_c2 -name '*kernel_trace.csv' -exec cp {} $OUT/c2_kernel_trace.csv \;
find $OUT/kt_c2 -name '*kernel_stats.csv' -exec cp {} $OUT/c2_kernel_stats.csv \;
python3 tools/trace_gaps.py $OUT/c2_kernel_trace.csv --seq k_scan_fast,k_select_ids --json $OUT/c2_gaps.json > /dev/null
cat $OUT/c2.jsonl $OUT/c2_gaps.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_c4 -o c4 --output-format csv -- python3 tools/bench_configs.py --configs C4 > $OUT/c4.jsonl 2> $OUT/c4.err || { echo KT_C4_FAIL; tail -20 $OUT/c4.err; exit 1; }
find $OUT/kt_c4 -name '*kernel_stats.csv' -exec cp {} $OUT/c4_kernel_stats.csv \;
cat $OUT/c4.jsonl
for b in 1 10; do
  MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python3 bench.py --rows 12500000 --steps 200 --warmup 20 --exchange-bucket $b --no-cpu-baseline > $OUT/shard_12m5_bucket$b.json 2> $OUT/shard_12m5_bucket$b.err || { echo SHARD_FAIL; tail -20 $OUT/shard_12m5_bucket$b.err; exit 1; }
  cat $OUT/shard_12m5_bucket$b.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('bucket', $b, d['phases_us'])"
done
df -h /tmp | tail -1
mkdir -p /tmp/mbx_delivery && rm -f /tmp/mbx_delivery/db
timeout -k 10 420 minibase-columnar-database_amd/host/bench_delivery /tmp/mbx_delivery 10000000 100000000 3 > $OUT/delivery.jsonl 2> $OUT/delivery.err || { echo DELIVERY_FAIL; tail -20 $OUT/delivery.err; exit 1; }
rm -rf /tmp/mbx_delivery
cat $OUT/delivery.err $OUT/delivery.jsonl
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo ANATOMY_OK
