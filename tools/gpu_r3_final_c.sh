# Round 3 validation, part B (count frames: the shard runs with --count auto = frames, and the finalize): the other configs (C2, C4, C5 125M / 1B) with
# rocprofv3 kernel traces of C2 and C4, the 12.5M-row strong-scaling shard
# with a per-query exchange (bucket 1) and bucketed (10), delivered rows
# through the C++ drop-ins, and the 2-rank same-GPU rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_final}
mkdir -p $OUT
timeout -k 10 600 python tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; tail -20 $OUT/configs.err; exit 1; }
cat $OUT/configs.jsonl
for c in C2 C4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$c -o $c --output-format csv -- python3 tools/bench_configs.py --configs $c > $OUT/kt_$c.jsonl 2> $OUT/kt_$c.err || { echo KT_${c}_FAIL; tail -20 $OUT/kt_$c.err; exit 1; }
  find $OUT/kt_$c -name '*kernel_stats.csv' -exec cp {} $OUT/${c}_kernel_stats.csv \;
  find $OUT/kt_$c -name '*kernel_trace.csv' -exec cp {} $OUT/${c}_kernel_trace.csv \;
done
python3 tools/trace_gaps.py $OUT/C2_kernel_trace.csv --seq k_scan_fast,k_select_ids --json $OUT/c2_gaps.json > /dev/null && cat $OUT/c2_gaps.json
rm -f $OUT/C2_kernel_trace.csv $OUT/C4_kernel_trace.csv
for b in 1 10; do for cnt in auto finalize; do
  MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python3 bench.py --rows 12500000 --steps 200 --warmup 20 --exchange-bucket $b --count $cnt --no-cpu-baseline > $OUT/shard_12m5_bucket$b.$cnt.json 2> $OUT/shard_12m5_bucket$b.$cnt.err || { echo SHARD_FAIL; tail -20 $OUT/shard_12m5_bucket$b.$cnt.err; exit 1; }
  cat $OUT/shard_12m5_bucket$b.$cnt.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('bucket', $b, '$cnt', d['phases_us'])"
done; done
mkdir -p /tmp/mbx_delivery && rm -f /tmp/mbx_delivery/db
timeout -k 10 420 minibase-columnar-database_amd/host/bench_delivery /tmp/mbx_delivery 10000000 100000000 3 > $OUT/delivery.jsonl 2> $OUT/delivery.err || { echo DELIVERY_FAIL; tail -20 $OUT/delivery.err; exit 1; }
rm -rf /tmp/mbx_delivery
cat $OUT/delivery.jsonl
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err || { echo REHEARSAL_FAIL; tail -20 $OUT/bench_2rank_gloo.err; exit 1; }
cat $OUT/bench_2rank_gloo.json
echo FINAL_B_OK
