# Round 4 part B: the full GPU suite (packed cursor, capacity-guarded
# k_cnf_select, column groups, JNI harness), bench_delivery, then C4 with and
# without the (c0, c1) column group: bench_configs line + kernel trace +
# FETCH_SIZE / WRITE_SIZE passes of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
mkdir -p /tmp/mbx_delivery && rm -f /tmp/mbx_delivery/db
timeout -k 10 420 minibase-columnar-database_amd/host/bench_delivery /tmp/mbx_delivery 10000000 100000000 3 > $OUT/delivery.jsonl 2> $OUT/delivery.err || { echo DELIVERY_FAIL; tail -20 $OUT/delivery.err; exit 1; }
rm -rf /tmp/mbx_delivery
cat $OUT/delivery.jsonl
for lay in cols group; do
  if [ $lay = group ]; then G=--c4-group; else G=; fi
  CMD="python3 tools/bench_configs.py --configs C4 $G"
  timeout -k 10 300 $CMD > $OUT/c4_$lay.jsonl 2> $OUT/c4_$lay.err || { echo C4_FAIL_$lay; tail -20 $OUT/c4_$lay.err; exit 1; }
  cat $OUT/c4_$lay.jsonl
  D=$OUT/c4_$lay
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o k --output-format csv -- $CMD > $D.kt.log 2>&1 || { echo KT_FAIL_$lay; tail -20 $D.kt.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o k --output-format csv -- $CMD > $D.fetch.log 2>&1 || { echo FETCH_FAIL_$lay; tail -20 $D.fetch.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $D/write -o k --output-format csv -- $CMD > $D.write.log 2>&1 || { echo WRITE_FAIL_$lay; tail -20 $D.write.log; exit 1; }
  python3 tools/kernel_pmc_table.py $D/kt $D/fetch $D/write > $OUT/c4_${lay}_kernels.jsonl || { echo TABLE_FAIL; exit 1; }
  find $D/kt -name '*kernel_stats.csv' -exec cp {} $OUT/c4_${lay}_kernel_stats.csv \;
  rm -rf $D/kt $D/fetch $D/write
  grep k_cnf_select $OUT/c4_${lay}_kernels.jsonl
done
echo R4_B_OK
