# Round 4: rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE (separate passes)
# of the C3 scan over rank 0's shard at N = 1, 2, 4, 8 (tools/c3_shard_scan.py,
# the COUNT form bench.py uses at that N), merged into
# gpurun_out/<tag>/c3_scan_pmc.json keyed ROWS:MODE; then bench.py's own
# N-rank launcher on one GPU (MBX_BENCH_SAME_DEVICE=1, no torch.distributed.run)
# and the N=1 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_shard_pmc}
mkdir -p $OUT
J=$OUT/c3_scan_pmc.json
rm -f $J
for n in 1 2 4 8; do
  if [ $n = 1 ]; then mode=finalize; else mode=frame; fi
  CMD="python3 tools/c3_shard_scan.py --gpus $n --launches 50 --count $mode"
  D=$OUT/n$n
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/kt -o k --output-format csv -- $CMD > $D.kt.log 2>&1 || { echo KT_FAIL_$n; tail -20 $D.kt.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o k --output-format csv -- $CMD > $D.fetch.log 2>&1 || { echo FETCH_FAIL_$n; tail -20 $D.fetch.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $D/write -o k --output-format csv -- $CMD > $D.write.log 2>&1 || { echo WRITE_FAIL_$n; tail -20 $D.write.log; exit 1; }
  rows=$(python3 -c "import sys; sys.path.insert(0,'.'); import mbx_pkg; b,e=mbx_pkg.load().mbx.shard_bounds(100000000,$n,0); print(e-b)")
  python3 tools/pmc_summary.py --kernel-substr k_scan_fast --rows $rows --algo-bytes $((rows*8)) --out $J --key $rows:$mode $D/kt $D/fetch $D/write > /dev/null || { echo SUMMARY_FAIL_$n; exit 1; }
  find $D/kt -name '*kernel_stats.csv' -exec cp {} $OUT/n${n}_kernel_stats.csv \;
  rm -rf $D/kt $D/fetch $D/write
done
cat $J
cp $J profiles/c3_scan_pmc.json
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_n2_same_device.json 2> $OUT/bench_n2_same_device.err || { echo N2_FAIL; tail -30 $OUT/bench_n2_same_device.err; exit 1; }
cat $OUT/bench_n2_same_device.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cat $OUT/bench_n1.json
timeout -k 10 600 python -u -m pytest tests/test_jni_harness.py tests/test_bench_launch.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_jni.log 2>&1 || { echo JNI_TESTS_FAIL; tail -40 $OUT/pytest_jni.log; exit 1; }
tail -3 $OUT/pytest_jni.log
echo R4_SHARD_PMC_OK
