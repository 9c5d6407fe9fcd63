# Round 3 validation of the tree, part A: every GPU test, smoke, the bench
# line (CPU baseline included), rocprofv3 kernel trace + FETCH_SIZE /
# WRITE_SIZE passes of the bench -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o c3 --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --graph-steps 0 > $OUT/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o c3 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --graph-steps 0 > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o c3 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --graph-steps 0 > $OUT/write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
python tools/pmc_summary.py $OUT/kt $OUT/fetch $OUT/write --rows 100000000 --algo-bytes 800000000 --out $OUT/c3_scan_pmc.json > $OUT/summary.log 2>&1 || { echo SUMMARY_FAIL; exit 1; }
cat $OUT/summary.log
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/c3_kernel_stats.csv \;
echo FINAL_A_OK
