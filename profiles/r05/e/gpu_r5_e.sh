# Round 5 (e): the driver's N=1 bench line, its rocprofv3 kernel stats, and
# FETCH_SIZE / WRITE_SIZE passes (separate runs) over a short bench run, so
# every config record's kernel gets its PMC traffic per launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_e}
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-300 $OUT/bench_n1.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { echo KT_FAIL; tail -20 $OUT/bench_kt.err; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/bench_n1_kernel_stats.csv \;
head -12 $OUT/bench_n1_kernel_stats.csv | cut -c1-160
CMD="python3 bench.py --steps 5 --warmup 1 --kernel-graph 5 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o k --output-format csv -- $CMD > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o k --output-format csv -- $CMD > $OUT/write.log 2>&1 || { echo WRITE_FAIL; tail -5 $OUT/write.log; exit 1; }
python3 tools/kernel_pmc_table.py $OUT/kt $OUT/fetch $OUT/write > $OUT/kernels.jsonl || { echo TABLE_FAIL; exit 1; }
rm -rf $OUT/kt $OUT/fetch $OUT/write
cut -c1-220 $OUT/kernels.jsonl
echo R5_E_OK
