# Round 5 final: C4 positions-only default check, the whole GPU suite and
# smoke, then the driver's N=1 bench line with its rocprofv3 kernel stats and
# FETCH_SIZE / WRITE_SIZE passes (tools/config_pmc.py reads them).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_final}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/c4_forms.py --check-rows 1000,1000003 --positions-only > $OUT/c4_pos.jsonl 2> $OUT/c4_pos.err || { echo C4P_FAIL; tail -5 $OUT/c4_pos.err; exit 1; }
grep '"us"' $OUT/c4_pos.jsonl | cut -c1-200
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-200 $OUT/bench_n1.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { echo KT_FAIL; tail -20 $OUT/bench_kt.err; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/bench_n1_kernel_stats.csv \;
CMD="python3 bench.py --steps 5 --warmup 1 --kernel-graph 5 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o k --output-format csv -- $CMD > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o k --output-format csv -- $CMD > $OUT/write.log 2>&1 || { echo WRITE_FAIL; tail -5 $OUT/write.log; exit 1; }
python3 tools/kernel_pmc_table.py $OUT/kt $OUT/fetch $OUT/write > $OUT/kernels.jsonl || { echo TABLE_FAIL; exit 1; }
rm -rf $OUT/kt $OUT/fetch $OUT/write
grep -E "k_scan|k_cnf" $OUT/kernels.jsonl | cut -c1-200
echo R5_FINAL_OK
