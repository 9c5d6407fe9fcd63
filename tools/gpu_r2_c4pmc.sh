# k_cnf_select (one-launch C4) kernel trace + FETCH_SIZE / WRITE_SIZE passes -> gpurun_out/r2_c4pmc
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r2_c4pmc
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o c4 --output-format csv -- python3 tools/bench_configs.py --configs C4 --steps 20 --warmup 3 > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail $OUT/kt.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o c4 --output-format csv -- python3 tools/bench_configs.py --configs C4 --steps 5 --warmup 1 > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; tail $OUT/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o c4 --output-format csv -- python3 tools/bench_configs.py --configs C4 --steps 5 --warmup 1 > $OUT/write.log 2>&1 || { echo WRITE_FAIL; tail $OUT/write.log; exit 1; }
python3 tools/kernel_pmc_table.py $OUT/kt $OUT/fetch $OUT/write > $OUT/table.txt 2>&1 || { echo TABLE_FAIL; exit 1; }
cat $OUT/table.txt
