# rocprofv3 kernel trace + stats of the C4 config (k_cnf_select, chained look-back)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2_c4kt}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o c4 --output-format csv -- python3 tools/bench_configs.py --configs C4 > $OUT/c4.jsonl 2> $OUT/c4.err || { echo KT_FAIL; tail -20 $OUT/c4.err; exit 1; }
cat $OUT/c4.jsonl
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/c4_kernel_stats.csv \;
head -8 $OUT/c4_kernel_stats.csv
echo KT_OK
