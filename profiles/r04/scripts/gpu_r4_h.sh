# Round 4 part H: PMC traffic of C2's k_scan_select (FETCH_SIZE and
# WRITE_SIZE in separate passes, gfx950 correction in tools/pmc_summary.py)
# against its algorithmic 49.25 MB per launch (40 MB of c0 read, 1.25 MB of
# BitSet and 8.0 MB of positions written).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_h}
mkdir -p $OUT
CMD="python3 tools/bench_configs.py --configs C2 --steps 20 --warmup 2"
D=$OUT/c2
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/kt -o k --output-format csv -- $CMD > $D.kt.log 2>&1 || { echo KT_FAIL; tail -20 $D.kt.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o k --output-format csv -- $CMD > $D.fetch.log 2>&1 || { echo FETCH_FAIL; tail -20 $D.fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $D/write -o k --output-format csv -- $CMD > $D.write.log 2>&1 || { echo WRITE_FAIL; tail -20 $D.write.log; exit 1; }
python3 tools/pmc_summary.py --kernel-substr k_scan_select --rows 10000000 --algo-bytes 49246272 --out $OUT/c2_pmc.json $D/kt $D/fetch $D/write || { echo SUMMARY_FAIL; exit 1; }
find $D/kt -name '*kernel_stats.csv' -exec cp {} $OUT/c2_kernel_stats.csv \;
rm -rf $D/kt $D/fetch $D/write
cat $OUT/c2_pmc.json
echo R4_H_OK
