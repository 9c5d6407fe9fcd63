# C3 kernel sweep + rocprofv3 kernel trace + PMC (FETCH_SIZE / WRITE_SIZE in
# separate passes) -> gpurun_out/, summarised by tools/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/${PROF_TAG:-prof}
mkdir -p $OUT
if [ -z "$SKIP_SWEEP" ]; then
timeout -k 10 420 python tools/scan_sweep.py --generic > $OUT/sweep.log 2>&1 || { echo SWEEP_FAIL; exit 1; }
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o c3 --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > $OUT/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o c3 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o c3 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
python tools/pmc_summary.py $OUT/kt $OUT/fetch $OUT/write --rows 100000000 --algo-bytes 800000000 --out $OUT/c3_scan_pmc.json > $OUT/summary.log 2>&1 || { echo SUMMARY_FAIL; exit 1; }
echo PROFILE_OK
