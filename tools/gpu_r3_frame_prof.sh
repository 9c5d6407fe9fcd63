# Round 3: full GPU suite + smoke after the count-frame change, then rocprofv3
# kernel traces of the 12.5M-row shard (per-query exchange forced on) with
# count frames and with the in-launch finalize -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_frame_prof}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $OUT/smoke.log; exit 1; }
for cnt in frame finalize; do
  MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$cnt -o s --output-format csv -- python3 bench.py --rows 12500000 --steps 200 --warmup 20 --count $cnt --no-cpu-baseline > $OUT/kt_$cnt.json 2> $OUT/kt_$cnt.err || { echo KT_FAIL; tail $OUT/kt_$cnt.err; exit 1; }
  find $OUT/kt_$cnt -name '*kernel_stats.csv' -exec cp {} $OUT/shard_${cnt}_kernel_stats.csv \;
  grep -h "k_scan_fast\|nccl\|rccl" $OUT/shard_${cnt}_kernel_stats.csv | cut -c1-160
done
echo PROF_OK
