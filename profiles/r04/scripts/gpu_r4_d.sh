# Round 4 part D: PMC traffic of the weak-scaling shard (100M rows, count
# frame) merged into the committed summary, the driver's N=1 bench line with
# a rocprofv3 kernel trace of the same command, the self-launched N=2 line
# (two ranks sharing the GPU, gloo exchange), smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_d}
mkdir -p $OUT
J=$OUT/c3_scan_pmc.json
cp profiles/c3_scan_pmc.json $J
CMD="python3 tools/c3_shard_scan.py --gpus 1 --launches 50 --count frame"
D=$OUT/w100
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/kt -o k --output-format csv -- $CMD > $D.kt.log 2>&1 || { echo KT_FAIL; tail -20 $D.kt.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o k --output-format csv -- $CMD > $D.fetch.log 2>&1 || { echo FETCH_FAIL; tail -20 $D.fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $D/write -o k --output-format csv -- $CMD > $D.write.log 2>&1 || { echo WRITE_FAIL; tail -20 $D.write.log; exit 1; }
python3 tools/pmc_summary.py --kernel-substr k_scan_fast --rows 100000000 --algo-bytes 800000000 --out $J --key 100000000:frame $D/kt $D/fetch $D/write > /dev/null || { echo SUMMARY_FAIL; exit 1; }
find $D/kt -name '*kernel_stats.csv' -exec cp {} $OUT/w100_frame_kernel_stats.csv \;
rm -rf $D/kt $D/fetch $D/write
python3 -c "import json; d=json.load(open('$J'))['shards']; print({k: round(v['traffic_over_algorithmic'], 5) for k, v in d.items()})"
cp $J profiles/c3_scan_pmc.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-600 $OUT/bench_n1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench_kt -o b --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { echo BENCH_KT_FAIL; tail -20 $OUT/bench_kt.err; exit 1; }
find $OUT/bench_kt -name '*kernel_stats.csv' -exec cp {} $OUT/bench_n1_kernel_stats.csv \;
rm -rf $OUT/bench_kt
head -3 $OUT/bench_n1_kernel_stats.csv
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_n2_same_device.json 2> $OUT/bench_n2_same_device.err || { echo N2_FAIL; tail -30 $OUT/bench_n2_same_device.err; exit 1; }
cut -c1-600 $OUT/bench_n2_same_device.json
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
echo R4_D_OK
