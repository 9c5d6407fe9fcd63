# Round 4 final: the whole GPU test suite, smoke, the driver's N=1 bench line
# with its rocprofv3 kernel stats, the self-launched N=2 line on one GPU, and
# the configs / delivery lines of the shipped library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-400 $OUT/bench_n1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench_kt -o b --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { echo BENCH_KT_FAIL; tail -20 $OUT/bench_kt.err; exit 1; }
find $OUT/bench_kt -name '*kernel_stats.csv' -exec cp {} $OUT/bench_n1_kernel_stats.csv \;
rm -rf $OUT/bench_kt
head -3 $OUT/bench_n1_kernel_stats.csv
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 2 > $OUT/bench_n2_same_device.json 2> $OUT/bench_n2_same_device.err || { echo N2_FAIL; tail -30 $OUT/bench_n2_same_device.err; exit 1; }
cut -c1-300 $OUT/bench_n2_same_device.json
timeout -k 10 300 python3 tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; tail -20 $OUT/configs.err; exit 1; }
timeout -k 10 300 python3 tools/bench_configs.py --configs C4 --c4-group > $OUT/c4_group.jsonl 2> $OUT/c4_group.err || { echo C4G_FAIL; tail -20 $OUT/c4_group.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/cfg_kt -o c --output-format csv -- python3 tools/bench_configs.py > $OUT/cfg_kt.jsonl 2> $OUT/cfg_kt.err || { echo CFG_KT_FAIL; tail -20 $OUT/cfg_kt.err; exit 1; }
find $OUT/cfg_kt -name '*kernel_stats.csv' -exec cp {} $OUT/configs_kernel_stats.csv \;
rm -rf $OUT/cfg_kt
mkdir -p /tmp/mbx_delivery && rm -f /tmp/mbx_delivery/db
timeout -k 10 420 minibase-columnar-database_amd/host/bench_delivery /tmp/mbx_delivery 10000000 100000000 3 > $OUT/delivery.jsonl 2> $OUT/delivery.err || { echo DELIVERY_FAIL; tail -20 $OUT/delivery.err; exit 1; }
rm -rf /tmp/mbx_delivery
cut -c1-300 $OUT/configs.jsonl $OUT/delivery.jsonl
echo R4_FINAL_OK
