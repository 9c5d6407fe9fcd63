# Round 5 (j): the driver's N=1 bench command and the same-device N=2
# rehearsal of the final bench.py (configs, strong sub-record, pre-check).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_j}
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-200 $OUT/bench_n1.json
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 500 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_n2_same_device.json 2> $OUT/bench_n2_same_device.err || { echo N2_FAIL; tail -30 $OUT/bench_n2_same_device.err; exit 1; }
cut -c1-200 $OUT/bench_n2_same_device.json
MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_n1_exchange.json 2> $OUT/bench_n1_exchange.err || { echo N1X_FAIL; tail -30 $OUT/bench_n1_exchange.err; exit 1; }
cut -c1-200 $OUT/bench_n1_exchange.json
echo R5_J_OK
