# Round 5 (a): the n-record device fold test, the new bench.py (all config
# records, graph-replay kernel times) at N=1, the same-device N=2 rehearsal
# (strong sub-record, pre-check) and the pre-check firing on a damaged frame.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_a}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_comm.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_comm.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_comm.log; exit 1; }
tail -1 $OUT/pytest_comm.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-300 $OUT/bench_n1.json
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 500 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_n2_same_device.json 2> $OUT/bench_n2_same_device.err || { echo N2_FAIL; tail -30 $OUT/bench_n2_same_device.err; exit 1; }
cut -c1-300 $OUT/bench_n2_same_device.json
# must fail with a one-line reason before timing
MBX_BENCH_SAME_DEVICE=1 MBX_BENCH_CORRUPT=frame timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --configs none --no-cpu-baseline > $OUT/bench_n2_corrupt.json 2> $OUT/bench_n2_corrupt.err
echo "corrupt-frame run exit: $?" | tee $OUT/bench_n2_corrupt.rc
grep -h "pre-check" $OUT/bench_n2_corrupt.err || true
echo R5_A_OK
