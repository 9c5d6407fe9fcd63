# Focused GPU check: selected parity tests (PYTEST_ARGS / TESTS), one bench
# line, feature timings under a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
timeout -k 10 900 python -m pytest ${TESTS:-tests} -m gpu -x -q ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py --cpu-seconds 5 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o feat --output-format csv -- python3 tools/bench_features.py > $OUT/features.jsonl 2> $OUT/features.err || { echo FEAT_FAIL; tail -20 $OUT/features.err; exit 1; }
cat $OUT/features.jsonl
echo QUICK_OK
