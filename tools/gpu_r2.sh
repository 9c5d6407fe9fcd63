# Round 2 GPU check: parity tests (TESTS, default all), smoke, one bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
if [ -z "$NO_BENCH" ]; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['measured_read_peak'])"
fi
echo R2_OK
