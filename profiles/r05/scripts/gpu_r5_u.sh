# Round 5 (u): C5's aggregate scan VALU load (SQ instruction counters beside
# the kernel trace) -- run before and after the 64-bit-key string terms and
# the NaN-free tile skip; with TESTS=1 the whole GPU suite runs first (or
# TESTS='tests/a.py tests/b.py').
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_u}
mkdir -p $OUT
if [ "${TESTS:-0}" != 0 ]; then
  # TESTS=1: the whole GPU suite; otherwise the test paths it names
  T=tests; [ "$TESTS" != 1 ] && T="$TESTS"
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
CMD="python3 bench.py --steps 5 --warmup 1 --kernel-graph 5 --no-cpu-baseline --configs ${CONFIGS:-C5}"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o k --output-format csv -- $CMD > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail -5 $OUT/kt.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/sq -o k --output-format csv -- $CMD > $OUT/sq.log 2>&1 || { echo SQ_FAIL; tail -5 $OUT/sq.log; exit 1; }
python3 tools/kernel_pmc_table.py $OUT/kt $OUT/sq > $OUT/table.jsonl || { echo TABLE_FAIL; exit 1; }
rm -rf $OUT/kt $OUT/sq
grep -E "k_scan|k_cnf" $OUT/table.jsonl
[ "${CONFIGS:-C5}" = C5 ] || { echo R5_U_OK; exit 0; }
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs C5 > $OUT/bench_c5_$i.json 2> $OUT/bench_c5_$i.err || { echo BENCH_FAIL; tail -5 $OUT/bench_c5_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_c5_$i.json')); c=d['configs']['C5']; print('C3', round(d['roofline']['kernel_ms']*1e3,2), 'C5', round(c['kernel_ms']*1e3,2), round(c['frac'],3))"
done
echo R5_U_OK
