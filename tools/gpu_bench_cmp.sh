# parity tests, then bench.py with 1 and 2 streams (interleaved, twice), then features
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-benchcmp}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
  for s in 1 2; do
    timeout -k 10 300 python3 bench.py --streams $s --no-cpu-baseline > $OUT/bench_s${s}_r${r}.json 2> $OUT/bench_s${s}_r${r}.err || { echo BENCH_FAIL; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_s${s}_r${r}.json'));print($s, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o feat --output-format csv -- python3 tools/bench_features.py > $OUT/features.jsonl 2> $OUT/features.err || { echo FEAT_FAIL; exit 1; }
cat $OUT/features.jsonl
echo CMP_OK
