# Round 3: typed range tests (scan_int_range = 2: float / char(16) literal
# terms too) -- GPU tests, then C5 (125M / 1B rows) with knob 2 vs 1, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_tr}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_typed_range.py tests/test_int_range.py tests/test_nan_order.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for k in 2 1; do
    MBX_SCAN_INT_RANGE=$k timeout -k 10 300 python3 tools/bench_configs.py --configs C5 > $OUT/c5_k$k.$r.jsonl 2> $OUT/c5_k$k.$r.err || { echo C5_FAIL; tail -20 $OUT/c5_k$k.$r.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/c5_k$k.$r.jsonl'):
    d=json.loads(l); print('C5 knob=$k', $r, d['rows'], round(d['ms_per_query']*1e3,1), 'us', round(d.get('scan_gbs_per_gpu',0)))"
  done
done
echo TR_OK
