# Round 3: aggregate scans over > 1024 blocks fold in a separate launch
# (default) vs the in-launch write-through finalize (MBX_FIN_MODE=0):
# aggregate / NaN / comm / shard GPU tests, then C5 125M / 1B interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_c5sep}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_nan_order.py tests/test_typed_range.py tests/test_comm.py tests/test_shards.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for fm in def 0; do
    if [ $fm = def ]; then E=""; else E="MBX_FIN_MODE=$fm"; fi
    env $E timeout -k 10 300 python3 tools/bench_configs.py --configs C5 > $OUT/c5_$fm.$r.jsonl 2> $OUT/c5_$fm.$r.err || { echo C5_FAIL; tail -20 $OUT/c5_$fm.$r.err; exit 1; }
    python3 -c "
import json
for l in open('$OUT/c5_$fm.$r.jsonl'):
    d=json.loads(l); print('C5 fin=$fm', $r, d['rows'], round(d['ms_per_query']*1e3,1), 'us')"
  done
done
echo C5SEP_OK
