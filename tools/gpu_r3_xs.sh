# round 3: the per-query exchange on the context stream (MBX_COMM_SAME_STREAM=1)
# vs the exchange stream, captured in graphs (bench.py's structure), with and
# without a stand-in real kernel per step (MBX_BENCH_XS_KERNEL=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_xs}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_comm.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
MBX_COMM_SAME_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_comm.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_same.log 2>&1 || { echo PYTEST_SAME_FAIL; tail -40 $OUT/pytest_same.log; exit 1; }
tail -1 $OUT/pytest_same.log
for cfg in "0 0" "1 0" "0 1" "1 1" "0 0" "1 0" "0 1" "1 1"; do
  set -- $cfg
  MBX_COMM_SAME_STREAM=$1 MBX_BENCH_XS_KERNEL=$2 MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python3 bench.py --rows 12500000 --steps 200 --warmup 20 --exchange-bucket 1 --no-cpu-baseline > $OUT/s$1_x$2.json 2> $OUT/s$1_x$2.err || { echo SHARD_FAIL; tail -20 $OUT/s$1_x$2.err; exit 1; }
  cat $OUT/s$1_x$2.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('same_stream', $1, 'xs_kernel', $2, round(d['ms_per_step'] * 1e3, 2), 'graph', d['config']['graph_steps'])"
done
echo XS_OK
