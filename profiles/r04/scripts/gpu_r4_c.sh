# Round 4 part C: delivery after the inline Jtuple fill and 256 Ki-row
# batches: the C++ drop-in / CLI GPU tests, then bench_delivery.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_c}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_cli_transcript.py tests/test_cnf_cursor.py tests/test_shards.py tests/test_joins.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
mkdir -p /tmp/mbx_delivery && rm -f /tmp/mbx_delivery/db
timeout -k 10 420 minibase-columnar-database_amd/host/bench_delivery /tmp/mbx_delivery 10000000 100000000 3 > $OUT/delivery.jsonl 2> $OUT/delivery.err || { echo DELIVERY_FAIL; tail -20 $OUT/delivery.err; exit 1; }
rm -rf /tmp/mbx_delivery
cut -c1-330 $OUT/delivery.jsonl
echo R4_C_OK
