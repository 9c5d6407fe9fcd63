# Round 5 (h): C4 k_cnf_select grid x look-back form (chained walk vs every
# predecessor polled, flags packed or one per 128-byte line), checked at every
# size first; then the CNF tests with the winning form via the environment.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_h}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/c4_forms.py --blocks 512,768,1024 --lookback chained,poll16,poll1 --check-rows 1000,70001,1000003,33554431 > $OUT/c4_lb.jsonl 2> $OUT/c4_lb.err || { echo C4_FAIL; tail -5 $OUT/c4_lb.err; grep -v '"us"' $OUT/c4_lb.jsonl | grep false; exit 1; }
grep '"us"' $OUT/c4_lb.jsonl | cut -c1-140
MBX_SELECT_DBG=128 MBX_CNF_FLAG_STRIDE=16 timeout -k 10 600 python -u -m pytest tests/test_cnf_cursor.py tests/test_cnf_materialize.py tests/test_column_group.py tests/test_shards.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_poll16.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_poll16.log; exit 1; }
tail -1 $OUT/pytest_poll16.log
echo R5_H_OK
