# Round 5 (i): k_cnf_select's automatic look-back form (polled for narrow
# projections read from column groups and for positions-only launches,
# chained otherwise) against both forced forms, with a projection and
# positions only; then the whole CNF / cursor / group test set on the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_i}
mkdir -p $OUT
timeout -k 10 240 python3 -u tools/c4_forms.py --lookback default,chained,poll1 --check-rows 1000,70001,1000003 > $OUT/c4_auto.jsonl 2> $OUT/c4_auto.err || { echo C4_FAIL; tail -5 $OUT/c4_auto.err; exit 1; }
timeout -k 10 240 python3 -u tools/c4_forms.py --lookback default,chained,poll1 --check-rows 1000,70001,1000003 --positions-only > $OUT/c4_auto_pos.jsonl 2> $OUT/c4_auto_pos.err || { echo C4P_FAIL; tail -5 $OUT/c4_auto_pos.err; exit 1; }
grep -h '"us"' $OUT/c4_auto.jsonl $OUT/c4_auto_pos.jsonl | cut -c1-150
timeout -k 10 600 python -u -m pytest tests/test_cnf_cursor.py tests/test_cnf_materialize.py tests/test_cnf_materialize_poll_all.py tests/test_column_group.py tests/test_shards.py tests/test_jni_harness.py tests/test_cli_transcript.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
echo R5_I_OK
