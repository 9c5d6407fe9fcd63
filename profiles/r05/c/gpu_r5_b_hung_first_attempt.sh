# Round 5 (b): C4 k_cnf_select in one or two rounds per block (cnf_rounds),
# checked and timed; the CNF / cursor / group tests under both forms.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_b}
mkdir -p $OUT
timeout -k 10 150 python3 -u tools/c4_forms.py > $OUT/c4_forms.jsonl 2> $OUT/c4_forms.err || { echo C4_FAIL; tail -20 $OUT/c4_forms.err; cat $OUT/c4_forms.jsonl; exit 1; }
cat $OUT/c4_forms.jsonl
MBX_CNF_ROUNDS=2 timeout -k 10 600 python -u -m pytest tests/test_cnf_cursor.py tests/test_cnf_materialize.py tests/test_column_group.py tests/test_shards.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_rounds2.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_rounds2.log; exit 1; }
tail -1 $OUT/pytest_rounds2.log
echo R5_B_OK
