# Round 5 (d): C4 gather of a grouped (c0, c1) row as one 8-byte load vs two
# 4-byte loads, checked and timed; the group / cursor tests with the pair form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_d}
mkdir -p $OUT
timeout -k 10 150 python3 -u tools/c4_forms.py > $OUT/c4_pair.jsonl 2> $OUT/c4_pair.err || { echo C4_FAIL; tail -5 $OUT/c4_pair.err; cat $OUT/c4_pair.jsonl; exit 1; }
MBX_GATHER_PAIR=0 timeout -k 10 150 python3 -u tools/c4_forms.py --check-rows 1000 > $OUT/c4_nopair.jsonl 2> $OUT/c4_nopair.err || { echo C4N_FAIL; tail -5 $OUT/c4_nopair.err; exit 1; }
timeout -k 10 150 python3 -u tools/c4_forms.py --check-rows 1000 > $OUT/c4_pair2.jsonl 2> $OUT/c4_pair2.err || { echo C4_FAIL; exit 1; }
cut -c1-200 $OUT/c4_pair.jsonl $OUT/c4_nopair.jsonl $OUT/c4_pair2.jsonl
timeout -k 10 600 python -u -m pytest tests/test_cnf_cursor.py tests/test_cnf_materialize.py tests/test_column_group.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
echo R5_D_OK
