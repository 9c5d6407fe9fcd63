# one-launch C4 (mbx_cnf_materialize_async): its tests, then the C4 config
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r2_c4}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_cnf_materialize.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/bench_configs.py --configs C4 > $OUT/c4.jsonl 2> $OUT/c4.err || { echo C4_FAIL; tail -20 $OUT/c4.err; exit 1; }
cat $OUT/c4.jsonl
timeout -k 10 300 python tools/bench_configs.py --configs C4 --c4-positions > $OUT/c4_pos.jsonl 2> $OUT/c4_pos.err || { echo C4POS_FAIL; tail -20 $OUT/c4_pos.err; exit 1; }
cat $OUT/c4_pos.jsonl
timeout -k 10 300 python tools/c4_anatomy.py > $OUT/anat.jsonl 2> $OUT/anat.err || { echo ANAT_FAIL; exit 1; }
cat $OUT/anat.jsonl
