# Round 4 part F: k_scan_select's look-back forms at C2 -- the chained walk
# (default), every predecessor polled with the count flags packed, and polled
# with one flag per 128-byte line (select_flag_stride 16): parity, then the
# interleaved timings with per-block stamps, and segment sizes 20-39 tiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_f}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_scan_select_fused.py tests/test_cnf_materialize.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 tools/bench_configs.py --configs C2 --c2-stamps --c2-tpb 26,39 > $OUT/c2.jsonl 2> $OUT/c2.err || { echo C2_FAIL; tail -20 $OUT/c2.err; exit 1; }
cut -c1-1500 $OUT/c2.jsonl
timeout -k 10 300 python3 tools/bench_configs.py --configs C4 > $OUT/c4.jsonl 2> $OUT/c4.err || { echo C4_FAIL; tail -20 $OUT/c4.err; exit 1; }
timeout -k 10 300 python3 tools/bench_configs.py --configs C4 --c4-group > $OUT/c4_group.jsonl 2> $OUT/c4_group.err || { echo C4G_FAIL; tail -20 $OUT/c4_group.err; exit 1; }
cut -c1-400 $OUT/c4.jsonl $OUT/c4_group.jsonl
echo R4_F_OK
