# round 3: the 4-per-lane chained look-back (k_cnf_select, k_scan_select) and
# the finalize-free async BitSet scan: parity tests, C2 stamps and A/B
# (select_dbg 256 = the round-2 one-per-lane walk), C4 A/B, C2 configs line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_lb}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_scan_select_fused.py tests/test_cnf_materialize.py tests/test_cnf_cursor.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python3 tools/anatomy_r2.py --parts c2 --rounds 3 \
  --variants "${VARIANTS:-base;scan_select_fused=1;scan_select_fused=1,scan_select_waves=4}" > $OUT/anat.jsonl 2> $OUT/anat.err || { echo ANAT_FAIL; tail -20 $OUT/anat.err; exit 1; }
cat $OUT/anat.jsonl
for v in ${C4DBG:-0 0}; do
  MBX_SELECT_DBG=$v timeout -k 10 300 python3 tools/bench_configs.py --configs C4 > $OUT/c4_dbg$v.jsonl 2> $OUT/c4_dbg$v.err || { echo C4_FAIL; tail -20 $OUT/c4_dbg$v.err; exit 1; }
  echo "select_dbg=$v $(cat $OUT/c4_dbg$v.jsonl)"
done
timeout -k 10 300 python3 tools/bench_configs.py --configs C2 > $OUT/c2_ab.jsonl 2> $OUT/c2_ab.err || { echo C2_FAIL; tail -20 $OUT/c2_ab.err; exit 1; }
cat $OUT/c2_ab.jsonl
echo LB_OK
