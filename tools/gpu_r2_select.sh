# Round 2: one-launch BitSet + positions (kModeSelect) -- its parity tests,
# the NaN-order matrix through scan_select, then the C2 anatomy A/B (fused vs
# two launches) -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2_select}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_nan_order.py -m gpu -x -v --timeout 120 --timeout-method thread -k "select or nan or c2 or segments" > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 240 python3 tools/anatomy_r2.py --parts ${PARTS:-c2} --variants "${VARIANTS:-base}" > $OUT/anatomy.jsonl 2> $OUT/anatomy.err || { echo ANAT_FAIL; tail -30 $OUT/anatomy.err; exit 1; }
cat $OUT/anatomy.jsonl
echo SELECT_OK
