# round 3: the segment-interleaved one-launch select at 10 M and 100 M rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_il2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_scan_select_fused.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python3 tools/anatomy_r2.py --parts c2 --c2-rows 100000000 --rounds 3 --variants "base;scan_select_fused=0" > $OUT/anat_100m.jsonl 2> $OUT/anat_100m.err || { echo ANAT_FAIL; tail -20 $OUT/anat_100m.err; exit 1; }
grep '"part": "c2"' $OUT/anat_100m.jsonl
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_configs.py --configs C2 > $OUT/c2_$r.jsonl 2> $OUT/c2_$r.err || { echo C2_FAIL; tail -20 $OUT/c2_$r.err; exit 1; }
  cat $OUT/c2_$r.jsonl
done
echo IL_OK
