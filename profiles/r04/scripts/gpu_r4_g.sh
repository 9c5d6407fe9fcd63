# Round 4 part G: C2 anatomy in production timing (a -DMBX_DIAG build with
# parts of k_scan_select's tail switched off, tools/c2_anatomy.py), then the
# production library's C2 / C4 lines and the fused-select parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_g}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_scan_select_fused.py tests/test_cnf_materialize.py tests/test_gpu_parity.py -k "fused or lookback or cnf or ab_only or c2" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 tools/c2_anatomy.py --lib minibase-columnar-database_amd/libmbx_diag.so > $OUT/c2_anatomy_diag.jsonl 2> $OUT/c2_anatomy_diag.err || { echo ANAT_FAIL; tail -20 $OUT/c2_anatomy_diag.err; exit 1; }
cat $OUT/c2_anatomy_diag.jsonl
timeout -k 10 300 python3 tools/bench_configs.py --configs C2,C4 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; tail -20 $OUT/configs.err; exit 1; }
cut -c1-700 $OUT/configs.jsonl
echo R4_G_OK
