set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp6; mkdir -p $OUT
timeout -k 10 200 python -u tools/c5_diag.py 200000000,1000000000 > $OUT/diag.jsonl 2> $OUT/diag.err || { tail $OUT/diag.err; cat $OUT/diag.jsonl; exit 1; }
cat $OUT/diag.jsonl
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -k "c5_full_table_1b" > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 4 $OUT/pytest.log
timeout -k 10 300 python -u tools/bench_configs.py --configs C5 --c5-rows 125000000,1000000000 > $OUT/c5.jsonl 2> $OUT/c5.err || { tail $OUT/c5.err; exit 1; }
cat $OUT/c5.jsonl
