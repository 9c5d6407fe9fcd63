set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-exp}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/small_sweep.py --tpb 0 --rounds 3 > $OUT/small.jsonl 2> $OUT/small.err || { tail $OUT/small.err; exit 1; }
cat $OUT/small.jsonl
