set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp16; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
for rep in 1 2; do
for fm in 0 3; do
MBX_FIN_MODE=$fm timeout -k 10 200 python -u tools/small_sweep.py --rows 10000000,12500000,100000000 --tpb 0 --rounds 3 > $OUT/fm$fm.$rep.jsonl 2> $OUT/fm$fm.err || { tail $OUT/fm$fm.err; exit 1; }
echo "fin_mode $fm rep $rep"; cat $OUT/fm$fm.$rep.jsonl
done
done
