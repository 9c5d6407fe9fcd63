set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp21; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
for rep in 1 2; do
for sl in 0 1; do
MBX_SINK_LDS=$sl timeout -k 10 200 python -u tools/small_sweep.py --rows 10000000,12500000,100000000 --tpb 0 --ops scan_bitmap,select,scan_select --rounds 3 > $OUT/sl$sl.$rep.jsonl 2> $OUT/sl$sl.err || { tail $OUT/sl$sl.err; exit 1; }
echo "sink_lds $sl rep $rep"; cat $OUT/sl$sl.$rep.jsonl
done
done
