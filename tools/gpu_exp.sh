set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp15; mkdir -p $OUT
for rep in 1 2; do
for v in 0 21; do
MBX_SCAN_VARIANT=$v timeout -k 10 200 python -u tools/small_sweep.py --rows 10000000,12500000,100000000 --tpb 0 --ops scan_count,scan_bitmap,select,scan_select --rounds 3 > $OUT/v$v.$rep.jsonl 2> $OUT/v$v.err || { tail $OUT/v$v.err; exit 1; }
echo "variant $v rep $rep"; cat $OUT/v$v.$rep.jsonl
done
done
