set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp41; mkdir -p $OUT
for r in 10000000 100000000; do
timeout -k 10 300 python -u tools/small_sweep.py --tpb 0 --rounds 3 --rows $r --ops scan_count,select > $OUT/a.jsonl 2>$OUT/a.err || exit 1
MBX_SCAN_VARIANT=41 timeout -k 10 300 python -u tools/small_sweep.py --tpb 0 --rounds 3 --rows $r --ops scan_count,select > $OUT/b.jsonl 2>$OUT/b.err || exit 1
cat $OUT/a.jsonl $OUT/b.jsonl
done
