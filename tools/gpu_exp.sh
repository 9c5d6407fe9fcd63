set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp22; mkdir -p $OUT
for rep in 1 2; do
for ri in 1 2; do
MBX_SCAN_RI=$ri timeout -k 10 200 python -u tools/small_sweep.py --rows 100000000 --tpb 0 --ops scan_count --rounds 3 > $OUT/ri$ri.$rep.jsonl 2> $OUT/ri$ri.err || { tail $OUT/ri$ri.err; exit 1; }
echo "ri $ri rep $rep"; cat $OUT/ri$ri.$rep.jsonl
done
done
