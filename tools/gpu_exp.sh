set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp10; mkdir -p $OUT
for r in 10000000 100000000; do
timeout -k 10 200 python -u tools/ab_tmp.py $r >> $OUT/ab.jsonl 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
done
cat $OUT/ab.jsonl
