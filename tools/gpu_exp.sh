set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp20; mkdir -p $OUT
timeout -k 10 400 python -u tools/scan_sweep.py --variants 0 --tpb 0 --fin 3 --groups 1,4,8,16,32 --rounds 7 > $OUT/sweep.jsonl 2> $OUT/sweep.err || { tail $OUT/sweep.err; exit 1; }
cat $OUT/sweep.jsonl
