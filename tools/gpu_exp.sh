set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-exp}; mkdir -p $OUT
timeout -k 10 600 python -u tools/bench_staging.py > $OUT/staging.jsonl 2> $OUT/staging.err || { tail $OUT/staging.err; exit 1; }
cat $OUT/staging.jsonl
