set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp18; mkdir -p $OUT
timeout -k 10 500 python -u tools/bench_configs.py > $OUT/configs_1gpu.jsonl 2> $OUT/configs.err || { tail $OUT/configs.err; exit 1; }
cat $OUT/configs_1gpu.jsonl
