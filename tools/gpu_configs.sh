# Per-config throughput (C2, C4, C5) on one GPU -> gpurun_out/<tag>/configs.jsonl
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-configs}
mkdir -p $OUT
timeout -k 10 900 python tools/bench_configs.py ${CFG_ARGS} > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; exit 1; }
echo CONFIGS_OK
