# Per-config throughput (C2, C4, C5) on one GPU -> gpurun_out/<tag>/configs.jsonl,
# plus a rocprofv3 kernel trace of the same run (per-kernel breakdown).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-configs}
mkdir -p $OUT
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/kt -o cfg --output-format csv -- python3 tools/bench_configs.py ${CFG_ARGS} > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; tail -20 $OUT/configs.err; exit 1; }
cat $OUT/configs.jsonl
echo CONFIGS_OK
