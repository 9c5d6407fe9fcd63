# Widened rows (DB staging, index persistence, joins): timings + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-features}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o feat --output-format csv -- python3 tools/bench_features.py > $OUT/features.jsonl 2> $OUT/features.err || { echo FEAT_FAIL; tail -20 $OUT/features.err; exit 1; }
cat $OUT/features.jsonl
FEAT_ROWS=100000000 timeout -k 10 900 python3 tools/bench_features.py > $OUT/features_100m.jsonl 2> $OUT/features_100m.err || { echo FEAT100_FAIL; tail -20 $OUT/features_100m.err; exit 1; }
cat $OUT/features_100m.jsonl
echo FEATURES_OK
