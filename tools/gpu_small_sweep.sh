# Segment-size sweep at latency-bound sizes (tools/small_sweep.py), fail-fast.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-small_sweep}
mkdir -p $OUT
timeout -k 10 600 python -u tools/small_sweep.py ${SWEEP_ARGS} > $OUT/sweep.jsonl 2> $OUT/sweep.err || { echo SWEEP_FAIL; exit 1; }
echo SWEEP_OK
