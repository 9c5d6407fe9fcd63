# Round 4 part I: per-block stamps of the shipped k_scan_select at C2 (start /
# staged / offset known / end, wall_clock64 at 100 MHz) for each look-back
# form, raw per block, plus the interleaved timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_i}
mkdir -p $OUT
timeout -k 10 300 python3 tools/bench_configs.py --configs C2 --c2-stamps --c2-stamps-out $OUT/c2_stamps > $OUT/c2.jsonl 2> $OUT/c2.err || { echo C2_FAIL; tail -20 $OUT/c2.err; exit 1; }
cut -c1-1200 $OUT/c2.jsonl
ls $OUT
echo R4_I_OK
