# Round 5 (k): C5 aggregate scan grid sweep (tiles_per_block), checked.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_k}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/c5_sweep.py > $OUT/c5_grid.jsonl 2> $OUT/c5_grid.err || { echo C5_FAIL; tail -5 $OUT/c5_grid.err; cat $OUT/c5_grid.jsonl; exit 1; }
cat $OUT/c5_grid.jsonl
echo R5_K_OK
