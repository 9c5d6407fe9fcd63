# Round 5 (g): C4 k_cnf_select grid sweep (tuning cnf_blocks: 1024 = the
# chip-resident grid of round 4, 1536 .. 8192 = later blocks' operand loads
# beside earlier blocks' gathers), checked at every size first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_g}
mkdir -p $OUT
timeout -k 10 240 python3 -u tools/c4_forms.py --blocks 0,1536,2048,3072,4096,8192 > $OUT/c4_blocks.jsonl 2> $OUT/c4_blocks.err || { echo C4_FAIL; tail -5 $OUT/c4_blocks.err; cat $OUT/c4_blocks.jsonl; exit 1; }
grep '"us"' $OUT/c4_blocks.jsonl | cut -c1-120
echo R5_G_OK
