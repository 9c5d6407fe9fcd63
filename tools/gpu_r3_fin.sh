# round 3: what the COUNT finalize and the segment size cost at the 8-GPU shard
# size (12.5M rows) and at C2 (10M rows): scan vs its read probe, A/B of
# finalize forms (fin_mode 4 = no finalize, diagnostic) and grids; the
# one-launch C2 form with per-block stamps, dense vs spread look-back flags
# (select_dbg 256), and C4 with both flag layouts
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_fin}
mkdir -p $OUT
timeout -k 10 500 python3 tools/anatomy_r2.py --parts c3small,c2 --c3-rows 12500000,100000000 --rounds 3 \
  --variants "${VARIANTS:-base;fin_mode=4;ticket_groups=8;tiles_per_block=24;tiles_per_block=32;scan_select_fused=1;scan_select_fused=1,select_dbg=256}" > $OUT/anat.jsonl 2> $OUT/anat.err || { echo ANAT_FAIL; tail -20 $OUT/anat.err; exit 1; }
cat $OUT/anat.jsonl
for v in 0 256 0 256; do
  MBX_SELECT_DBG=$v timeout -k 10 300 python3 tools/bench_configs.py --configs C4 > $OUT/c4_dbg$v.jsonl 2> $OUT/c4_dbg$v.err || { echo C4_FAIL; tail -20 $OUT/c4_dbg$v.err; exit 1; }
  echo "select_dbg=$v $(cat $OUT/c4_dbg$v.jsonl)"
done
echo FIN_OK
