# Round 2: BitSet vs COUNT scan of one column at 100M rows -- timing A/B over
# the BitSink knobs, then kernel trace + PMC passes (separate runs) of the
# default pair -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2_bitset}
mkdir -p $OUT
timeout -k 10 240 python3 tools/anatomy_r2.py --parts bitset --launches 40 --rounds 3 --variants "base;sink_lds=0;sink_lds=2;scan_ri=0;tiles_per_block=191;tiles_per_block=96" > $OUT/ab.jsonl 2> $OUT/ab.err || { echo AB_FAIL; tail -20 $OUT/ab.err; exit 1; }
cat $OUT/ab.jsonl
CMD="python3 tools/anatomy_r2.py --parts bitset --launches 5 --rounds 1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o k --output-format csv -- $CMD > $OUT/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d $OUT/sq -o k --output-format csv -- $CMD > $OUT/sq.log 2>&1 || { echo SQ_FAIL; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d $OUT/sq2 -o k --output-format csv -- $CMD > $OUT/sq2.log 2>&1 || { echo SQ2_FAIL; tail -5 $OUT/sq2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o k --output-format csv -- $CMD > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o k --output-format csv -- $CMD > $OUT/write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
python3 tools/kernel_pmc_table.py $OUT/kt $OUT/sq $OUT/sq2 $OUT/fetch $OUT/write > $OUT/table.jsonl || { echo TABLE_FAIL; exit 1; }
cat $OUT/table.jsonl
echo BITSET_OK
