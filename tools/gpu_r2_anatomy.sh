# Round 2: C2 compaction anatomy + k_gather line-granularity calibration
# (tools/anatomy_r2.py) with a kernel trace and separate FETCH_SIZE /
# WRITE_SIZE / TCC_EA0_RDREQ passes -> gpurun_out/<tag>/
#   VARIANTS="base;knob=1" TAG=... bash tools/gpu_r2_anatomy.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2_anat}
mkdir -p $OUT
V="${VARIANTS:-base}"
timeout -k 10 240 python3 tools/anatomy_r2.py --variants "$V" > $OUT/anatomy.jsonl 2> $OUT/anatomy.err || { echo ANAT_FAIL; tail -30 $OUT/anatomy.err; exit 1; }
cat $OUT/anatomy.jsonl
CMD="python3 tools/anatomy_r2.py --variants base --rounds 1 --launches 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o k --output-format csv -- $CMD > $OUT/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o k --output-format csv -- $CMD > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o k --output-format csv -- $CMD > $OUT/write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
if grep -q "TCC_EA0_RDREQ_32B" $OUT/counters.txt && grep -q "TCC_EA0_RDREQ\b" $OUT/counters.txt; then
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B -d $OUT/rdreq -o k --output-format csv -- $CMD > $OUT/rdreq.log 2>&1 || echo RDREQ_FAIL
fi
python3 tools/kernel_pmc_table.py $OUT/kt $OUT/fetch $OUT/write $OUT/rdreq > $OUT/table.jsonl || { echo TABLE_FAIL; exit 1; }
cat $OUT/table.jsonl
echo ANAT_OK
