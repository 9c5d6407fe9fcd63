# Kernel trace + FETCH_SIZE + WRITE_SIZE passes (separate runs) over one
# command, summarised per kernel by tools/kernel_pmc_table.py.
#   CMD="tools/c4_req_probe 100000000 10 10" TAG=... bash tools/gpu_kernel_pmc.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-kpmc}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o k --output-format csv -- $CMD > $OUT/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o k --output-format csv -- $CMD > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o k --output-format csv -- $CMD > $OUT/write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
python3 tools/kernel_pmc_table.py $OUT/kt $OUT/fetch $OUT/write > $OUT/table.jsonl || { echo TABLE_FAIL; exit 1; }
cat $OUT/table.jsonl
echo KPMC_OK
