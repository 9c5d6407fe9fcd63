# Round 3: sparse gather / stream over coarse, fine-grained and uncached
# allocations (tools/gather_mtype_probe.hip) at 0.1 / 1 / 5 % selectivity,
# plus one FETCH_SIZE pass at 1 % -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_mtype}
mkdir -p $OUT
for pm in 10 1 50; do
  timeout -k 10 120 tools/gather_mtype_probe 100000000 $pm >> $OUT/mtype.jsonl 2>> $OUT/mtype.err || { echo PROBE_FAIL; tail $OUT/mtype.err; exit 1; }
done
cat $OUT/mtype.jsonl
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d $OUT/fetch -o m --output-format csv -- tools/gather_mtype_probe 100000000 10 > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; tail $OUT/fetch.log; exit 1; }
echo MTYPE_OK
