# Round 6: the C3 scan over rank 0's shard at N = 1, 2, 4, 8 (tools/c3_shard_scan.py,
# the COUNT form bench.py uses at that N) with the shipped kernel: kernel trace +
# read-request size split + WRITE_SIZE passes -> one kernels.jsonl per N, merged
# into profiles/c3_scan_pmc.json by tools/c3_pmc_merge.py (bench.py's
# roofline.traffic at every N).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6_e}
mkdir -p $OUT
for tag in ${TAGS:-n1 n1frame n2 n4 n8}; do
  case $tag in n1) n=1; mode=finalize;; n1frame) n=1; mode=frame;; *) n=${tag#n}; mode=frame;; esac
  CMD="python3 tools/c3_shard_scan.py --gpus $n --launches 50 --count $mode"
  D=$OUT/$tag
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D/kt -o k --output-format csv -- $CMD > $D.kt.log 2>&1 || { echo KT_FAIL_$n; tail -20 $D.kt.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $D/split -o k --output-format csv -- $CMD > $D.split.log 2>&1 || { echo SPLIT_FAIL_$n; tail -20 $D.split.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $D/write -o k --output-format csv -- $CMD > $D.write.log 2>&1 || { echo WRITE_FAIL_$n; tail -20 $D.write.log; exit 1; }
  python3 tools/kernel_pmc_table.py $D/kt $D/split $D/write > $OUT/${tag}_kernels.jsonl || { echo TABLE_FAIL_$tag; exit 1; }
  find $D/kt -name '*kernel_stats.csv' -exec cp {} $OUT/${tag}_kernel_stats.csv \;
  rm -rf $D/kt $D/split $D/write
  grep k_scan_fast $OUT/${tag}_kernels.jsonl | cut -c1-250
done
echo R6_E_OK
