# Round 6 validation of the shipped tree + the config records' traffic from
# the read-request size split: the whole GPU suite
# and smoke, the driver's N = 1 line, its rocprofv3 kernel stats, then PMC
# passes (request split, write split, FETCH_SIZE, WRITE_SIZE; one pass each)
# over a short bench.py with every config record -> kernels.jsonl, which
# tools/config_pmc.py turns into profiles/config_pmc.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6_b}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-300 $OUT/bench_n1.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o b --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_kt.json 2> $OUT/bench_kt.err || { echo KT_FAIL; tail -20 $OUT/bench_kt.err; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/bench_n1_kernel_stats.csv \;
B="python3 bench.py --steps 5 --warmup 1 --kernel-graph 5 --no-cpu-baseline"
timeout -k 10 300 $B > $OUT/bench_pmc.json 2> $OUT/bench_pmc.err || { echo BPMC_FAIL; tail -20 $OUT/bench_pmc.err; exit 1; }
i=0
for CTRS in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CTRS -d $OUT/p$i -o p --output-format csv -- $B > $OUT/p$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/kernel_pmc_table.py $OUT/kt $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 > $OUT/kernels.jsonl || { echo TABLE_FAIL; exit 1; }
rm -rf $OUT/kt $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4
grep -E "k_scan|k_cnf" $OUT/kernels.jsonl | cut -c1-300
echo R6_B_OK
