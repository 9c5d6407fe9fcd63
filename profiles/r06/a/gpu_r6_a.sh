# Round 6, first GPU session: the default library's new tests + the whole
# GPU suite + smoke; the graph-phase fallback rehearsed twice (same-device
# N = 2 through bench.py's own launcher; torch.distributed.run N = 1 with a
# one-rank RCCL clique, i.e. the supervisor path the driver's N > 1 run takes);
# the driver's N = 1 line; then C4's read-request size split (VERDICT r5 item
# 2): rocprofv3 passes over tools/c4_req_probe (known footprints) and over
# bench.py's C3 + C4 kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6_a}
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || echo LIST_FAIL
grep -E "TCC_EA0_RDREQ|TCC_BUBBLE|TCC_EA0_WRREQ" $OUT/counters_list.txt | head -40 > $OUT/counters_tcc.txt || true
timeout -k 10 300 python -u -m pytest tests/test_tuning_and_materialize.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { echo NEW_FAIL; tail -40 $OUT/pytest_new.log; exit 1; }
tail -1 $OUT/pytest_new.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
# (a) same-device N = 2, rank 0's first graph replay forced to mismatch: the
# launcher must start fresh ranks with eager steps and print a complete line
MBX_BENCH_SAME_DEVICE=1 MBX_BENCH_FORCE_GRAPH_FAIL=verify timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/fallback_same_device_n2.json 2> $OUT/fallback_same_device_n2.err || { echo FB_A_FAIL; tail -30 $OUT/fallback_same_device_n2.err; exit 1; }
cut -c1-300 $OUT/fallback_same_device_n2.json
# (b) torch.distributed.run N = 1 + a one-rank RCCL clique (graphs with the
# collective inside), the first replay forced to time out: the supervisor path
MBX_BENCH_FORCE_EXCHANGE=1 MBX_BENCH_FORCE_GRAPH_FAIL=timeout timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --configs C4,C5 > $OUT/fallback_torchrun_n1.json 2> $OUT/fallback_torchrun_n1.err || { echo FB_B_FAIL; tail -30 $OUT/fallback_torchrun_n1.err; exit 1; }
cut -c1-300 $OUT/fallback_torchrun_n1.json
# (c) the same without forcing: graphs kept, first replay verified
MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/torchrun_n1.json 2> $OUT/torchrun_n1.err || { echo TR_FAIL; tail -30 $OUT/torchrun_n1.err; exit 1; }
cut -c1-300 $OUT/torchrun_n1.json
# the driver's N = 1 command
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-300 $OUT/bench_n1.json
# C4 read-request sizes: the probe (known footprints) and bench.py's C3 + C4
P="tools/c4_req_probe 100000000 10 10"
B="python3 bench.py --steps 5 --warmup 1 --kernel-graph 5 --no-cpu-baseline --configs C4"
timeout -k 10 120 $P > $OUT/probe.jsonl 2> $OUT/probe.err || { echo PROBE_FAIL; tail -5 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl | cut -c1-300
i=0
for CTRS in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_DRAM_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CTRS -d $OUT/pp$i -o p --output-format csv -- $P > $OUT/pp$i.log 2>&1 || { echo PMC_PROBE_FAIL $i; tail -5 $OUT/pp$i.log; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc $CTRS -d $OUT/pb$i -o p --output-format csv -- $B > $OUT/pb$i.log 2>&1 || { echo PMC_BENCH_FAIL $i; tail -5 $OUT/pb$i.log; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/ktp -o k --output-format csv -- $P > $OUT/ktp.log 2>&1 || { echo KTP_FAIL; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ktb -o k --output-format csv -- $B > $OUT/ktb.log 2>&1 || { echo KTB_FAIL; exit 1; }
python3 tools/kernel_pmc_table.py $OUT/ktp $OUT/pp1 $OUT/pp2 $OUT/pp3 $OUT/pp4 $OUT/pp5 > $OUT/probe_table.jsonl || { echo TABLE_FAIL; exit 1; }
python3 tools/kernel_pmc_table.py $OUT/ktb $OUT/pb1 $OUT/pb2 $OUT/pb3 $OUT/pb4 $OUT/pb5 > $OUT/bench_table.jsonl || { echo TABLE_FAIL; exit 1; }
find $OUT/ktb -name '*kernel_stats.csv' -exec cp {} $OUT/bench_c4_kernel_stats.csv \;
rm -rf $OUT/pp? $OUT/pb? $OUT/ktp $OUT/ktb
cut -c1-400 $OUT/probe_table.jsonl
grep -E "k_scan_fast|k_cnf" $OUT/bench_table.jsonl | cut -c1-400
echo R6_A_OK
