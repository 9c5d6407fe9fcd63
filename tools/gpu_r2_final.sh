# Round 2 validation of the tree: GPU tests, smoke, the bench line (CPU
# baseline included), rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes
# of the bench, the other configs (C2, C4, C5 125M / 1B), the 12.5M-row
# strong-scaling shard with its exchange, ticket-group A/B at the shard sizes,
# and the 2-rank same-GPU rehearsal -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2_final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o c3 --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --graph-steps 0 > $OUT/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o c3 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --graph-steps 0 > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o c3 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --graph-steps 0 > $OUT/write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
python tools/pmc_summary.py $OUT/kt $OUT/fetch $OUT/write --rows 100000000 --algo-bytes 800000000 --out $OUT/c3_scan_pmc.json > $OUT/summary.log 2>&1 || { echo SUMMARY_FAIL; exit 1; }
cat $OUT/summary.log
timeout -k 10 600 python tools/bench_configs.py > $OUT/configs.jsonl 2> $OUT/configs.err || { echo CONFIGS_FAIL; tail -20 $OUT/configs.err; exit 1; }
cat $OUT/configs.jsonl
MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --rows 12500000 > $OUT/shard_12m5_x.json 2> $OUT/shard_12m5_x.err || { echo SHARD_FAIL; exit 1; }
cat $OUT/shard_12m5_x.json
timeout -k 10 300 python3 tools/anatomy_r2.py --parts c3small --c3-rows 12500000,100000000 --launches 100 --rounds 5 --variants "base;ticket_groups=8;ticket_groups=16;ticket_groups=4" > $OUT/groups.jsonl 2> $OUT/groups.err || { echo GROUPS_FAIL; exit 1; }
cat $OUT/groups.jsonl
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err || { echo REHEARSAL_FAIL; tail -20 $OUT/bench_2rank_gloo.err; exit 1; }
cat $OUT/bench_2rank_gloo.json
MBX_BENCH_BACKEND=gloo MBX_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 tools/bench_configs.py --configs C4,C5 --c5-rows 125000000 > $OUT/configs_2rank_gloo.jsonl 2> $OUT/configs_2rank_gloo.err || { echo CFG_REHEARSAL_FAIL; tail -20 $OUT/configs_2rank_gloo.err; exit 1; }
cat $OUT/configs_2rank_gloo.jsonl
echo FINAL_OK
