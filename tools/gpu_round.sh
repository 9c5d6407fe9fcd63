# Full GPU check: parity tests, smoke, bench (with CPU baseline), rocprofv3
# kernel trace + PMC (FETCH_SIZE / WRITE_SIZE in separate passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-round}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o c3 --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o c3 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o c3 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
python tools/pmc_summary.py $OUT/kt $OUT/fetch $OUT/write --rows 100000000 --algo-bytes 800000000 --out $OUT/c3_scan_pmc.json > $OUT/summary.log 2>&1 || { echo SUMMARY_FAIL; exit 1; }
echo ROUND_OK
# N>1 flow rehearsal on this one GPU: 2 ranks, gloo for the combine (RCCL
# refuses two ranks on one device), short run
MBX_BENCH_BACKEND=gloo MBX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --rows 20000000 > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err || { echo REHEARSAL_FAIL; exit 1; }
cat $OUT/bench_2rank_gloo.json
echo REHEARSAL_OK
