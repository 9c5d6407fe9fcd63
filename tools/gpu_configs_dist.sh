# GPU tests, per-config timings on one GPU (C2, C4, C5 at 125M and 1B rows),
# and the N-rank flow of C4 / C5 rehearsed with 2 ranks on this one GPU
# (gloo for the exchange: RCCL refuses two ranks on one device).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cfgdist}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 600 python -u tools/bench_configs.py > $OUT/configs_1gpu.jsonl 2> $OUT/configs_1gpu.err || { echo CFG1_FAIL; tail -20 $OUT/configs_1gpu.err; exit 1; }
MBX_BENCH_BACKEND=gloo MBX_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 tools/bench_configs.py --configs C4,C5 --c5-rows 250000000 --steps 20 > $OUT/configs_2rank_gloo.jsonl 2> $OUT/configs_2rank_gloo.err || { echo CFG2_FAIL; tail -30 $OUT/configs_2rank_gloo.err; exit 1; }
timeout -k 10 300 python -u tools/small_sweep.py --tpb 0 --rounds 3 > $OUT/small.jsonl 2> $OUT/small.err || { echo SMALL_FAIL; exit 1; }
cat $OUT/configs_1gpu.jsonl $OUT/configs_2rank_gloo.jsonl $OUT/small.jsonl
echo CFGDIST_OK
