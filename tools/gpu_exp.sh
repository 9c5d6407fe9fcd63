set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp19; mkdir -p $OUT
MBX_BENCH_BACKEND=gloo MBX_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 tools/bench_configs.py --configs C4,C5 --c5-rows 250000000 --steps 20 > $OUT/configs_2rank_gloo.jsonl 2> $OUT/configs_2rank_gloo.err || { echo CFG2_FAIL; tail -30 $OUT/configs_2rank_gloo.err; exit 1; }
cat $OUT/configs_2rank_gloo.jsonl
