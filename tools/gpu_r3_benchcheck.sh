# Round 3: bench.py sanity after the exchange fallback: N=1, the 12.5M shard
# with its exchange forced on, and the 2-rank same-GPU rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_benchcheck}
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/n1.json 2> $OUT/n1.err || { echo N1_FAIL; tail -20 $OUT/n1.err; exit 1; }
MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python3 bench.py --rows 12500000 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/shard.json 2> $OUT/shard.err || { echo SHARD_FAIL; tail -20 $OUT/shard.err; exit 1; }
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/r2.json 2> $OUT/r2.err || { echo R2_FAIL; tail -20 $OUT/r2.err; exit 1; }
for f in n1 shard r2; do python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['config']['exchange'][:40], d['config']['count'][:10])"; done
echo CHECK_OK
