# round 3: bench.py's N>1 step structure on one GPU (one-rank clique, 12.5M-row
# shard, one collective per query): graphs of scans with the collectives
# enqueued after each graph vs eager, with and without one extra real kernel
# per step on the exchange stream (MBX_BENCH_XS_KERNEL=1, standing in for an
# N-rank collective's kernel)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_parts3}
mkdir -p $OUT
for cfg in "0 10" "1 10" "0 0" "1 0" "0 10" "1 10"; do
  set -- $cfg
  MBX_BENCH_XS_KERNEL=$1 MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python3 bench.py --rows 12500000 --steps 200 --warmup 20 --exchange-bucket 1 --graph-steps $2 --no-cpu-baseline > $OUT/shard_x$1_g$2.json 2> $OUT/shard_x$1_g$2.err || { echo SHARD_FAIL; tail -20 $OUT/shard_x$1_g$2.err; exit 1; }
  cat $OUT/shard_x$1_g$2.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('xs_kernel', $1, 'graph', $2, round(d['ms_per_step'] * 1e3, 2), d['phases_us'], d['config']['exchange'])"
done
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err || { echo REHEARSAL_FAIL; tail -20 $OUT/bench_2rank_gloo.err; exit 1; }
cut -c1-300 $OUT/bench_2rank_gloo.json
echo PARTS3_OK
