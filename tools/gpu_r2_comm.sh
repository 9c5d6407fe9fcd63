# Round 2: the C-ABI exchange (RCCL one-rank cliques, graphs) + bench lines:
# N=1 default, N=1 with the forced exchange, a 12.5M-row shard (the N=8
# strong-scaling per-GPU size) with the forced exchange, graph vs eager.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2_comm}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_comm.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_comm.log 2>&1 || { echo PYTEST_FAIL; tail -60 $OUT/pytest_comm.log; exit 1; }
tail -3 $OUT/pytest_comm.log
b() { name=$1; shift; timeout -k 10 200 "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo BENCH_FAIL $name; tail -30 $OUT/$name.err; exit 1; }; python -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', '%.4g'%d['value'], 'ms/step %.4f'%d['ms_per_step'], d['phases_us'])"; }
b n1 python bench.py --no-cpu-baseline --steps 200 --warmup 20
b n1_eager python bench.py --no-cpu-baseline --steps 200 --warmup 20 --graph-steps 0
MBX_BENCH_FORCE_EXCHANGE=1 b n1_x python bench.py --no-cpu-baseline --steps 200 --warmup 20
MBX_BENCH_FORCE_EXCHANGE=1 b r12_x python bench.py --no-cpu-baseline --steps 200 --warmup 20 --rows 12500000
MBX_BENCH_FORCE_EXCHANGE=1 b r12_x_eager python bench.py --no-cpu-baseline --steps 200 --warmup 20 --rows 12500000 --graph-steps 0
b r12 python bench.py --no-cpu-baseline --steps 200 --warmup 20 --rows 12500000
b r12_g50 python bench.py --no-cpu-baseline --steps 200 --warmup 20 --rows 12500000 --graph-steps 50
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/rehearsal2.json 2> $OUT/rehearsal2.err || { echo REHEARSAL_FAIL; tail -30 $OUT/rehearsal2.err; exit 1; }
cat $OUT/rehearsal2.json
echo COMM_OK
