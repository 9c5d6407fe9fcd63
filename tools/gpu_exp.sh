set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-exp}; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/b0.json 2>$OUT/b0.err || { tail $OUT/b0.err; exit 1; }
MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/b1.json 2>$OUT/b1.err || { tail $OUT/b1.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/b2.json 2>$OUT/b2.err || { tail $OUT/b2.err; exit 1; }
MBX_BENCH_BACKEND=gloo MBX_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --rows 20000000 > $OUT/b3.json 2> $OUT/b3.err || { tail $OUT/b3.err; exit 1; }
for f in b0 b1 b2 b3; do python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['parallelism'])"; done
