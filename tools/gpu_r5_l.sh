# Round 5 (l): the fallback exchange (torch.distributed's RCCL group, taken
# when libmbx's communicator fails on any rank) forced on one GPU, and the
# default N=1 line after the change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_l}
mkdir -p $OUT
MBX_BENCH_TORCH_EXCHANGE=1 timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_torch_exchange.json 2> $OUT/bench_torch_exchange.err || { echo TX_FAIL; tail -30 $OUT/bench_torch_exchange.err; exit 1; }
cut -c1-200 $OUT/bench_torch_exchange.json
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-200 $OUT/bench_n1.json
echo R5_L_OK
