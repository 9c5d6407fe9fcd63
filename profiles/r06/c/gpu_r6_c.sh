# Round 6: the exchange fallback rehearsed (extended): the
# driver's launch form (torch.distributed.run -> per-rank supervisors ->
# workers) with a one-rank RCCL clique whose setup is forced to fail -> fresh
# workers with the host exchange; then torch.distributed.run N = 2 with both
# workers on this one GPU (MBX_BENCH_SAME_DEVICE=1, gloo exchange: RCCL refuses
# two ranks on one device) -> the supervisors' N > 1 path end to end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6_c}
mkdir -p $OUT
MBX_BENCH_FORCE_EXCHANGE=1 MBX_BENCH_FORCE_COMM_FAIL=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/host_fallback_torchrun_n1.json 2> $OUT/host_fallback_torchrun_n1.err || { echo HOSTFB_FAIL; tail -30 $OUT/host_fallback_torchrun_n1.err; exit 1; }
cut -c1-400 $OUT/host_fallback_torchrun_n1.json
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/torchrun_same_device_n2.json 2> $OUT/torchrun_same_device_n2.err || { echo TR2_FAIL; tail -30 $OUT/torchrun_same_device_n2.err; exit 1; }
cut -c1-400 $OUT/torchrun_same_device_n2.json
echo R6_C_OK
