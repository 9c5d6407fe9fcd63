# Round 6: the driver's N > 1 launch form at N = 4 and N = 8 --
# torch.distributed.run -> one supervisor per rank -> one worker each -- with
# every worker on this one GPU (MBX_BENCH_SAME_DEVICE=1: gloo exchange, since
# RCCL refuses two ranks on one device).  Checks the supervisors, the weak /
# strong / bucketed records and the per-phase deadlines at the rank counts the
# 8-GPU node will run; the numbers are N ranks sharing one GPU, not scaling.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6_f}
mkdir -p $OUT
for n in 4 8; do
  MBX_BENCH_SAME_DEVICE=1 timeout -k 10 540 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr 127.0.0.1 --master-port $((29550 + n)) bench.py --gpus $n --steps 20 --warmup 5 > $OUT/torchrun_same_device_n$n.json 2> $OUT/torchrun_same_device_n$n.err || { echo TR_FAIL_$n; tail -30 $OUT/torchrun_same_device_n$n.err; exit 1; }
  cut -c1-300 $OUT/torchrun_same_device_n$n.json
done
echo R6_F_OK
