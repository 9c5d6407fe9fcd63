# Round 5 (w): same-device N = 4 rehearsal of the driver's multi-GPU bench
# (four ranks on one card, gloo exchange: every config record, the strong
# sub-record, cpu_baseline null at N > 1) and the N = 1 torch.distributed
# fallback exchange.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_w}
mkdir -p $OUT
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 4 --steps 20 --warmup 5 > $OUT/bench_n4_same_device.json 2> $OUT/bench_n4_same_device.err || { echo N4_FAIL; tail -30 $OUT/bench_n4_same_device.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_n4_same_device.json'))
print(d['n_gpus'], d['value'], d['config']['exchange'], 'cpu_baseline', d['cpu_baseline'], 'strong', round(d['strong']['value']), list(d['configs']))
for k, v in d['configs'].items(): print(k, v['gpus'], v['exchange'], v['pre_check'], round(v['ms_per_query'] * 1e3, 1))"
MBX_BENCH_TORCH_EXCHANGE=1 timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_n1_torch_exchange.json 2> $OUT/bench_n1_torch_exchange.err || { echo N1T_FAIL; tail -30 $OUT/bench_n1_torch_exchange.err; exit 1; }
cut -c1-300 $OUT/bench_n1_torch_exchange.json
echo R5_W_OK
