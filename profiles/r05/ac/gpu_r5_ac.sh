# Round 5 (ac): the bucketed sub-records -- same-device N = 2 rehearsal
# (gloo exchange) and the one-rank RCCL clique with a bucketed headline
# (the captured bucketed all-reduce the 8-GPU run will replay).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_ac}
mkdir -p $OUT
MBX_BENCH_SAME_DEVICE=1 timeout -k 10 500 python3 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_n2_same_device.json 2> $OUT/bench_n2_same_device.err || { echo N2_FAIL; tail -30 $OUT/bench_n2_same_device.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_n2_same_device.json'))
print('weak', round(d['value']), 'bucketed', d['bucketed'] and round(d['bucketed']['value']), 'strong', round(d['strong']['value']), 'strong.bucketed', d['strong']['bucketed'] and round(d['strong']['bucketed']['value']), list(d['configs']))"
for b in 1 20; do
  MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --configs none --exchange-bucket $b > $OUT/bench_n1_x_b$b.json 2> $OUT/bench_n1_x_b$b.err || { echo N1X_FAIL; tail -30 $OUT/bench_n1_x_b$b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_n1_x_b$b.json')); print('bucket $b', d['config']['exchange'][:60], round(d['ms_per_step']*1e3,2), d['config']['exchange_bucket_steps'])"
done
echo R5_AC_OK
