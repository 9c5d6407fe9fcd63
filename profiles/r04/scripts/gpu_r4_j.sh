# Round 4 part J: the N > 1 step on one GPU -- the C3 scan plus its per-query
# COUNT all-reduce through a one-rank RCCL clique captured in the HIP graphs
# (MBX_BENCH_FORCE_EXCHANGE=1, count frames), beside the plain N = 1 line:
# the exchange's own cost per step, for the weak-scaling estimate.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_j}
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -20 $OUT/bench_n1.err; exit 1; }
MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench_n1_exchange.json 2> $OUT/bench_n1_exchange.err || { echo XCH_FAIL; tail -20 $OUT/bench_n1_exchange.err; exit 1; }
MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o x --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/kt.json 2> $OUT/kt.err || { echo KT_FAIL; tail -20 $OUT/kt.err; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/bench_n1_exchange_kernel_stats.csv \;
rm -rf $OUT/kt
python3 -c "
import json
a = json.load(open('$OUT/bench_n1.json')); b = json.load(open('$OUT/bench_n1_exchange.json'))
print({'plain_ms_per_step': a['ms_per_step'], 'exchange_ms_per_step': b['ms_per_step'], 'exchange_us': round((b['ms_per_step'] - a['ms_per_step']) * 1e3, 2), 'count': b['config'].get('count')})
"
head -6 $OUT/bench_n1_exchange_kernel_stats.csv | cut -c1-160
echo R4_J_OK
