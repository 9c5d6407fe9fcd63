# Round 5 (m): is C5's record slower inside the full bench line than alone?
# The same bench with C5 alone, C5 first, and the default order.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_m}
mkdir -p $OUT
for cfg in C5 C5,C4,C2 C2,C4,C5; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --configs $cfg > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { echo FAIL $cfg; tail -10 $OUT/bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$cfg.json')); print('$cfg', round(d['roofline']['kernel_ms']*1e3,2), {k: (round(v['ms_per_query']*1e3,1), round(v['kernel_ms']*1e3,1)) for k,v in d['configs'].items()})"
done
echo R5_M_OK
