# Round 2 planning probe: the C3 step at the per-GPU sizes a strong-scaling
# run over the fixed 100M-row table gives (100M / N rows), with and without
# the per-step RCCL exchange (one-rank group at N=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2_sizes}
mkdir -p $OUT
for r in 12500000 25000000 50000000 100000000; do
  timeout -k 10 120 python bench.py --rows $r --steps 200 --warmup 20 --no-cpu-baseline > $OUT/b_$r.json 2> $OUT/b_$r.err || { echo BENCH_FAIL $r; tail -5 $OUT/b_$r.err; exit 1; }
  MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 120 python bench.py --rows $r --steps 200 --warmup 20 --no-cpu-baseline > $OUT/x_$r.json 2> $OUT/x_$r.err || { echo XBENCH_FAIL $r; tail -5 $OUT/x_$r.err; exit 1; }
  python - $OUT/b_$r.json $OUT/x_$r.json <<'PY'
import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read())
    print(f, "ms/step %.4f"%d["ms_per_step"], "kernel ms %.4f"%d["roofline"]["kernel_ms"], "GB/s %.0f"%d["roofline"]["achieved"], "probe %.0f"%d["roofline"]["measured_read_peak"])
PY
done
echo SIZES_OK
