# Round 3: tiles in flight per wave for the branch-free C3 kernel: U = 2
# (default, knob 2) vs 3 / 4 (knob 3 / 4), full table and 12.5M shard, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_u}
mkdir -p $OUT
for r in 1 2; do
  for k in 2 3 4; do
    MBX_SCAN_INT_RANGE=$k timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/full_k$k.$r.json 2> $OUT/full_k$k.$r.err || { echo FULL_FAIL; tail -20 $OUT/full_k$k.$r.err; exit 1; }
    MBX_SCAN_INT_RANGE=$k MBX_BENCH_FORCE_EXCHANGE=1 timeout -k 10 200 python3 bench.py --rows 12500000 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/shard_k$k.$r.json 2> $OUT/shard_k$k.$r.err || { echo SHARD_FAIL; tail -20 $OUT/shard_k$k.$r.err; exit 1; }
    python3 -c "import json; a=json.load(open('$OUT/full_k$k.$r.json')); b=json.load(open('$OUT/shard_k$k.$r.json')); print('knob=$k', $r, 'full', round(a['phases_us']['step_wall'],2), round(a['roofline']['kernel_ms']*1e3,2), 'shard', round(b['phases_us']['step_wall'],2))"
  done
done
echo U_OK
