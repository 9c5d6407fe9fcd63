set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp14; mkdir -p $OUT
for mode in none marker exchange; do
env_args=""
[ $mode = marker ] && export MARKER_ONLY=1 || unset MARKER_ONLY
[ $mode = exchange ] && export MBX_BENCH_FORCE_EXCHANGE=1 || unset MBX_BENCH_FORCE_EXCHANGE
timeout -k 10 200 python -u tools/bench_marker_tmp.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/b_$mode.json 2> $OUT/b_$mode.err || { tail $OUT/b_$mode.err; exit 1; }
echo $mode; grep 'host enqueue' $OUT/b_$mode.err
done
