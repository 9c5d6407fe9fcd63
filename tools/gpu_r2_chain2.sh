# chained look-back as the default of k_cnf_select: the whole GPU suite (incl.
# the every-predecessor form under its knob), then C4 default vs
# MBX_SELECT_DBG=128 (the old poll) A/B/A/B, with positions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r2_chain2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $OUT/smoke.log; exit 1; }
for r in 1 2 3; do
  timeout -k 10 300 python tools/bench_configs.py --configs C4 > $OUT/c4_chain_$r.jsonl 2> $OUT/c4_chain_$r.err || { echo C4_FAIL; tail -20 $OUT/c4_chain_$r.err; exit 1; }
  cat $OUT/c4_chain_$r.jsonl
  MBX_SELECT_DBG=128 timeout -k 10 300 python tools/bench_configs.py --configs C4 > $OUT/c4_pollall_$r.jsonl 2> $OUT/c4_pollall_$r.err || { echo C4P_FAIL; tail -20 $OUT/c4_pollall_$r.err; exit 1; }
  cat $OUT/c4_pollall_$r.jsonl
done
timeout -k 10 300 python tools/bench_configs.py --configs C4 --c4-positions > $OUT/c4_chain_pos.jsonl 2> $OUT/c4_chain_pos.err || { echo C4CP_FAIL; exit 1; }
cat $OUT/c4_chain_pos.jsonl
echo CHAIN2_OK
