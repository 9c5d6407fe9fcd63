# First A/B of k_cnf_select's chained look-back, run while it was opt-in
# (MBX_SELECT_DBG=128 selected it then; it is the default now and the knob
# selects the every-predecessor poll -- see tools/gpu_r2_chain2.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r2_chain}
mkdir -p $OUT
MBX_SELECT_DBG=128 timeout -k 10 400 python -u -m pytest tests/test_cnf_materialize.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_chain.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_chain.log; exit 1; }
tail -1 $OUT/pytest_chain.log
for r in 1 2; do
  timeout -k 10 300 python tools/bench_configs.py --configs C4 > $OUT/c4_base_$r.jsonl 2> $OUT/c4_base_$r.err || { echo C4_FAIL; tail -20 $OUT/c4_base_$r.err; exit 1; }
  cat $OUT/c4_base_$r.jsonl
  MBX_SELECT_DBG=128 timeout -k 10 300 python tools/bench_configs.py --configs C4 > $OUT/c4_chain_$r.jsonl 2> $OUT/c4_chain_$r.err || { echo C4C_FAIL; tail -20 $OUT/c4_chain_$r.err; exit 1; }
  cat $OUT/c4_chain_$r.jsonl
done
MBX_SELECT_DBG=128 timeout -k 10 300 python tools/bench_configs.py --configs C4 --c4-positions > $OUT/c4_chain_pos.jsonl 2> $OUT/c4_chain_pos.err || { echo C4CP_FAIL; exit 1; }
cat $OUT/c4_chain_pos.jsonl
echo CHAIN_OK
