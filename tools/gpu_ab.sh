# A/B of a library tuning knob: GPU tests under the default and the
# alternative setting, then per-config timings under each setting.
#   KNOB=MBX_SCAN_RI VALUES="0 2" TAG=... bash tools/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for v in $VALUES; do
  env $KNOB=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$v.log 2>&1 || { echo PYTEST_${v}_FAIL; exit 1; }
done
for v in $VALUES; do
  env $KNOB=$v timeout -k 10 300 python -u tools/small_sweep.py --tpb 0 --rounds 3 > $OUT/small_$v.jsonl 2> $OUT/small_$v.err || { echo SMALL_${v}_FAIL; exit 1; }
  env $KNOB=$v timeout -k 10 300 python -u tools/bench_configs.py --configs C2,C4,C5 --c5-rows 125000000 > $OUT/configs_$v.jsonl 2> $OUT/configs_$v.err || { echo CFG_${v}_FAIL; exit 1; }
  env $KNOB=$v timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo BENCH_${v}_FAIL; exit 1; }
done
echo AB_OK
