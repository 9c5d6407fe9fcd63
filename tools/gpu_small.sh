# GPU parity tests, then ticket-group / grid sweeps at C2 and C3 sizes and a
# kernel trace of the C2/C4/C5 configs -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-small}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python tools/scan_sweep.py --rows 10000000 --variants 0 --tpb 0,10,20 --groups 1,8,32,64 --rounds 3 > $OUT/sweep_c2.log 2>&1 || { echo SWEEP_FAIL; exit 1; }
timeout -k 10 300 python tools/scan_sweep.py --variants 0 --tpb 0,48,96 --groups 1,32 --rounds 3 > $OUT/sweep_c3.log 2>&1 || { echo SWEEP3_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o cfg --output-format csv -- python3 tools/bench_configs.py --configs C2,C4,C5 --c5-rows 125000000 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo KT_FAIL; exit 1; }
echo SMALL_OK
