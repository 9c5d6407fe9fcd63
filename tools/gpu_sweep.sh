# GPU tests + C3 kernel sweep (variants x grid sizes), fail-fast.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 600 python tools/scan_sweep.py ${SWEEP_ARGS} > $OUT/sweep.log 2>&1 || { echo SWEEP_FAIL; exit 1; }
echo SWEEP_OK
