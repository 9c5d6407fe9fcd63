# GPU parity tests only -> gpurun_out/<tag>/pytest_gpu.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tests}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo TESTS_OK
