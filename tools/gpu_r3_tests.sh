# round 3: selected GPU test files -> gpurun_out/<tag>/pytest.log
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3tests}
mkdir -p $OUT
timeout -k 10 ${TLIM:-600} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
echo TESTS_OK
