set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/cli2
timeout -k 10 600 python -m pytest tests/test_cli_transcript.py -x -q > gpurun_out/cli2/pytest.log 2>&1; rc=$?
tail -30 gpurun_out/cli2/pytest.log
exit $rc
