# C3 anatomy: probe vs scan variants / finalize modes under a kernel trace,
# plus an interleaved A/B sweep of the variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-anatomy}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o an --output-format csv -- python3 tools/scan_anatomy.py ${ANATOMY_ARGS} > $OUT/anatomy.log 2>&1 || { echo ANATOMY_FAIL; tail -20 $OUT/anatomy.log; exit 1; }
timeout -k 10 600 python tools/scan_sweep.py ${SWEEP_ARGS} > $OUT/sweep.log 2>&1 || { echo SWEEP_FAIL; tail -20 $OUT/sweep.log; exit 1; }
cat $OUT/sweep.log
echo ANATOMY_DONE
