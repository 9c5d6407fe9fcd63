# Round 4 part E: k_scan_select's dry tail pass under the first loads
# (scan_select_warm) -- parity, then C2 interleaved two-launch / one-launch /
# one-launch-warm with per-block stamps and a kernel trace (the WARM
# instantiation has its own kernel name); delivery after the all-int bulk
# Jtuple copy and the inline get_next; then part D.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4_e}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_scan_select_fused.py tests/test_gpu_parity.py -k "fused or ab_only or finalize" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 tools/bench_configs.py --configs C2 --c2-stamps --c2-tpb 10,13,20,26,39 > $OUT/c2.jsonl 2> $OUT/c2.err || { echo C2_FAIL; tail -20 $OUT/c2.err; exit 1; }
cut -c1-900 $OUT/c2.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2_kt -o c --output-format csv -- python3 tools/bench_configs.py --configs C2 > $OUT/c2_kt.jsonl 2> $OUT/c2_kt.err || { echo C2_KT_FAIL; tail -20 $OUT/c2_kt.err; exit 1; }
find $OUT/c2_kt -name '*kernel_stats.csv' -exec cp {} $OUT/c2_kernel_stats.csv \;
rm -rf $OUT/c2_kt
grep -E "scan_select|select_ids|scan_fast" $OUT/c2_kernel_stats.csv | cut -c1-260
mkdir -p /tmp/mbx_delivery && rm -f /tmp/mbx_delivery/db
timeout -k 10 420 minibase-columnar-database_amd/host/bench_delivery /tmp/mbx_delivery 10000000 100000000 3 > $OUT/delivery.jsonl 2> $OUT/delivery.err || { echo DELIVERY_FAIL; tail -20 $OUT/delivery.err; exit 1; }
rm -rf /tmp/mbx_delivery
cut -c1-330 $OUT/delivery.jsonl
echo R4_E_OK
TAG=r4_d bash tools/gpu_r4_d.sh
