# round 3: k_scan_select (one-launch BitSet + positions) parity tests, the C2
# A/B of both forms (+ rocprofv3 kernel trace), delivered-rows bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_fused}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_scan_select_fused.py tests/test_gpu_parity.py -k "fused or c2 or scan_select" -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 tools/bench_configs.py --configs C2 > $OUT/c2_ab.jsonl 2> $OUT/c2_ab.err || { echo C2_FAIL; tail -20 $OUT/c2_ab.err; exit 1; }
cat $OUT/c2_ab.jsonl
MBX_SCAN_SELECT_FUSED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o c2f --output-format csv -- python3 tools/bench_configs.py --configs C2 > $OUT/c2_fused_kt.jsonl 2> $OUT/c2_fused_kt.err || { echo KT_FAIL; tail -20 $OUT/c2_fused_kt.err; exit 1; }
find $OUT/kt -name '*kernel_stats.csv' -exec cp {} $OUT/c2_fused_kernel_stats.csv \;
head -6 $OUT/c2_fused_kernel_stats.csv
mkdir -p /tmp/mbx_delivery && rm -f /tmp/mbx_delivery/db
timeout -k 10 420 minibase-columnar-database_amd/host/bench_delivery /tmp/mbx_delivery 10000000 100000000 3 > $OUT/delivery.jsonl 2> $OUT/delivery.err || { echo DELIVERY_FAIL; tail -20 $OUT/delivery.err; exit 1; }
rm -rf /tmp/mbx_delivery
cat $OUT/delivery.jsonl
echo FUSED_OK
