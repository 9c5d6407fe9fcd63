set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-exp}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/b$i.json 2>$OUT/b$i.err || { tail $OUT/b$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b$i.json')); r=d['roofline']; print(d['value'], r['kernel_ms'], r['achieved'], r['measured_read_peak'], r['frac_of_measured_read_peak'])"
done
