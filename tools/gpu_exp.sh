set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/exp8; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
for rep in 1 2; do
for fm in 0 3; do
MBX_FIN_MODE=$fm timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/b_$fm.json 2> $OUT/b_$fm.err || { tail $OUT/b_$fm.err; exit 1; }
python -c "
import json,sys; d=json.load(open('$OUT/b_$fm.json')); r=d['roofline']
print('fin_mode $fm', round(r['kernel_ms']*1e3,2), 'us', round(r['achieved']), 'GB/s', 'value', '%.4g' % d['value'], 'ms/step', round(d['ms_per_step']*1e3,2), 'probe', round(r['measured_read_peak']))"
done
done
