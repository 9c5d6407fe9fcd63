# Round 3: C5 (125M rows) anatomy -- the aggregate finalize as its own launch
# (MBX_FIN_MODE=2) under rocprofv3, beside the default in-launch finalize
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_c5fin}
mkdir -p $OUT
for fm in 2 0; do
  MBX_FIN_MODE=$fm timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt$fm -o c5 --output-format csv -- python3 tools/bench_configs.py --configs C5 --c5-rows 125000000 > $OUT/c5_fm$fm.jsonl 2> $OUT/c5_fm$fm.err || { echo KT_FAIL; tail -20 $OUT/c5_fm$fm.err; exit 1; }
  find $OUT/kt$fm -name '*kernel_stats.csv' -exec cp {} $OUT/c5_fm${fm}_kernel_stats.csv \;
  echo "fin_mode=$fm"; grep -h "k_scan_fast\|k_finalize" $OUT/c5_fm${fm}_kernel_stats.csv | cut -c1-200
  python3 -c "import json; d=json.loads(open('$OUT/c5_fm$fm.jsonl').readline()); print('query us', round(d['ms_per_query']*1e3,1))"
done
echo C5FIN_OK
