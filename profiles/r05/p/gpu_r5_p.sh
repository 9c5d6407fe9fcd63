# Round 5 (p): k_cnf_select in 16-wave blocks (256 blocks at C4) vs 4-wave
# blocks (1024): checked at every size, timed with a projection and positions
# only, group and no group; per-block stamps of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_p}
mkdir -p $OUT
timeout -k 10 240 python3 -u tools/c4_forms.py --waves 4,16 --check-rows 1000,70001,1000003,33554431 > $OUT/c4_waves.jsonl 2> $OUT/c4_waves.err || { echo C4_FAIL; tail -5 $OUT/c4_waves.err; grep false $OUT/c4_waves.jsonl | head; exit 1; }
timeout -k 10 240 python3 -u tools/c4_forms.py --waves 4,16 --check-rows 1000,1000003 --positions-only > $OUT/c4_waves_pos.jsonl 2> $OUT/c4_waves_pos.err || { echo C4P_FAIL; tail -5 $OUT/c4_waves_pos.err; exit 1; }
python3 -c "
import json
for f in ['$OUT/c4_waves.jsonl', '$OUT/c4_waves_pos.jsonl']:
    for l in open(f):
        d = json.loads(l)
        if 'us' in d: print(d['positions_only'], d['group'], d['waves'], round(d['us'], 2))
"
timeout -k 10 120 python3 -u tools/c4_stamps.py 16 > $OUT/c4_stamps16.jsonl 2> $OUT/c4_stamps16.err || { echo ST_FAIL; tail -5 $OUT/c4_stamps16.err; exit 1; }
cut -c1-330 $OUT/c4_stamps16.jsonl
echo R5_P_OK
