# Round 5 (s): dynamically scheduled k_cnf_select (cnf_dyn = S segments taken
# from 8 per-XCD counters by 1024 resident blocks) vs the static grid:
# checked at every size (repeated launches: the counters must come back to
# 0), timed with a projection and positions only.  Every run under its own
# short limit: a scheduling bug shows as a hang, not a fault.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_s}
mkdir -p $OUT
timeout -k 5 90 python3 -u tools/c4_forms.py --dyn 0,2048,4096,8192 --check-rows 1000,70001,1000003,33554431 > $OUT/c4_dyn.jsonl 2> $OUT/c4_dyn.err || { echo C4_FAIL; tail -5 $OUT/c4_dyn.err; grep false $OUT/c4_dyn.jsonl | head -3; exit 1; }
timeout -k 5 90 python3 -u tools/c4_forms.py --dyn 0,4096 --check-rows 1000 --positions-only > $OUT/c4_dyn_pos.jsonl 2> $OUT/c4_dyn_pos.err || { echo C4P_FAIL; tail -5 $OUT/c4_dyn_pos.err; exit 1; }
python3 -c "
import json
for f in ['$OUT/c4_dyn.jsonl', '$OUT/c4_dyn_pos.jsonl']:
    for l in open(f):
        d = json.loads(l)
        if 'us' in d: print(d['positions_only'], d['group'], d['dyn'], round(d['us'], 2))
"
echo R5_S_OK
