# Round 2: load flavour of the fused gather (plain / nt / sc1 / sc0 sc1):
# timing A/B over the line-calibration BitSets, then RDREQ / RDREQ_32B /
# FETCH_SIZE per flavour (separate PMC runs) -> gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2_gload}
mkdir -p $OUT
timeout -k 10 300 python3 tools/anatomy_r2.py --parts gather --variants "base;gather_load=1;gather_load=2;gather_load=3" > $OUT/ab.jsonl 2> $OUT/ab.err || { echo AB_FAIL; tail -20 $OUT/ab.err; exit 1; }
cat $OUT/ab.jsonl
for v in 0 1 2 3; do
  MBX_GATHER_LOAD=$v timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B -d $OUT/rdreq$v -o k --output-format csv -- python3 tools/anatomy_r2.py --parts gather --rounds 1 --launches 5 > $OUT/rdreq$v.log 2>&1 || { echo RDREQ_FAIL $v; exit 1; }
done
echo GLOAD_OK
