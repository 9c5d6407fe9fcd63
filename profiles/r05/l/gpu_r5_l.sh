# Round 5 (l): the fallback exchange (torch.distributed's RCCL group, taken
# when libmbx's communicator fails on any rank) forced on one GPU, and the
# default N=1 line after the change; C4 output stores (cnf_store: default,
# plain, write-through, nontemporal), with a projection and positions only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5_l}
mkdir -p $OUT
MBX_BENCH_TORCH_EXCHANGE=1 timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_torch_exchange.json 2> $OUT/bench_torch_exchange.err || { echo TX_FAIL; tail -30 $OUT/bench_torch_exchange.err; exit 1; }
cut -c1-200 $OUT/bench_torch_exchange.json
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { echo N1_FAIL; tail -30 $OUT/bench_n1.err; exit 1; }
cut -c1-200 $OUT/bench_n1.json
timeout -k 10 240 python3 -u tools/c4_forms.py --store 0,1,2,3 --check-rows 1000,1000003 > $OUT/c4_wt.jsonl 2> $OUT/c4_wt.err || { echo C4_FAIL; tail -5 $OUT/c4_wt.err; exit 1; }
timeout -k 10 240 python3 -u tools/c4_forms.py --store 0,1,2,3 --check-rows 1000,1000003 --positions-only > $OUT/c4_wt_pos.jsonl 2> $OUT/c4_wt_pos.err || { echo C4P_FAIL; tail -5 $OUT/c4_wt_pos.err; exit 1; }
grep -h '"us"' $OUT/c4_wt.jsonl $OUT/c4_wt_pos.jsonl | cut -c1-200
echo R5_L_OK
