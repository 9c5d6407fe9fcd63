"""k_cnf_select (mbx_cnf_materialize_async) counts vs numpy at 150 M,
2^31 + 4133, 2^32 - 64 and 2^32 + 4133 bits, 2 or 4 operand BitSets,
positions only or one projected column, beside k_bitmap_cnf's count.
Round 5 (profiles/r05/y): the first run zeroed its count on torch's stream
without a synchronize before the launch on the context stream and read 0 --
a stream race in the harness, not the kernel."""
import sys, json
sys.path.insert(0, '/root/repo')
import numpy as np, torch, mbx_pkg
m = mbx_pkg.load(); M = m.mbx
ctx = m.Context(0)
for N in [150_000_037, (1 << 31) + 4133, (1 << 32) - 64, (1 << 32) + 4133]:
    nw = (N + 63) // 64
    g = torch.Generator(device="cuda"); g.manual_seed(7)
    ops = [torch.randint(-(1 << 63), (1 << 63) - 1, (nw,), dtype=torch.int64, device="cuda", generator=g) for _ in range(4)]
    col = torch.empty(N, dtype=torch.int32, device="cuda")
    t = ctx.wrap([(M.INTEGER, 4)], [col.data_ptr()], N)
    bms = [ctx.bitmap_upload(N, w.cpu().numpy().view(np.uint64)) for w in ops]
    for nb in [2, 4]:
        a = ops[0]
        for k in range(1, nb): a = a & ops[k]
        a = a.clone(); a[-1] &= (1 << (N % 64)) - 1 if N % 64 else -1
        want = int(np.bitwise_count(a.cpu().numpy().view(np.uint64)).sum())
        ids = torch.zeros(want + 64, dtype=torch.int64, device="cuda")
        out = torch.zeros(want + 64, dtype=torch.int32, device="cuda")
        for proj in ([], [0]):
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            ctx.cnf_materialize_async(t, [[b] for b in bms[:nb]], proj, ids.data_ptr(), [out.data_ptr()] if proj else [], cnt.data_ptr())
            ctx.sync()
            c2 = ctx.bitmap_cnf(N, [[b] for b in bms[:nb]]).count
            print(json.dumps(dict(N=N, nb=nb, proj=proj, want=want, got=int(cnt.item()), bitmap_cnf=c2)), flush=True)
        del ids, out
    del ops, col, bms, t
    torch.cuda.empty_cache()
