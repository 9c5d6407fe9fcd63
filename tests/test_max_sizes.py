"""Tables past Java's int positions.  The reference's positions are Java ints
(`TID.position`, `BitSet` indexes: R/iterator/ColumnarFileScan.java:174-188,
R/index/ColumnarIndexScan.java:287-308), so its tables end at 2^31 - 1 rows;
this library's positions are int64.  These tests cross 2^31 rows with the file
scan (COUNT, BitSet + ascending positions) and 2^32 bits with the one-launch
ColumnarIndexScan (k_cnf_select, whose 32-bit inclusive prefixes make tables
of >= 2^32 rows take the polled look-back) on ragged sizes, checked against
torch through size-independent properties: the count equals torch's, the
positions are strictly increasing and every one is selected -- together,
exactly the selected set -- and the projected values equal the column at
those positions.
"""
import numpy as np
import pytest

import mbx_pkg

pytestmark = pytest.mark.gpu

N31 = (1 << 31) + 4099          # rows: past the largest Java int position
N32 = (1 << 32) + 4096 + 37     # bits: past 2^32, a ragged last word


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


def _ascending_and_selected(p, ok):
    assert bool((p[1:] > p[:-1]).all()), "positions not strictly increasing"
    assert bool(ok.all()), "a position outside the selection"


def test_file_scan_past_2_31_rows(m, ctx):
    import torch
    g = torch.Generator(device="cuda")
    g.manual_seed(31)
    c0 = torch.randint(0, 1 << 20, (N31,), dtype=torch.int32, device="cuda", generator=g)
    t = ctx.wrap([(m.mbx.INTEGER, 4)], [c0.data_ptr()], N31)
    lit = 1 << 16  # ~6 %: ~134 M positions
    plan = ctx.compile(t, [[(m.mbx.LT, ("sym", 1), ("int", lit))]])
    want = int((c0 < lit).sum().item())
    assert ctx.scan_count(plan) == want
    # COUNT / SUM / MIN / MAX of the selected rows (int64 sum)
    sel = c0 < lit  # (boolean indexing of > 2^31 elements fails in torch: masked reductions instead)
    agg = ctx.scan_aggregate(plan, 0)
    assert agg == dict(count=want, sum=int(torch.where(sel, c0, 0).sum(dtype=torch.int64).item()),
                       min=int(torch.where(sel, c0, (1 << 31) - 1).min().item()),
                       max=int(torch.where(sel, c0, -(1 << 31)).max().item()))
    del sel
    bm = ctx.bitmap_alloc(N31)
    ids = torch.zeros(want + 64, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # torch's fills (its stream) before the library's launch (the context stream)
    ctx.scan_select_async(plan, bm, ids.data_ptr(), cnt.data_ptr())
    ctx.sync()
    assert int(cnt.item()) == want
    p = ids[:want]
    _ascending_and_selected(p, (p >= 0) & (p < N31) & (c0[p.clamp(0, N31 - 1)] < lit))
    assert int(p[-1]) >= 1 << 31
    assert bm.count in (want, -1)
    del c0, ids, p, t, plan, bm
    torch.cuda.empty_cache()


def test_index_scan_past_2_32_bits(m, ctx):
    import torch
    nw = (N32 + 63) // 64
    g = torch.Generator(device="cuda")
    g.manual_seed(32)
    ops = [torch.randint(-(1 << 63), (1 << 63) - 1, (nw,), dtype=torch.int64, device="cuda", generator=g)
           for _ in range(4)]
    anded = ops[0] & ops[1] & ops[2] & ops[3]  # ~1/16 of the bits
    tail = N32 % 64
    anded[-1] &= (1 << tail) - 1
    want = int(np.bitwise_count(anded.cpu().numpy().view(np.uint64)).sum())
    bms = [ctx.bitmap_upload(N32, w.cpu().numpy().view(np.uint64)) for w in ops]
    col = torch.randint(-(1 << 31), (1 << 31) - 1, (N32,), dtype=torch.int32, device="cuda", generator=g)
    t = ctx.wrap([(m.mbx.INTEGER, 4)], [col.data_ptr()], N32)
    ids = torch.zeros(want + 64, dtype=torch.int64, device="cuda")
    out = torch.zeros(want + 64, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    # four one-BitSet conjuncts: a & b & c & d
    torch.cuda.synchronize()  # torch's fills (its stream) before the library's launch (the context stream)
    ctx.cnf_materialize_async(t, [[b] for b in bms], [0], ids.data_ptr(), [out.data_ptr()], cnt.data_ptr())
    ctx.sync()
    assert int(cnt.item()) == want
    p = ids[:want].clone()
    q = p.clamp(0, N32 - 1)
    bit = torch.bitwise_right_shift(anded[q >> 6], q & 63) & 1
    _ascending_and_selected(p, (p >= 0) & (p < N32) & (bit == 1))
    assert int(p[-1]) >= 1 << 32
    assert bool((out[:want] == col[q]).all()), "projected values differ from the column"
    # positions only (write-through stores, the other launch form)
    ids.zero_()
    cnt.zero_()
    torch.cuda.synchronize()
    ctx.cnf_materialize_async(t, [[b] for b in bms], [], ids.data_ptr(), [], cnt.data_ptr())
    ctx.sync()
    assert int(cnt.item()) == want and bool((ids[:want] == p).all())
    del ops, anded, col, ids, out, p, q, bit, t, bms
    torch.cuda.empty_cache()
