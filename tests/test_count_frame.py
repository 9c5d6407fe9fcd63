"""Count frames (include/mbx.h mbx_scan_count_frame_async): the ColumnarFileScan
COUNT (Query.executeFileScan's resultCount, R/input/Query.java:137-152; the
predicate is PredEval.Eval, R/iterator/PredEval.java:25-183) enqueued with no
in-launch finalize -- every block adds a packed (count, NaN block, arrival)
word into one of 32 slots of a caller-zeroed frame, and the reader (or an
all-reduce of whole frames) adds the slots.

Checked against the oracle (COUNT and the PredEval NaN order), against the
finalizing scan of the same plan, for additivity (two scans into one frame,
an RCCL one-rank all-reduce of a frame) and for the arrival bookkeeping.
"""
import numpy as np
import pytest

import helpers
import mbx_pkg
import oracle

pytestmark = pytest.mark.gpu

LT, GT, GE, EQ = oracle.LT, oracle.GT, oracle.GE, oracle.EQ
W = 512  # MBX_COUNT_FRAME_WORDS


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.fixture(scope="module")
def ctx(m):
    c = m.Context(0)
    yield c
    c.close()


def _frames(torch, k):
    return torch.zeros((k, W), dtype=torch.int64, device="cuda")


def _int_table(n, seed, deleted_frac=0.0):
    rng = np.random.Generator(np.random.PCG64(seed))
    cols = [(oracle.INTEGER, 4, rng.integers(0, 1 << 20, n, dtype=np.int32)) for _ in range(4)]
    dele = None
    if deleted_frac:
        bits = rng.random(n) < deleted_frac
        dele = np.frombuffer(np.pad(np.packbits(bits, bitorder="little"), (0, (-((n + 7) // 8)) % 8)).tobytes(),
                             dtype=np.uint64).copy()
    return cols, dele


C3 = [[(LT, ("sym", 1), ("int", 1 << 19))], [(GE, ("sym", 2), ("int", 1 << 19))]]
OR3 = [[(LT, ("sym", 1), ("int", 1000)), (GT, ("sym", 3), ("int", (1 << 20) - 5000))],
       [(GE, ("sym", 2), ("int", 1 << 18))], [(LT, ("sym", 4), ("int", 900_000))]]


@pytest.mark.parametrize("n", [1, 63, 64, 1000, 65_537, 1_000_003, 12_500_000])
@pytest.mark.parametrize("cnf", [C3, OR3], ids=["c3", "or3"])
def test_frame_count_equals_oracle(m, ctx, n, cnf):
    import torch
    cols, _ = _int_table(n, 11 + n % 7)
    t = ctx.stage(cols)
    plan = ctx.compile(t, cnf)
    fr = _frames(torch, 1)
    torch.cuda.synchronize()
    ctx.scan_count_frame_async(plan, fr.data_ptr())
    ctx.sync()
    count, nan, arr = m.mbx.count_frame_decode(fr[0].cpu().numpy())
    if n <= 1_000_003:
        want = oracle.filescan_count(oracle.Table(cols), cnf)
    else:
        want = ctx.scan_count(plan)
    assert count == want == ctx.scan_count(plan)
    assert nan == 0
    assert arr == ctx.scan_blocks(plan)
    # only slot words carry data; the rest of each 128-byte line stays zero
    h = fr[0].cpu().numpy().reshape(32, 16)
    assert not h[:, 1:].any()


def test_frame_with_deleted_rows(m, ctx):
    import torch
    n = 300_001
    cols, dele = _int_table(n, 5, deleted_frac=0.1)
    t = ctx.stage(cols, dele)
    plan = ctx.compile(t, C3)
    fr = _frames(torch, 1)
    torch.cuda.synchronize()
    ctx.scan_count_frame_async(plan, fr.data_ptr())
    ctx.sync()
    count, _, _ = m.mbx.count_frame_decode(fr[0].cpu().numpy())
    assert count == oracle.filescan_count(oracle.Table(cols, dele), C3)


def test_frames_are_additive(m, ctx):
    """Two scans into one frame add; a frame all-reduced over a one-rank RCCL
    clique decodes to the same count (the exchange sums whole frames)."""
    import torch
    cols, _ = _int_table(2_000_000, 9)
    t = ctx.stage(cols)
    plan = ctx.compile(t, C3)
    want = ctx.scan_count(plan)
    fr = _frames(torch, 2)
    torch.cuda.synchronize()
    ctx.scan_count_frame_async(plan, fr[0].data_ptr())
    ctx.scan_count_frame_async(plan, fr[0].data_ptr())
    ctx.scan_count_frame_async(plan, fr[1].data_ptr())
    comm = ctx.comm_init_rank(1, 0, m.mbx.comm_unique_id())
    try:
        comm.allreduce_count_async(fr.data_ptr(), 2 * W)
        ctx.sync()
    finally:
        comm.close()
    a = m.mbx.count_frame_decode(fr[0].cpu().numpy())
    b = m.mbx.count_frame_decode(fr[1].cpu().numpy())
    nb = ctx.scan_blocks(plan)
    assert a == (2 * want, 0, 2 * nb)
    assert b == (want, 0, nb)


def test_frame_in_a_graph(m, ctx):
    """Captured and replayed (the bench's timed form): every replay adds."""
    import torch
    cols, _ = _int_table(1_000_000, 4)
    t = ctx.stage(cols)
    plan = ctx.compile(t, C3)
    want = ctx.scan_count(plan)
    fr = _frames(torch, 3)
    torch.cuda.synchronize()
    ctx.sync()
    ctx.graph_begin()
    try:
        for k in range(3):
            ctx.scan_count_frame_async(plan, fr[k].data_ptr())
    finally:
        g = ctx.graph_end()
    g.launch()
    g.launch()
    ctx.sync()
    g.close()
    for k in range(3):
        assert m.mbx.count_frame_decode(fr[k].cpu().numpy())[0] == 2 * want


def test_frame_nan_follows_predeval_order(m, ctx):
    """A NaN compare the PredEval order reaches is counted per block in the
    frame and raised at the next sync; one it does not reach is neither."""
    import torch
    from test_nan_order import CASES, _table
    cols, dele = _table()
    t = ctx.stage(cols, dele)
    ot = oracle.Table(cols, dele)
    for name, cnf, raises in CASES:
        plan = ctx.compile(t, cnf)
        fr = _frames(torch, 1)
        torch.cuda.synchronize()
        ctx.scan_count_frame_async(plan, fr.data_ptr())
        if raises:
            with pytest.raises(m.MbxError) as e:
                ctx.sync()
            assert e.value.code == m.mbx.E_TYPE, name
        else:
            ctx.sync()
        count, nan, arr = m.mbx.count_frame_decode(fr[0].cpu().numpy())
        assert (nan > 0) == raises, name
        if not raises:
            assert count == oracle.filescan_count(ot, cnf), name
        ctx.sync()


def test_frame_rejects_misaligned(m, ctx):
    import torch
    cols, _ = _int_table(1000, 2)
    t = ctx.stage(cols)
    plan = ctx.compile(t, C3)
    fr = _frames(torch, 1)
    with pytest.raises(m.MbxError):
        ctx.scan_count_frame_async(plan, fr.data_ptr() + 8)


def test_frame_decode_host_only(m):
    """The decode is plain host arithmetic over the 32 slot words."""
    f = np.zeros(W, dtype=np.int64)
    for s, (cnt, nan, arr) in enumerate([(5, 0, 3), (7, 1, 2), (1 << 30, 0, 255)]):
        f[16 * s] = (cnt << 24) | (nan << 12) | arr
    assert m.mbx.count_frame_decode(f) == (5 + 7 + (1 << 30), 1, 260)
