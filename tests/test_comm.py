"""The multi-GPU exchange step behind the C-ABI (include/mbx.h, mbx_comm_*):
row-range shard bounds, RCCL collectives on a context's exchange stream, and
HIP-graph capture of a repeated scan + exchange.

The GPU box has one MI355X, so the RCCL tests run one-rank cliques (through
both mbx_comm_init_rank and mbx_comm_init_all): the combine there must equal
the host-side fold of dist.py bit for bit.  The N-rank data flow (shards,
global positions, rank-ordered folds) is covered by tests/test_dist.py over
gloo and by bench.py's strong-scaling run, whose global COUNT is asserted
against the unsharded table at every N.
"""
import numpy as np
import pytest

import helpers  # noqa: F401  (puts oracle/ on sys.path)
import mbx_pkg
import oracle


@pytest.fixture(scope="module")
def m():
    return mbx_pkg.load()


@pytest.mark.parametrize("world", [1, 2, 3, 7, 8])
def test_c_shard_bounds_match_dist(m, world):
    """mbx_shard_bounds (C) == dist.shard_bounds (the Python restatement the
    gloo tests use), 64-aligned, tiling [0, nrows)."""
    for n in [0, 1, 63, 64, 65, 1000, 100_003, 100_000_000, 1_000_000_000]:
        for r in range(world):
            assert m.mbx.shard_bounds(n, world, r) == m.dist.shard_bounds(n, world, r), (n, world, r)


def test_c_shard_bounds_rejects_bad_arguments(m):
    for args in [(-1, 2, 0), (10, 0, 0), (10, 2, 2), (10, 2, -1)]:
        with pytest.raises(m.MbxError):
            m.mbx.shard_bounds(*args)


# ---------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    return torch


def _table(m, ctx, n=1_000_003, seed=3):
    rng = np.random.Generator(np.random.PCG64(seed))
    cols = [(oracle.INTEGER, 4, rng.integers(-1000, 1000, n, dtype=np.int32)),
            (oracle.REAL, 4, (rng.random(n, dtype=np.float32) - 0.5) * 100)]
    return cols, ctx.stage(cols, row_offset=0)


CNF = [[(oracle.GT, ("sym", 1), ("int", -100))], [(oracle.LT, ("sym", 2), ("real", 10.0))]]


@pytest.mark.gpu
@pytest.mark.parametrize("init", ["rank", "all"])
def test_one_rank_rccl_combine_is_exact(m, torch_cuda, init):
    """COUNT all-reduce, the aggregate all-gather + rank-ordered device fold
    and the count all-gather on a one-rank clique equal dist.fold_aggregates
    of the same records bit for bit."""
    torch = torch_cuda
    ctx = m.Context(0)
    try:
        cols, t = _table(m, ctx)
        plan = ctx.compile(t, CNF)
        if init == "rank":
            comm = ctx.comm_init_rank(1, 0, m.mbx.comm_unique_id())
        else:
            (comm,) = m.mbx.comm_init_all([ctx])
        want = ctx.scan_count(plan)
        buf = torch.zeros(4, dtype=torch.int64, device="cuda")
        allc = torch.zeros(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()  # torch's zero fills run on its own stream, not the library's
        ctx.scan_count_async(plan, buf.data_ptr())
        comm.allreduce_count_async(buf.data_ptr(), 1)
        comm.allgather_count_async(buf.data_ptr(), allc.data_ptr())
        ctx.sync()
        assert int(buf[0]) == want and int(allc[0]) == want
        for col in (0, 1):
            rec = torch.zeros(6, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            ctx.scan_aggregate_async(plan, col, rec.data_ptr())
            ctx.sync()
            local = rec.cpu().numpy().copy()
            if init == "rank":
                comm.allreduce_agg_async(rec.data_ptr())
            else:
                m.mbx.comm_allreduce_agg_all([comm], [rec.data_ptr()])
            ctx.sync()
            folded = m.dist.fold_aggregates(local)
            got = m.dist.fold_aggregates(rec.cpu().numpy())
            assert got == folded
            ref = oracle.aggregate(oracle.Table(cols), CNF, col)
            assert got["count"] == ref["count"] and got["min"] == ref["min"] and got["max"] == ref["max"]
        if init == "all":
            m.mbx.comm_allreduce_count_all([comm], [buf.data_ptr()], 1)
            ctx.sync()
            assert int(buf[0]) == want
    finally:
        ctx.close()


@pytest.mark.gpu
def test_comm_rejects_misuse(m):
    ctx = m.Context(0)
    try:
        with pytest.raises(m.MbxError):
            ctx.comm_init_rank(2, 2, m.mbx.comm_unique_id())
        comm = ctx.comm_init_rank(1, 0, m.mbx.comm_unique_id())
        with pytest.raises(m.MbxError):  # one communicator per context
            ctx.comm_init_rank(1, 0, m.mbx.comm_unique_id())
        with pytest.raises(m.MbxError):
            m.mbx.comm_init_all([ctx])
        comm.close()
        ctx2 = m.Context(0)
        with pytest.raises(m.MbxError):  # one device, two ranks
            m.mbx.comm_init_all([ctx, ctx2])
        ctx2.close()
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("with_comm", [False, True])
def test_graph_replays_scan_and_exchange(m, torch_cuda, with_comm):
    """A captured batch of steps (scan -> exchange each, as bench.py times
    them) replays to the same counts as the eager calls, launch after
    launch; a NaN-free plan leaves mbx_sync clean."""
    torch = torch_cuda
    ctx = m.Context(0)
    try:
        cols, t = _table(m, ctx, n=3_000_017)
        plan = ctx.compile(t, CNF)
        comm = ctx.comm_init_rank(1, 0, m.mbx.comm_unique_id()) if with_comm else None
        want = ctx.scan_count(plan)
        k = 7
        buf = torch.zeros(k, dtype=torch.int64, device="cuda")
        ctx.scan_count_async(plan, buf.data_ptr())  # sizes scratch before the capture
        ctx.sync()
        ctx.graph_begin()
        for i in range(k):
            ctx.scan_count_async(plan, buf.data_ptr() + 8 * i)
            if comm is not None:
                comm.allreduce_count_async(buf.data_ptr() + 8 * i, 1)
        g = ctx.graph_end()
        ctx.sync()
        for _ in range(3):
            buf.zero_()
            torch.cuda.synchronize()
            g.launch()
            ctx.sync()
            assert buf.cpu().tolist() == [want] * k
        with pytest.raises(m.MbxError):  # no nested capture / sync inside a capture
            ctx.graph_begin()
            ctx.graph_begin()
        with pytest.raises(m.MbxError):
            ctx.sync()
        ctx.graph_end().close()
        g.close()
    finally:
        ctx.close()


INT_CNFS = [
    [[(oracle.LT, ("sym", 1), ("int", 1 << 19))], [(oracle.GE, ("sym", 2), ("int", 1 << 19))]],
    [[(oracle.EQ, ("sym", 1), ("int", 7)), (oracle.GT, ("sym", 2), ("int", 1000))]],
]


@pytest.mark.gpu
@pytest.mark.parametrize("deleted", [False, True])
def test_comm_scan_count_parts_and_exchange(m, torch_cuda, deleted):
    """mbx_comm_scan_count_async (one-rank clique): the scan leaves one count
    per block in dev_parts, the exchange stream sums and all-reduces them --
    equal to the scan's own COUNT for int plans, eagerly and replayed from a
    graph; a float plan keeps the finalize (scan, then the collective); too
    small a parts buffer is refused"""
    torch = torch_cuda
    ctx = m.Context(0)
    try:
        n = 3_000_017
        cols = [(oracle.INTEGER, 4, c) for c in helpers.synthetic_int_table(n, 2, hi=1 << 20, seed=9)]
        cols.append((oracle.REAL, 4, np.random.Generator(np.random.PCG64(2)).random(n, dtype=np.float32)))
        dele = helpers.random_deleted(n, 0.05, seed=4) if deleted else None
        t = ctx.stage(cols, dele, row_offset=128)
        comm = ctx.comm_init_rank(1, 0, m.mbx.comm_unique_id())
        cap = 2048
        parts = torch.zeros(8 * cap, dtype=torch.int64, device="cuda")
        out = torch.zeros(8, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        float_cnf = [[(oracle.LT, ("sym", 1), ("int", 1 << 19))], [(oracle.LT, ("sym", 3), ("real", 0.25))]]
        plans = [ctx.compile(t, cnf) for cnf in INT_CNFS] + [ctx.compile(t, float_cnf)]
        wants = [ctx.scan_count(p) for p in plans]
        for i, p in enumerate(plans):
            comm.scan_count_async(p, parts.data_ptr() + 8 * cap * i, cap, out.data_ptr() + 8 * i)
        ctx.sync()
        assert out[:len(plans)].cpu().tolist() == wants
        # a graph of the int queries, replayed
        ctx.graph_begin()
        for i, p in enumerate(plans[:2]):
            comm.scan_count_async(p, parts.data_ptr() + 8 * cap * (4 + i), cap, out.data_ptr() + 8 * (4 + i))
        g = ctx.graph_end()
        for _ in range(3):
            out.zero_()
            torch.cuda.synchronize()
            g.launch()
            ctx.sync()
            assert out[4:6].cpu().tolist() == wants[:2]
        g.close()
        with pytest.raises(m.MbxError):
            comm.scan_count_async(plans[0], parts.data_ptr(), 4, out.data_ptr())
        ctx.sync()
    finally:
        ctx.close()


def _records(m, kind, n, seed):
    """n rank records of one aggregate kind, rank 1 and rank n-2 empty shards
    (count 0 and the identities the scan writes for them); float partial sums
    spread over 1e-3..1e16 so that only the rank-order fold reproduces them."""
    rng = np.random.Generator(np.random.PCG64(seed))
    recs = np.zeros(n, dtype=m.dist.AGG_RECORD)
    for r in range(n):
        empty = n > 2 and r in (1, n - 2)
        if kind == "int":
            lo, hi = sorted(int(x) for x in rng.integers(-2 ** 31, 2 ** 31 - 1, 2))
            agg = dict(count=0, sum=0, min=2 ** 31 - 1, max=-2 ** 31) if empty else dict(
                count=int(rng.integers(1, 1 << 40)), sum=int(rng.integers(-(1 << 60), 1 << 60)), min=lo, max=hi)
        else:
            lo, hi = sorted(float(np.float32(x)) for x in rng.normal(0, 1e6, 2))
            agg = dict(count=0, sum=0.0, min=float("inf"), max=float("-inf")) if empty else dict(
                count=int(rng.integers(1, 1 << 40)), sum=float(rng.choice([1e16, -1e16, 1.0, 3.3e-3, 7.77e8])
                                                          * rng.random()), min=lo, max=hi)
        recs[r] = m.dist.pack_aggregate(agg, kind == "int")[0]
    return recs


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["int", "float"])
@pytest.mark.parametrize("n", [1, 2, 8])
def test_device_fold_of_n_rank_records_is_exact(m, torch_cuda, kind, n):
    """mbx_agg_fold_async -- the fold the aggregate exchange runs after its
    RCCL all-gather -- over n gathered records (n = 8: the driver's 8-GPU
    C5 combine, run here without RCCL), with empty shards: equal to
    dist.fold_aggregates bit for bit, also folded in place."""
    torch = torch_cuda
    ctx = m.Context(0)
    try:
        recs = _records(m, kind, n, seed=10 * n + (kind == "int"))
        want = m.dist.fold_aggregates(recs)
        dev = torch.from_numpy(recs.view(np.int64).copy()).cuda()
        out = torch.zeros(m.dist.AGG_WORDS, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        ctx.agg_fold_async(dev.data_ptr(), n, out.data_ptr())
        ctx.agg_fold_async(dev.data_ptr(), n, dev.data_ptr())  # in place over record 0
        ctx.sync()
        for got_words in (out.cpu().numpy(), dev.cpu().numpy()[:m.dist.AGG_WORDS]):
            got = m.dist.fold_aggregates(got_words)
            assert got == want
            if kind == "float":
                assert np.float64(got["sum"]).tobytes() == np.float64(want["sum"]).tobytes()
        with pytest.raises(m.MbxError):
            ctx.agg_fold_async(dev.data_ptr(), 0, out.data_ptr())
    finally:
        ctx.close()
