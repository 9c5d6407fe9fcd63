"""Worker for the multi-rank tests (tests/test_dist.py): one process per rank,
row-range shards, torch.distributed (gloo) for the single exchange step."""
import os

import numpy as np

import helpers
import mbx_pkg
import oracle

N = 100_003
CNF = [[(oracle.LT, ("sym", 1), ("int", 300))], [(oracle.GE, ("sym", 2), ("int", 100)),
                                                  (oracle.EQ, ("sym", 3), ("int", 7))]]


def full_table():
    rng = np.random.Generator(np.random.PCG64(123))
    cols = [(oracle.INTEGER, 4, rng.integers(0, 1000, N, dtype=np.int32)) for _ in range(3)]
    cols.append((oracle.REAL, 4, rng.random(N, dtype=np.float32)))
    return cols, helpers.random_deleted(N, 0.05, seed=9)


def run(rank, world, port, executor):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = mbx_pkg.load()
    D = m.dist
    cols, dele = full_table()
    s, e = D.shard_bounds(N, world, rank)
    assert s % 64 == 0
    shard = [(t, sz, a[s:e]) for t, sz, a in cols]
    sdel = dele[s // 64:(e + 63) // 64].copy()
    if executor == "oracle":  # CPU stand-in for the per-rank scan
        ot = oracle.Table(shard, sdel)
        n, _, ids = oracle.filescan(ot, CNF)
        ids = ids + s
        agg_i, agg_f = oracle.aggregate(ot, CNF, 0), oracle.aggregate(ot, CNF, 3)
    else:  # the HIP path, every rank on cuda:0
        ctx = m.Context(0)
        t = ctx.stage(shard, sdel, row_offset=s)
        plan = ctx.compile(t, CNF)
        bm = ctx.scan_bitmap(plan)
        n = bm.count
        ids = ctx.select(bm, row_offset=s)
        agg_i, agg_f = ctx.scan_aggregate(plan, 0), ctx.scan_aggregate(plan, 3)
        ctx.close()
    total = D.combine_count(n)
    all_ids = D.gather_positions(ids)
    gi, gf = D.combine_aggregate(agg_i), D.combine_aggregate(agg_f)
    ft = oracle.Table(cols, dele)
    n_o, _, ids_o = oracle.filescan(ft, CNF)
    assert total == n_o, (total, n_o)
    assert np.array_equal(all_ids, ids_o)
    ai, af = oracle.aggregate(ft, CNF, 0), oracle.aggregate(ft, CNF, 3)
    assert gi == ai, (gi, ai)
    assert gf["count"] == af["count"] and gf["min"] == af["min"] and gf["max"] == af["max"]
    assert abs(gf["sum"] - af["sum"]) <= 1e-6 * abs(af["sum"])
    dist.barrier()
    dist.destroy_process_group()
