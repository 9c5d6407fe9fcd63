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


# ---- DB-file shards (mbx_db_stage_range): C4- and C5-shaped Columnarfiles

C4_CNF = [[(oracle.EQ, ("sym", 3), ("int", 3))], [(oracle.EQ, ("sym", 4), ("int", 7)),
                                                   (oracle.LT, ("sym", 4), ("int", 1))]]
C5_CNF = [[(oracle.LT, ("sym", 1), ("int", 1 << 19))], [(oracle.GE, ("sym", 2), ("real", 0.25))],
          [(oracle.GE, ("sym", 3), ("str", "M"))]]
NAMES = ["Alabama", "Colorado", "Iowa", "Maine", "Montana", "Ohio", "South_Dakota", "Texas", "Utah", "Zed"]


def c4_columns(n, seed=4):
    """C4 shape: c0, c1 int32 uniform [0, 2^20); c2, c3 in [0, 10)"""
    rng = np.random.Generator(np.random.PCG64(seed))
    return [(oracle.INTEGER, 4, rng.integers(0, 1 << 20, n, dtype=np.int32)) for _ in range(2)] + \
           [(oracle.INTEGER, 4, rng.integers(0, 10, n, dtype=np.int32)) for _ in range(2)]


def c5_columns(n, seed=5):
    """C5 shape: int32 c0 [0, 2^20), float c1 [0, 1), char(16) c2 of a dictionary"""
    rng = np.random.Generator(np.random.PCG64(seed))
    return [(oracle.INTEGER, 4, rng.integers(0, 1 << 20, n, dtype=np.int32)),
            (oracle.REAL, 4, rng.random(n, dtype=np.float32)),
            (oracle.STRING, 16, helpers.encode_strings([NAMES[i] for i in rng.integers(0, len(NAMES), n)], 16))]


def write_db(m, path, cols, names, deleted_every=0):
    with m.mbx.Db(path, 1 << 17) as db:
        db.columnar_create("cf", [(t, s) for t, s, _ in cols], names)
        db.columnar_insert("cf", cols)
        if deleted_every:
            db.mark_deleted_many("cf", np.arange(0, len(cols[0][2]), deleted_every, dtype=np.int64))


def run_db(rank, world, port, executor, c4_path, c5_path):
    """Each rank owns positions [s, e) of both DB files (dist.shard_bounds):
    C4 -- the ColumnarIndexScan CNF's positions + projected c0, c1;
    C5 -- COUNT/SUM/MIN/MAX of c1 under the 3-conjunct filter.  One combine
    each (counts -> concatenation offsets, positions / rows in rank order;
    the 48-byte aggregate records folded in rank order) must equal the
    whole-file oracle answer."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = mbx_pkg.load()
    D = m.dist
    import minibase_pages as mp
    n4, cols4, del4 = mp.columnar_table(mp.DbImage(c4_path), "cf")
    n5, cols5, del5 = mp.columnar_table(mp.DbImage(c5_path), "cf")
    s4, e4 = D.shard_bounds(n4, world, rank)
    s5, e5 = D.shard_bounds(n5, world, rank)
    if executor == "oracle":  # the shard as the reader restatement decodes it
        sh4 = oracle.Table([(t, z, a[s4:e4]) for t, z, a in cols4], del4[s4 // 64:(e4 + 63) // 64].copy())
        k, w = oracle.columnar_index_scan(sh4, C4_CNF)
        ids = oracle.words_to_positions(w)
        v0, v1 = oracle.gather(sh4, ids, [0, 1])
        ids = ids + s4
        sh5 = oracle.Table([(t, z, a[s5:e5]) for t, z, a in cols5], del5[s5 // 64:(e5 + 63) // 64].copy())
        agg = oracle.aggregate(sh5, C5_CNF, 1)
    else:  # every rank on cuda:0: the shard staged from the DB file by range
        ctx = m.Context(0)
        with m.mbx.Db(c4_path) as db:
            t = ctx.stage_db_range(db, "cf", s4, e4)
            assert (t.row_offset, t.nrows) == (s4, e4 - s4)
            regs = {}
            for c in (2, 3):
                vals = [int(v) for v in db.bitmap_values("cf", c)]
                regs[c] = {v: ctx.stage_db_bitmap_range(db, f"cf.bm.{c}.{v}", s4, e4 - s4) for v in vals}
            dele = ctx.stage_db_bitmap_range(db, "cf.md", s4, e4 - s4)
        conj = helpers.index_conjuncts(regs, C4_CNF, [oracle.INTEGER] * 4)
        cur = ctx.cnf_cursor(t, conj, [0, 1], deleted=dele)
        ids, (v0, v1) = cur.next(max(1, e4 - s4))
        with m.mbx.Db(c5_path) as db:
            t5 = ctx.stage_db_range(db, "cf", s5, e5)
        agg = ctx.scan_aggregate(ctx.compile(t5, C5_CNF), 1)
    all_ids = D.gather_positions(ids)
    all_v0 = D.gather_positions(np.asarray(v0, dtype=np.int64))
    all_v1 = D.gather_positions(np.asarray(v1, dtype=np.int64))
    total = D.combine_count(len(ids))
    g5 = D.combine_aggregate(agg)
    ft4 = oracle.Table(cols4, del4)
    k_o, w_o = oracle.columnar_index_scan(ft4, C4_CNF)
    ids_o = oracle.words_to_positions(w_o)
    assert total == k_o and np.array_equal(all_ids, ids_o)
    o0, o1 = oracle.gather(ft4, ids_o, [0, 1])
    assert np.array_equal(all_v0, o0) and np.array_equal(all_v1, o1)
    a5 = oracle.aggregate(oracle.Table(cols5, del5), C5_CNF, 1)
    assert g5["count"] == a5["count"] and g5["min"] == a5["min"] and g5["max"] == a5["max"]
    assert abs(g5["sum"] - a5["sum"]) <= 1e-6 * abs(a5["sum"])
    dist.barrier()
    dist.destroy_process_group()
