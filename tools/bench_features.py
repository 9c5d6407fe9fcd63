#!/usr/bin/env python3
"""Timings of the widened rows on one GPU, one JSON line each:

  stage     mbx_db_stage of a 10M-row 4 x int32 Columnarfile written by the
            Minibase DB writer (pages -> HBM -> k_page_decode); wall time incl.
            the host -> device copy, plus the writer's own time
  index     mbx_db_create_bitmap_index on the staged table (10 values):
            k_distinct + k_index_build4 + BitMapFile writes
  join      mbx_join BMJ and NLJ orders over 20k x 20k selections of an int
            equality + range CNF (k_join_matrix over 4e8 pairs)
Kernel durations come from rocprofv3 when run under it (tools/gpu_features.sh).
"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import mbx_pkg

    m = mbx_pkg.load()
    M = m.mbx
    ctx = m.Context(0)
    n = int(os.environ.get("FEAT_ROWS", 10_000_000))
    rng = np.random.Generator(np.random.PCG64(42))
    cols = [(M.INTEGER, 4, rng.integers(0, 1 << 20, n, dtype=np.int32)) for _ in range(3)]
    cols.append((M.INTEGER, 4, rng.integers(0, 10, n, dtype=np.int32)))
    tmp = tempfile.mkdtemp(prefix="mbx_feat_")
    path = os.path.join(tmp, "db")
    t0 = time.perf_counter()
    db = M.Db(path, 1 << 20 if n <= 20_000_000 else (n // 100) * 5)
    db.columnar_create("cf", [(t, s) for t, s, _ in cols], ["c0", "c1", "c2", "c3"])
    db.columnar_insert("cf", cols)
    write_s = time.perf_counter() - t0
    pages = db.info()[1]
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        t = ctx.stage_db(db, "cf")
        ts.append(time.perf_counter() - t0)
        if _ < 2:
            t.close()
    plan = ctx.compile(t, [[(M.LT, ("sym", 1), ("int", 1 << 19))], [(M.GE, ("sym", 2), ("int", 1 << 19))]])
    want = int(np.count_nonzero((cols[0][2] < (1 << 19)) & (cols[1][2] >= (1 << 19))))
    assert ctx.scan_count(plan) == want
    print(json.dumps({"feature": "db_stage", "rows": n, "db_pages": pages, "db_mb": pages * 1024 / 1e6,
                      "write_s": write_s, "stage_s_min": min(ts), "stage_rows_per_s": n / min(ts)}), flush=True)
    t0 = time.perf_counter()
    nv = ctx.create_bitmap_index(db, "cf", t, 3)
    idx_s = time.perf_counter() - t0
    print(json.dumps({"feature": "bitmap_index_persist", "rows": n, "values": nv, "seconds": idx_s}), flush=True)
    db.close()

    # joins: 20k x 20k selections of a 1M-row table
    nj = 1_000_000
    jc = [(M.INTEGER, 4, rng.integers(0, 5000, nj, dtype=np.int32)),
          (M.INTEGER, 4, rng.integers(0, 1000, nj, dtype=np.int32))]
    tj = ctx.stage(jc)
    sel = np.zeros((nj + 63) // 64, dtype=np.uint64)
    pick = rng.choice(nj, 20_000, replace=False)
    np.bitwise_or.at(sel, pick // 64, np.uint64(1) << (pick % 64).astype(np.uint64))
    s = ctx.bitmap_upload(nj, sel)
    cnf = [[(M.EQ, 0, 0)], [(M.LT, 1, 1)]]
    for order, name, block in ((M.JOIN_BMJ, "bmj", 0), (M.JOIN_NLJ, "nlj", 4000)):
        ctx.join(tj, s, tj, s, cnf, order, block)
        t0 = time.perf_counter()
        op_, ip_, ps, passes = ctx.join(tj, s, tj, s, cnf, order, block)
        dt = time.perf_counter() - t0
        print(json.dumps({"feature": f"join_{name}", "outer": 20_000, "inner": 20_000, "pairs_evaluated": 4e8,
                          "result_pairs": int(len(op_)), "passes": passes, "seconds": dt,
                          "pairs_per_s": 4e8 / dt}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
