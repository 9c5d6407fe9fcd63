#!/usr/bin/env python3
"""PCIe-inclusive rate of the C3 query: the boundary hands the
library host arrays (mbx_table_stage copies them to HBM), so a query whose
table is not resident yet pays the host -> HBM copy.  Times, on the C3 table
(100M rows x 4 int32, the 2 referenced columns staged or all 4):
  stage_s   mbx_table_stage of pageable numpy arrays (hipMalloc + H2D copies)
  stage_pinned_s  the same from page-locked host memory (torch.pin_memory)
  scan_ms   the resident COUNT scan (bench.py's step)
and reports rows/s with the staging included next to the resident rate.
One JSON line per (columns staged, host memory kind)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch

    import mbx_pkg

    m = mbx_pkg.load()
    M = m.mbx
    torch.cuda.init()
    ctx = m.Context(0)
    n = 100_000_000
    rng = [np.random.Generator(np.random.PCG64(42 + j)) for j in range(4)]
    host = [r.integers(0, 1 << 20, size=n, dtype=np.int32) for r in rng]
    want = int(np.count_nonzero((host[0] < (1 << 19)) & (host[1] >= (1 << 19))))
    cnf = [[(M.LT, ("sym", 1), ("int", 1 << 19))], [(M.GE, ("sym", 2), ("int", 1 << 19))]]
    for ncols in (2, 4):
        for kind in ("pageable", "pinned"):
            if kind == "pinned":
                arrs = [torch.from_numpy(h).pin_memory().numpy() for h in host[:ncols]]
            else:
                arrs = host[:ncols]
            cols = [(M.INTEGER, 4, a) for a in arrs]
            best = None
            for _ in range(3):
                t0 = time.perf_counter()
                t = ctx.stage(cols)
                ctx.sync()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
                plan = ctx.compile(t, cnf)
                got = ctx.scan_count(plan)
                assert got == want, (got, want)
                t.close()
            t = ctx.stage(cols)
            plan = ctx.compile(t, cnf)
            out = torch.zeros(1, dtype=torch.int64, device="cuda")
            ext = torch.cuda.ExternalStream(ctx.stream)
            for _ in range(5):
                ctx.scan_count_async(plan, out.data_ptr())
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(ext)
            for _ in range(50):
                ctx.scan_count_async(plan, out.data_ptr())
            b.record(ext)
            ctx.sync()
            scan_ms = a.elapsed_time(b) / 50
            t.close()
            byts = ncols * 4 * n
            print(json.dumps({"columns_staged": ncols, "host_memory": kind, "stage_s": best,
                              "h2d_gbs": byts / best / 1e9, "scan_ms": scan_ms,
                              "rows_per_s_resident": n / (scan_ms * 1e-3),
                              "rows_per_s_pcie_inclusive": n / (best + scan_ms * 1e-3)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
