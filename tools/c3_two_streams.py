#!/usr/bin/env python3
"""C3 steps on one stream vs alternating over two contexts (two streams,
each with its own tickets and look-back state): does the next query's scan
filling the CUs the previous one's tail leaves idle (and hiding the launch
boundary) raise the step rate?  Same table (zero-copy wraps of the same
device columns), same plan, every step's COUNT checked against torch.
Forms, each timed as wall time of K steps between device-wide syncs:
  one     : one HIP graph of K scans on one stream (bench.py's form)
  two     : two graphs of K/2 scans (even / odd steps), one per context,
            launched back to back, so they run concurrently
  eager2  : K eager launches alternating between the two contexts
One JSON line per form and repetition."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

THRESH = 1 << 19


def main():
    import torch
    import mbx_pkg
    m = mbx_pkg.load()
    M = m.mbx
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    cols = []
    for j in range(4):
        g = torch.Generator(device="cuda")
        g.manual_seed(42 + j)
        cols.append(torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g))
    want = int(((cols[0] < THRESH) & (cols[1] >= THRESH)).sum().item())
    ctxs = [m.Context(0), m.Context(0)]
    cnf = [[(M.LT, ("sym", 1), ("int", THRESH))], [(M.GE, ("sym", 2), ("int", THRESH))]]
    tabs = [c.wrap([(M.INTEGER, 4)] * 4, [x.data_ptr() for x in cols], n) for c in ctxs]
    plans = [c.compile(t, cnf) for c, t in zip(ctxs, tabs)]
    counts = torch.zeros(K, dtype=torch.int64, device="cuda")
    base = counts.data_ptr()
    torch.cuda.synchronize()

    def sync_all():
        for c in ctxs:
            c.sync()
        torch.cuda.synchronize()

    def check(tag):
        got = counts.cpu().tolist()
        if any(x != want for x in got):
            print(json.dumps({"form": tag, "error": f"counts {got[:4]}... != {want}"}), flush=True)
            sys.exit(1)
        counts.zero_()
        torch.cuda.synchronize()

    # graphs
    ctxs[0].graph_begin()
    for k in range(K):
        ctxs[0].scan_count_async(plans[0], base + 8 * k)
    g_one = ctxs[0].graph_end()
    halves = []
    for i, c in enumerate(ctxs):
        c.graph_begin()
        for k in range(i, K, 2):
            c.scan_count_async(plans[i], base + 8 * k)
        halves.append(c.graph_end())

    def run_one():
        g_one.launch()

    def run_two():
        halves[0].launch()
        halves[1].launch()

    def run_eager2():
        for k in range(K):
            ctxs[k % 2].scan_count_async(plans[k % 2], base + 8 * k)

    forms = [("one", run_one), ("two", run_two), ("eager2", run_eager2)]
    for f in forms:  # warm-up + check
        f[1]()
        sync_all()
        check(f[0])
    for rep in range(5):
        for name, f in forms:
            sync_all()
            t0 = time.perf_counter()
            f()
            sync_all()
            dt = time.perf_counter() - t0
            check(name)
            print(json.dumps({"form": name, "rep": rep, "K": K, "us_per_step": dt / K * 1e6,
                              "rows_per_s": n * K / dt}), flush=True)
    for g in [g_one] + halves:
        g.close()
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
