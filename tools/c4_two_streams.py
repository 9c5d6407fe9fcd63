#!/usr/bin/env python3
"""C4 (ColumnarIndexScan: bm(c2=3) AND bm(c3=7) -> positions + c0, c1 with
the (c0, c1) column group, 100M rows) queries on one stream vs alternating
over two contexts: the next query's operand-word phase can then run under
the previous query's gathers (the overlap one launch cannot give itself,
DESIGN.md section 3).  Each context wraps the same device columns, builds
its own BitMapFiles and group, and writes its own outputs; every query's
count is checked against torch, the outputs of the last query of each
context against torch's selection.  Forms as tools/c3_two_streams.py."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mbx_pkg
    m = mbx_pkg.load()
    M = m.mbx
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    cols = [torch.randint(0, hi, (n,), dtype=torch.int32, device="cuda", generator=g)
            for hi in (1 << 20, 1 << 20, 10, 10)]
    sel = (cols[2] == 3) & (cols[3] == 7)
    want = int(sel.sum().item())
    wids = torch.nonzero(sel).flatten()
    ctxs = [m.Context(0), m.Context(0)]
    st = []
    for c in ctxs:
        t = c.wrap([(M.INTEGER, 4)] * 4, [x.data_ptr() for x in cols], n)
        a = c.index_build(t, 2, [("int", 3)])[0]
        b = c.index_build(t, 3, [("int", 7)])[0]
        c.group(t, [0, 1])
        outs = [torch.zeros(want + 64, dtype=dt, device="cuda") for dt in (torch.int64, torch.int32, torch.int32)]
        st.append((t, a, b, outs))
    counts = torch.zeros(K, dtype=torch.int64, device="cuda")
    base = counts.data_ptr()
    torch.cuda.synchronize()

    def launch(i, k):
        t, a, b, (ids, o0, o1) = st[i]
        ctxs[i].cnf_materialize_async(t, [[a], [b]], [0, 1], ids.data_ptr(), [o0.data_ptr(), o1.data_ptr()],
                                      base + 8 * k)

    def sync_all():
        for c in ctxs:
            c.sync()
        torch.cuda.synchronize()

    def check(tag, used):
        got = counts.cpu().tolist()
        bad = any(x != want for x in got)
        for i in used:
            ids, o0, o1 = st[i][3]
            bad = bad or not (bool((ids[:want] == wids).all()) and bool((o0[:want] == cols[0][sel]).all())
                              and bool((o1[:want] == cols[1][sel]).all()))
        if bad:
            print(json.dumps({"form": tag, "error": "counts or rows differ from torch"}), flush=True)
            sys.exit(1)
        counts.zero_()
        torch.cuda.synchronize()

    ctxs[0].graph_begin()
    for k in range(K):
        launch(0, k)
    g_one = ctxs[0].graph_end()
    halves = []
    for i, c in enumerate(ctxs):
        c.graph_begin()
        for k in range(i, K, 2):
            launch(i, k)
        halves.append(c.graph_end())

    forms = [("one", lambda: g_one.launch()), ("two", lambda: (halves[0].launch(), halves[1].launch())),
             ("eager2", lambda: [launch(k % 2, k) for k in range(K)])]
    used = {"one": [0], "two": [0, 1], "eager2": [0, 1]}  # the contexts whose outputs a form wrote
    for name, f in forms:
        f()
        sync_all()
        check(name, used[name])
    for rep in range(5):
        for name, f in forms:
            sync_all()
            t0 = time.perf_counter()
            f()
            sync_all()
            dt = time.perf_counter() - t0
            check(name, used[name])
            print(json.dumps({"form": name, "rep": rep, "K": K, "us_per_query": dt / K * 1e6}), flush=True)
    for gr in [g_one] + halves:
        gr.close()
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
