#!/usr/bin/env python3
"""Per-block timeline of C4's one-launch ColumnarIndexScan (k_cnf_select,
(c0, c1) column group, positions + c0, c1): wall_clock64() stamps at block
start / count published / offset known / end (tuning select_dbg bit 3,
mbx_diag_select_stamps), as percentiles in us from the earliest block start,
for a projection and for positions only.  The stamps' own stores move the
times a little; the kernel time without them is profiles/r05/scripts/c4_forms.py's."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import mbx_pkg
    m = mbx_pkg.load()
    M = m.mbx
    L = M.lib()
    ctx = m.Context(0)
    n = 100_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(42)
    c = [torch.randint(0, hi, (n,), dtype=torch.int32, device="cuda", generator=g)
         for hi in (1 << 20, 1 << 20, 10, 10)]
    t = ctx.wrap([(M.INTEGER, 4)] * 4, [x.data_ptr() for x in c], n)
    a = ctx.index_build(t, 2, [("int", 3)])[0]
    b = ctx.index_build(t, 3, [("int", 7)])[0]
    ctx.group(t, [0, 1])
    k = int(((c[2] == 3) & (c[3] == 7)).sum().item())
    ids = torch.zeros(k + 64, dtype=torch.int64, device="cuda")
    o0 = torch.zeros(k + 64, dtype=torch.int32, device="cuda")
    o1 = torch.zeros(k + 64, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    waves = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    if waves != 4:  # round 5's 16-wave A/B (profiles/r05/p) ran a build with the cnf_waves knob, since removed
        raise SystemExit("c4_stamps: the library launches 4-wave blocks only (knob cnf_waves removed)")
    nb = 1024
    for proj, outs in (([0, 1], [o0.data_ptr(), o1.data_ptr()]), ([], [])):
        for rep in range(3):
            ctx.set_tuning("select_dbg", 8)
            torch.cuda.synchronize()
            ctx.cnf_materialize_async(t, [[a], [b]], proj, ids.data_ptr(), outs, cnt.data_ptr())
            ctx.sync()
            st = np.zeros(4 * nb, dtype=np.int64)
            M._chk(L.mbx_diag_select_stamps(ctx.h, st.ctypes.data, nb))
            ctx.set_tuning("select_dbg", 0)
            st = st.reshape(nb, 4).astype(np.float64) / 100.0  # 100 MHz -> us
            st = st[st[:, 0] > 0]
            st -= st[:, 0].min()
            pct = lambda x: [round(float(v), 2) for v in np.percentile(x, [0, 10, 50, 90, 100])]
            print(json.dumps({"waves": waves, "proj": proj, "rep": rep, "blocks": int(st.shape[0]), "count_ok": int(cnt.item()) == k,
                              "start": pct(st[:, 0]), "published": pct(st[:, 1]), "offset_known": pct(st[:, 2]),
                              "end": pct(st[:, 3]), "end_minus_offset": pct(st[:, 3] - st[:, 2]),
                              "offset_minus_published": pct(st[:, 2] - st[:, 1])}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
