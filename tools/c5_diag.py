#!/usr/bin/env python3
"""C5 diagnostic: per-conjunct kernel counts vs torch counts over the same
device columns, at several table sizes (one JSON line per size/term)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    import torch
    import helpers
    import mbx_pkg
    import oracle
    m = mbx_pkg.load()
    M = m.mbx
    ctx = m.Context(0)
    names = [f"{chr(65 + (i * 7) % 26)}{'abcdefghijklmnop'[:(i % 15) + 1]}"[:16] for i in range(50)]
    dic = torch.from_numpy(helpers.encode_strings(names, 16).reshape(50, 16)).cuda()
    name_ok = torch.tensor([oracle.java_mutf8(s) >= b"M" for s in names], device="cuda")
    for n in map(int, sys.argv[1].split(",")):
        g = torch.Generator(device="cuda")
        g.manual_seed(1234)
        c0 = torch.randint(0, 1 << 20, (n,), dtype=torch.int32, device="cuda", generator=g)
        c1 = torch.rand(n, dtype=torch.float32, device="cuda", generator=g)
        idx = torch.randint(0, 50, (n,), dtype=torch.int32, device="cuda", generator=g)
        c2 = helpers.device_dictionary_column(dic, idx)
        print(json.dumps({"rows": n, "stage": "generated"}), flush=True)
        torch.cuda.synchronize()
        t = ctx.wrap([(M.INTEGER, 4), (M.REAL, 4), (M.STRING, 16)], [c0.data_ptr(), c1.data_ptr(), c2.data_ptr()], n)
        terms = {"c0": ([[(M.LT, ("sym", 1), ("int", 1 << 19))]], c0 < (1 << 19)),
                 "c1": ([[(M.GE, ("sym", 2), ("real", 0.25))]], c1 >= 0.25),
                 "c2": ([[(M.GE, ("sym", 3), ("str", "M"))]], name_ok[idx.long()]),
                 "c2_first_byte": (None, c2[:, 0] >= ord("M")),
                 "idx_hist_lo": (None, idx < 25)}
        for k, (cnf, mask) in terms.items():
            got = ctx.scan_count(ctx.compile(t, cnf)) if cnf else None
            want = int(mask.sum())
            print(json.dumps({"rows": n, "term": k, "kernel": got, "torch": want}), flush=True)
        for gen in ("0", "1"):
            os.environ["MBX_FORCE_GENERIC"] = gen
            got = ctx.scan_count(ctx.compile(t, terms["c2"][0]))
            print(json.dumps({"rows": n, "term": "c2", "generic": gen, "kernel": got}), flush=True)
        os.environ.pop("MBX_FORCE_GENERIC")
        t.close()
        del c0, c1, c2, idx
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
