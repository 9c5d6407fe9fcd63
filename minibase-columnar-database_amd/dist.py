"""Row-range sharding of one Columnarfile over ranks, and the single exchange
step of the path.

Every rank owns positions [start, end) of the logical table, with shard
boundaries on multiples of 64 rows so BitSet words never straddle ranks; its
HBM table is staged with row_offset = start so positions it returns are
global.  Rows are independent, so scans need no communication; the only
collective combines the per-rank results:

  COUNT / SUM(int)  -> all_reduce(SUM) on int64
  MIN / MAX         -> all_reduce(MIN / MAX)
  SUM(float)        -> all_gather of the per-rank double partials, summed in
                       rank order (bit-reproducible for a given world size)
  positions / rows  -> all_gather, concatenated in rank order (= ascending
                       global position order, the reference's nextSetBit order)

Backend-agnostic torch.distributed: "nccl" (RCCL over xGMI) with one process
per MI355X, "gloo" for the CPU tests.
"""
import numpy as np


def shard_bounds(nrows, world, rank, align=64):
    """[start, end) of `rank`'s row range; starts are multiples of `align`.
    Non-empty ranges tile [0, nrows) in rank order; a rank left without rows
    gets an empty range at an aligned start."""
    words = (nrows + align - 1) // align
    per = words // world
    extra = words % world
    w0 = rank * per + min(rank, extra)
    w1 = w0 + per + (1 if rank < extra else 0)
    if w0 == w1:
        s = min(w0 * align, (nrows // align) * align)
        return s, s
    return w0 * align, min(w1 * align, nrows)


def _dev(group_device):
    import torch
    return torch.device(group_device) if group_device else torch.device("cpu")


def combine_count(count, device=None, group=None):
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(count)], dtype=torch.int64, device=_dev(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item())


def combine_aggregate(agg, device=None, group=None):
    """agg: dict(count, sum, min, max) of one rank (mbx_agg / oracle layout)."""
    import torch
    import torch.distributed as dist
    dev = _dev(device)
    is_float = isinstance(agg["sum"], float)
    cnt = torch.tensor([int(agg["count"])], dtype=torch.int64, device=dev)
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
    if is_float:
        mn = torch.tensor([agg["min"]], dtype=torch.float32, device=dev)
        mx = torch.tensor([agg["max"]], dtype=torch.float32, device=dev)
        parts = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, torch.tensor([agg["sum"]], dtype=torch.float64, device=dev), group=group)
        total = 0.0
        for p in parts:  # rank order: deterministic
            total += float(p.item())
    else:
        mn = torch.tensor([agg["min"]], dtype=torch.int64, device=dev)
        mx = torch.tensor([agg["max"]], dtype=torch.int64, device=dev)
        s = torch.tensor([int(agg["sum"])], dtype=torch.int64, device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
        total = int(s.item())
    dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    cast = float if is_float else int
    return dict(count=int(cnt.item()), sum=total, min=cast(mn.item()), max=cast(mx.item()))


def gather_positions(ids, device=None, group=None):
    """Concatenate every rank's ascending global positions in rank order."""
    import torch
    import torch.distributed as dist
    dev = _dev(device)
    world = dist.get_world_size(group)
    n = torch.tensor([len(ids)], dtype=torch.int64, device=dev)
    ns = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    cap = max(int(x.item()) for x in ns)
    buf = torch.zeros(max(cap, 1), dtype=torch.int64, device=dev)
    if len(ids):
        buf[:len(ids)] = torch.as_tensor(np.asarray(ids, dtype=np.int64), device=dev)
    outs = [torch.zeros(max(cap, 1), dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return np.concatenate([o[:int(k.item())].cpu().numpy() for o, k in zip(outs, ns)])
