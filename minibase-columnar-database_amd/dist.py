"""Row-range sharding of one Columnarfile over ranks, and the single exchange
step of the path.

Every rank owns positions [start, end) of the logical table, with shard
boundaries on multiples of 64 rows so BitSet words never straddle ranks; its
HBM table is staged with row_offset = start so positions it returns are
global.  Rows are independent, so scans need no communication; the only
collective combines the per-rank results:

  COUNT             -> all_reduce(SUM) on int64
  COUNT/SUM/MIN/MAX -> ONE all_gather of every rank's 48-byte aggregate
                       record (the kernel's mbx_agg, straight from device
                       memory), folded in rank order: int64 sums exact, the
                       double SUM of the per-rank partials in rank order
                       (bit-reproducible for a given world size), MIN / MAX
  positions / rows  -> all_gather, concatenated in rank order (= ascending
                       global position order, the reference's nextSetBit order)

Two transports for the same combine:
  * libmbx's own RCCL communicator (include/mbx.h mbx_comm_*, RcclExchange
    below): the product path -- the collective runs on the communicator's
    exchange stream over xGMI, the fold of an aggregate is a one-wave kernel
    in rank order (identical to fold_aggregates), no host round trip.
    torch.distributed (any backend) only carries the 128-byte RCCL id.
  * torch.distributed ("gloo") for the CPU tests: the host-side restatement.
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


# one rank's aggregate in the C-ABI's mbx_agg layout (48 bytes = 6 int64),
# the unit the combine step exchanges
AGG_RECORD = np.dtype([("count", "<i8"), ("agg_type", "<i4"), ("pad", "<i4"), ("isum", "<i8"), ("imin", "<i4"),
                       ("imax", "<i4"), ("fsum", "<f8"), ("fmin", "<f4"), ("fmax", "<f4")])
AGG_WORDS = AGG_RECORD.itemsize // 8
_INTEGER = 1  # AttrType.attrInteger


def pack_aggregate(agg, integer):
    """dict(count, sum, min, max) -> one AGG_RECORD (the kernel's AggOut)."""
    r = np.zeros(1, dtype=AGG_RECORD)
    r["count"] = int(agg["count"])
    r["agg_type"] = _INTEGER if integer else 2
    if integer:
        r["isum"], r["imin"], r["imax"] = int(agg["sum"]), int(agg["min"]), int(agg["max"])
    else:
        r["fsum"], r["fmin"], r["fmax"] = float(agg["sum"]), float(agg["min"]), float(agg["max"])
    return r


def fold_aggregates(recs):
    """Rank-ordered AGG_RECORDs -> the global dict(count, sum, min, max).
    COUNT / int SUM add exactly; the double SUM adds the per-rank partials
    in rank order (bit-reproducible for a given world size); MIN / MAX fold
    the per-rank values, whose empty-shard values are the identities
    (INT32_MAX / INT32_MIN, +inf / -inf, like the oracle)."""
    recs = np.asarray(recs).view(AGG_RECORD).reshape(-1)
    integer = int(recs["agg_type"][0]) == _INTEGER
    count = int(recs["count"].sum())
    if integer:
        return dict(count=count, sum=int(recs["isum"].sum()), min=int(recs["imin"].min()),
                    max=int(recs["imax"].max()))
    total = 0.0
    for v in recs["fsum"]:
        total += float(v)
    return dict(count=count, sum=total, min=float(recs["fmin"].min()), max=float(recs["fmax"].max()))


def _all_gather_words(t, group):
    """ONE collective: every rank's int64 vector, concatenated in rank order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=group)
        return out
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    return torch.cat(parts)


def combine_aggregate(agg, device=None, group=None):
    """agg: dict(count, sum, min, max) of one rank (mbx_agg / oracle layout).
    The exchange is one all_gather of the 48-byte record."""
    import torch
    integer = not isinstance(agg["sum"], float)
    rec = pack_aggregate(agg, integer)
    t = torch.from_numpy(rec.view(np.int64).copy()).to(_dev(device))
    return fold_aggregates(_all_gather_words(t, group).cpu().numpy())


def combine_aggregate_device(rec_words, group=None):
    """rec_words: the int64[6] device tensor mbx_scan_aggregate_async wrote
    (RCCL over xGMI when the group is "nccl").  Returns the rank-ordered
    AGG_RECORDs gathered on the device; fold_aggregates() reads them."""
    return _all_gather_words(rec_words, group)


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


class RcclExchange:
    """The exchange step of one rank through libmbx (mbx_comm_init_rank):
    rank 0's RCCL id is broadcast over the torch.distributed group (gloo is
    enough: 128 bytes, once), then every collective is libmbx's, enqueued
    after the context's scans on its exchange stream."""

    def __init__(self, ctx, group=None):
        import torch.distributed as dist
        from . import mbx
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        box = [mbx.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        self.ctx, self.world, self.rank = ctx, world, rank
        self.comm = ctx.comm_init_rank(world, rank, box[0])

    def count_async(self, dev_ptr, n=1):
        """in place: dev_ptr[0..n) = the sum over ranks (int64)"""
        self.comm.allreduce_count_async(dev_ptr, n)

    def aggregate_async(self, dev_rec_ptr):
        """in place: the 48-byte mbx_agg record becomes the rank-ordered fold"""
        self.comm.allreduce_agg_async(dev_rec_ptr)

    def counts_async(self, dev_count_ptr, dev_all_ptr):
        """dev_all[r] = rank r's count (the concatenation offsets of the
        per-rank positions / rows, shard order)"""
        self.comm.allgather_count_async(dev_count_ptr, dev_all_ptr)
