// mbx_comm.cpp -- the multi-GPU exchange step (RCCL over xGMI) and HIP-graph
// capture of repeated queries, behind include/mbx.h.
//
// rows shard by range (64-aligned, mbx_shard_bounds), every
// shard is scanned by its own GPU with no communication, and ONE collective
// combines the per-shard results.  Each communicator owns an exchange stream:
// a collective waits (event) for the work already enqueued on its context's
// stream and runs beside the scans enqueued after it.  The combine of an
// aggregate is an all-gather of the 48-byte records plus a one-wave fold in
// rank order, so the double SUM is bit-reproducible for a given world size
// and equal to dist.fold_aggregates (minibase-columnar-database_amd/dist.py).
#include "../../include/mbx.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>
#include <vector>

#include "mbx_internal.hpp"
#include "mbx_objects.hpp"

using namespace mbx;

struct mbx_comm {
  mbx_ctx* ctx = nullptr;
  ncclComm_t nc = nullptr;
  int32_t nranks = 1, rank = 0;
  hipStream_t xs = nullptr;          // exchange stream (same device as ctx)
  hipEvent_t ev_main = nullptr;      // recorded on ctx->stream before a collective
  hipEvent_t ev_x = nullptr;         // recorded on xs after the collectives (mbx_comm_wait, graph join)
  AggOut* gathered = nullptr;        // nranks records (aggregate all-gather)
};

struct mbx_graph {
  mbx_ctx* ctx = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
};

#define NCCLCHK(expr)                                                                             \
  do {                                                                                            \
    ncclResult_t r_ = (expr);                                                                     \
    if (r_ != ncclSuccess) return fail(MBX_E_DEVICE, "%s: %s", #expr, ncclGetErrorString(r_));    \
  } while (0)

namespace {

// dist.fold_aggregates on the device: rank order, one lane.  out may alias
// recs[0] (mbx_agg_fold_async folds in place), so neither is __restrict__.
__global__ void k_fold_agg(const AggOut* recs, int32_t n, AggOut* out) {
  if (threadIdx.x != 0) return;
  AggOut r = recs[0];
  double fsum = 0.0;
  int64_t count = 0, isum = 0;
  int32_t imin = INT32_MAX, imax = INT32_MIN;
  float fmin = __builtin_inff(), fmax = -__builtin_inff();
  for (int32_t k = 0; k < n; ++k) {
    const AggOut& a = recs[k];
    count += a.count;
    isum += a.isum;
    imin = a.imin < imin ? a.imin : imin;
    imax = a.imax > imax ? a.imax : imax;
    fsum += a.fsum;
    fmin = a.fmin < fmin ? a.fmin : fmin;
    fmax = a.fmax > fmax ? a.fmax : fmax;
  }
  r.count = count;
  r.isum = isum;
  r.imin = imin;
  r.imax = imax;
  r.fsum = fsum;
  r.fmin = fmin;
  r.fmax = fmax;
  *out = r;
}

int comm_setup(mbx_ctx* c, mbx_comm* m) {
  m->ctx = c;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamCreateWithFlags(&m->xs, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&m->ev_main, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&m->ev_x, hipEventDisableTiming));
  HIPCHK(hipMalloc(&m->gathered, sizeof(AggOut) * (size_t)(m->nranks > 0 ? m->nranks : 1)));
  return MBX_OK;
}

void comm_release(mbx_comm* m) {
  if (!m) return;
  if (m->ctx) hipSetDevice(m->ctx->device);
  if (m->xs) hipStreamSynchronize(m->xs);
  if (m->nc) ncclCommDestroy(m->nc);
  hipFree(m->gathered);
  if (m->ev_main) hipEventDestroy(m->ev_main);
  if (m->ev_x) hipEventDestroy(m->ev_x);
  if (m->xs) hipStreamDestroy(m->xs);
  if (m->ctx && m->ctx->comm == m) m->ctx->comm = nullptr;
  delete m;
}

// where a collective runs: the context stream itself, right after the query
// that feeds it (knob comm_same_stream, default), or the communicator's
// exchange stream (the next scans could overlap it).  Measured on one GPU,
// 12.5 M-row shard, one collective per query, HIP graphs of 10 steps, with a
// stand-in real kernel per step beside the one-rank all-reduce: 20.4-20.6
// us per step on the context stream vs 34-35 us on the exchange stream (a
// kernel forked to a second stream inside a graph is not overlapped on this
// ROCm); 17.5-17.7 vs 18.0-18.2 without it (profiles/r03/parts)
bool same_stream(const mbx_comm* m) { return m->ctx->tune.comm_same_stream != 0; }
hipStream_t xstream(const mbx_comm* m) { return same_stream(m) ? m->ctx->stream : m->xs; }

// the exchange stream waits for the context stream's work so far
int fork_after_main(mbx_comm* m) {
  if (same_stream(m)) return MBX_OK;
  HIPCHK(hipEventRecord(m->ev_main, m->ctx->stream));
  HIPCHK(hipStreamWaitEvent(m->xs, m->ev_main, 0));
  return MBX_OK;
}

int check_all(mbx_comm* const* comms, int32_t n) {
  if (!comms || n <= 0) return fail(MBX_E_INVALID, "comm: %d communicators", n);
  for (int32_t i = 0; i < n; ++i) {
    if (!comms[i]) return fail(MBX_E_INVALID, "comm: null communicator %d", i);
    if (comms[i]->nranks != n || comms[i]->rank != i)
      return fail(MBX_E_INVALID, "comm: communicator %d is rank %d of %d, expected rank %d of %d", i, comms[i]->rank,
                  comms[i]->nranks, i, n);
  }
  return MBX_OK;
}

}  // namespace

extern "C" int mbx_shard_bounds(int64_t nrows, int32_t nshards, int32_t shard, int64_t* begin, int64_t* end) {
  NOTNULL(begin);
  NOTNULL(end);
  if (nrows < 0 || nshards <= 0 || shard < 0 || shard >= nshards)
    return fail(MBX_E_INVALID, "shard_bounds: nrows %lld, shard %d of %d", (long long)nrows, shard, nshards);
  const int64_t words = (nrows + 63) / 64;
  const int64_t per = words / nshards, extra = words % nshards;
  const int64_t w0 = shard * per + (shard < extra ? shard : extra);
  const int64_t w1 = w0 + per + (shard < extra ? 1 : 0);
  if (w0 == w1) {
    const int64_t s = w0 * 64 < (nrows / 64) * 64 ? w0 * 64 : (nrows / 64) * 64;
    *begin = *end = s;
    return MBX_OK;
  }
  *begin = w0 * 64;
  *end = w1 * 64 < nrows ? w1 * 64 : nrows;
  return MBX_OK;
}

extern "C" int mbx_comm_unique_id(void* id) {
  NOTNULL(id);
  static_assert(sizeof(ncclUniqueId) == MBX_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  NCCLCHK(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof(u));
  return MBX_OK;
}

extern "C" int mbx_comm_init_rank(mbx_ctx* c, int32_t nranks, int32_t rank, const void* id, mbx_comm** out) {
  NOTNULL(c);
  NOTNULL(id);
  NOTNULL(out);
  *out = nullptr;
  if (nranks <= 0 || rank < 0 || rank >= nranks) return fail(MBX_E_INVALID, "comm: rank %d of %d", rank, nranks);
  if (c->comm) return fail(MBX_E_INVALID, "comm: context already has a communicator");
  mbx_comm* m = new (std::nothrow) mbx_comm();
  if (!m) return fail(MBX_E_NOMEM, "comm: host allocation");
  m->nranks = nranks;
  m->rank = rank;
  int rc = comm_setup(c, m);
  if (!rc) {
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    const ncclResult_t r = ncclCommInitRank(&m->nc, nranks, u, rank);
    if (r != ncclSuccess) rc = fail(MBX_E_DEVICE, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  if (rc) {
    comm_release(m);
    return rc;
  }
  c->comm = m;
  *out = m;
  return MBX_OK;
}

extern "C" int mbx_comm_init_all(mbx_ctx* const* ctxs, int32_t n, mbx_comm** outs) {
  NOTNULL(ctxs);
  NOTNULL(outs);
  if (n <= 0) return fail(MBX_E_INVALID, "comm_init_all: %d contexts", n);
  std::vector<int> devs((size_t)n);
  for (int32_t i = 0; i < n; ++i) {
    if (!ctxs[i]) return fail(MBX_E_INVALID, "comm_init_all: null context %d", i);
    if (ctxs[i]->comm) return fail(MBX_E_INVALID, "comm_init_all: context %d already has a communicator", i);
    devs[(size_t)i] = ctxs[i]->device;
    for (int32_t j = 0; j < i; ++j)
      if (devs[(size_t)j] == devs[(size_t)i])
        return fail(MBX_E_INVALID, "comm_init_all: contexts %d and %d share device %d", j, i, devs[(size_t)i]);
    outs[i] = nullptr;
  }
  std::vector<mbx_comm*> ms((size_t)n, nullptr);
  std::vector<ncclComm_t> ncs((size_t)n, nullptr);
  int rc = MBX_OK;
  for (int32_t i = 0; i < n && !rc; ++i) {
    ms[(size_t)i] = new (std::nothrow) mbx_comm();
    if (!ms[(size_t)i]) {
      rc = fail(MBX_E_NOMEM, "comm: host allocation");
      break;
    }
    ms[(size_t)i]->nranks = n;
    ms[(size_t)i]->rank = i;
    rc = comm_setup(ctxs[i], ms[(size_t)i]);
  }
  if (!rc) {
    const ncclResult_t r = ncclCommInitAll(ncs.data(), n, devs.data());
    if (r != ncclSuccess) rc = fail(MBX_E_DEVICE, "ncclCommInitAll: %s", ncclGetErrorString(r));
  }
  if (rc) {
    for (int32_t i = 0; i < n; ++i) {
      if (ms[(size_t)i]) ms[(size_t)i]->nc = ncs[(size_t)i];
      comm_release(ms[(size_t)i]);
    }
    return rc;
  }
  for (int32_t i = 0; i < n; ++i) {
    ms[(size_t)i]->nc = ncs[(size_t)i];
    ctxs[i]->comm = ms[(size_t)i];
    outs[i] = ms[(size_t)i];
  }
  return MBX_OK;
}

extern "C" int mbx_comm_free(mbx_comm* m) {
  comm_release(m);
  return MBX_OK;
}

extern "C" int mbx_comm_info(const mbx_comm* m, int32_t* nranks, int32_t* rank) {
  NOTNULL(m);
  if (nranks) *nranks = m->nranks;
  if (rank) *rank = m->rank;
  return MBX_OK;
}

extern "C" int mbx_comm_wait(mbx_comm* m) {
  NOTNULL(m);
  HIPCHK(hipSetDevice(m->ctx->device));
  if (same_stream(m)) return MBX_OK;  // already in the context stream's order
  HIPCHK(hipEventRecord(m->ev_x, m->xs));
  HIPCHK(hipStreamWaitEvent(m->ctx->stream, m->ev_x, 0));
  return MBX_OK;
}

extern "C" int mbx_comm_allreduce_count_async(mbx_comm* m, int64_t* dev_counts, int64_t n) {
  NOTNULL(m);
  NOTNULL(dev_counts);
  if (n <= 0) return fail(MBX_E_INVALID, "allreduce_count: n = %lld", (long long)n);
  HIPCHK(hipSetDevice(m->ctx->device));
  if (int rc = fork_after_main(m)) return rc;
  NCCLCHK(ncclAllReduce(dev_counts, dev_counts, (size_t)n, ncclInt64, ncclSum, m->nc, xstream(m)));
  return MBX_OK;
}

extern "C" int mbx_comm_scan_count_async(mbx_comm* m, const mbx_plan* p, int64_t* dev_parts, int64_t parts_cap,
                                         int64_t* dev_count) {
  NOTNULL(m);
  NOTNULL(p);
  NOTNULL(dev_count);
  HIPCHK(hipSetDevice(m->ctx->device));
  if (plan_has_real(p)) {  // the NaN check needs the scan's own finalize: scan, then the collective
    if (int rc = mbx_scan_count_async(m->ctx, p, dev_count)) return rc;
    return mbx_comm_allreduce_count_async(m, dev_count, 1);
  }
  NOTNULL(dev_parts);
  int64_t nb = 0;
  if (int rc = scan_count_parts(m->ctx, p, dev_parts, parts_cap, &nb)) return rc;
  if (int rc = fork_after_main(m)) return rc;
  HIPCHK(launch_count_sum(dev_parts, nb, dev_count, xstream(m)));
  NCCLCHK(ncclAllReduce(dev_count, dev_count, 1, ncclInt64, ncclSum, m->nc, xstream(m)));
  return MBX_OK;
}

extern "C" int mbx_comm_allreduce_agg_async(mbx_comm* m, mbx_agg* dev_rec) {
  NOTNULL(m);
  NOTNULL(dev_rec);
  static_assert(sizeof(mbx_agg) == sizeof(AggOut), "mbx_agg layout");
  HIPCHK(hipSetDevice(m->ctx->device));
  if (int rc = fork_after_main(m)) return rc;
  NCCLCHK(ncclAllGather(dev_rec, m->gathered, sizeof(AggOut) / sizeof(int64_t), ncclInt64, m->nc, xstream(m)));
  hipLaunchKernelGGL(k_fold_agg, dim3(1), dim3(64), 0, xstream(m), m->gathered, m->nranks, (AggOut*)dev_rec);
  HIPCHK(hipGetLastError());
  return MBX_OK;
}

// the fold alone, over a caller's record array (a one-process caller that
// gathered the records itself; the 8-rank combine exercised on one GPU)
extern "C" int mbx_agg_fold_async(mbx_ctx* c, const mbx_agg* dev_recs, int32_t n, mbx_agg* dev_out) {
  NOTNULL(c);
  NOTNULL(dev_recs);
  NOTNULL(dev_out);
  if (n <= 0) return fail(MBX_E_INVALID, "agg_fold: %d records", n);
  HIPCHK(hipSetDevice(c->device));
  hipLaunchKernelGGL(k_fold_agg, dim3(1), dim3(64), 0, c->stream, (const AggOut*)dev_recs, n, (AggOut*)dev_out);
  HIPCHK(hipGetLastError());
  return MBX_OK;
}

extern "C" int mbx_comm_allgather_count_async(mbx_comm* m, const int64_t* dev_count, int64_t* dev_all) {
  NOTNULL(m);
  NOTNULL(dev_count);
  NOTNULL(dev_all);
  HIPCHK(hipSetDevice(m->ctx->device));
  if (int rc = fork_after_main(m)) return rc;
  NCCLCHK(ncclAllGather(dev_count, dev_all, 1, ncclInt64, m->nc, xstream(m)));
  return MBX_OK;
}

extern "C" int mbx_comm_allreduce_count_all(mbx_comm* const* comms, int32_t n, int64_t* const* dev_counts,
                                            int64_t count) {
  if (int rc = check_all(comms, n)) return rc;
  NOTNULL(dev_counts);
  if (count <= 0) return fail(MBX_E_INVALID, "allreduce_count_all: count = %lld", (long long)count);
  for (int32_t i = 0; i < n; ++i) {
    NOTNULL(dev_counts[i]);
    HIPCHK(hipSetDevice(comms[i]->ctx->device));
    if (int rc = fork_after_main(comms[i])) return rc;
  }
  NCCLCHK(ncclGroupStart());
  for (int32_t i = 0; i < n; ++i) {
    const ncclResult_t r =
        ncclAllReduce(dev_counts[i], dev_counts[i], (size_t)count, ncclInt64, ncclSum, comms[i]->nc, xstream(comms[i]));
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return fail(MBX_E_DEVICE, "ncclAllReduce (rank %d): %s", i, ncclGetErrorString(r));
    }
  }
  NCCLCHK(ncclGroupEnd());
  return MBX_OK;
}

extern "C" int mbx_comm_allgather_count_all(mbx_comm* const* comms, int32_t n, const int64_t* const* dev_counts,
                                            int64_t* const* dev_alls) {
  if (int rc = check_all(comms, n)) return rc;
  NOTNULL(dev_counts);
  NOTNULL(dev_alls);
  for (int32_t i = 0; i < n; ++i) {
    NOTNULL(dev_counts[i]);
    NOTNULL(dev_alls[i]);
    HIPCHK(hipSetDevice(comms[i]->ctx->device));
    if (int rc = fork_after_main(comms[i])) return rc;
  }
  NCCLCHK(ncclGroupStart());
  for (int32_t i = 0; i < n; ++i) {
    const ncclResult_t r = ncclAllGather(dev_counts[i], dev_alls[i], 1, ncclInt64, comms[i]->nc, xstream(comms[i]));
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return fail(MBX_E_DEVICE, "ncclAllGather (rank %d): %s", i, ncclGetErrorString(r));
    }
  }
  NCCLCHK(ncclGroupEnd());
  return MBX_OK;
}

extern "C" int mbx_comm_allreduce_agg_all(mbx_comm* const* comms, int32_t n, mbx_agg* const* dev_recs) {
  if (int rc = check_all(comms, n)) return rc;
  NOTNULL(dev_recs);
  for (int32_t i = 0; i < n; ++i) {
    NOTNULL(dev_recs[i]);
    HIPCHK(hipSetDevice(comms[i]->ctx->device));
    if (int rc = fork_after_main(comms[i])) return rc;
  }
  NCCLCHK(ncclGroupStart());
  for (int32_t i = 0; i < n; ++i) {
    const ncclResult_t r = ncclAllGather(dev_recs[i], comms[i]->gathered, sizeof(AggOut) / sizeof(int64_t),
                                         ncclInt64, comms[i]->nc, xstream(comms[i]));
    if (r != ncclSuccess) {
      ncclGroupEnd();
      return fail(MBX_E_DEVICE, "ncclAllGather (rank %d): %s", i, ncclGetErrorString(r));
    }
  }
  NCCLCHK(ncclGroupEnd());
  // the folds follow their all-gathers on each exchange stream
  for (int32_t i = 0; i < n; ++i) {
    HIPCHK(hipSetDevice(comms[i]->ctx->device));
    hipLaunchKernelGGL(k_fold_agg, dim3(1), dim3(64), 0, xstream(comms[i]), comms[i]->gathered, n,
                       (AggOut*)dev_recs[i]);
    HIPCHK(hipGetLastError());
  }
  return MBX_OK;
}

// ------------------------------------------------------------------ graphs

extern "C" int mbx_graph_begin(mbx_ctx* c) {
  NOTNULL(c);
  if (c->capturing) return fail(MBX_E_INVALID, "graph_begin: capture already open");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed));
  c->capturing = true;
  return MBX_OK;
}

extern "C" int mbx_graph_end(mbx_ctx* c, mbx_graph** out) {
  NOTNULL(c);
  NOTNULL(out);
  *out = nullptr;
  if (!c->capturing) return fail(MBX_E_INVALID, "graph_end: no capture open");
  HIPCHK(hipSetDevice(c->device));
  c->capturing = false;
  // the exchange stream's captured work joins the origin stream (a capture
  // ends only with every forked stream joined back); the capture is ended
  // even when the join (or anything captured before it) failed, so the
  // stream never stays in capture mode
  hipError_t je = hipSuccess;
  if (c->comm && !same_stream(c->comm)) {
    je = hipEventRecord(c->comm->ev_x, c->comm->xs);
    if (je == hipSuccess) je = hipStreamWaitEvent(c->stream, c->comm->ev_x, 0);
  }
  hipGraph_t g = nullptr;
  const hipError_t ee = hipStreamEndCapture(c->stream, &g);
  if (je != hipSuccess || ee != hipSuccess) {
    if (g) hipGraphDestroy(g);
    return fail(MBX_E_DEVICE, "graph_end: %s", hipGetErrorString(je != hipSuccess ? je : ee));
  }
  mbx_graph* mg = new (std::nothrow) mbx_graph();
  if (!mg) {
    hipGraphDestroy(g);
    return fail(MBX_E_NOMEM, "graph: host allocation");
  }
  mg->ctx = c;
  mg->graph = g;
  const hipError_t e = hipGraphInstantiate(&mg->exec, g, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    hipGraphDestroy(g);
    delete mg;
    return fail(MBX_E_DEVICE, "hipGraphInstantiate: %s", hipGetErrorString(e));
  }
  *out = mg;
  return MBX_OK;
}

extern "C" int mbx_graph_launch(mbx_graph* g) {
  NOTNULL(g);
  HIPCHK(hipSetDevice(g->ctx->device));
  HIPCHK(hipGraphLaunch(g->exec, g->ctx->stream));
  return MBX_OK;
}

extern "C" int mbx_graph_free(mbx_graph* g) {
  if (!g) return MBX_OK;
  hipSetDevice(g->ctx->device);
  hipStreamSynchronize(g->ctx->stream);
  if (g->exec) hipGraphExecDestroy(g->exec);
  if (g->graph) hipGraphDestroy(g->graph);
  delete g;
  return MBX_OK;
}

// mbx_sync's part for the exchange stream (mbx_api.cpp)
int mbx::comm_sync(mbx_ctx* c) {
  if (c->comm) HIPCHK(hipStreamSynchronize(c->comm->xs));
  return MBX_OK;
}

// mbx_free's part: a context's communicator goes with it
void mbx::comm_release_of(mbx_ctx* c) {
  if (c->comm) comm_release(c->comm);
}
