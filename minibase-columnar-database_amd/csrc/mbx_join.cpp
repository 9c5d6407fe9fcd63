// mbx_join.cpp -- C-ABI of the join operators (include/mbx_join.h) over the
// kernels of mbx_join.hip.  Host work: term validation, the two selections
// turned into position arrays (the scan's compaction kernel), chunking of the
// pair matrix so its scratch stays bounded, and result bookkeeping.  Every
// pair is evaluated on the GPU.
#include "../../include/mbx_join.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "mbx_internal.hpp"
#include "mbx_objects.hpp"

using namespace mbx;

struct mbx_join_result {
  mbx_ctx* ctx = nullptr;
  int64_t count = 0;
  int64_t passes = 1;
  int64_t cap = 0;
  int64_t* outer = nullptr;  // device, global positions
  int64_t* inner = nullptr;
  int32_t* pass = nullptr;
  ~mbx_join_result() {
    hipFree(outer);
    hipFree(inner);
    hipFree(pass);
  }
};

namespace {

int32_t cmp_op(int32_t op) {
  switch (op) {
    case MBX_OP_EQ: return kEQ;
    case MBX_OP_LT: return kLT;
    case MBX_OP_GT: return kGT;
    case MBX_OP_NE: return kNE;
    case MBX_OP_NOT: return kNE;  // PredEval: aopNOT behaves as !=
    case MBX_OP_LE: return kLE;
    case MBX_OP_GE: return kGE;
    default: return -1;           // aopNOP / opRANGE: never true
  }
}

int kind_of(int32_t attr) { return attr == MBX_ATTR_INTEGER ? kInt : (attr == MBX_ATTR_REAL ? kReal : kStr); }

// ascending table-local rows of a selection, on the device
int positions(mbx_ctx* c, const mbx_bitmap* sel, int64_t** dev, int64_t* n) {
  *dev = nullptr;
  int rc = ensure_count(c, const_cast<mbx_bitmap*>(sel));
  if (rc) return rc;
  *n = sel->count;
  HIPCHK(hipMalloc(dev, sizeof(int64_t) * (size_t)(*n > 0 ? *n : 1)));
  int64_t* dtotal = c->dcount + 1;
  hipError_t e = launch_materialize(sel->words, sel->nwords, sel->wpb, sel->segc, 0, *dev, nullptr, nullptr, 0, dtotal,
                                    c->stream);
  if (e != hipSuccess) {
    hipFree(*dev);
    *dev = nullptr;
    return fail(MBX_E_DEVICE, "join: selection positions: %s", hipGetErrorString(e));
  }
  return MBX_OK;
}

int grow(mbx_join_result* r, int64_t need, hipStream_t s) {
  if (need <= r->cap) return MBX_OK;
  int64_t cap = std::max<int64_t>(need, r->cap * 2);
  int64_t *o = nullptr, *i = nullptr;
  int32_t* p = nullptr;
  hipError_t e = hipMalloc(&o, sizeof(int64_t) * (size_t)cap);
  if (e == hipSuccess) e = hipMalloc(&i, sizeof(int64_t) * (size_t)cap);
  if (e == hipSuccess) e = hipMalloc(&p, sizeof(int32_t) * (size_t)cap);
  if (e == hipSuccess && r->count > 0) {
    e = hipMemcpyAsync(o, r->outer, sizeof(int64_t) * (size_t)r->count, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(i, r->inner, sizeof(int64_t) * (size_t)r->count, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(p, r->pass, sizeof(int32_t) * (size_t)r->count, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
  }
  if (e != hipSuccess) {
    hipFree(o);
    hipFree(i);
    hipFree(p);
    return fail(MBX_E_NOMEM, "join: %lld result pairs: %s", (long long)cap, hipGetErrorString(e));
  }
  hipFree(r->outer);
  hipFree(r->inner);
  hipFree(r->pass);
  r->outer = o;
  r->inner = i;
  r->pass = p;
  r->cap = cap;
  return MBX_OK;
}

}  // namespace

extern "C" int mbx_join(mbx_ctx* c, const mbx_table* outer, const mbx_bitmap* outer_sel, const mbx_table* inner,
                        const mbx_bitmap* inner_sel, const mbx_join_cnf* cnf, int32_t order, int64_t outer_block,
                        mbx_join_result** out) {
  NOTNULL(c);
  NOTNULL(outer);
  NOTNULL(outer_sel);
  NOTNULL(inner);
  NOTNULL(inner_sel);
  NOTNULL(cnf);
  NOTNULL(out);
  *out = nullptr;
  if (order != MBX_JOIN_BMJ && order != MBX_JOIN_NLJ) return fail(MBX_E_INVALID, "join: order %d", order);
  if (order == MBX_JOIN_NLJ && outer_block <= 0) return fail(MBX_E_INVALID, "join: outer_block %lld",
                                                             (long long)outer_block);
  if (outer_sel->nbits != outer->nrows || inner_sel->nbits != inner->nrows)
    return fail(MBX_E_INVALID, "join: selection / table size mismatch");
  if (cnf->nconj < 0 || cnf->nconj > 32) return fail(MBX_E_UNSUPPORTED, "join: %d conjuncts", cnf->nconj);
  JoinArgs A;
  memset(&A, 0, sizeof(A));
  const int32_t nterms = cnf->nconj > 0 ? cnf->conj_offsets[cnf->nconj] : 0;
  if (nterms > kMaxJoinTerms) return fail(MBX_E_UNSUPPORTED, "join: %d terms (max %d)", nterms, kMaxJoinTerms);
  if (nterms > 0) NOTNULL(cnf->terms);
  for (int32_t k = 0; k < cnf->nconj; ++k) {
    A.all_conj |= 1u << k;
    for (int32_t t = cnf->conj_offsets[k]; t < cnf->conj_offsets[k + 1]; ++t) {
      const mbx_join_term& jt = cnf->terms[t];
      if (jt.outer_col < 0 || jt.outer_col >= (int32_t)outer->cols.size() || jt.inner_col < 0 ||
          jt.inner_col >= (int32_t)inner->cols.size())
        return fail(MBX_E_RANGE, "join: term %d names a column outside the tables", t);
      const TCol& oc = outer->cols[(size_t)jt.outer_col];
      const TCol& ic = inner->cols[(size_t)jt.inner_col];
      if (oc.attr_type != ic.attr_type) return fail(MBX_E_TYPE, "Invalid JOIN COLUMN ATTR TYPE NOT MATCH.");
      JoinTerm& T = A.terms[t];
      T.kind = kind_of(oc.attr_type);
      T.op = cmp_op(jt.op);
      T.ocol = oc.dev;
      T.icol = ic.dev;
      T.ostride_w = oc.stride_w;
      T.istride_w = ic.stride_w;
      T.conj_bit = 1u << k;
    }
  }
  for (int32_t t = 0; t < nterms; ++t) A.terms[t].req_below = A.all_conj & (A.terms[t].conj_bit - 1u);
  A.nterms = nterms;
  A.plain = c->tune.join_plain;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t s = c->stream;
  mbx_join_result* r = new (std::nothrow) mbx_join_result();
  if (!r) return fail(MBX_E_NOMEM, "join: host allocation");
  r->ctx = c;
  int64_t *opos = nullptr, *ipos = nullptr;
  int64_t no = 0, ni = 0;
  if ((rc = positions(c, outer_sel, &opos, &no)) || (rc = positions(c, inner_sel, &ipos, &ni))) {
    hipFree(opos);
    delete r;
    return rc;
  }
  A.mode = order == MBX_JOIN_BMJ ? 0 : 1;
  A.opos = opos;
  A.no = no;
  A.ipos = ipos;
  A.ni = ni;
  A.nan = c->dnan;
  int64_t total_rows, wpr;
  if (order == MBX_JOIN_BMJ) {
    total_rows = no;
    wpr = (ni + 63) / 64;
    r->passes = 1;
  } else {
    const int64_t blk = std::min(outer_block, std::max<int64_t>(no, 1));
    A.block = outer_block;
    r->passes = no == 0 ? 1 : (no + outer_block - 1) / outer_block;
    total_rows = no == 0 ? 0 : r->passes * ni;
    wpr = (blk + 63) / 64;
  }
  A.words_per_row = wpr;
  // the pair matrix in chunks of rows: <= 2^24 words (128 MiB) of scratch
  const int64_t chunk_rows = wpr > 0 ? std::max<int64_t>(1, ((int64_t)1 << 24) / wpr) : 1;
  mbx_bitmap* m = nullptr;
  int64_t* ids = nullptr;
  int64_t ids_cap = 0;
  hipError_t e = hipMemsetAsync(c->dnan, 0, sizeof(int32_t), s);
  const int64_t rows_here0 = std::min(chunk_rows, total_rows);
  if (e == hipSuccess && rows_here0 > 0 && wpr > 0) rc = bitmap_new(c, rows_here0 * wpr * 64, &m);
  for (int64_t row0 = 0; !rc && e == hipSuccess && row0 < total_rows && wpr > 0; row0 += chunk_rows) {
    const int64_t rows = std::min(chunk_rows, total_rows - row0);
    A.row0 = row0;
    A.nrows = rows;
    A.out = m->words;
    e = launch_join_matrix(A, s);
    // the chunk as a BitSet of rows * wpr * 64 bits (a shorter last chunk
    // uses a prefix of the scratch BitSet: its segments are the same)
    const int64_t nw = rows * wpr;
    const int64_t nseg = (nw + m->wpb - 1) / m->wpb;
    if (e == hipSuccess) e = launch_seg_popcount(m->words, nw, m->wpb, m->segc, s);
    int64_t* dtotal = c->dcount + 1;
    if (e == hipSuccess) e = launch_count_sum(m->segc, nseg, dtotal, s);
    int64_t got = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&got, dtotal, sizeof(int64_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess || got == 0) continue;
    if (got > ids_cap) {
      hipFree(ids);
      ids = nullptr;
      ids_cap = 0;
      e = hipMalloc(&ids, sizeof(int64_t) * (size_t)got);
      if (e != hipSuccess) break;
      ids_cap = got;
    }
    e = launch_materialize(m->words, nw, m->wpb, m->segc, 0, ids, nullptr, nullptr, 0, dtotal, s);
    if (e != hipSuccess || (rc = grow(r, r->count + got, s))) break;
    JoinDecode D;
    memset(&D, 0, sizeof(D));
    D.mode = A.mode;
    D.opos = opos;
    D.ipos = ipos;
    D.ni = ni;
    D.block = A.block;
    D.row0 = row0;
    D.words_per_row = wpr;
    D.outer_offset = outer->row_offset;
    D.inner_offset = inner->row_offset;
    D.base = r->count;
    D.out_outer = r->outer;
    D.out_inner = r->inner;
    D.out_pass = r->pass;
    e = launch_join_decode(ids, dtotal, got, D, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    r->count += got;
  }
  int32_t nan = 0;
  if (!rc && e == hipSuccess) e = hipMemcpy(&nan, c->dnan, sizeof(int32_t), hipMemcpyDeviceToHost);
  if (m) mbx_bitmap_free(m);
  hipFree(ids);
  hipFree(opos);
  hipFree(ipos);
  if (!rc && e != hipSuccess) rc = fail(MBX_E_DEVICE, "join: %s", hipGetErrorString(e));
  if (!rc && nan) rc = fail(MBX_E_TYPE, "NaN in a float join comparison (TupleUtils falls through and raises)");
  if (rc) {
    delete r;
    return rc;
  }
  *out = r;
  return MBX_OK;
}

extern "C" int mbx_join_info(const mbx_join_result* r, int64_t* count, int64_t* passes) {
  NOTNULL(r);
  if (count) *count = r->count;
  if (passes) *passes = r->passes;
  return MBX_OK;
}

extern "C" int mbx_join_fetch(mbx_ctx* c, const mbx_join_result* r, int64_t start, int64_t n, int64_t* outer_pos,
                              int64_t* inner_pos, int32_t* pass) {
  NOTNULL(c);
  NOTNULL(r);
  if (start < 0 || n < 0 || start + n > r->count)
    return fail(MBX_E_RANGE, "join_fetch: [%lld, %lld) outside %lld pairs", (long long)start, (long long)(start + n),
                (long long)r->count);
  if (n == 0) return MBX_OK;
  int rc = set_device(c);
  if (rc) return rc;
  if (outer_pos) HIPCHK(hipMemcpy(outer_pos, r->outer + start, sizeof(int64_t) * (size_t)n, hipMemcpyDeviceToHost));
  if (inner_pos) HIPCHK(hipMemcpy(inner_pos, r->inner + start, sizeof(int64_t) * (size_t)n, hipMemcpyDeviceToHost));
  if (pass) HIPCHK(hipMemcpy(pass, r->pass + start, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost));
  return MBX_OK;
}

extern "C" int mbx_join_free(mbx_join_result* r) {
  delete r;
  return MBX_OK;
}

extern "C" int mbx_gather(mbx_ctx* c, const mbx_table* t, const int64_t* positions_h, int64_t n, const int32_t* proj,
                          int32_t nproj, void* const* host_out) {
  NOTNULL(c);
  NOTNULL(t);
  if (n < 0 || nproj < 0) return fail(MBX_E_INVALID, "gather: n %lld, nproj %d", (long long)n, nproj);
  if (n == 0 || nproj == 0) return MBX_OK;
  NOTNULL(positions_h);
  NOTNULL(proj);
  NOTNULL(host_out);
  for (int64_t k = 0; k < n; ++k)
    if (positions_h[k] < t->row_offset || positions_h[k] >= t->row_offset + t->nrows)
      return fail(MBX_E_RANGE, "gather: position %lld outside the table", (long long)positions_h[k]);
  for (int32_t j = 0; j < nproj; ++j)
    if (proj[j] < 0 || proj[j] >= (int32_t)t->cols.size()) return fail(MBX_E_RANGE, "gather: column %d", proj[j]);
  int rc = set_device(c);
  if (rc) return rc;
  int64_t* dpos = nullptr;
  void* dout = nullptr;
  int32_t maxw = 1;
  for (int32_t j = 0; j < nproj; ++j) maxw = std::max(maxw, t->cols[(size_t)proj[j]].stride_w);
  HIPCHK(hipMalloc(&dpos, sizeof(int64_t) * (size_t)n));
  hipError_t e = hipMalloc(&dout, sizeof(uint32_t) * (size_t)n * (size_t)maxw);
  if (e == hipSuccess) e = hipMemcpy(dpos, positions_h, sizeof(int64_t) * (size_t)n, hipMemcpyHostToDevice);
  std::vector<uint8_t> img;
  for (int32_t j = 0; j < nproj && e == hipSuccess; ++j) {
    const TCol& tc = t->cols[(size_t)proj[j]];
    e = launch_gather_pos(dpos, n, t->row_offset, tc.dev, tc.stride_w, dout, c->stream);
    img.resize((size_t)n * (size_t)tc.stride_w * 4);
    if (e == hipSuccess) e = hipMemcpyAsync(img.data(), dout, img.size(), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess) unpack_rows(tc, img.data(), n, host_out[j]);
  }
  hipFree(dpos);
  hipFree(dout);
  if (e != hipSuccess) return fail(MBX_E_DEVICE, "gather: %s", hipGetErrorString(e));
  return MBX_OK;
}
