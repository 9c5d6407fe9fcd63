// mbx_join.hip -- CDNA4 kernels of the join operators (include/mbx_join.h).
//
//   k_join_matrix  the pair matrix of a join CNF: one wave evaluates one
//                  64-bit word = 64 pairs sharing one "row" side value (read
//                  once, wave-uniform) against 64 "lane" side values; the wave
//                  ballot is the word.  BMJ: row = outer, lanes = inner
//                  (outer-major order, BitMapQuery.executeJoin); NLJ: row =
//                  (pass, inner), lanes = outer rows of the pass's block
//                  (ColumnarNestedLoopJoins.get_next).  Row-major compaction
//                  of the matrix (the scan's k_select_ids) is then exactly the
//                  reference's output order.
//   k_join_decode  flat matrix bit index -> (outer position, inner position,
//                  pass) through the two selections' position arrays.
//   k_gather_pos   late materialisation by explicit positions.
//
// Term semantics are PredEval's (R/iterator/PredEval.java:137-162): signed int
// compare, float compare (NaN flagged), String.compareTo order for char(n)
// (big-endian word compare of the device string images, any two strides).
#include <algorithm>

#include "mbx_internal.hpp"

namespace mbx {

__device__ __forceinline__ int jstr_cmp(const uint32_t* a, int aw, const uint32_t* b, int bw) {
  const int n = aw > bw ? aw : bw;
  for (int i = 0; i < n; ++i) {
    const uint32_t x = i < aw ? __builtin_bswap32(a[i]) : 0u;
    const uint32_t y = i < bw ? __builtin_bswap32(b[i]) : 0u;
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

__device__ __forceinline__ bool jop(int op, int c) {
  switch (op) {
    case kLT: return c < 0;
    case kLE: return c <= 0;
    case kGT: return c > 0;
    case kGE: return c >= 0;
    case kEQ: return c == 0;
    case kNE: return c != 0;
    default: return false;  // aopNOP / opRANGE
  }
}

__device__ __forceinline__ uint32_t eval_pair(const JoinArgs& A, int64_t orow, int64_t irow, int32_t& nan) {
  uint32_t cb = 0;
  for (int t = 0; t < A.nterms; ++t) {
    const JoinTerm& T = A.terms[t];
    int c;
    if (T.kind == kStr) {
      c = jstr_cmp((const uint32_t*)T.ocol + orow * T.ostride_w, T.ostride_w,
                   (const uint32_t*)T.icol + irow * T.istride_w, T.istride_w);
    } else if (T.kind == kInt) {
      const int32_t a = ((const int32_t*)T.ocol)[orow], b = ((const int32_t*)T.icol)[irow];
      c = a < b ? -1 : (a > b ? 1 : 0);
    } else {
      const float a = ((const float*)T.ocol)[orow], b = ((const float*)T.icol)[irow];
      nan |= (a != a) || (b != b);
      c = a < b ? -1 : (a > b ? 1 : 0);
    }
    cb |= jop(T.op, c) ? T.conj_bit : 0u;
  }
  return cb;
}

// Grid: blockIdx.y strides over the matrix words w (64 lane-side entries,
// fixed per wave, so their positions are read once), blockIdx.x * 4 + wave
// strides over rows.  The row side is wave-uniform: one scalar read per term
// per row.
__global__ __launch_bounds__(kBlock) void k_join_matrix(JoinArgs A) {
  const int lane = threadIdx.x & 63;
  const int64_t rstride = (int64_t)gridDim.x * kWaves;
  int32_t nan = 0;
  for (int64_t w = blockIdx.y; w < A.words_per_row; w += gridDim.y) {
    const int64_t col = w * 64 + lane;
    int64_t lane_pos = -1;  // BMJ: inner position of this lane; NLJ: outer, per pass
    int64_t cached_pass = -1;
    if (A.mode == 0 && col < A.ni) lane_pos = A.ipos[col];
    for (int64_t r = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); r < A.nrows; r += rstride) {
      const int64_t row = A.row0 + r;
      int64_t orow, irow;
      if (A.mode == 0) {  // BMJ: row = outer index (uniform), lanes = inner
        orow = A.opos[row];
        irow = lane_pos;
      } else {            // NLJ: row = pass * ni + inner index (uniform), lanes = outer of the block
        const int64_t p = row / A.ni;
        irow = A.ipos[row - p * A.ni];
        if (p != cached_pass) {
          cached_pass = p;
          const int64_t oi = p * A.block + col;
          lane_pos = (col < A.block && oi < A.no) ? A.opos[oi] : -1;
        }
        orow = lane_pos;
      }
      bool hit = false;
      if (lane_pos >= 0) hit = eval_pair(A, orow, irow, nan) == A.all_conj;
      const uint64_t m = __ballot(hit);
      if (lane == 0) A.out[r * A.words_per_row + w] = m;
    }
  }
  if (nan) atomicOr(A.nan, 1);
}

__global__ __launch_bounds__(kBlock) void k_join_decode(const int64_t* __restrict__ ids, const int64_t* __restrict__ n,
                                                        JoinDecode D) {
  const int64_t total = *n;
  const int64_t bits_per_row = D.words_per_row * 64;
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < total; k += (int64_t)gridDim.x * kBlock) {
    const int64_t id = ids[k];
    const int64_t row = D.row0 + id / bits_per_row;
    const int64_t col = id % bits_per_row;
    int64_t oi, ii;
    int32_t pass = 0;
    if (D.mode == 0) {
      oi = row;
      ii = col;
    } else {
      const int64_t p = row / D.ni;
      ii = row - p * D.ni;
      oi = p * D.block + col;
      pass = (int32_t)p;
    }
    D.out_outer[D.base + k] = D.opos[oi] + D.outer_offset;
    D.out_inner[D.base + k] = D.ipos[ii] + D.inner_offset;
    D.out_pass[D.base + k] = pass;
  }
}

__global__ __launch_bounds__(kBlock) void k_gather_pos(const int64_t* __restrict__ pos, int64_t n, int64_t row_offset,
                                                       const uint32_t* __restrict__ col, int32_t stride_w,
                                                       uint32_t* __restrict__ out) {
  const int64_t total = n * stride_w;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (int64_t)gridDim.x * kBlock) {
    const int64_t k = i / stride_w, w = i - k * stride_w;
    out[i] = col[(pos[k] - row_offset) * stride_w + w];
  }
}

static int64_t grid_for(int64_t work, int64_t per_block, int64_t cap) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return g > cap ? cap : g;
}

hipError_t launch_join_matrix(const JoinArgs& A, hipStream_t s) {
  if (A.nrows <= 0 || A.words_per_row <= 0) return hipSuccess;
  // ~2048 blocks across the words of a row and the rows
  const int64_t gy = std::min<int64_t>(A.words_per_row, 65535);
  const int64_t want = std::max<int64_t>(1, 2048 / gy);
  const int64_t gx = std::min<int64_t>(want, (A.nrows + kWaves - 1) / kWaves);
  hipLaunchKernelGGL(k_join_matrix, dim3((unsigned)std::max<int64_t>(gx, 1), (unsigned)gy), dim3(kBlock), 0, s, A);
  return hipGetLastError();
}

hipError_t launch_join_decode(const int64_t* ids, const int64_t* n, int64_t max_n, const JoinDecode& D,
                              hipStream_t s) {
  if (max_n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_join_decode, dim3((unsigned)grid_for(max_n, kBlock, 4096)), dim3(kBlock), 0, s, ids, n, D);
  return hipGetLastError();
}

hipError_t launch_gather_pos(const int64_t* pos, int64_t n, int64_t row_offset, const void* col, int32_t stride_w,
                             void* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_pos, dim3((unsigned)grid_for(n * stride_w, kBlock, 4096)), dim3(kBlock), 0, s, pos, n,
                     row_offset, (const uint32_t*)col, stride_w, (uint32_t*)out);
  return hipGetLastError();
}

}  // namespace mbx
