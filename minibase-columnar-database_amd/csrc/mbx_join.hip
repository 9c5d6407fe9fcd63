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
#include <cstdint>
#include <cstdlib>

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
      // raises only where PredEval evaluates this compare (R/iterator/PredEval.java:164-175)
      const bool reach = ((cb & T.req_below) == T.req_below) && !(cb & T.conj_bit);
      nan |= reach && ((a != a) || (b != b));
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

// Fast form for CNFs of at most kFastJoinTerms int / float terms.  A wave
// owns 64 matrix rows x one word: lane k loads row k's side (position and the
// term values, one coalesced load per term) and the lanes' side is held in
// registers; the 64 rows are then swept with v_readlane, so the dependent
// row-side loads of the plain form become one batch per 64 ballots.  Each
// term is reduced to a 3-bit outcome mask {x<y, x==y, x>y} over x = lane
// value, y = row value (the BMJ masks are mirrored host-side since the row
// is the outer side there).  Lane k keeps ballot k; one store per lane.
constexpr int kFastJoinTerms = 4;

struct FastJoin {
  const int32_t* lane_col[kFastJoinTerms];
  const int32_t* row_col[kFastJoinTerms];
  int32_t is_real[kFastJoinTerms];
  uint32_t mask[kFastJoinTerms];   // bit0: x<y, bit1: x==y, bit2: x>y
  uint32_t bit[kFastJoinTerms];
  uint32_t below[kFastJoinTerms];  // JoinTerm.req_below
};

__device__ __forceinline__ void lane_values(const JoinArgs& A, const FastJoin& F, int64_t pos, int32_t* lv) {
#pragma unroll
  for (int t = 0; t < kFastJoinTerms; ++t) lv[t] = (t < A.nterms && pos >= 0) ? F.lane_col[t][pos] : 0;
}

__global__ __launch_bounds__(kBlock) void k_join_matrix_fast(JoinArgs A, FastJoin F) {
  const int lane = threadIdx.x & 63;
  const int wave = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nchunks = (A.nrows + 63) >> 6;
  const int64_t cstride = (int64_t)gridDim.x * kWaves;
  int32_t nan = 0;
  for (int64_t w = blockIdx.y; w < A.words_per_row; w += gridDim.y) {
    const int64_t col = w * 64 + lane;
    int64_t lane_pos = -1;
    int32_t lv[kFastJoinTerms];
    int64_t pass = -1;                        // NLJ: the pass the lane values belong to
    if (A.mode == 0) {
      lane_pos = col < A.ni ? A.ipos[col] : -1;
      lane_values(A, F, lane_pos, lv);
    }
    for (int64_t ch = (int64_t)blockIdx.x * kWaves + wave; ch < nchunks; ch += cstride) {
      const int64_t r0 = ch * 64;
      // row side of rows r0 .. r0 + 63 (lane k holds row r0 + k)
      const int64_t rr = r0 + lane;
      const bool rvalid = rr < A.nrows;
      const int64_t row = A.row0 + rr;
      int64_t rpos = -1;
      if (rvalid) {
        if (A.mode == 0) {
          rpos = A.opos[row];
        } else {
          const int64_t p = row / A.ni;
          rpos = A.ipos[row - p * A.ni];
        }
      }
      int32_t rv[kFastJoinTerms];
#pragma unroll
      for (int t = 0; t < kFastJoinTerms; ++t) rv[t] = (t < A.nterms && rpos >= 0) ? F.row_col[t][rpos] : 0;
      // NLJ: matrix row -> pass changes at multiples of ni
      int64_t next_pass_row = INT64_MAX;
      if (A.mode == 1) {
        const int64_t p = (A.row0 + r0) / A.ni;
        if (p != pass) {
          pass = p;
          const int64_t oi = p * A.block + col;
          lane_pos = (col < A.block && oi < A.no) ? A.opos[oi] : -1;
          lane_values(A, F, lane_pos, lv);
        }
        next_pass_row = (p + 1) * A.ni - A.row0;  // launch-local row where the next pass starts
      }
      const int kmax = (int)min<int64_t>(64, A.nrows - r0);
      uint64_t mine = 0;
      for (int k = 0; k < kmax; ++k) {
        if (A.mode == 1 && r0 + k == next_pass_row) {  // uniform: the block of outer rows moves on
          ++pass;
          const int64_t oi = pass * A.block + col;
          lane_pos = (col < A.block && oi < A.no) ? A.opos[oi] : -1;
          lane_values(A, F, lane_pos, lv);
          next_pass_row += A.ni;
        }
        uint32_t cb = 0;
#pragma unroll
        for (int t = 0; t < kFastJoinTerms; ++t) {
          if (t < A.nterms) {
            const int32_t y = __builtin_amdgcn_readlane(rv[t], k);
            bool lt, gt;
            if (F.is_real[t]) {
              const float xf = __int_as_float(lv[t]), yf = __int_as_float(y);
              lt = xf < yf;
              gt = xf > yf;
              const bool reach = ((cb & F.below[t]) == F.below[t]) && !(cb & F.bit[t]);
              nan |= (lane_pos >= 0) && reach && ((xf != xf) || (yf != yf));
            } else {
              lt = lv[t] < y;
              gt = lv[t] > y;
            }
            const uint32_t m = F.mask[t];
            const bool r = lt ? (m & 1u) : (gt ? (m & 4u) : (m & 2u));
            cb |= r ? F.bit[t] : 0u;
          }
        }
        const uint64_t b = __ballot(lane_pos >= 0 && cb == A.all_conj);
        mine = lane == k ? b : mine;
      }
      if (lane < kmax) A.out[(r0 + lane) * A.words_per_row + w] = mine;
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
  bool fast = A.nterms <= kFastJoinTerms && !A.plain;
  uint32_t covered = 0;  // an empty conjunct is never true: leave it to the plain kernel
  for (int t = 0; t < A.nterms; ++t) {
    fast = fast && A.terms[t].kind != kStr;
    covered |= A.terms[t].conj_bit;
  }
  fast = fast && covered == A.all_conj;
  const int64_t gy = std::min<int64_t>(A.words_per_row, 65535);
  if (fast) {
    FastJoin F{};
    for (int t = 0; t < A.nterms; ++t) {
      const JoinTerm& T = A.terms[t];
      // lanes: inner side (BMJ) / outer side (NLJ)
      F.lane_col[t] = (const int32_t*)(A.mode == 0 ? T.icol : T.ocol);
      F.row_col[t] = (const int32_t*)(A.mode == 0 ? T.ocol : T.icol);
      F.is_real[t] = T.kind == kReal;
      // outcome of cmp(outer, inner) per op
      uint32_t m = 0;
      switch (T.op) {
        case kLT: m = 1; break;
        case kLE: m = 3; break;
        case kGT: m = 4; break;
        case kGE: m = 6; break;
        case kEQ: m = 2; break;
        case kNE: m = 5; break;
        default: m = 0;
      }
      // x = lane value: in BMJ x is the inner side, so mirror < and >
      if (A.mode == 0) m = (m & 2u) | ((m & 1u) << 2) | ((m & 4u) >> 2);
      F.mask[t] = m;
      F.bit[t] = T.conj_bit;
      F.below[t] = T.req_below;
    }
    const int64_t nchunks = (A.nrows + 63) / 64;
    const int64_t want = std::max<int64_t>(1, 8192 / gy);
    const int64_t gx = std::min<int64_t>(want, (nchunks + kWaves - 1) / kWaves);
    hipLaunchKernelGGL(k_join_matrix_fast, dim3((unsigned)std::max<int64_t>(gx, 1), (unsigned)gy), dim3(kBlock), 0,
                       s, A, F);
    return hipGetLastError();
  }
  // ~2048 blocks across the words of a row and the rows
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
