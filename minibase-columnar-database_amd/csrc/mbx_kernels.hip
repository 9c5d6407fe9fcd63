// mbx_kernels.hip -- CDNA4 (gfx950) kernels of the columnar scan path.
//
//   k_scan_fast      PredEval over 4-byte columns (ColumnarFileScan.get_next,
//                    R/iterator/ColumnarFileScan.java:156-172): 16-byte loads,
//                    4 rows per lane, 256-row wave tiles; COUNT / BitSet /
//                    COUNT+SUM+MIN+MAX outputs.  HBM-read bound.
//   k_scan_generic   same contract for any CNF (char(n) strings, column-vs-
//                    column terms): one row per lane, the wave ballot is the
//                    BitSet word.
//   k_bitmap_cnf     ColumnarIndexScan OR/AND over index BitSets
//                    (R/index/ColumnarIndexScan.java:130-181) AND NOT deleted.
//   k_bitmap_combine BitSet.and / or / andNot.
//   k_seg_popcount / k_select_ids / k_gather
//                    nextSetBit compaction + late materialisation
//                    (R/index/ColumnarIndexScan.java:287-308): per-segment
//                    counts -> each block sums the counts before it and writes
//                    its ascending positions -> thread-per-row gather of the
//                    projected values.
//   k_index_build    Columnarfile.createBitMapIndex (R/columnar/Columnarfile.java:698-753).
//   k_finalize       deterministic fixed-order reduction of per-block partials.
//
// No atomics on the data path: every reduction is per block into a partial
// slot, then a single-block pass in a fixed order (bit-reproducible sums).
#include <cstdlib>

#include "mbx_internal.hpp"

namespace mbx {

// ----------------------------------------------------------------- helpers

template <typename T>
__device__ __forceinline__ bool cmp1(int op, T a, T b) {
  switch (op) {
    case kLT: return a < b;
    case kLE: return a <= b;
    case kGT: return a > b;
    case kGE: return a >= b;
    case kEQ: return a == b;
    case kNE: return a != b;
    default: return false;  // kNever
  }
}

// one uniform switch, four rows
template <typename T>
__device__ __forceinline__ void cmp4(int op, const T (&a)[4], T b, bool (&r)[4]) {
  switch (op) {
    case kLT:
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = a[j] < b;
      break;
    case kLE:
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = a[j] <= b;
      break;
    case kGT:
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = a[j] > b;
      break;
    case kGE:
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = a[j] >= b;
      break;
    case kEQ:
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = a[j] == b;
      break;
    case kNE:
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = a[j] != b;
      break;
    default:  // kNever
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = false;
      break;
  }
}

// String.compareTo sign over the device string image: big-endian unsigned
// word compare, missing words read as zero padding.
__device__ __forceinline__ int str_cmp(const uint32_t* a, int aw, const uint32_t* b, int bw) {
  const int n = aw > bw ? aw : bw;
  for (int i = 0; i < n; ++i) {
    const uint32_t x = i < aw ? __builtin_bswap32(a[i]) : 0u;
    const uint32_t y = i < bw ? __builtin_bswap32(b[i]) : 0u;
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

struct Acc {
  int64_t count;  // meaningful in lane 0 only (scalar ballot counts)
  int64_t isum;
  double fsum;
  int32_t imin, imax;
  float fmin, fmax;
  int32_t nan;
};

__device__ __forceinline__ void acc_init(Acc& a) {
  a.count = 0;
  a.isum = 0;
  a.fsum = 0.0;
  a.imin = INT32_MAX;
  a.imax = INT32_MIN;
  a.fmin = __builtin_inff();
  a.fmax = -__builtin_inff();
  a.nan = 0;
}

__device__ __forceinline__ void acc_merge(Acc& a, const Acc& b) {
  a.count += b.count;
  a.isum += b.isum;
  a.fsum += b.fsum;
  a.imin = b.imin < a.imin ? b.imin : a.imin;
  a.imax = b.imax > a.imax ? b.imax : a.imax;
  a.fmin = b.fmin < a.fmin ? b.fmin : a.fmin;
  a.fmax = b.fmax > a.fmax ? b.fmax : a.fmax;
  a.nan |= b.nan;
}

__device__ __forceinline__ Acc shfl_xor_acc(const Acc& a, int m) {
  Acc b;
  b.count = __shfl_xor(a.count, m);
  b.isum = __shfl_xor(a.isum, m);
  b.fsum = __shfl_xor(a.fsum, m);
  b.imin = __shfl_xor(a.imin, m);
  b.imax = __shfl_xor(a.imax, m);
  b.fmin = __shfl_xor(a.fmin, m);
  b.fmax = __shfl_xor(a.fmax, m);
  b.nan = __shfl_xor(a.nan, m);
  return b;
}

__device__ __forceinline__ Acc from_partial(const Partial& p) {
  Acc b;
  b.count = p.count;
  b.isum = p.isum;
  b.fsum = p.fsum;
  b.imin = p.imin;
  b.imax = p.imax;
  b.fmin = p.fmin;
  b.fmax = p.fmax;
  b.nan = p.nan_seen;
  return b;
}

// write-through (sc1) store / load of one Partial, 8 bytes at a time
__device__ __forceinline__ void store_partial_sc1(Partial* dst, const Partial& p) {
  const uint64_t* s = reinterpret_cast<const uint64_t*>(&p);
  uint64_t* d = reinterpret_cast<uint64_t*>(dst);
#pragma unroll
  for (int i = 0; i < kSegStride; ++i) __hip_atomic_store(d + i, s[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ Partial load_partial_sc1(const Partial* src) {
  Partial p;
  uint64_t* d = reinterpret_cast<uint64_t*>(&p);
  uint64_t* s = reinterpret_cast<uint64_t*>(const_cast<Partial*>(src));
#pragma unroll
  for (int i = 0; i < kSegStride; ++i) d[i] = __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return p;
}

// COUNT / BitSet scans (no aggregate): only the count and nan words of a
// Partial are stored and read back -- 2 of its 6 words
__device__ __forceinline__ void store_count_sc1(Partial* dst, const Partial& p) {
  const uint64_t* s = reinterpret_cast<const uint64_t*>(&p);
  uint64_t* d = reinterpret_cast<uint64_t*>(dst);
  __hip_atomic_store(d, s[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(d + kSegStride - 1, s[kSegStride - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ Acc load_count_sc1(const Partial* src) {
  uint64_t* s = reinterpret_cast<uint64_t*>(const_cast<Partial*>(src));
  Partial p;
  uint64_t* d = reinterpret_cast<uint64_t*>(&p);
  d[0] = __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  d[kSegStride - 1] = __hip_atomic_load(s + kSegStride - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  Acc b;
  acc_init(b);
  b.count = p.count;
  b.nan = p.nan_seen;
  return b;
}

// Reduce n partials with one block in a fixed order (thread i folds i, i+256,
// ... sequentially, then a fixed xor tree and wave order) and write the
// results.  Bit-reproducible for a given grid.  SC1: the partials were
// stored write-through in this launch and are read with sc1 loads; LITE: only
// their count and nan words were stored.
// NF partials' loads in flight per thread; the fold order (i, i + 256, ...
// per thread, then the wave / block tree) does not depend on NF
template <bool SC1, bool LITE = false, int NF = 4>
__device__ __forceinline__ void finalize_block(const Partial* parts, int64_t n, int32_t agg_kind, AggOut* out,
                                               int64_t* count_out, int32_t* nan_flag) {
  __shared__ Acc fsh[kWaves];
  Acc a;
  acc_init(a);
  // 4 partials' loads in flight per thread, then folded in the same order
  // (i, i + 256, ...) -- one at a time, each sc1 load's trip to memory was
  // paid serially (4 per thread at 1024 blocks)
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += NF * kBlock) {
    Acc b[NF];
#pragma unroll
    for (int k = 0; k < NF; ++k) {
      const int64_t i = i0 + (int64_t)k * kBlock;
      if (i < n)
        b[k] = LITE ? load_count_sc1(parts + i) : from_partial(SC1 ? load_partial_sc1(parts + i) : parts[i]);
      else
        acc_init(b[k]);
    }
#pragma unroll
    for (int k = 0; k < NF; ++k) acc_merge(a, b[k]);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    Acc b = shfl_xor_acc(a, m);
    acc_merge(a, b);
  }
  if ((threadIdx.x & 63) == 0) fsh[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    Acc r = fsh[0];
    for (int w = 1; w < kWaves; ++w) acc_merge(r, fsh[w]);
    if (out) {
      AggOut o;
      o.count = r.count;
      o.agg_type = agg_kind == kReal ? 2 : 1;  // MBX_ATTR_REAL / MBX_ATTR_INTEGER
      o.pad_ = 0;
      o.isum = r.isum;
      o.imin = r.imin;
      o.imax = r.imax;
      o.fsum = r.fsum;
      o.fmin = r.fmin;
      o.fmax = r.fmax;
      *out = o;
    }
    if (count_out) *count_out = r.count;
    if (nan_flag) {  // [0] this launch, [1] sticky until mbx_sync reads it
      nan_flag[0] = r.nan;
      if (r.nan) nan_flag[1] = 1;
    }
  }
}

// One block arrives (thread 0, after its partial is drained); true for the
// last block of the grid.  Every ticket it exhausts is reset to 0 for the next
// launch on the stream (only the last arriver of a ticket touches it again).
__device__ __forceinline__ bool arrive(uint32_t* ticket, int groups) {
  const uint32_t nb = gridDim.x;
  if (groups <= 1 || nb <= (uint32_t)groups) {
    const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t != nb - 1) return false;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  const uint32_t G = (uint32_t)groups;
  const uint32_t g = blockIdx.x % G;
  const uint32_t members = (nb - g + G - 1) / G;  // blocks b < nb with b % G == g
  uint32_t* gt = ticket + (1 + g) * kTicketStride;
  const uint32_t t = __hip_atomic_fetch_add(gt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t != members - 1) return false;
  __hip_atomic_store(gt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t u = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (u != G - 1) return false;
  __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// COUNT finalize without partials (kFinPackedCount).  One 64-bit atomic word
// per ticket: bits 0..11 arrivals, 12..23 blocks that saw a NaN, 24..63 the
// row count.  Integer addition is order-free, so the total is exact and the
// same for every arrival order.  The last arriver of a group adds the group's
// sum to the top word; the last arriver of the top word holds the launch's
// total, writes it, and (like every last arriver) resets its word for the
// next launch on the stream.  One dependent atomic round trip per level, no
// partial stores or loads (the sc1 path pays store, ticket and load trips).
constexpr int kPackArrBits = 12, kPackNanBits = 12;
constexpr uint64_t kPackArrMask = (1ull << kPackArrBits) - 1;
constexpr uint64_t kPackNanMask = (1ull << kPackNanBits) - 1;

__device__ __forceinline__ uint64_t pack_count(int64_t count, uint32_t nan_blocks) {
  return ((uint64_t)count << (kPackArrBits + kPackNanBits)) | ((uint64_t)nan_blocks << kPackArrBits) | 1ull;
}

// true for the last arriver; *sum = the word's total including this add
__device__ __forceinline__ bool packed_arrive(uint64_t* w, uint64_t add, uint32_t members, uint64_t* sum) {
  const uint64_t prev = __hip_atomic_fetch_add(w, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((prev & kPackArrMask) != members - 1) return false;
  __hip_atomic_store(w, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  *sum = prev + add;
  return true;
}

// true for the final arriver of the launch
__device__ __forceinline__ bool packed_count_finalize(uint32_t* ticket, int groups, int64_t count, int nan,
                                                      int64_t* count_out, int32_t* nan_out) {
  const uint32_t nb = gridDim.x;
  uint64_t add = pack_count(count, nan ? 1u : 0u), sum;
  if (groups > 1 && nb > (uint32_t)groups) {
    const uint32_t G = (uint32_t)groups;
    const uint32_t g = blockIdx.x % G;
    const uint32_t members = (nb - g + G - 1) / G;
    if (!packed_arrive(reinterpret_cast<uint64_t*>(ticket + (1 + g) * kTicketStride), add, members, &sum)) return false;
    const uint64_t nan_g = (sum >> kPackArrBits) & kPackNanMask;
    add = pack_count((int64_t)(sum >> (kPackArrBits + kPackNanBits)), nan_g ? 1u : 0u);
    if (!packed_arrive(reinterpret_cast<uint64_t*>(ticket), add, G, &sum)) return false;
  } else if (!packed_arrive(reinterpret_cast<uint64_t*>(ticket), add, nb, &sum)) {
    return false;
  }
  if (count_out) *count_out = (int64_t)(sum >> (kPackArrBits + kPackNanBits));
  if (nan_out) {  // [0] this launch, [1] sticky until mbx_sync reads it
    const int32_t nan_any = ((sum >> kPackArrBits) & kPackNanMask) ? 1 : 0;
    nan_out[0] = nan_any;
    if (nan_any) nan_out[1] = 1;
  }
  return true;
}

// Block-wide fixed-order reduction of per-thread accumulators into this
// block's Partial; with a ticket, the last block to arrive then finalizes all
// partials inside the same launch.  Hand-off (MI355X: per-XCD L2s are not
// coherent): the storing thread drains its store, releases at agent scope and
// takes a relaxed agent-scope ticket; the last arriver acquires at agent scope
// before the whole block reads the partials with plain loads.
template <bool FULL>
__device__ __forceinline__ void block_reduce_store(Acc a, const ScanLaunch& L) {
  __shared__ Acc sh[kWaves];
  __shared__ int is_last;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  if (FULL) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      Acc b = shfl_xor_acc(a, m);
      acc_merge(a, b);
    }
  } else {
    int nn = a.nan;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) nn |= __shfl_xor(nn, m);
    a.nan = nn;
  }
  if (lane == 0) sh[wave] = a;
  __syncthreads();
  if (!FULL && L.fin_mode == kFinSegOnly) {
    if (threadIdx.x == 0 && L.seg_counts) {
      int64_t cnt = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) cnt += sh[w].count;
      __hip_atomic_store(L.seg_counts + blockIdx.x, cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (!FULL && L.fin_mode == kFinFrame) {
    if (threadIdx.x == 0) {
      Acc r = sh[0];
#pragma unroll
      for (int w = 1; w < kWaves; ++w) acc_merge(r, sh[w]);
      // result unused: a no-return atomic, nothing waits for it in the block
      __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(L.count_out) + (blockIdx.x % kFrameSlots) * kFrameSlotStride,
                             pack_count(r.count, r.nan ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (r.nan && L.nan_out) __hip_atomic_store(L.nan_out + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (!FULL && L.ticket && L.fin_mode == kFinPackedCount) {
    if (threadIdx.x == 0) {
      Acc r = sh[0];
#pragma unroll
      for (int w = 1; w < kWaves; ++w) acc_merge(r, sh[w]);
      if (L.seg_counts)  // the BitSet's segment count, for a later compaction launch: not waited for
        __hip_atomic_store(L.seg_counts + blockIdx.x, r.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      packed_count_finalize(L.ticket, L.ticket_groups, r.count, r.nan, L.count_out, L.nan_out);
    }
    return;
  }
  if (threadIdx.x == 0) {
    Acc r = sh[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) acc_merge(r, sh[w]);
    if (L.seg_counts)
      __hip_atomic_store(L.seg_counts + blockIdx.x, r.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    Partial p;
    p.count = r.count;
    p.isum = r.isum;
    p.fsum = r.fsum;
    p.imin = r.imin;
    p.imax = r.imax;
    p.fmin = r.fmin;
    p.fmax = r.fmax;
    p.nan_seen = r.nan;
    p.pad_ = 0;
    if (L.ticket && L.fin_mode == kFinWriteThrough) {
      // write-through (sc1) partial, drained, then the ticket: no L2
      // write-back fence needed (MI355X_MICROARCH.md, Valid forms row 1)
      if (FULL)
        store_partial_sc1(L.partials + blockIdx.x, p);
      else
        store_count_sc1(L.partials + blockIdx.x, p);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      is_last = arrive(L.ticket, L.ticket_groups);
#ifdef MBX_DIAG
    } else if (L.ticket) {  // kFinFences: plain stores + release / acquire fences (the A/B reference form)
      L.partials[blockIdx.x] = p;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      is_last = arrive(L.ticket, L.ticket_groups);
      if (is_last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
#endif
    } else {
      L.partials[blockIdx.x] = p;
    }
  }
  if (!L.ticket) return;
  __syncthreads();
  if (is_last) {
#ifdef MBX_DIAG
    if (L.fin_mode != kFinWriteThrough) {
      finalize_block<false>(L.partials, gridDim.x, L.agg_kind, L.agg_out, L.count_out, L.nan_out);
      return;
    }
#endif
    finalize_block<true, !FULL>(L.partials, gridDim.x, L.agg_kind, L.agg_out, L.count_out, L.nan_out);
  }
}

// Pack the 4-row nibbles of 16 consecutive lanes into one BitSet word.
// Lane l holds rows 4l..4l+3 of the tile; word k of the tile = lanes 16k..16k+15.
__device__ __forceinline__ uint64_t pack_word16(uint32_t nib, int lane) {
  uint32_t o = __shfl_xor(nib, 1);
  uint32_t v8 = (lane & 1) ? (o | (nib << 4)) : (nib | (o << 4));
  o = __shfl_xor(v8, 2);
  uint32_t v16 = (lane & 2) ? (o | (v8 << 8)) : (v8 | (o << 8));
  o = __shfl_xor(v16, 4);
  uint32_t v32 = (lane & 4) ? (o | (v16 << 16)) : (v16 | (o << 16));
  o = __shfl_xor(v32, 8);
  return (lane & 8) ? (((uint64_t)v32 << 32) | o) : ((uint64_t)v32 | ((uint64_t)o << 32));
}

// Positions of one step of 64 consecutive BitSet words (lane = word `base +
// lane`, mw = its bits) to ids[off ...]; off advances by the step's count.
// Steps of <= kStageIds positions go through the wave's LDS stage `st`
// (12-bit offsets within the step) and are copied out with coalesced 512-byte
// wave stores; the stage is filled by whichever loop is shorter -- each lane
// peeling its own word's bits (iterations = the largest popcount) or the wave
// visiting the non-zero words with lane = bit (iterations = non-zero words).
// Denser steps store straight from the lane = bit loop: one store per
// non-zero word, each with > 32 active lanes on average.  (A direct store per
// non-zero word on moderately sparse steps made the slowest wave of a 10M-row
// compaction 3.6x the median: profiles/r02/anatomy.)
constexpr uint32_t kStageIds = 2048;

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int j) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), j);
  return ((uint64_t)hi << 32) | lo;
}

// One step in two halves, so a caller can stage a step before it knows the
// step's output offset: stage_step returns the step's count (uniform) and,
// for <= kStageIds positions, leaves their 12-bit in-step offsets in `st`;
// store_step writes them (or, for a denser step, stores straight from the
// lane = bit loop) at ids[off ...].  cap: positions at or beyond it are not
// stored (a caller buffer smaller than the selection; the count covers them).
struct StepScan {
  uint32_t excl;   // this lane's word's first slot within the step
  uint32_t total;  // the step's positions (uniform)
};

// sbase / pbase: stage from st[sbase] on, offsets + pbase; nothing is staged
// unless the step's positions fit below kStageIds
// Wave-wide inclusive prefix sum / max on the DPP paths (VALU only, no LDS
// permute traffic): row_shr 1, 2, 4, 8 inside each 16-lane row, then
// row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry the rows'
// totals upwards.  Lanes a DPP step does not write keep `old` = 0.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, true);
}
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += dpp0<0x111>(x);
  x += dpp0<0x112>(x);
  x += dpp0<0x114>(x);
  x += dpp0<0x118>(x);
  x += dpp0<0x142, 0xa>(x);
  x += dpp0<0x143, 0xc>(x);
  return x;
}
// lane 63 holds the maximum of every lane's (unsigned) value
__device__ __forceinline__ uint32_t wave_max_to_63(uint32_t x) {
  x = max(x, dpp0<0x111>(x));
  x = max(x, dpp0<0x112>(x));
  x = max(x, dpp0<0x114>(x));
  x = max(x, dpp0<0x118>(x));
  x = max(x, dpp0<0x142, 0xa>(x));
  x = max(x, dpp0<0x143, 0xc>(x));
  return x;
}

__device__ __forceinline__ StepScan stage_step(uint64_t mw, uint16_t* st, int lane, uint32_t sbase = 0,
                                               uint32_t pbase = 0) {
  const uint32_t pc = (uint32_t)__popcll(mw);
  const uint32_t incl = wave_incl_sum(pc);
  StepScan r;
  r.excl = incl - pc;
  r.total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  if (r.total == 0 || sbase + r.total > kStageIds) return r;
  st += sbase;
  uint64_t nz = __ballot(mw != 0ull);
  const uint32_t maxpc = (uint32_t)__builtin_amdgcn_readlane((int)wave_max_to_63(pc), 63);
  if (maxpc <= (uint32_t)__popcll(nz)) {
    uint64_t m = mw;
    uint32_t o = r.excl;
    while (m) {
      st[o++] = (uint16_t)(pbase + lane * 64 + __builtin_ctzll(m));
      m &= m - 1ull;
    }
  } else {
    while (nz) {
      const int j = __builtin_ctzll(nz);
      nz &= nz - 1ull;
      const uint64_t m = readlane64(mw, j);
      const uint32_t slot = (uint32_t)__builtin_amdgcn_readlane((int)r.excl, j);
      if ((m >> lane) & 1ull) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        st[slot + below] = (uint16_t)(pbase + j * 64 + lane);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();  // LDS ops of one wave complete in order
  return r;
}

// Late materialisation fused into the compaction (C4: positions + projected
// int / float columns): where a step's positions are written, the values of
// up to 4 four-byte columns at those rows are loaded (every load of two rows
// per lane issued before their stores) and written beside them.
struct Gather4 {
  const int32_t* col[4];
  uint32_t* out[4];
  int32_t n;  // projected columns (0: positions only)
  int64_t cap = INT64_MAX;  // rows the outputs (and positions) hold
  // words between rows of col[g]: 1 for a column, the group's width when the
  // column is read from a column group (its row's projected values share a line)
  int32_t stride[4] = {1, 1, 1, 1};
  // two projected columns side by side in a group (C4's (c0, c1)): a row's
  // values are one aligned 8-byte load (gather4_pairing)
  int32_t pair = 0;
};

// the 8-byte pair form applies: 2 columns, adjacent words of one row of a
// group (even stride, 8-byte aligned); allow = false (tuning gather_pair 0)
// keeps two 4-byte loads per row (A/B)
inline void gather4_pairing(Gather4& G, bool allow) {
  G.pair = allow && G.n == 2 && G.col[1] == G.col[0] + 1 && G.stride[0] == G.stride[1] && G.stride[0] % 2 == 0 &&
           ((uintptr_t)G.col[0] & 7) == 0;
}

// one row's projected values (every load issued before any is used)
template <int G4>
__device__ __forceinline__ void gather_row(const Gather4& G, int64_t p, uint32_t (&v)[G4 > 0 ? G4 : 1]) {
  if constexpr (G4 >= 2) {
    if (G.pair) {
      const uint2 x = *reinterpret_cast<const uint2*>(G.col[0] + p * G.stride[0]);
      v[0] = x.x;
      v[1] = x.y;
      return;
    }
  }
#pragma unroll
  for (int g = 0; g < G4; ++g)
    if (g < G.n) v[g] = (uint32_t)G.col[g][p * G.stride[g]];
}

// the narrow gather's source of a projected 4-byte column: its column group
// when it has one, else the column
__device__ __host__ inline void gather4_source(Gather4& G, int g, const ProjCol& pc) {
  if (pc.gstride > 0) {
    G.col[g] = (const int32_t*)pc.gbase;
    G.stride[g] = pc.gstride;
  } else {
    G.col[g] = (const int32_t*)pc.base;
    G.stride[g] = 1;
  }
}

// Any projection (ColumnarIndexScan's out_indexes with char(n) columns, or
// more than 4 columns): template argument G4 == kWide.  Column g's rows are
// sw[g] 32-bit words (the device row image: 1 for int / float, stride_w for
// char(n)); a lane copies its row's words, all loads before the stores.
constexpr int kWide = -1;
struct GatherW {
  const uint32_t* col[kMaxProj];
  uint32_t* out[kMaxProj];
  int32_t sw[kMaxProj];
  int32_t n;
  int64_t cap = INT64_MAX;  // rows the outputs (and positions) hold
};

// An output store of the compaction: plain, or write-through (`sc1`: the
// line leaves the XCD's L2 with the store instead of staying dirty there
// for the end-of-kernel write-back).  Write-through is the default for
// positions-only compactions (G4 == 0): C2 k_select_ids 7.5 -> 7.0 us, C2
// query 16.7 -> 15.6 us (one launch 16.3 -> 15.2); with gathered values
// (C4) it is neutral for the projection and +1.2 us with positions, so
// those stay plain.  Kernel dbg bit 5 (select_dbg 512) flips the choice
// (profiles/r03/lb/wt_*).
// wt: 0 plain, 1 write-through, 2 nontemporal (the line is not kept in L2)
template <class T>
__device__ __forceinline__ void put(T* p, T v, int wt) {
  if (wt == 1)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else if (wt == 2)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

__device__ __forceinline__ void wide_row(const GatherW& G, int64_t p, int64_t o) {
  for (int g = 0; g < G.n; ++g) {
    const int sw = G.sw[g];
    const uint32_t* __restrict__ s = G.col[g] + p * sw;
    uint32_t* __restrict__ d = G.out[g] + o * sw;
    if (sw == 1) {
      d[0] = s[0];
      continue;
    }
    int k = 0;
    for (; k + 4 <= sw; k += 4) {
      const uint32_t a = s[k], b = s[k + 1], c = s[k + 2], e = s[k + 3];
      d[k] = a;
      d[k + 1] = b;
      d[k + 2] = c;
      d[k + 3] = e;
    }
    for (; k < sw; ++k) d[k] = s[k];
  }
}

template <int G4, class GT = Gather4>
__device__ __forceinline__ void store_step(int64_t base, uint64_t mw, const StepScan& r, int64_t& off,
                                           int64_t row_offset, int64_t* __restrict__ ids, const uint16_t* st,
                                           int lane, const GT& G, uint32_t first = 0, int wt = 0,
                                           bool nt = false) {
  if (r.total == 0) return;
  const int64_t lbase = base * 64;  // table-local row of bit 0 of word `base`
  if (r.total <= kStageIds && G4 == 0) {
    // positions only: 4 staged positions per lane read together, then
    // their 4 stores (one LDS round trip per 256 positions, not per 64)
    for (uint32_t i0 = first + lane; i0 < r.total; i0 += 256) {
      uint32_t q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = i0 + 64u * u < r.total ? st[i0 + 64u * u] : 0u;
      if (ids) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (i0 + 64u * u < r.total) {
            if (nt)  // diagnostic (-DMBX_DIAG, dbg bit 9): nontemporal positions stores
              __builtin_nontemporal_store(row_offset + lbase + q[u], &ids[off + i0 + 64u * u]);
            else
              put(&ids[off + i0 + 64u * u], row_offset + lbase + q[u], wt);
          }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the stage is rewritten by the next step
  } else if (r.total <= kStageIds) {
    // staged positions from `first` on (the caller wrote those below it)
    for (uint32_t i0 = first + lane; i0 < r.total; i0 += 128) {
      const uint32_t i1 = i0 + 64;
      const bool two = i1 < r.total;
      const int64_t p0 = lbase + st[i0];
      const int64_t p1 = two ? lbase + st[i1] : p0;
      if constexpr (G4 == kWide) {
        if (ids) {
          ids[off + i0] = row_offset + p0;
          if (two) ids[off + i1] = row_offset + p1;
        }
        wide_row(G, p0, off + i0);
        if (two) wide_row(G, p1, off + i1);
      } else {
        uint32_t v0[G4 > 0 ? G4 : 1], v1[G4 > 0 ? G4 : 1];
        gather_row<G4>(G, p0, v0);
        gather_row<G4>(G, p1, v1);
        if (ids) {
          put(&ids[off + i0], row_offset + p0, wt);
          if (two) put(&ids[off + i1], row_offset + p1, wt);
        }
#pragma unroll
        for (int g = 0; g < G4; ++g)
          if (g < G.n) {
            put(&G.out[g][off + i0], v0[g], wt);
            if (two) put(&G.out[g][off + i1], v1[g], wt);
          }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the stage is rewritten by the next step
  } else {
    uint64_t nz = __ballot(mw != 0ull);
    while (nz) {
      const int j = __builtin_ctzll(nz);
      nz &= nz - 1ull;
      const uint64_t m = readlane64(mw, j);
      const uint32_t slot = (uint32_t)__builtin_amdgcn_readlane((int)r.excl, j);
      if ((m >> lane) & 1ull) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const int64_t p = lbase + j * 64 + lane;
        const int64_t o = off + slot + below;
        if (ids) put(&ids[o], row_offset + p, wt);
        if constexpr (G4 == kWide) {
          wide_row(G, p, o);
        } else {
          uint32_t v[G4 > 0 ? G4 : 1];
          gather_row<G4>(G, p, v);
#pragma unroll
          for (int g = 0; g < G4; ++g)
            if (g < G.n) put(&G.out[g][o], v[g], wt);
        }
      }
    }
  }
  off += r.total;
}

template <int G4 = 0, class GT = Gather4>
__device__ __forceinline__ void emit_step(int64_t base, uint64_t mw, int64_t& off, int64_t row_offset,
                                          int64_t* __restrict__ ids, uint16_t* st, int lane, const GT& G,
                                          int wt = 0) {
  const StepScan r = stage_step(mw, st, lane);
  store_step<G4, GT>(base, mw, r, off, row_offset, ids, st, lane, G, 0, wt);
}

// ------------------------------------------------------------- fast scan
//
// K 4-byte columns in plan slots 0..K-1, every term `slot OP literal`.
// Each wave streams whole 256-row tiles of its block's segment: one
// global_load_dwordx4 per column per tile, terms folded into per-row
// conjunct bitmasks (cb), the CNF holds when cb == all_conj.
// One tile's column data in registers: K 4-byte slots (lane l holds rows
// 4l..4l+3) and KS 16-byte string slots (char(13..16)).  String rows are
// loaded so that every load instruction reads one contiguous KiB -- load j of
// lane l holds row 64j + l -- and their compare results are moved back to the
// 4-rows-per-lane layout through the wave ballots (= the tile's 4 BitSet words).
template <int K, int KS>
struct TileRegs {
  int32_t v[K > 0 ? K : 1][4];
  uint32_t s[KS > 0 ? KS : 1][4][4];
};

// String.compareTo sign of four zero-padded 16-byte rows against a literal of
// <= 4 words (big-endian word order = modified-UTF-8 byte order)
__device__ __forceinline__ void str16_cmp4(const uint32_t (&rows)[4][4], const uint32_t (&lit)[4], int32_t (&c)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int32_t r = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t x = __builtin_bswap32(rows[j][i]);
      const int32_t d = x < lit[i] ? -1 : (x > lit[i] ? 1 : 0);
      r = r != 0 ? r : d;
    }
    c[j] = r;
  }
}

// A string term of the range-test body (IR = 2) over four zero-padded
// 16-byte rows: rs[j] = the term holds for row j.  Each row is two 64-bit
// big-endian keys (hi = bytes 0..7, lo = bytes 8..15), so its compareTo sign
// against the literal (lhi, llo) comes from two 64-bit compares per key, and
// the range test of that sign is the acceptance of lt / eq / gt (a_lt, a_eq,
// a_gt: uniform, from the term's rlo / rspan / rneg) -- the same results as
// str16_cmp4 + the range test, a third of the VALU instructions (C5's
// aggregate scan was 62 % VALU-busy, profiles/r05/u).
__device__ __forceinline__ void str16_accept4(const uint32_t (&rows)[4][4], uint64_t lhi, uint64_t llo, bool a_lt,
                                              bool a_eq, bool a_gt, bool (&rs)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint64_t hi = ((uint64_t)__builtin_bswap32(rows[j][0]) << 32) | __builtin_bswap32(rows[j][1]);
    const uint64_t lo = ((uint64_t)__builtin_bswap32(rows[j][2]) << 32) | __builtin_bswap32(rows[j][3]);
    const bool heq = hi == lhi;
    const bool lt = hi < lhi || (heq && lo < llo);
    const bool eq = heq && lo == llo;
    rs[j] = lt ? a_lt : (eq ? a_eq : a_gt);
  }
}

// per-tile body shared by every unroll depth: folds the CNF, applies deleted
// rows and emits the requested output.
// TQ > 0: the first TQ terms were hoisted into registers (th) before the
// tile loop and the term loop is unrolled over them (nterms <= TQ); TQ = 0:
// terms are read from the plan per tile.
// RI (row-interleaved tile layout): register j of lane l holds row 64j + l of
// the tile instead of row 4l + j, so the wave ballot of row group j *is*
// BitSet word j of the tile -- no cross-lane packing for BitSet output, the
// deleted words apply as they are, string compares need no re-layout.
// NaN: a row raises only where PredEval would evaluate the float compare --
// the row is live (TupleScan skips deleted rows, R/columnar/TupleScan.java:80-87),
// every required conjunct before the term held and no earlier term of its
// own conjunct did (R/iterator/PredEval.java:164-175); KTerm.req_below.
// WHOLE: the tile is one of the table's full tiles (the main loop's): no row
// bound checks -- only the one partial tile needs them
// IR = 1: every term is an int `column OP literal` (ScanLaunch.int_range): the
// term body is one unsigned range test per row, no branch on the operator or
// the comparison type (KTerm.rlo / rspan / rneg, mbx_api.cpp int_range_of).
// IR = 2: literal terms of any type, one range test over a signed-ordered key
// (KTerm.rm31: float bits; a char(16) term's compareTo sign); a float term
// still tracks PredEval's NaN reach
template <int K, int KS, int MODE, bool DEL, int TQ = 0, bool RI = false, bool WHOLE = false, int IR = 0>
__device__ __forceinline__ void fast_tile(const ScanLaunch& L, const KPlan* __restrict__ P, const TileRegs<K, KS>& D,
                                          int64_t t, int lane, int nterms, uint32_t all, int agg_slot, bool agg_real,
                                          Acc& acc, uint64_t& wave_count, const KTerm* th = nullptr,
                                          uint64_t* ws = nullptr) {
  const int64_t nrows = L.nrows;
  const int64_t nwords = (nrows + 63) >> 6;
  const int64_t row0 = t * kTileRows + lane * (RI ? 1 : 4);
  constexpr int kRowStep = RI ? 64 : 1;  // row of register j = row0 + j * kRowStep
  uint32_t cb[4] = {0u, 0u, 0u, 0u};
  bool nanr[4] = {false, false, false, false};  // reached a float compare on a NaN
#pragma unroll
  for (int ti = 0; ti < (TQ > 0 ? TQ : nterms); ++ti) {
    if (TQ > 0 && ti > 0 && ti >= nterms) break;  // TQ > 0 implies nterms >= 1
    const KTerm& T = TQ > 0 ? th[ti] : P->terms[ti];
    const int lhs = T.lhs;
    bool r[4];
    if constexpr (IR == 2) {
      const uint32_t lo = (uint32_t)T.rlo, span = T.rspan;
      const bool neg = T.rneg != 0;
      if (KS > 0 && T.kind == kStr) {
        uint32_t lit[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) lit[i] = i < T.swords ? __builtin_bswap32(P->pool[T.soff + i]) : 0u;
        const uint64_t lhi = ((uint64_t)lit[0] << 32) | lit[1], llo = ((uint64_t)lit[2] << 32) | lit[3];
        // the range test of each compareTo sign, decided once per term
        const bool a_lt = (0xffffffffu - lo <= span) != neg;
        const bool a_eq = (0u - lo <= span) != neg;
        const bool a_gt = (1u - lo <= span) != neg;
        bool rs[4];  // rs[j] is row 64j + lane (string slots load row-interleaved)
        if (KS == 1 || lhs == K)
          str16_accept4(D.s[0], lhi, llo, a_lt, a_eq, a_gt, rs);
        else
          str16_accept4(D.s[KS > 1 ? 1 : 0], lhi, llo, a_lt, a_eq, a_gt, rs);
        if (RI) {
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] = rs[j];
        } else {
          const uint64_t w0 = __ballot(rs[0]), w1 = __ballot(rs[1]), w2 = __ballot(rs[2]), w3 = __ballot(rs[3]);
          const int q = lane >> 4;
          const uint64_t w = q == 0 ? w0 : (q == 1 ? w1 : (q == 2 ? w2 : w3));
          const uint32_t nib = (uint32_t)(w >> ((lane & 15) * 4));
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] = (nib >> j) & 1u;
        }
      } else {
        int32_t a[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = D.v[0][j];
#pragma unroll
        for (int s = 1; s < K; ++s)
          if (lhs == s) {
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = D.v[s][j];
          }
        if (T.kind == kReal) {
          // PredEval's NaN reach, worked out only for a tile that holds a
          // NaN (or a NaN literal): one compare per row otherwise
          bool isn[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) isn[j] = __int_as_float(a[j]) != __int_as_float(a[j]);
          if (T.nan_lit || __ballot(isn[0] || isn[1] || isn[2] || isn[3]) != 0ull) {
            const uint32_t below = T.req_below, own = T.conj_bit;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const bool reach = ((cb[j] & below) == below) && !(cb[j] & own);
              nanr[j] = nanr[j] || (reach && (T.nan_lit || isn[j]));
            }
          }
        }
        const uint32_t rm = T.rm31;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t x = (uint32_t)a[j] ^ ((uint32_t)(a[j] >> 31) & rm);
          r[j] = ((x - lo) <= span) != neg;
        }
      }
    } else if constexpr (IR == 1) {
      int32_t a[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = D.v[0][j];
#pragma unroll
      for (int s = 1; s < K; ++s)
        if (lhs == s) {
#pragma unroll
          for (int j = 0; j < 4; ++j) a[j] = D.v[s][j];
        }
      const uint32_t lo = (uint32_t)T.rlo, span = T.rspan;
      const bool neg = T.rneg != 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = (((uint32_t)a[j] - lo) <= span) != neg;
    } else if (KS > 0 && T.kind == kStr) {
      uint32_t lit[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) lit[i] = i < T.swords ? __builtin_bswap32(P->pool[T.soff + i]) : 0u;
      int32_t c[4];
      if (KS == 1 || lhs == K) {
        str16_cmp4(D.s[0], lit, c);
      } else {
        str16_cmp4(D.s[KS > 1 ? 1 : 0], lit, c);
      }
      bool rs[4];
      cmp4<int32_t>(T.op, c, 0, rs);
      // rs[j] is row 64j + lane; ballot j is BitSet word j of the tile
      if (RI) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = rs[j];
      } else {
        const uint64_t w0 = __ballot(rs[0]), w1 = __ballot(rs[1]), w2 = __ballot(rs[2]), w3 = __ballot(rs[3]);
        const int q = lane >> 4;
        const uint64_t w = q == 0 ? w0 : (q == 1 ? w1 : (q == 2 ? w2 : w3));
        const uint32_t nib = (uint32_t)(w >> ((lane & 15) * 4));
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = (nib >> j) & 1u;
      }
    } else {
      int32_t a[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = D.v[0][j];
#pragma unroll
      for (int s = 1; s < K; ++s)
        if (lhs == s) {
#pragma unroll
          for (int j = 0; j < 4; ++j) a[j] = D.v[s][j];
        }
      if (T.kind == kInt) {
        cmp4<int32_t>(T.op, a, T.ilit, r);
      } else {
        float f[4];
        const uint32_t below = T.req_below, own = T.conj_bit;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f[j] = __int_as_float(a[j]);
          const bool reach = ((cb[j] & below) == below) && !(cb[j] & own);
          nanr[j] = nanr[j] || (reach && (T.nan_lit || f[j] != f[j]));
        }
        cmp4<float>(T.op, f, T.flit, r);
      }
    }
    const uint32_t bit = T.conj_bit;
#pragma unroll
    for (int j = 0; j < 4; ++j) cb[j] |= r[j] ? bit : 0u;
  }

  bool live[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) live[j] = WHOLE || row0 + j * kRowStep < nrows;
  const int64_t word = t * kWordsPerTile + (RI ? 0 : (lane >> 4));
  if (DEL && RI) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t dw = (WHOLE || word + j < nwords) ? L.deleted[word + j] : 0ull;  // uniform: one scalar load
      live[j] = live[j] && !((dw >> lane) & 1ull);
    }
  } else if (DEL) {
    const uint64_t dw = (WHOLE || word < nwords) ? L.deleted[word] : 0ull;
    const uint32_t dn = (uint32_t)(dw >> ((lane & 15) * 4)) & 0xFu;
#pragma unroll
    for (int j = 0; j < 4; ++j) live[j] = live[j] && !((dn >> j) & 1u);
  }
  bool p[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    // a conjunct folded to `true` on the host may keep terms for their NaN
    // reach, so its bit can be set without being required
    p[j] = ((cb[j] & all) == all) && live[j];
    acc.nan |= nanr[j] && live[j];
  }
  if (MODE == kModeBitmap && RI) {
    const uint64_t w0 = __ballot(p[0]), w1 = __ballot(p[1]), w2 = __ballot(p[2]), w3 = __ballot(p[3]);
    if (ws) {  // the caller buffers the words (BitSink)
      ws[0] = w0;
      ws[1] = w1;
      ws[2] = w2;
      ws[3] = w3;
    } else {
      const uint64_t w = lane == 0 ? w0 : (lane == 1 ? w1 : (lane == 2 ? w2 : w3));
      if (lane < 4 && (WHOLE || word + lane < nwords)) L.out_words[word + lane] = w;
    }
  } else if (MODE == kModeBitmap) {
    const uint32_t nib = (uint32_t)p[0] | ((uint32_t)p[1] << 1) | ((uint32_t)p[2] << 2) | ((uint32_t)p[3] << 3);
    const uint64_t w = pack_word16(nib, lane);
    if ((lane & 15) == 0 && (WHOLE || word < nwords)) L.out_words[word] = w;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) wave_count += __popcll(__ballot(p[j]));
  if (MODE == kModeAgg && K > 0) {
    int32_t g[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = D.v[0][j];
#pragma unroll
    for (int s = 1; s < K; ++s)
      if (agg_slot == s) {
#pragma unroll
        for (int j = 0; j < 4; ++j) g[j] = D.v[s][j];
      }
    if (agg_real) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float f = __int_as_float(g[j]);
        acc.fsum += p[j] ? (double)f : 0.0;
        acc.fmin = p[j] && f < acc.fmin ? f : acc.fmin;
        acc.fmax = p[j] && f > acc.fmax ? f : acc.fmax;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc.isum += p[j] ? (int64_t)g[j] : 0;
        acc.imin = p[j] && g[j] < acc.imin ? g[j] : acc.imin;
        acc.imax = p[j] && g[j] > acc.imax ? g[j] : acc.imax;
      }
    }
  }
}

typedef int32_t v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4i gv4i;
typedef __attribute__((address_space(1))) const int32_t gi32;

// Column loads through global (address space 1) pointers: global_load, not
// flat_load -- a flat load also counts on lgkmcnt, which forces a full
// s_waitcnt before the first compare and so defeats the load pipeline below.
template <bool NT>
__device__ __forceinline__ v4i load16(const int32_t* p) {
  gv4i* q = (gv4i*)p;
  if (NT) return __builtin_nontemporal_load(q);
  return *q;
}

__device__ __forceinline__ int32_t load4(const int32_t* p) { return *(gi32*)p; }

template <bool NT>
__device__ __forceinline__ int32_t load4n(const int32_t* p) {
  if (NT) return __builtin_nontemporal_load((gi32*)p);
  return *(gi32*)p;
}

// One full tile's 4-byte slot s: dwordx4 rows 4l..4l+3 (RI = false) or four
// 256-byte wave loads, register j = row 64j + l (RI = true).
template <int K, int KS, bool NT, bool RI>
__device__ __forceinline__ void load_slot(TileRegs<K, KS>& D, int s, const int32_t* col, int64_t t, int lane) {
  if (RI) {
#pragma unroll
    for (int j = 0; j < 4; ++j) D.v[s][j] = load4n<NT>(col + t * kTileRows + j * 64 + lane);
  } else {
    const v4i q = load16<NT>(col + t * kTileRows + lane * 4);
    D.v[s][0] = q.x;
    D.v[s][1] = q.y;
    D.v[s][2] = q.z;
    D.v[s][3] = q.w;
  }
}

// The full tiles base + u * ustep (u < U, below tf) of one wave into
// registers.  Loads only, no else path: a branch that also wrote the
// registers would make the compiler join the two and wait for the loads
// right where they are issued.
template <int K, int KS, int U, bool NT, bool RI = false>
__device__ __forceinline__ void load_tiles(TileRegs<K, KS> (&D)[U], int64_t base, int64_t ustep, int64_t tf,
                                           const int32_t* const (&colp)[K > 0 ? K : 1],
                                           const int32_t* const (&strp)[KS > 0 ? KS : 1], int lane) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t t = base + (int64_t)u * ustep;
    if (t < tf) {
#pragma unroll
      for (int s = 0; s < K; ++s) load_slot<K, KS, NT, RI>(D[u], s, colp[s], t, lane);
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const v4i q = load16<NT>(strp[s] + (t * kTileRows + j * 64 + lane) * 4);
          D[u].s[s][j][0] = (uint32_t)q.x;
          D[u].s[s][j][1] = (uint32_t)q.y;
          D[u].s[s][j][2] = (uint32_t)q.z;
          D[u].s[s][j][3] = (uint32_t)q.w;
        }
    }
  }
}

// Clamped form: the same loads, unconditional -- a tile index past tf is
// clamped to tf - 1 (a re-read of a tile in flight anyway, served by L2), so
// every path issues the same number of loads and the waitcnt pass can wait
// for exactly the older group (vmcnt(N)) instead of draining all loads.
template <int K, int KS, int U, bool NT, bool RI = false>
__device__ __forceinline__ void load_tiles_clamped(TileRegs<K, KS> (&D)[U], int64_t base, int64_t ustep, int64_t tf,
                                                   const int32_t* const (&colp)[K > 0 ? K : 1],
                                                   const int32_t* const (&strp)[KS > 0 ? KS : 1], int lane) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    int64_t t = base + (int64_t)u * ustep;
    t = t < tf ? t : tf - 1;
#pragma unroll
    for (int s = 0; s < K; ++s) load_slot<K, KS, NT, RI>(D[u], s, colp[s], t, lane);
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const v4i q = load16<NT>(strp[s] + (t * kTileRows + j * 64 + lane) * 4);
        D[u].s[s][j][0] = (uint32_t)q.x;
        D[u].s[s][j][1] = (uint32_t)q.y;
        D[u].s[s][j][2] = (uint32_t)q.z;
        D[u].s[s][j][3] = (uint32_t)q.w;
      }
  }
}

// The table's one partial tile t (rows t * 256 .. nrows - 1): guarded loads.
template <int K, int KS, bool RI = false>
__device__ __forceinline__ void load_partial(TileRegs<K, KS>& D, int64_t t, int64_t nrows,
                                             const int32_t* const (&colp)[K > 0 ? K : 1],
                                             const int32_t* const (&strp)[KS > 0 ? KS : 1], int lane) {
  const int64_t row0 = t * kTileRows + lane * (RI ? 1 : 4);
  constexpr int kRowStep = RI ? 64 : 1;
#pragma unroll
  for (int s = 0; s < K; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      D.v[s][j] = row0 + j * kRowStep < nrows ? load4(colp[s] + row0 + j * kRowStep) : 0;
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t r = t * kTileRows + j * 64 + lane;
        D.s[s][j][i] = r < nrows ? (uint32_t)load4(strp[s] + r * 4 + i) : 0u;
      }
}

// U tiles per wave iteration: all loads of the U tiles are issued before the
// first compare (U x (K + 4 KS) x 1 KiB in flight per wave).  A block owns a
// contiguous segment of tiles, dealt round-robin to its 4 waves (per-segment
// counts feed compaction).  A grid-stride interleave measured equal on MI355X
// (DESIGN.md section 5).
// TQ > 0: <= TQ literal terms hoisted into registers, term loop unrolled.
template <int K, int KS, int MODE, bool DEL, int U, bool NT, int TQ = 0, bool RI = false, int IR = 0>
__global__ __launch_bounds__(kBlock) void k_scan_fast(ScanLaunch L) {
  const KPlan* __restrict__ P = L.plan;
  const int lane = threadIdx.x & 63;
  const int wave = (int)uniform(threadIdx.x >> 6);
  const int64_t nrows = L.nrows;
  const int64_t ntiles = (nrows + kTileRows - 1) / kTileRows;
  const int64_t t0 = (int64_t)blockIdx.x * L.tiles_per_block;
  const int64_t t1 = min(t0 + L.tiles_per_block, ntiles);
  constexpr int64_t ustep = kWaves;  // between the U tiles of one wave
  const int nterms = P->nterms;
  const uint32_t all = P->all_conj;
  const int agg_slot = MODE == kModeAgg ? P->agg_slot : 0;
  const bool agg_real = L.agg_kind == kReal;

  const int32_t* colp[K > 0 ? K : 1];
#pragma unroll
  for (int s = 0; s < K; ++s) colp[s] = (const int32_t*)P->cols[s].base;
  const int32_t* strp[KS > 0 ? KS : 1];
#pragma unroll
  for (int s = 0; s < KS; ++s) strp[s] = (const int32_t*)P->cols[K + s].base;

  Acc acc;
  acc_init(acc);
  uint64_t wave_count = 0;
  KTerm th[TQ > 0 ? TQ : 1];
#pragma unroll
  for (int ti = 0; ti < TQ; ++ti)
    if (ti < nterms) th[ti] = P->terms[ti];

  // full tiles in the main loop; the partial last tile (if any) after it
  const int64_t tf = min(t1, nrows / kTileRows);
  // BitSink (BitSet output, RI layout): a wave's full tiles come in the order
  // t0 + wave + i * ustep; the 4 words of its i-th tile go to lanes
  // 4 (i % 16) .. 4 (i % 16) + 3 of one register, stored with ONE store per
  // 16 tiles -- a store in every tile iteration holds up the next loads
  // (their registers wait for the store's data to be read), 91 vs 70 us at
  // 100M rows.
  constexpr bool kSink = MODE == kModeBitmap && RI;
  uint64_t sink = 0;
  int64_t sink_t = t0 + wave;  // tile of slot 0 of the current 16-tile chunk
  int sink_n = 0;              // tiles captured in the chunk (uniform)
  // L.sink_lds: the words go to this block's LDS stage instead and are stored
  // in one burst when the block's loads are done -- BitSet stores spread
  // through the read stream cost ~16 us at 100M rows (82 vs 66 us for the
  // COUNT scan of the same column) for 12.5 MB written
  extern __shared__ uint64_t sink_stage[];
  auto sink_flush = [&]() {
    if (sink_n > 0) {
      const int sl = lane >> 2;
      if (sl < sink_n) {
        const int64_t t = sink_t + (int64_t)sl * ustep;
        if (L.sink_lds)
          sink_stage[(t - t0) * kWordsPerTile + (lane & 3)] = sink;
        else
          put(&L.out_words[t * kWordsPerTile + (lane & 3)], sink, L.words_wt != 0);
      }
      sink_t += 16 * ustep;
      sink_n = 0;
    }
  };
  auto compute = [&](TileRegs<K, KS>(&D)[U], int64_t base) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t t = base + (int64_t)u * ustep;
      if (t < tf) {
        if constexpr (kSink) {
          uint64_t w[4];
          fast_tile<K, KS, MODE, DEL, TQ, RI, true, IR>(L, P, D[u], t, lane, nterms, all, agg_slot, agg_real, acc,
                                                  wave_count, th, w);
          if ((lane >> 2) == sink_n) {
            const int j = lane & 3;
            sink = j == 0 ? w[0] : (j == 1 ? w[1] : (j == 2 ? w[2] : w[3]));
          }
          if (++sink_n == 16) sink_flush();
        } else {
          fast_tile<K, KS, MODE, DEL, TQ, RI, true, IR>(L, P, D[u], t, lane, nterms, all, agg_slot, agg_real, acc,
                                                  wave_count, th);
        }
      }
    }
  };
  const int64_t step = ustep * U;
  for (int64_t base = t0 + wave; base < tf; base += step) {
    TileRegs<K, KS> D[U];
    if (TQ > 0)  // every path issues all U loads: exact vmcnt waits
      load_tiles_clamped<K, KS, U, NT, RI>(D, base, ustep, tf, colp, strp, lane);
    else
      load_tiles<K, KS, U, NT, RI>(D, base, ustep, tf, colp, strp, lane);
    compute(D, base);
  }
  if constexpr (kSink) {
    sink_flush();
    if (L.sink_lds) {  // uniform
      __syncthreads();
      const int64_t nw = (tf > t0 ? tf - t0 : 0) * kWordsPerTile;
      uint64_t* dst = L.out_words + t0 * kWordsPerTile;
      for (int64_t i = threadIdx.x; i < nw; i += kBlock) put(&dst[i], sink_stage[i], L.words_wt != 0);
    }
  }
  const int64_t tp = nrows / kTileRows;  // the partial tile, owned like any other tile of [t0, t1)
  if ((nrows % kTileRows) != 0 && tp >= t0 + wave && tp < t1 && (tp - t0 - wave) % ustep == 0) {
    TileRegs<K, KS> D;
    load_partial<K, KS, RI>(D, tp, nrows, colp, strp, lane);
    fast_tile<K, KS, MODE, DEL, TQ, RI, false, IR>(L, P, D, tp, lane, nterms, all, agg_slot, agg_real, acc, wave_count,
                                                 th);
  }
  acc.count = lane == 0 ? (int64_t)wave_count : 0;
  block_reduce_store<MODE == kModeAgg>(acc, L);
}

// ---------------------------------------------------------- generic scan
//
// Any CNF the host accepted: char(n) strings, column-vs-column terms, more
// than 4 columns.  One row per lane; the ballot of a wave is one BitSet word.
template <int MODE, bool DEL>
__global__ __launch_bounds__(kBlock) void k_scan_generic(ScanLaunch L) {
  const KPlan* __restrict__ P = L.plan;
  const int lane = threadIdx.x & 63;
  const int wave = (int)uniform(threadIdx.x >> 6);
  const int64_t nrows = L.nrows;
  const int64_t nwords = (nrows + 63) >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * L.tiles_per_block * kWordsPerTile;
  const int64_t w1 = min(w0 + L.tiles_per_block * kWordsPerTile, nwords);
  const int nterms = P->nterms;
  const uint32_t all = P->all_conj;
  const bool agg_real = L.agg_kind == kReal;

  Acc acc;
  acc_init(acc);
  uint64_t wave_count = 0;

  for (int64_t w = w0 + wave; w < w1; w += kWaves) {
    const int64_t row = w * 64 + lane;
    const bool valid = row < nrows;
    uint32_t cb = 0;
    bool nanr = false;  // reached a float compare on a NaN (fast_tile's rule)
    for (int ti = 0; ti < nterms; ++ti) {
      const KTerm& T = P->terms[ti];
      bool r = false;
      if (valid) {
        const KCol& A = P->cols[T.lhs];
        if (T.kind == kStr) {
          const uint32_t* ap = (const uint32_t*)A.base + row * A.stride_w;
          int c;
          if (T.rhs >= 0) {
            const KCol& B = P->cols[T.rhs];
            c = str_cmp(ap, A.stride_w, (const uint32_t*)B.base + row * B.stride_w, B.stride_w);
          } else {
            c = str_cmp(ap, A.stride_w, P->pool + T.soff, T.swords);
          }
          r = cmp1<int>(T.op, c, 0);
        } else if (T.kind == kInt) {
          const int32_t a = ((const int32_t*)A.base)[row];
          const int32_t b = T.rhs >= 0 ? ((const int32_t*)P->cols[T.rhs].base)[row] : T.ilit;
          r = cmp1<int32_t>(T.op, a, b);
        } else {
          const float a = ((const float*)A.base)[row];
          const float b = T.rhs >= 0 ? ((const float*)P->cols[T.rhs].base)[row] : T.flit;
          const bool reach = ((cb & T.req_below) == T.req_below) && !(cb & T.conj_bit);
          nanr = nanr || (reach && (T.nan_lit || a != a || b != b));
          r = cmp1<float>(T.op, a, b);
        }
      }
      cb |= r ? T.conj_bit : 0u;
    }
    bool live = valid;
    if (DEL) live = live && !((L.deleted[w] >> lane) & 1ull);
    const bool p = live && (cb & all) == all;
    acc.nan |= nanr && live;
    const uint64_t m = __ballot(p);
    if (MODE == kModeBitmap && lane == 0) L.out_words[w] = m;
    wave_count += __popcll(m);
    if (MODE == kModeAgg && p) {
      const KCol& G = P->cols[P->agg_slot];
      if (agg_real) {
        const float f = ((const float*)G.base)[row];
        acc.fsum += (double)f;
        acc.fmin = f < acc.fmin ? f : acc.fmin;
        acc.fmax = f > acc.fmax ? f : acc.fmax;
      } else {
        const int32_t g = ((const int32_t*)G.base)[row];
        acc.isum += g;
        acc.imin = g < acc.imin ? g : acc.imin;
        acc.imax = g > acc.imax ? g : acc.imax;
      }
    }
  }
  acc.count = lane == 0 ? (int64_t)wave_count : 0;
  block_reduce_store<MODE == kModeAgg>(acc, L);
}

// --------------------------------------------------------------- finalize

__global__ __launch_bounds__(kBlock) void k_finalize(const Partial* __restrict__ parts, int64_t n,
                                                     int32_t agg_kind, AggOut* out, int64_t* count_out,
                                                     int32_t* nan_flag) {
  // its own launch, its own registers: 16 partials in flight per thread
  // (4096 blocks' partials in one memory round trip instead of four)
  finalize_block<false, false, 16>(parts, n, agg_kind, out, count_out, nan_flag);
}

// ---------------------------------------------------------- bitmap kernels

// result = AND_c OR_{k in c} bms[k], AND NOT deleted; two words per thread.
constexpr int kCnfBatch = 4;  // operand bitmaps whose loads k_bitmap_cnf issues together

__global__ __launch_bounds__(kBlock) void k_bitmap_cnf(BitmapCnf C, const uint64_t* __restrict__ del,
                                                       int64_t nwords, uint64_t tail_mask,
                                                       int64_t words_per_block, uint64_t* __restrict__ out,
                                                       int64_t* __restrict__ segc) {
  const int64_t w0 = (int64_t)blockIdx.x * words_per_block;
  const int64_t w1 = min(w0 + words_per_block, nwords);
  int64_t cnt = 0;
  const int nbm = C.conj_off[C.nconj];
  for (int64_t w = w0 + 2 * threadIdx.x; w < w1; w += 2 * kBlock) {
    const bool two = w + 1 < w1;
    uint64_t r0 = ~0ull, r1 = ~0ull;
    if (nbm <= kCnfBatch && two && (w & 1) == 0) {
      // every operand's 16 bytes in flight at once, then the CNF in registers
      ulonglong2 q[kCnfBatch];
#pragma unroll
      for (int k = 0; k < kCnfBatch; ++k)
        if (k < nbm) q[k] = *reinterpret_cast<const ulonglong2*>(C.bms[k] + w);
      for (int c = 0; c < C.nconj; ++c) {
        uint64_t o0 = 0, o1 = 0;
#pragma unroll
        for (int k = 0; k < kCnfBatch; ++k)
          if (k >= C.conj_off[c] && k < C.conj_off[c + 1]) {
            o0 |= q[k].x;
            o1 |= q[k].y;
          }
        r0 &= o0;
        r1 &= o1;
      }
    } else {
      for (int c = 0; c < C.nconj; ++c) {
        uint64_t o0 = 0, o1 = 0;
        for (int k = C.conj_off[c]; k < C.conj_off[c + 1]; ++k) {
          const uint64_t* b = C.bms[k];
          if (two && ((w & 1) == 0)) {
            const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(b + w);
            o0 |= q.x;
            o1 |= q.y;
          } else {
            o0 |= b[w];
            if (two) o1 |= b[w + 1];
          }
        }
        r0 &= o0;
        r1 &= o1;
      }
    }
    if (del) {
      r0 &= ~del[w];
      if (two) r1 &= ~del[w + 1];
    }
    if (w == nwords - 1) r0 &= tail_mask;
    if (two && w + 1 == nwords - 1) r1 &= tail_mask;
    out[w] = r0;
    cnt += __popcll(r0);
    if (two) {
      out[w + 1] = r1;
      cnt += __popcll(r1);
    }
  }
  // block sum of counts (fixed order)
  __shared__ int64_t sh[kWaves];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) cnt += __shfl_xor(cnt, m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t s = 0;
    for (int i = 0; i < kWaves; ++i) s += sh[i];
    segc[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(kBlock) void k_bitmap_combine(int32_t op, const uint64_t* __restrict__ a,
                                                           const uint64_t* __restrict__ b, int64_t nwords,
                                                           uint64_t tail_mask, int64_t words_per_block,
                                                           uint64_t* __restrict__ out,
                                                           int64_t* __restrict__ segc) {
  const int64_t w0 = (int64_t)blockIdx.x * words_per_block;
  const int64_t w1 = min(w0 + words_per_block, nwords);
  int64_t cnt = 0;
  for (int64_t w = w0 + threadIdx.x; w < w1; w += kBlock) {
    uint64_t r = op == 0 ? (a[w] & b[w]) : (op == 1 ? (a[w] | b[w]) : (a[w] & ~b[w]));
    if (w == nwords - 1) r &= tail_mask;
    out[w] = r;
    cnt += __popcll(r);
  }
  __shared__ int64_t sh[kWaves];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) cnt += __shfl_xor(cnt, m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t s = 0;
    for (int i = 0; i < kWaves; ++i) s += sh[i];
    segc[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(kBlock) void k_seg_popcount(const uint64_t* __restrict__ words, int64_t nwords,
                                                         int64_t words_per_block,
                                                         int64_t* __restrict__ segc) {
  const int64_t w0 = (int64_t)blockIdx.x * words_per_block;
  const int64_t w1 = min(w0 + words_per_block, nwords);
  int64_t cnt = 0;
  for (int64_t w = w0 + threadIdx.x; w < w1; w += kBlock) cnt += __popcll(words[w]);
  __shared__ int64_t sh[kWaves];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) cnt += __shfl_xor(cnt, m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t s = 0;
    for (int i = 0; i < kWaves; ++i) s += sh[i];
    segc[blockIdx.x] = s;
  }
}

// Compaction (nextSetBit order): one block per segment; each wave owns a
// contiguous run of the segment's words.  64 words per step are loaded
// coalesced (lane = word); an exclusive scan of their popcounts gives each
// word's output slot; then either each lane peels its own word's bits
// (sparse steps: iterations = the largest popcount) or the wave visits only
// the non-zero words with lane = bit, writing ascending global positions
// densely (dense steps; stores only -- no load sits between two iterations).
// A block's output offset is the sum of the segment counts before it (read
// straight from the producers' per-segment counts -- no separate scan
// launch); the last block also writes the total.
constexpr int kSelRegs = 8;  // a wave's words (x64) held in registers between the count and the write pass

template <int G4>
__global__ __launch_bounds__(kBlock) void k_select_ids(const uint64_t* __restrict__ words, int64_t nwords,
                                                       int64_t words_per_block,
                                                       const int64_t* __restrict__ segc, int64_t segs_per_block,
                                                       int64_t row_offset, int64_t* __restrict__ ids,
                                                       int64_t* __restrict__ total, int32_t dbg,
                                                       int64_t* __restrict__ stamps, Gather4 G) {
  // dbg (diagnostic A/B, mbx_set_tuning "select_dbg"; -DMBX_DIAG builds
  // only): bit 0 skips the prefix loads, bit 1 the emission; stamps: per
  // block wall_clock64() at start / words + prefix in / after the block
  // barrier / end
  dbg &= kDiagDbg;
  if (stamps && threadIdx.x == 0) stamps[4 * blockIdx.x] = wall_clock64();
  __shared__ int64_t wcount[kWaves];
  __shared__ int64_t wpre[kWaves];
  __shared__ uint16_t stage[kWaves][32 * 64];
  const int lane = threadIdx.x & 63;
  const int wave = (int)uniform(threadIdx.x >> 6);
  const int64_t s0 = (int64_t)blockIdx.x * words_per_block;
  const int64_t s1 = min(s0 + words_per_block, nwords);
  const int64_t per = (s1 - s0 + kWaves - 1) / kWaves;
  const int64_t a0 = min(s0 + wave * per, s1);
  const int64_t a1 = min(a0 + per, s1);
  // a wave range of <= 64 * kSelRegs words is loaded once, all loads in
  // flight together, and kept in registers for the write pass
  const bool cached = a1 - a0 <= 64 * kSelRegs;
  // this block's output offset: the segment counts before it (a compact
  // int64 array, two per 16-byte load, 4 loads in flight per thread), issued
  // before the word loads so both latencies overlap
  const int64_t npre = (dbg & 1) ? 0 : (int64_t)blockIdx.x * segs_per_block;
  const int64_t npairs = npre >> 1;
  const ulonglong2* __restrict__ sp = reinterpret_cast<const ulonglong2*>(segc);
  int64_t pre = 0;
  for (int64_t i0 = 0; i0 < npairs; i0 += 4 * kBlock) {
    ulonglong2 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = i0 + k * kBlock + threadIdx.x;
      v[k] = i < npairs ? sp[i] : ulonglong2{0ull, 0ull};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) pre += (int64_t)(v[k].x + v[k].y);
  }
  if ((npre & 1) && threadIdx.x == 0) pre += segc[npre - 1];
  uint64_t wr[kSelRegs];
  int64_t c = 0;
  if (cached) {
#pragma unroll
    for (int r = 0; r < kSelRegs; ++r) {
      const int64_t w = a0 + r * 64 + lane;
      wr[r] = w < a1 ? words[w] : 0ull;
    }
#pragma unroll
    for (int r = 0; r < kSelRegs; ++r) c += __popcll(wr[r]);
  } else {
    for (int64_t w = a0 + lane; w < a1; w += 64) c += __popcll(words[w]);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    c += __shfl_xor(c, m);
    pre += __shfl_xor(pre, m);
  }
  if (lane == 0) {
    wcount[wave] = c;
    wpre[wave] = pre;
  }
  if (stamps && threadIdx.x == 0) stamps[4 * blockIdx.x + 1] = wall_clock64();
  __syncthreads();
  if (stamps && threadIdx.x == 0) stamps[4 * blockIdx.x + 2] = wall_clock64();
  int64_t off = 0;
  for (int k = 0; k < kWaves; ++k) off += wpre[k];
  if (threadIdx.x == 0 && blockIdx.x == gridDim.x - 1) {
    int64_t all = off;
    for (int k = 0; k < kWaves; ++k) all += wcount[k];
    *total = all;
  }
  for (int k = 0; k < wave; ++k) off += wcount[k];
  // one step = 64 consecutive words, lane = word
  const bool wt = (G4 == 0) != ((dbg & 32) != 0);
  auto step = [&](int64_t base, uint64_t mw) {
    emit_step<G4>(base, mw, off, row_offset, ids, stage[wave], lane, G, wt);
  };
  if (dbg & 2) {
  } else if (cached) {
#pragma unroll
    for (int r = 0; r < kSelRegs; ++r) {
      const int64_t base = a0 + r * 64;
      if (base >= a1) break;
      step(base, wr[r]);
    }
  } else {
    for (int64_t base = a0; base < a1; base += 64) step(base, base + lane < a1 ? words[base + lane] : 0ull);
  }
  if (stamps && threadIdx.x == 0) stamps[4 * blockIdx.x + 3] = wall_clock64();
}

// ColumnarIndexScan in one launch (mbx_cnf_materialize_async,
// R/index/ColumnarIndexScan.java:130-181 then :287-308): each block forms its
// words of the CNF of index BitSets in registers (as k_bitmap_cnf; the CNF's
// BitSet is never stored), publishes its count at once, sums its
// predecessors' published counts for its output offset (decoupled look-back:
// blocks are dispatched in index order, so every predecessor is resident or
// done and publishes without waiting on anything) and writes its positions
// (ids may be null) + up to G4 projected 4-byte columns.
// Each wave stages the positions of its leading steps together (while they
// fit the stage) and loads the values of the first 256 of them BEFORE the
// look-back resolves: the look-back's round trips overlap those gathers, and
// a sparse wave (C4: ~250 rows) needs one gather round trip, not one per
// 64-word step.
// lb[0] = the epoch of the previous launch; lb[1 + b * fs] = epoch << 32 |
// count of block b.  Every launch's epoch differs from the stale flags it
// finds (they carry earlier launches' epochs; the words are set back to
// epoch 0 around the wrap, select_tail), so nothing is cleared between
// launches (graph replays included: the epoch is read from lb[0], not baked
// into the launch); the last block, having seen every other block's flag (so
// every block has read lb[0]), stores the new epoch.
constexpr int kLookbackBlocks = 4 * kBlock;  // one poll load per thread per 256 predecessors
// staged rows per lane whose values load before the look-back: 6 x 64 covers
// a 1 % wave of ~245 rows with 9 sd to spare; 4 columns hold fewer (occupancy)
template <int G4>
constexpr int prefetch_rows() { return G4 <= 2 ? 6 : 3; }

__device__ __forceinline__ uint64_t cnf_word(const BitmapCnf& C, int64_t w) {
  uint64_t r = ~0ull;
  for (int c = 0; c < C.nconj; ++c) {
    uint64_t o = 0;
    for (int k = C.conj_off[c]; k < C.conj_off[c + 1]; ++k) o |= C.bms[k][w];
    r &= o;
  }
  return r;
}

// G4: projected 4-byte columns the registers hold (kWide: any projection,
// GT = GatherW); NB: 1..4 operands batched, 0: any
// The part of a one-launch selection after each wave has formed its words
// (k_cnf_select from index BitSets, k_scan_select from a predicate scan):
// the block count is published, the output offset taken from the
// predecessors (decoupled look-back), the leading steps' positions staged and
// their projected values loaded before the offset is known, then positions +
// values written.  wr / cached: the wave's words (lane = word) when its range
// fits kSelRegs x 64 words; word_at(w) re-forms word w otherwise.  segc (may
// be null): the block's count is also stored there.
// The chained look-back of one block (wave 0): the sum of every
// predecessor's count.  Each round reads the count and inclusive-prefix
// flags of the 64 predecessors below e (lane l: e - 64 + l, one line group
// of each, all loads in flight together); the nearest published inclusive
// prefix ends the walk, otherwise the window's counts are added once all are
// published and the walk moves 64 further down.  The cost is the flag lines'
// request queue, not the number of rounds: 4 predecessors per lane (4x the
// requests, a quarter of the rounds) measured slower -- C2 one launch 22.5
// vs 18.6 us, C4 51-52 vs 45 us (profiles/r03/lb).
__device__ __forceinline__ int64_t lookback_window(int64_t* __restrict__ lb, int64_t* __restrict__ inc, int64_t e,
                                                   int64_t epoch, int lane, int64_t& in) {
  const int64_t j = e - 64 + lane;
  in = j >= 0 ? __hip_atomic_load(&inc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  return j >= 0 ? __hip_atomic_load(&lb[1 + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (epoch << 32);
}

// in0 / a0: the first window's flags (below blockIdx.x), loaded by the caller
__device__ __forceinline__ int64_t chained_lookback(int64_t* __restrict__ lb, int64_t* __restrict__ inc,
                                                    int64_t epoch, int lane, int64_t in0, int64_t a0, int64_t bid) {
  constexpr int64_t kLow = 0xffffffffll;
  int64_t pre = 0;
  int64_t e = bid;
  bool first = true;
  while (e > 0) {
    const int64_t j = e - 64 + lane;
    const bool live = j >= 0;
    int64_t in = in0, a = a0;
    if (!first) a = lookback_window(lb, inc, e, epoch, lane, in);
    first = false;
    for (;;) {
      const bool ok_in = live && (in >> 32) == epoch;
      const bool ok_a = (a >> 32) == epoch;
      const uint64_t im = __ballot(ok_in);
      if (im) {
        const int L = 63 - __clzll((long long)im);
        if (!__any(lane > L && !ok_a)) {
          pre += lane == L ? (in & kLow) : (lane > L ? (a & kLow) : 0);
          e = 0;
          break;
        }
      } else if (!__any(!ok_a)) {
        pre += a & kLow;
        e -= 64;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      if (live && !ok_in) in = __hip_atomic_load(&inc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!ok_a) a = __hip_atomic_load(&lb[1 + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  return pre;
}

// the chained look-back's inclusive prefixes: lb[1 + kIncBase + segment]
// (count flags below, one per segment, <= kIncBase segments)
constexpr int64_t kIncBase = 8192;
static_assert(1 + 2 * kIncBase <= kLookbackWords, "look-back buffer");
struct NoAfter {
  __device__ void operator()() const {}
};

// bid / nblk: the segment this call completes and the launch's segment count
// (default: blockIdx.x / gridDim.x, one segment per block); after(): run by
// every wave once its leading steps are staged and their values' loads are
// issued, before the look-back (k_cnf_select's next round issues its operand
// loads there)
template <int G4, class GT, class WordAt, int NW = kWaves, int NR = kSelRegs, class After = NoAfter>
__device__ __forceinline__ void select_tail(const uint64_t (&wr)[NR], int64_t c, bool cached, int64_t a0,
                                            int64_t a1, WordAt word_at, int lane, int wave, int64_t* __restrict__ lb,
                                            int64_t epoch, int64_t row_offset, int64_t* __restrict__ ids,
                                            int64_t* __restrict__ total, const GT& G, int64_t* __restrict__ stamps,
                                            int32_t dbg, int64_t* __restrict__ segc, int64_t nseg, int64_t* wcount,
                                            int64_t* wpre, uint16_t (*stage)[32 * 64],
                                            uint64_t* __restrict__ words_out = nullptr, int32_t fs = 1,
                                            int64_t bid = -1, int64_t nblk = -1, After after = After{}) {
  // fs: int64 words between two blocks' count flags (1, or 16 = one 128-byte
  // line per flag for the polling form: the polls of every block do not queue
  // on the same few lines); the chained form needs 1
  dbg &= kDiagDbg;  // bits 0-2: A/B poll forms, -DMBX_DIAG builds only
  int64_t* const inc = lb + 1 + kIncBase;  // chained form (dbg bit 3): epoch << 32 | inclusive prefix
  const int64_t B = bid < 0 ? (int64_t)blockIdx.x : bid;
  const int64_t NB = nblk < 0 ? (int64_t)gridDim.x : nblk;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
  if (lane == 0) wcount[wave] = c;
  __syncthreads();
  // the block's count and this wave's offset within it, read now (every
  // count unrolled, the loads in flight together) rather than after the
  // offset barrier, where a loop over the lower waves' counts was a chain
  // of dependent LDS round trips on every wave's critical path
  int64_t bc = 0, wpos = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const int64_t x = wcount[k];
    bc += x;
    wpos += k < wave ? x : 0;
  }
  // The count is published by the LAST wave, which then loads nothing until
  // the emission: vmcnt counts loads and stores in issue order, so a wave
  // that waits for anything after the publishing store also waits for that
  // store's write-through round trip (~1.5 us at C2).  The compiler places
  // waits wherever a register of a load that may be in flight on some path
  // is touched, so no look-back load may be in flight on any path into code
  // the publishing wave runs before the offset barrier: the staging comes
  // first for every wave, the look-back loads are issued after it, in
  // branches the publishing wave does not take, and consumed there; their
  // result reaches the block through LDS.  The flag store itself is inline
  // asm -- the write-through vector store the relaxed agent-scope atomic
  // store compiles to -- with its address and data moved into VGPRs by an
  // asm of their own and kept live to the end of the function, so no later
  // write of those registers calls for a wait; the compiler does not count
  // the store, and a wait it emits for its own operations can only wait
  // longer (completion is in issue order), never less.
  constexpr int kPub = NW - 1;
  constexpr int kPollers = 64 * (NW - 1);
  constexpr int kPolls = (kLookbackBlocks + kPollers - 1) / kPollers;
  int64_t* flag_at = nullptr;
  int64_t flag = 0;
  if (wave == kPub) {
    flag_at = &lb[1 + B * fs];
    flag = (epoch << 32) | bc;
    asm volatile("" : "+v"(flag_at), "+v"(flag));
    // vmcnt(0) before the flag: free (nothing of this wave is in flight here
    // but a diagnostic stamp), and the compiler then counts nothing in flight
    // on this path, so it places no wait after the flag
    __builtin_amdgcn_s_waitcnt(0x0f70);
    if (lane == 0) {
      asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(flag_at), "v"(flag) : "memory");
      wpre[kPub] = 0;
    }
  }
  if (dbg & 128) {  // diagnostic: the count only (wrong output by design)
    if (B == NB - 1 && threadIdx.x == 0) lb[0] = epoch;
    return;
  }
  // the wave's leading steps staged together, the first kPrefetch x 64
  // rows' values loaded
  uint16_t* const st = stage[wave];
  uint32_t tot = 0;  // staged positions (offsets from bit 0 of word a0: < 8 x 4096)
  int nst = 0;       // steps staged
  constexpr int kPrefetch = prefetch_rows<G4>();
  uint32_t pv[kPrefetch > 0 ? kPrefetch : 1][G4 > 0 ? G4 : 1];
  if (cached && !(dbg & 16)) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if (a0 + r * 64 >= a1) break;
      const StepScan q = stage_step(wr[r], st, lane, tot, (uint32_t)r * 4096u);
      if (tot + q.total > kStageIds) break;
      tot += q.total;
      nst = r + 1;
    }
    if constexpr (G4 != kWide) {
#pragma unroll
      for (int k = 0; k < kPrefetch; ++k) {
        const uint32_t i = (uint32_t)lane + 64u * k;
        if (i < tot) {
          const int64_t p = a0 * 64 + st[i];
          gather_row<G4>(G, p, pv[k]);
        }
      }
    }
  }
  after();
  if (wave == kPub) {
  } else if (dbg & 8) {
    // chained form: wave 0 walks back over its predecessors, 64 per round,
    // stops at the nearest one whose inclusive prefix is published and adds
    // the counts after it, and publishes this block's inclusive prefix at
    // once; the other waves contribute 0
    if (stamps && threadIdx.x == 64) stamps[4 * B + 1] = wall_clock64();
    if (wave == 0) {
      int64_t in0 = 0, a0f = epoch << 32;
      if (B > 0) a0f = lookback_window(lb, inc, B, epoch, lane, in0);
      int64_t pre = chained_lookback(lb, inc, epoch, lane, in0, a0f, B);
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) pre += __shfl_xor(pre, m);
      if (lane == 0) {
        wpre[0] = pre;
        __hip_atomic_store(&inc[B], (epoch << 32) | (pre + bc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else if (lane == 0) {
      wpre[wave] = 0;
    }
  } else {
    // polling form: every predecessor's count, one per thread of the other
    // waves, all in flight together
    if (stamps && threadIdx.x == 64) stamps[4 * B + 1] = wall_clock64();
    int64_t v[kPolls];
#pragma unroll
    for (int k = 0; k < kPolls; ++k) {
      const int64_t j = (int64_t)k * kPollers + threadIdx.x;
      if (j >= B)
        v[k] = epoch << 32;
      else if (dbg & 4)  // first round through L2 (a stale line only reads as "not yet"), then coherent polls
        v[k] = __builtin_nontemporal_load(&lb[1 + j * fs]);
      else
        v[k] = __hip_atomic_load(&lb[1 + j * fs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    int64_t pre = 0;
#pragma unroll
    for (int k = 0; k < kPolls; ++k) {
      const int64_t j = (int64_t)k * kPollers + threadIdx.x;
      while (!(dbg & 2) && (v[k] >> 32) != epoch) {
        if (dbg & 1)
          __builtin_amdgcn_s_sleep(16);
        else
          __builtin_amdgcn_s_sleep(1);
        v[k] = __hip_atomic_load(&lb[1 + j * fs], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      pre += v[k] & 0xffffffffll;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) pre += __shfl_xor(pre, m);
    if (lane == 0) wpre[wave] = pre;
  }
  __syncthreads();
  if (stamps && threadIdx.x == 0) stamps[4 * B + 2] = wall_clock64();
  int64_t off = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) off += wpre[k];
  // the last block: the total, and the epoch the next launch starts from
  // (every block has read it: the last block's offset needs every other
  // block's count)
  if (B == NB - 1 && threadIdx.x == 0) {
    *total = off + bc;
    lb[0] = epoch;
  }
  // a block whose rows would end past the outputs' capacity writes none of
  // them: the caller sees *total > cap and fails, with nothing out of bounds
  // (dbg bit 6, -DMBX_DIAG builds: no positions written -- the emission's
  // cost, for the C2 anatomy)
  const bool fits = off + bc <= G.cap && !(dbg & (64 | 16));
  off += wpos;
  // the outputs' stores (dbg bits 12-13, tuning cnf_store): 0 the default --
  // write-through for positions only (k_cnf_select with no projected column
  // too: 13.7-14.0 vs 14.9 us at C4's 1 M positions, profiles/r05/l), plain
  // with gathered values (write-through 33.1 vs 30.0 us, nontemporal 30.4-30.7;
  // dbg bit 5 flips the default) -- 1 plain, 2 write-through, 3 nontemporal
  const int smode = (dbg >> 12) & 3;
  const bool positions_only = G4 == 0 || G.n == 0;
  const int wt = smode == 0 ? ((positions_only != ((dbg & 32) != 0)) ? 1 : 0) : (smode == 1 ? 0 : (smode == 2 ? 1 : 2));
  if (!fits) {
  } else if (cached) {
    // the prefetched rows, then the rest of the staged ones, then the steps
    // that did not fit the stage one by one
#pragma unroll
    for (int k = 0; k < kPrefetch; ++k) {
      const uint32_t i = (uint32_t)lane + 64u * k;
      if (i < tot) {
        if (ids) put(&ids[off + i], row_offset + a0 * 64 + st[i], wt);
        if constexpr (G4 == kWide) {
          wide_row(G, a0 * 64 + st[i], off + i);
        } else {
#pragma unroll
          for (int g = 0; g < G4; ++g)
            if (g < G.n) put(&G.out[g][off + i], pv[k][g], wt);
        }
      }
    }
    const StepScan all{0u, tot};
    store_step<G4, GT>(a0, 0ull, all, off, row_offset, ids, st, lane, G, 64u * kPrefetch, wt, (dbg & 512) != 0);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int64_t base = a0 + r * 64;
      if (r < nst) continue;
      if (base >= a1) break;
      emit_step<G4, GT>(base, wr[r], off, row_offset, ids, st, lane, G, wt);
    }
  } else {
    for (int64_t base = a0; base < a1; base += 64)
      emit_step<G4, GT>(base, base + lane < a1 ? word_at(base + lane) : 0ull, off, row_offset, ids, st, lane, G,
                        wt);
  }
  // the BitSet (k_scan_select): its words and one segment count per 4 waves
  if (words_out && !(dbg & 256)) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int64_t wd = a0 + r * 64 + lane;
      if (wd < a1) put(&words_out[wd], wr[r], wt);
    }
  }
  if (segc && threadIdx.x < NW / kWaves) {
    const int64_t sg = (int64_t)blockIdx.x * (NW / kWaves) + threadIdx.x;
    if (sg < nseg) {
      int64_t sc = 0;
      for (int k = 0; k < kWaves; ++k) sc += wcount[threadIdx.x * kWaves + k];
      segc[sg] = sc;
    }
  }
  // Epochs run 1 .. 2^31 - 1 and wrap, every launch of either kernel on this
  // look-back buffer taking the next one, so a word can only be mistaken for
  // this launch's if it was written exactly one cycle earlier and never
  // since.  The last two launches before the wrap (their last block, once
  // its offset -- i.e. every other block's count -- is known) set every
  // word they do not use back to epoch 0, which no launch has: by induction
  // no word holds the epoch of a launch before that launch writes it.
  if (B == NB - 1 && epoch >= 0x7ffffffe) {
    for (int64_t w = 1 + threadIdx.x; w < kLookbackWords; w += 64 * NW) {
      const int64_t x = w - 1;
      const bool live = (dbg & 8) ? (x < NB || (x >= kIncBase && x - kIncBase < NB)) : (x % fs == 0 && x / fs < NB);
      if (!live) lb[w] = 0;
    }
  }
  if (stamps) {
    __syncthreads();
    if (threadIdx.x == 0) stamps[4 * B + 3] = wall_clock64();
  }
  asm volatile("" ::"v"(flag_at), "v"(flag));  // the flag store's registers, live to here
}

// R rounds: the launch covers gridDim.x x R segments of words_per_block
// words, block b completing segment b, then b + gridDim.x, the next round's
// operand words loaded while this round's gathers are in flight (the after()
// hook of select_tail); NR: the registers holding a wave's words per round.
// Production launches R = 1 only: R = 2 measured slower at C4 (36.6 vs 31.8
// us, profiles/r05/c: its extra registers cut residency from 4 to 3 blocks
// per CU, and round 2 waits on every block's round 1, so the grid must be
// resident at once -- DESIGN.md section 3).
// NW: waves per block.  Production launches 4: workgroups reach the CUs at
// ~220 per us, so C4's 1024 four-wave blocks take ~4.6 us to all start
// (profiles/r05/o) -- 256 sixteen-wave blocks start within ~2 us but run the
// query in 41 vs 30 us: a block's count waits for its slowest of 16 waves
// while its other waves' gathers already load HBM (profiles/r05/p)
template <int G4, int NB, class GT = Gather4, int R = 1, int NR = kSelRegs, int NW = kWaves>
__global__ __launch_bounds__(64 * NW) void k_cnf_select(BitmapCnf C, const uint64_t* __restrict__ del,
                                                       int64_t nwords, uint64_t tail_mask, int64_t words_per_block,
                                                       int64_t* __restrict__ lb, int64_t row_offset,
                                                       int64_t* __restrict__ ids, int64_t* __restrict__ total,
                                                       GT G, int64_t* __restrict__ stamps, int32_t dbg,
                                                       int32_t fs) {
  // fs: int64 words between two blocks' count flags (the polling form: 16 =
  // one 128-byte line per flag, or 1; the chained form: 1)
  // dbg bit 3: the chained look-back -- each block also publishes its
  // inclusive prefix, and wave 0 walks back 64 predecessors per round to the
  // nearest published one (~4 flag lines per block instead of every
  // predecessor's); without it, every thread polls its predecessors' counts
  // (diagnostic A/B of that form, select_dbg >> 4: bit 0 polls with a
  // 1024-clock back-off, bit 1 skips the look-back's wait (wrong output: its
  // cost), bit 2 takes the first poll round as plain nontemporal loads)
  // stamps (diagnostic, select_dbg bit 3): per block wall_clock64() at start /
  // count published / offset known / end
  if (stamps && threadIdx.x == 0) stamps[4 * blockIdx.x] = wall_clock64();
  __shared__ int64_t wcount[NW];
  __shared__ int64_t wpre[NW];
  __shared__ uint16_t stage[NW][32 * 64];
  const int lane = threadIdx.x & 63;
  const int wave = (int)uniform(threadIdx.x >> 6);
  // epochs 1 .. 2^31 - 1: epoch << 32 stays a positive int64
  const uint32_t prev = (uint32_t)lb[0];
  const int64_t epoch = prev >= 0x7fffffffu ? 1 : (int64_t)prev + 1;
  const int64_t nseg = (int64_t)gridDim.x * R;
  auto range = [&](int64_t seg, int64_t& a0, int64_t& a1) {
    const int64_t s0 = min(seg * words_per_block, nwords);
    const int64_t s1 = min(s0 + words_per_block, nwords);
    const int64_t per = (s1 - s0 + NW - 1) / NW;
    a0 = min(s0 + wave * per, s1);
    a1 = min(a0 + per, s1);
  };
  auto word_at = [&](int64_t w) -> uint64_t {
    uint64_t r = cnf_word(C, w);
    if (del) r &= ~del[w];
    if (w == nwords - 1) r &= tail_mask;
    return r;
  };
  // every operand word of a wave's range in flight at once (NB x NR
  // register pairs: sized to the operand count)
  uint64_t q[NR][NB > 0 ? NB : 1];
  auto load_ops = [&](int64_t a0, int64_t a1) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int64_t w = a0 + r * 64 + lane;
#pragma unroll
      for (int k = 0; k < NB; ++k) q[r][k] = w < a1 ? C.bms[k][w] : 0ull;
    }
  };
  int64_t a0, a1;
  range(blockIdx.x, a0, a1);
  if (NB > 0 && a1 - a0 <= 64 * NR) load_ops(a0, a1);
#pragma unroll
  for (int round = 0; round < R; ++round) {
    const int64_t seg = (int64_t)round * gridDim.x + blockIdx.x;
    if (round > 0) range(seg, a0, a1);
    const bool cached = a1 - a0 <= 64 * NR;
    uint64_t wr[NR];
    int64_t c = 0;
    if (NB > 0 && cached) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int64_t w = a0 + r * 64 + lane;
        uint64_t x = ~0ull;
        for (int cj = 0; cj < C.nconj; ++cj) {
          uint64_t o = 0;
#pragma unroll
          for (int k = 0; k < NB; ++k)
            if (k >= C.conj_off[cj] && k < C.conj_off[cj + 1]) o |= q[r][k];
          x &= o;
        }
        if (del && w < a1) x &= ~del[w];
        if (w == nwords - 1) x &= tail_mask;
        wr[r] = w < a1 ? x : 0ull;
        c += __popcll(wr[r]);
      }
    } else if (cached) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int64_t w = a0 + r * 64 + lane;
        wr[r] = w < a1 ? word_at(w) : 0ull;
        c += __popcll(wr[r]);
      }
    } else {
      for (int64_t w = a0 + lane; w < a1; w += 64) c += __popcll(word_at(w));
    }
    // the next round's operand loads, issued behind this round's gathers
    auto after = [&]() {
      if (round + 1 < R && NB > 0) {
        int64_t n0, n1;
        range(seg + gridDim.x, n0, n1);
        if (n1 - n0 <= 64 * NR) load_ops(n0, n1);
      }
    };
    select_tail<G4, GT, decltype(word_at), NW, NR>(wr, c, cached, a0, a1, word_at, lane, wave, lb, epoch,
                                                         row_offset, ids, total, G, R == 1 ? stamps : nullptr, dbg,
                                                         nullptr, 0, wcount, wpre, stage, nullptr, fs, seg, nseg,
                                                         after);
    if (round + 1 < R) __syncthreads();  // LDS counts / stage reused by the next round
  }
}

constexpr int kDefaultU = 2;
// measured on MI355X (profiles/r01/sweep3.log, C3 100M rows): U=2 tiles in
// flight per wave with non-temporal loads, 4 blocks per CU, write-through
// partials -> 135 us = 5.9 TB/s; plain loads +3 %, 8 blocks/CU +7 %,
// 2 blocks/CU +56 %, release-fence partials +22 %.
constexpr bool kDefaultNT = true;

// ColumnarFileScan's get_next_tid stream as BitSet + ascending positions +
// COUNT (R/iterator/ColumnarFileScan.java:174-188) in ONE launch
// (mbx_scan_select_async, knob scan_select_fused): each wave scans a
// contiguous run of its block's full tiles with the fast scan's tile body
// (hoisted literal terms; row-interleaved loads, so each row group's ballot
// is one BitSet word) and collects its words lane = word (the 4 words of its
// i-th tile go to lanes 4i..4i+3 of register i / 16), stores them as the
// BitSet (coalesced, after its loads) with the block's segment count, then
// select_tail turns them into positions: count published, offset from the
// predecessors (chained look-back), leading steps staged before the offset
// is known -- no second launch, no re-read of the BitSet.  Plans of 1..4
// 4-byte int literal terms (no float compare: no NaN reach), wave ranges of
// <= kSelRegs x 16 tiles (tables up to ~134 M rows), <= kLookbackBlocks blocks.
template <int K, bool DEL, int U, int TQ, int NW, int NR, int IR = 0>
__global__ __launch_bounds__(64 * NW) void k_scan_select(ScanLaunch L, int64_t* __restrict__ lb, int64_t row_offset,
                                                         int64_t* __restrict__ ids, int64_t* __restrict__ total,
                                                         int64_t* __restrict__ stamps, int32_t dbg, int32_t fs) {
#ifndef MBX_DIAG
  dbg &= 8;  // the look-back form (bit 3: chained, else every predecessor polled); write-through positions
#endif
  if (stamps && threadIdx.x == 0) stamps[4 * blockIdx.x] = wall_clock64();
  __shared__ int64_t wcount[NW];
  __shared__ int64_t wpre[NW];
  __shared__ __attribute__((aligned(16))) uint16_t stage[NW][32 * 64];  // also the segment words (uint64)
  const KPlan* __restrict__ P = L.plan;
  const int lane = threadIdx.x & 63;
  const int wave = (int)uniform(threadIdx.x >> 6);
  const uint32_t prev = (uint32_t)lb[0];
  const int64_t epoch = prev >= 0x7fffffffu ? 1 : (int64_t)prev + 1;
  const int64_t nrows = L.nrows;
  const int64_t nwords = (nrows + 63) >> 6;
  const int64_t ntiles = (nrows + kTileRows - 1) / kTileRows;
  // NW / 4 BitSet segments per block, 4 waves per segment: wave w scans
  // its quarter of segment blockIdx * NW / 4 + w / 4
  const int64_t nseg = (ntiles + L.tiles_per_block - 1) / L.tiles_per_block;
  const int64_t tb0 = min(((int64_t)blockIdx.x * (NW / kWaves) + wave / kWaves) * L.tiles_per_block, ntiles);
  const int64_t tb1 = min(tb0 + L.tiles_per_block, ntiles);
  const int64_t per = (tb1 - tb0 + kWaves - 1) / kWaves;  // tiles per wave (<= 16 * NR, launcher-checked)
  const int64_t wt0 = min(tb0 + (wave % kWaves) * per, tb1);
  const int64_t wt1 = min(wt0 + per, tb1);
  const int64_t a0 = wt0 * kWordsPerTile;
  const int64_t a1 = min(wt1 * kWordsPerTile, nwords);
  const int nterms = P->nterms;
  const uint32_t all = P->all_conj;
  const int32_t* colp[K];
#pragma unroll
  for (int s = 0; s < K; ++s) colp[s] = (const int32_t*)P->cols[s].base;
  const int32_t* const strp[1] = {nullptr};
  KTerm th[TQ];
#pragma unroll
  for (int ti = 0; ti < TQ; ++ti)
    if (ti < nterms) th[ti] = P->terms[ti];
  Acc acc;
  acc_init(acc);
  uint64_t wave_count = 0;
  uint64_t wr[NR];
  int64_t c = 0;
  {
    // the segment's 4 waves read its tiles interleaved (wave w % 4 takes
    // tiles w % 4, + 4, + 8, ... as the fast scan does: at any moment the
    // waves of a segment stream adjacent tiles), the words go to LDS (the
    // stage, not yet in use) and each wave then takes its contiguous quarter
    // of them into registers -- the positions stay ascending by wave
    uint64_t* const segw =
        reinterpret_cast<uint64_t*>(&stage[0][0]) + (int64_t)(wave / kWaves) * L.tiles_per_block * kWordsPerTile;
    const int sub = wave % kWaves;
    const int64_t tf = min(tb1, nrows / kTileRows);  // the segment's full tiles end here
    for (int64_t base = tb0 + sub; base < tb1; base += (int64_t)kWaves * U) {
      TileRegs<K, 0> D[U];
      load_tiles<K, 0, U, kDefaultNT, true>(D, base, kWaves, tf, colp, strp, lane);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t t = base + (int64_t)u * kWaves;
        uint64_t w[4] = {0ull, 0ull, 0ull, 0ull};
        if (t < tf) {
          fast_tile<K, 0, kModeBitmap, DEL, TQ, true, true, IR>(L, P, D[u], t, lane, nterms, all, 0, false, acc,
                                                           wave_count, th, w);
        } else if (t < tb1) {  // the table's one partial tile
          TileRegs<K, 0> Dp;
          load_partial<K, 0, true>(Dp, t, nrows, colp, strp, lane);
          fast_tile<K, 0, kModeBitmap, DEL, TQ, true, false, IR>(L, P, Dp, t, lane, nterms, all, 0, false, acc,
                                                            wave_count, th, w);
        }
        if (t < tb1 && lane < 4)
          segw[(t - tb0) * kWordsPerTile + lane] = lane == 0 ? w[0] : (lane == 1 ? w[1] : (lane == 2 ? w[2] : w[3]));
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int64_t wd = a0 + (int64_t)r * 64 + lane;
      wr[r] = wd < a1 ? segw[wd - tb0 * kWordsPerTile] : 0ull;
      c += __popcll(wr[r]);
    }
    __syncthreads();  // select_tail stages positions over the same LDS
  }
  auto word_at = [&](int64_t) -> uint64_t { return 0ull; };  // never called: every range is cached
  const Gather4 G{};
  select_tail<0, Gather4, decltype(word_at), NW, NR>(wr, c, true, a0, a1, word_at, lane, wave, lb, epoch, row_offset,
                                                     ids, total, G, stamps, dbg, L.seg_counts, nseg, wcount, wpre,
                                                     stage, L.out_words, fs);
}

// Late materialisation (Heapfile.findRID + getRecord per output column,
// R/index/ColumnarIndexScan.java:292-297): out_p[i] = column_p[ids[i]] for
// the *total selected rows; thread per output row, 4 rows in flight per
// thread, writes coalesced, reads ascending.
struct MatArgs {
  ProjCol proj[kMaxProj];
  void* out[kMaxProj];
  int32_t nproj;
};

// Late materialisation.  G4 > 0: every projected column is 4 bytes wide and
// there are at most G4 of them -- all their loads are issued before the
// first store (4 rows x G4 columns in flight per thread: the row reads are
// random, so this is a request-rate-bound kernel).
template <int G4>
__global__ __launch_bounds__(kBlock) void k_gather(const int64_t* __restrict__ ids, const int64_t* __restrict__ total,
                                                   int64_t row_offset, MatArgs M) {
  const int64_t n = *total;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; i0 < n; i0 += 4 * stride) {
    int64_t row[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * stride;
      row[u] = i < n ? ids[i] - row_offset : -1;
    }
    if constexpr (G4 > 0) {
      uint32_t v[G4][4];
#pragma unroll
      for (int p = 0; p < G4; ++p) {
        const gi32* src = (const gi32*)M.proj[p].base;
#pragma unroll
        for (int u = 0; u < 4; ++u) v[p][u] = (p < M.nproj && row[u] >= 0) ? (uint32_t)src[row[u]] : 0u;
      }
#pragma unroll
      for (int p = 0; p < G4; ++p)
        if (p < M.nproj) {
          uint32_t* dst = (uint32_t*)M.out[p];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (row[u] >= 0) dst[i0 + u * stride] = v[p][u];
        }
    } else {
      for (int p = 0; p < M.nproj; ++p) {
        const int sw = M.proj[p].stride_w;
        const uint32_t* src = (const uint32_t*)M.proj[p].base;
        uint32_t* dst = (uint32_t*)M.out[p];
        if (sw == 1) {
          uint32_t v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = row[u] >= 0 ? src[row[u]] : 0u;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (row[u] >= 0) dst[i0 + u * stride] = v[u];
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (row[u] >= 0)
              for (int k = 0; k < sw; ++k) dst[(i0 + u * stride) * sw + k] = src[row[u] * sw + k];
        }
      }
    }
  }
}

// One pass over a column building the BitSet of each listed value.  Deleted
// positions stay clear: createBitMapIndex walks a ColumnScan, which skips them
// (R/columnar/ColumnScan.java:49-65).
struct IndexArgs {
  uint64_t* out[64];
};

__global__ __launch_bounds__(kBlock) void k_index_build(KCol col, int64_t nrows, const uint64_t* __restrict__ del,
                                                        const uint32_t* __restrict__ vals, int32_t nvalues,
                                                        int32_t vwords, IndexArgs A, int64_t words_per_block) {
  const int lane = threadIdx.x & 63;
  const int wave = (int)uniform(threadIdx.x >> 6);
  const int64_t nwords = (nrows + 63) >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * words_per_block;
  const int64_t w1 = min(w0 + words_per_block, nwords);
  for (int64_t w = w0 + wave; w < w1; w += kWaves) {
    const int64_t row = w * 64 + lane;
    const bool valid = row < nrows && !(del && ((del[w] >> lane) & 1ull));
    uint32_t x0 = 0;
    if (valid && col.kind != kStr) x0 = ((const uint32_t*)col.base)[row];
    for (int v = 0; v < nvalues; ++v) {
      bool eq = false;
      if (valid) {
        if (col.kind == kStr) {
          eq = str_cmp((const uint32_t*)col.base + row * col.stride_w, col.stride_w, vals + v * vwords, vwords) == 0;
        } else if (col.kind == kInt) {
          eq = (int32_t)x0 == (int32_t)vals[v];
        } else {
          eq = __uint_as_float(x0) == __uint_as_float(vals[v]);
        }
      }
      const uint64_t m = __ballot(eq);
      if (lane == 0) A.out[v][w] = m;
    }
  }
}

// The same for a 4-byte column: lane l of a wave loads rows l, 64+l, 128+l,
// 192+l of a 256-row tile (four coalesced 256-byte loads), so the wave ballot
// of each compare IS one BitSet word -- per value and tile: 4 compares, 4
// ballots, 4 scalar popcounts, one store by lanes 0..3.  U tiles in flight
// per wave; every output's segment count is accumulated in wave-private LDS
// slots (no separate popcount pass).
struct IndexArgs4 {
  uint64_t* out[64];
  int64_t* segs[64];
};

template <int U>
__global__ __launch_bounds__(kBlock) void k_index_build4(const int32_t* __restrict__ col, int32_t kind,
                                                         int64_t nrows, const uint64_t* __restrict__ del,
                                                         const uint32_t* __restrict__ vals, int32_t nvalues,
                                                         IndexArgs4 A, int64_t tiles_per_block) {
  __shared__ uint32_t cnt[kWaves][64];
  const int lane = threadIdx.x & 63;
  const int wave = (int)uniform(threadIdx.x >> 6);
  cnt[wave][lane] = 0u;
  const int64_t ntiles = (nrows + kTileRows - 1) / kTileRows;
  const int64_t nwords = (nrows + 63) >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_block;
  const int64_t t1 = min(t0 + tiles_per_block, ntiles);
  for (int64_t base = t0 + wave; base < t1; base += (int64_t)kWaves * U) {
    int32_t x[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t t = base + (int64_t)u * kWaves;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t r = t * kTileRows + j * 64 + lane;
        x[u][j] = (t < t1 && r < nrows) ? __builtin_nontemporal_load(col + r) : 0;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t t = base + (int64_t)u * kWaves;
      if (t >= t1) continue;
      uint64_t live[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t w = t * kWordsPerTile + j;
        live[j] = __ballot(w * 64 + lane < nrows) & ((del && w < nwords) ? ~del[w] : ~0ull);
      }
      for (int v = 0; v < nvalues; ++v) {
        const uint32_t lit = vals[v];
        uint64_t m[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool eq = kind == kReal ? __int_as_float(x[u][j]) == __uint_as_float(lit) : x[u][j] == (int32_t)lit;
          m[j] = __ballot(eq) & live[j];
        }
        const uint64_t mine = lane == 0 ? m[0] : (lane == 1 ? m[1] : (lane == 2 ? m[2] : m[3]));
        const int64_t w = t * kWordsPerTile + lane;
        if (lane < 4 && w < nwords) A.out[v][w] = mine;
        if (lane == 0) cnt[wave][v] += (uint32_t)(__popcll(m[0]) + __popcll(m[1]) + __popcll(m[2]) + __popcll(m[3]));
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < nvalues) {
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) c += cnt[k][threadIdx.x];
    A.segs[threadIdx.x][blockIdx.x] = c;
  }
}

// ------------------------------------------------------------ read probe
//
// The scan's load pattern with the predicate removed: the same 256-row tiles,
// U tiles in flight per wave, non-temporal dwordx4 loads, the same segment
// (or grid-stride) mapping; the words are XOR-folded and one word per block
// is stored.  Its time is the read-bandwidth ceiling the scan is held to
// ("measured read peak").
template <int U>
__global__ __launch_bounds__(kBlock) void k_read_probe(ProbeArgs A) {
  const int lane = threadIdx.x & 63;
  const int wave = (int)uniform(threadIdx.x >> 6);
  const int64_t ntiles = A.nrows / kTileRows;  // full tiles only
  const bool il = A.interleave != 0;
  const int64_t t0 = il ? (int64_t)blockIdx.x * kWaves : (int64_t)blockIdx.x * A.tiles_per_block;
  const int64_t t1 = il ? ntiles : min(t0 + A.tiles_per_block, ntiles);
  const int64_t ustep = il ? (int64_t)gridDim.x * kWaves : kWaves;
  v4i acc = {0, 0, 0, 0};
  for (int64_t base = t0 + wave; base < t1; base += ustep * U) {
    v4i q[U][kMaxProbeCols];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t t = base + (int64_t)u * ustep;
#pragma unroll
      for (int c = 0; c < kMaxProbeCols; ++c)
        q[u][c] = (t < t1 && c < A.ncols) ? load16<true>(A.cols[c] + t * kTileRows + lane * 4) : v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < kMaxProbeCols; ++c) acc ^= q[u][c];
  }
  int32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  for (int off = 32; off > 0; off >>= 1) x ^= __shfl_xor(x, off);
  __shared__ int32_t red[kWaves];
  if (lane == 0) red[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) A.sink[blockIdx.x] = (uint32_t)(red[0] ^ red[1] ^ red[2] ^ red[3]);
}

hipError_t launch_read_probe(const ProbeArgs& A, hipStream_t s) {
  const int64_t ntiles = A.nrows / kTileRows;
  if (ntiles <= 0) return hipSuccess;
  const int64_t g = A.interleave ? A.grid : (ntiles + A.tiles_per_block - 1) / A.tiles_per_block;
  hipLaunchKernelGGL(k_read_probe<2>, dim3((unsigned)g), dim3(kBlock), 0, s, A);
  return hipGetLastError();
}

// ---------------------------------------------------------------- launchers

int64_t choose_tiles_per_block(int64_t nrows) {
  const int64_t ntiles = (nrows + kTileRows - 1) / kTileRows;
  // ~1024 blocks (4 per CU on 256 CUs, 16 waves/CU) for large inputs,
  // >= 4 tiles per block
  int64_t tpb = (ntiles + 1023) / 1024;
  return tpb < 4 ? 4 : tpb;
}

int64_t grid_blocks(int64_t nrows, int64_t tiles_per_block) {
  const int64_t ntiles = (nrows + kTileRows - 1) / kTileRows;
  const int64_t g = (ntiles + tiles_per_block - 1) / tiles_per_block;
  return g < 1 ? 1 : g;
}

// the production kernel of one (K, KS, MODE, DEL) class in either tile layout
template <int K, int KS, int MODE, bool DEL, bool RI>
static void prod_launch(const ScanLaunch& L, dim3 grid, hipStream_t s) {
  // 4-byte slots only and 1..kHoistTerms literal terms (L.hoist_terms): the terms
  // are hoisted into registers (TQ) and the per-row tile body is unrolled over
  // them -- measured 2.5 % faster than reading them from the plan per tile
  // and than an SGPR-lane-mask body, profiles/r01/an3
  constexpr int TQ = KS == 0 ? kHoistTerms : 0;
  // one 4-byte column: 4 tiles in flight per wave (the same bytes in flight as
  // two columns at U=2); 100M rows: COUNT 69.7 -> 67.3 us, BitSet 87.5 -> 81.0 us
  // two-column COUNT scans (C3): 3 tiles in flight per wave -- 117.4 vs
  // 117.8-119.4 us (U = 2) and 120.3-120.7 (U = 4) at 100M rows, alternating
  // A/B builds on one box (profiles/r05/ak; MBX_SCAN_U2 overrides it in
  // tools/build_variant.sh builds)
#ifndef MBX_SCAN_U2
#define MBX_SCAN_U2 3
#endif
  // MBX_SCAN_U_AGG (A/B builds): tiles in flight for aggregate scans
#ifndef MBX_SCAN_U_AGG
#define MBX_SCAN_U_AGG kDefaultU
#endif
  constexpr int kU = K == 1 && KS == 0 ? 4
                     : (K == 2 && KS == 0 && MODE == kModeCount ? MBX_SCAN_U2
                                                                : (MODE == kModeAgg ? MBX_SCAN_U_AGG : kDefaultU));
  const unsigned lds = L.sink_lds ? (unsigned)(L.tiles_per_block * kWordsPerTile * sizeof(uint64_t)) : 0u;
  // int literal terms as branch-free range tests
  if constexpr (KS == 0) {
    if (L.hoist_terms && L.int_range == 1) {
      hipLaunchKernelGGL((k_scan_fast<K, KS, MODE, DEL, kU, kDefaultNT, TQ, RI, 1>), grid, dim3(kBlock), lds, s, L);
      return;
    }
  }
  // literal terms of any type as range tests over ordered keys, hoisted
  // (COUNT / aggregate scans in the 4-rows-per-lane layout)
  if constexpr (MODE != kModeBitmap && !RI) {
    if (L.int_range == 2) {
      hipLaunchKernelGGL((k_scan_fast<K, KS, MODE, DEL, kU, kDefaultNT, kHoistTerms, RI, 2>), grid, dim3(kBlock), lds, s,
                         L);
      return;
    }
  }
  if (KS == 0 && L.hoist_terms)
    hipLaunchKernelGGL((k_scan_fast<K, KS, MODE, DEL, kU, kDefaultNT, TQ, RI>), grid, dim3(kBlock), lds, s, L);
  else
    hipLaunchKernelGGL((k_scan_fast<K, KS, MODE, DEL, kU, kDefaultNT, 0, RI>), grid, dim3(kBlock), lds, s, L);
}

template <int K, int KS, int MODE>
static void fast_launch(const ScanLaunch& L, dim3 grid, hipStream_t s) {
  if (L.deleted) {
    if (L.ri)
      prod_launch<K, KS, MODE, true, true>(L, grid, s);
    else
      prod_launch<K, KS, MODE, true, false>(L, grid, s);
  } else if (L.ri) {
    prod_launch<K, KS, MODE, false, true>(L, grid, s);
  } else {
    prod_launch<K, KS, MODE, false, false>(L, grid, s);
  }
}

// fast_k = number of 4-byte slots, fast_ks = number of 16-byte string slots;
// anything else goes to the one-row-per-lane generic kernel
template <int MODE>
static void mode_launch(const ScanLaunch& L, dim3 grid, hipStream_t s) {
  const int code = L.fast_ks * 8 + L.fast_k;
  switch (code) {
    case 1: fast_launch<1, 0, MODE>(L, grid, s); return;
    case 2: fast_launch<2, 0, MODE>(L, grid, s); return;
    case 3: fast_launch<3, 0, MODE>(L, grid, s); return;
    case 4: fast_launch<4, 0, MODE>(L, grid, s); return;
    case 8 + 0: fast_launch<0, 1, MODE>(L, grid, s); return;
    case 8 + 1: fast_launch<1, 1, MODE>(L, grid, s); return;
    case 8 + 2: fast_launch<2, 1, MODE>(L, grid, s); return;
    case 8 + 3: fast_launch<3, 1, MODE>(L, grid, s); return;
    case 16 + 0: fast_launch<0, 2, MODE>(L, grid, s); return;
    case 16 + 1: fast_launch<1, 2, MODE>(L, grid, s); return;
    case 16 + 2: fast_launch<2, 2, MODE>(L, grid, s); return;
    default:
      if (L.deleted)
        hipLaunchKernelGGL((k_scan_generic<MODE, true>), grid, dim3(kBlock), 0, s, L);
      else
        hipLaunchKernelGGL((k_scan_generic<MODE, false>), grid, dim3(kBlock), 0, s, L);
  }
}

hipError_t launch_scan(const ScanLaunch& L, hipStream_t s) {
  const dim3 grid((unsigned)grid_blocks(L.nrows, L.tiles_per_block));
  switch (L.mode) {
    case kModeCount: mode_launch<kModeCount>(L, grid, s); break;
    case kModeBitmap: mode_launch<kModeBitmap>(L, grid, s); break;
    default: mode_launch<kModeAgg>(L, grid, s); break;
  }
  return hipGetLastError();
}

hipError_t launch_finalize(const Partial* partials, int64_t nblocks, int32_t agg_kind, AggOut* out,
                           int64_t* count_out, int32_t* nan_flag, hipStream_t s) {
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(kBlock), 0, s, partials, nblocks, agg_kind, out, count_out,
                     nan_flag);
  return hipGetLastError();
}

static uint64_t tail_mask_of(int64_t nbits) {
  const int r = (int)(nbits & 63);
  return r == 0 ? ~0ull : ((1ull << r) - 1ull);
}

hipError_t launch_bitmap_cnf(const BitmapCnf& c, const uint64_t* deleted, int64_t nwords, int64_t nbits,
                             int64_t words_per_block, uint64_t* out, int64_t* segc, hipStream_t s) {
  const int64_t g = nwords == 0 ? 1 : (nwords + words_per_block - 1) / words_per_block;
  hipLaunchKernelGGL(k_bitmap_cnf, dim3((unsigned)g), dim3(kBlock), 0, s, c, deleted, nwords,
                     tail_mask_of(nbits), words_per_block, out, segc);
  return hipGetLastError();
}

hipError_t launch_bitmap_combine(int32_t op, const uint64_t* a, const uint64_t* b, int64_t nwords, int64_t nbits,
                                 int64_t words_per_block, uint64_t* out, int64_t* segc, hipStream_t s) {
  const int64_t g = nwords == 0 ? 1 : (nwords + words_per_block - 1) / words_per_block;
  hipLaunchKernelGGL(k_bitmap_combine, dim3((unsigned)g), dim3(kBlock), 0, s, op, a, b, nwords,
                     tail_mask_of(nbits), words_per_block, out, segc);
  return hipGetLastError();
}

hipError_t launch_seg_popcount(const uint64_t* words, int64_t nwords, int64_t words_per_block, int64_t* segc,
                               hipStream_t s) {
  const int64_t g = nwords == 0 ? 1 : (nwords + words_per_block - 1) / words_per_block;
  hipLaunchKernelGGL(k_seg_popcount, dim3((unsigned)g), dim3(kBlock), 0, s, words, nwords, words_per_block,
                     segc);
  return hipGetLastError();
}

// the sum of n segment counts (a BitSet's cardinality), one block, fixed order
__global__ __launch_bounds__(kBlock) void k_count_sum(const int64_t* __restrict__ segc, int64_t n,
                                                     int64_t* __restrict__ out) {
  __shared__ int64_t sh[kWaves];
  int64_t c = 0;
  for (int64_t i = threadIdx.x; i < n; i += kBlock) c += segc[i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) *out = sh[0] + sh[1] + sh[2] + sh[3];
}

hipError_t launch_count_sum(const int64_t* segc, int64_t n, int64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_count_sum, dim3(1), dim3(kBlock), 0, s, segc, n, out);
  return hipGetLastError();
}


hipError_t launch_materialize(const uint64_t* words, int64_t nwords, int64_t words_per_block,
                              const int64_t* segc, int64_t row_offset, int64_t* ids, const ProjCol* proj,
                              void* const* out, int32_t nproj, int64_t* total, hipStream_t s, int32_t dbg,
                              int64_t* stamps, bool fuse_gather, int64_t max_blocks, bool gather_pair) {
  if (nwords == 0) return hipMemsetAsync(total, 0, sizeof(int64_t), s);
  if (max_blocks < 1) max_blocks = 1024;
  // ~max_blocks (1024) compaction blocks whatever the segment size: S segments per block
  const int64_t nseg = (nwords + words_per_block - 1) / words_per_block;
  const int64_t S = (nseg + max_blocks - 1) / max_blocks;
  const int64_t wpb = S * words_per_block;
  const int64_t g = (nwords + wpb - 1) / wpb;
  // up to 4 int / float columns: gathered by the compaction itself (no
  // second launch, no re-read of the positions)
  bool all4 = nproj <= 4;
  for (int j = 0; j < nproj && j < kMaxProj; ++j) all4 = all4 && proj[j].stride_w == 1;
  Gather4 G{};
  if (nproj > 0 && all4 && fuse_gather) {
    for (int j = 0; j < nproj; ++j) {
      gather4_source(G, j, proj[j]);
      G.out[j] = (uint32_t*)out[j];
    }
    G.n = nproj;
    gather4_pairing(G, gather_pair);
    hipLaunchKernelGGL(k_select_ids<4>, dim3((unsigned)g), dim3(kBlock), 0, s, words, nwords, wpb, segc, S,
                       row_offset, ids, total, dbg, stamps, G);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_select_ids<0>, dim3((unsigned)g), dim3(kBlock), 0, s, words, nwords, wpb, segc, S,
                     row_offset, ids, total, dbg, stamps, G);
  if (nproj > 0) {
    MatArgs M;
    M.nproj = nproj;
    for (int j = 0; j < nproj && j < kMaxProj; ++j) {
      M.proj[j] = proj[j];
      M.out[j] = out[j];
    }
    if (all4)
      hipLaunchKernelGGL(k_gather<4>, dim3(1024), dim3(kBlock), 0, s, ids, total, row_offset, M);
    else
      hipLaunchKernelGGL(k_gather<0>, dim3(1024), dim3(kBlock), 0, s, ids, total, row_offset, M);
  }
  return hipGetLastError();
}

hipError_t launch_cnf_materialize(const BitmapCnf& c, const uint64_t* deleted, int64_t nwords, int64_t nbits,
                                  int64_t* lb, int64_t row_offset, int64_t* ids, const ProjCol* proj,
                                  void* const* out, int32_t nproj, int64_t* total, hipStream_t s,
                                  int64_t* stamps, int32_t dbg, int64_t cap, const CnfTune* tune) {
  if (nwords == 0) return hipMemsetAsync(total, 0, sizeof(int64_t), s);
  const CnfTune knobs = tune ? *tune : CnfTune{};
  const int32_t blocks = knobs.blocks, flag_stride = knobs.flag_stride, lookback = knobs.lookback;
  dbg = (dbg & ~(3 << 12)) | ((knobs.store & 3) << 12);
  if (nproj < 0 || nproj > kMaxProj) return hipErrorInvalidValue;
  // <= 4 four-byte columns: values prefetched in registers (Gather4); any
  // other projection (char(n) rows, more columns): row copies (GatherW)
  bool narrow = nproj <= 4;
  for (int j = 0; j < nproj; ++j) narrow = narrow && proj[j].stride_w == 1;
  Gather4 G{};
  GatherW W{};
  for (int j = 0; j < nproj; ++j) {
    if (proj[j].stride_w < 1) return hipErrorInvalidValue;
    if (narrow) {
      gather4_source(G, j, proj[j]);
      G.out[j] = (uint32_t*)out[j];
    }
    W.col[j] = (const uint32_t*)proj[j].base;
    W.out[j] = (uint32_t*)out[j];
    W.sw[j] = proj[j].stride_w;
  }
  G.n = narrow ? nproj : 0;
  gather4_pairing(G, knobs.gather_pair != 0);
  W.n = nproj;
  G.cap = W.cap = cap;
  // kernel dbg bit 3 = the chained look-back: each block walks back 64
  // predecessors per round to the nearest published inclusive prefix;
  // without it every thread polls its share of the predecessors' counts, all
  // in flight together.  Measured at C4 (100 M rows, 1 % AND, 1024 blocks,
  // profiles/r05/h): with the projected pair gathered from a column group,
  // polling (flags packed) 29.8 us vs chained 32.1 us; with the columns
  // gathered separately (one more line per row) chained 45.1 vs polling
  // 46.6-48.0.  So (lookback 0, auto) narrow projections read from column
  // groups -- and positions-only launches -- poll, the rest walk the chain;
  // inclusive prefixes are 32-bit, so tables of >= 2^32 rows always poll.
  // lookback 1 / 2 (tuning cnf_lookback) force the chain / the polls, as
  // select_dbg bit 7 (MBX_SELECT_DBG=128) forces the polls.
  bool grouped = narrow;
  for (int j = 0; j < nproj; ++j) grouped = grouped && proj[j].gstride > 0;
  const bool chained = nbits < (int64_t(1) << 32) && !(dbg & 8) &&
                       (lookback == 1 || (lookback == 0 && !grouped));
  dbg = (dbg & ~8) | (chained ? 8 : 0);
  // <= kLookbackBlocks blocks for the polling form (one poll load per thread
  // per 256 predecessors); the chained form takes up to kIncBase (tuning
  // cnf_blocks: more blocks than the chip holds at once, so the later ones'
  // operand loads run beside the earlier ones' gathers)
  const int64_t want = blocks > 0 ? ((dbg & 8) ? (blocks < kIncBase ? blocks : kIncBase)
                                                : (blocks < kLookbackBlocks ? blocks : kLookbackBlocks))
                                   : kLookbackBlocks;
  const int32_t fs = (dbg & 8) || flag_stride != kFlagStride ? 1 : kFlagStride;
  const int64_t wpb = (nwords + want - 1) / want;
  const int64_t g = (nwords + wpb - 1) / wpb;
  const int nbm = c.conj_off[c.nconj];
  // the prefetch registers sized to the projection: <= 2 columns or <= 4
#define MBX_CNF_SELECT(NB)                                                                                  \
  if (!narrow)                                                                                              \
    hipLaunchKernelGGL((k_cnf_select<kWide, NB, GatherW>), dim3((unsigned)g), dim3(kBlock), 0, s, c, deleted, \
                       nwords, tail_mask_of(nbits), wpb, lb, row_offset, ids, total, W, stamps, dbg, fs);            \
  else if (nproj <= 2)                                                                                      \
    hipLaunchKernelGGL((k_cnf_select<2, NB>), dim3((unsigned)g), dim3(kBlock), 0, s, c, deleted, nwords,    \
                       tail_mask_of(nbits), wpb, lb, row_offset, ids, total, G, stamps, dbg, fs);                    \
  else                                                                                                      \
    hipLaunchKernelGGL((k_cnf_select<4, NB>), dim3((unsigned)g), dim3(kBlock), 0, s, c, deleted, nwords,    \
                       tail_mask_of(nbits), wpb, lb, row_offset, ids, total, G, stamps, dbg, fs)
  switch (nbm) {
    case 1: MBX_CNF_SELECT(1); break;
    case 2: MBX_CNF_SELECT(2); break;
    case 3: MBX_CNF_SELECT(3); break;
    case 4: MBX_CNF_SELECT(4); break;
    default: MBX_CNF_SELECT(0); break;
  }
#undef MBX_CNF_SELECT
  return hipGetLastError();
}

bool scan_select_fusable(int64_t nrows, int64_t tiles_per_block, int32_t fast_k, int32_t fast_ks, int32_t nterms,
                         int32_t has_real, int32_t waves) {
  const int64_t ntiles = (nrows + kTileRows - 1) / kTileRows;
  const int64_t nseg = ntiles == 0 ? 1 : (ntiles + tiles_per_block - 1) / tiles_per_block;
  // look-back flags per block: a 16-wave block holds 4 segments
  const int64_t spb = waves == 16 ? 16 / kWaves : 1;
  const int64_t nb = (nseg + spb - 1) / spb;
  return fast_k >= 1 && fast_k <= 4 && fast_ks == 0 && !has_real && nterms >= 1 && nterms <= kHoistTerms &&
         nrows > 0 && nb <= kLookbackBlocks && (tiles_per_block + kWaves - 1) / kWaves <= 16 * kSelRegs &&
         nrows < (int64_t(1) << 32);
}

hipError_t launch_scan_select(const ScanLaunch& L, int64_t* lb, int64_t row_offset, int64_t* ids, int64_t* total,
                              hipStream_t s, int64_t* stamps, int32_t dbg, int32_t waves, int32_t flag_stride) {
  // waves per block: 4 (one BitSet segment per block) or 16 (four): a
  // quarter of the blocks publish and walk back
  const int nw = waves == 16 ? 16 : kWaves;
  const int64_t nseg = grid_blocks(L.nrows, L.tiles_per_block);
  const int64_t g = (nseg + nw / kWaves - 1) / (nw / kWaves);
  // every predecessor's count polled (<= 256 blocks: one poll per thread of
  // 15 waves), one flag per 128-byte line (flag_stride kFlagStride, the
  // default: the polls of all blocks do not queue on a few lines) -- C2
  // 11.8-12.1 us vs 13.4-13.6 for the chained walk and 12.0-12.2 with the
  // flags packed (profiles/r04/f1); select_dbg bit 7: the chained walk
  // (32-bit inclusive prefixes: tables < 2^32 rows)
  const int32_t fs = (dbg & 8) || flag_stride != kFlagStride ? 1 : kFlagStride;
  const bool del = L.deleted != nullptr;
  const bool ir = L.int_range != 0;  // branch-free int terms (every fused plan qualifies; the knob can turn it off)
  // registers of 64 words per wave: only as many as a wave's quarter
  // segment needs (C2: one) -- the unrolled count / staging / emission code
  // of unused registers is not instantiated (a smaller kernel for the
  // instruction cache, fewer VGPRs)
  const int64_t wave_words = (L.tiles_per_block + kWaves - 1) / kWaves * kWordsPerTile;
  const int nr = wave_words <= 64 ? 1 : wave_words <= 128 ? 2 : wave_words <= 256 ? 4 : kSelRegs;
#define MBX_SCAN_SELECT_NW(KK, UU, NW, NR)                                                                       \
  if (del && ir)                                                                                               \
    hipLaunchKernelGGL((k_scan_select<KK, true, UU, kHoistTerms, NW, NR, 1>), dim3((unsigned)g), dim3(64 * NW), \
                       0, s, L, lb, row_offset, ids, total, stamps, dbg, fs);                                  \
  else if (del)                                                                                                \
    hipLaunchKernelGGL((k_scan_select<KK, true, UU, kHoistTerms, NW, NR>), dim3((unsigned)g), dim3(64 * NW), 0, \
                       s, L, lb, row_offset, ids, total, stamps, dbg, fs);                                     \
  else if (ir)                                                                                                 \
    hipLaunchKernelGGL((k_scan_select<KK, false, UU, kHoistTerms, NW, NR, 1>), dim3((unsigned)g),            \
                       dim3(64 * NW), 0, s, L, lb, row_offset, ids, total, stamps, dbg, fs);                   \
  else                                                                                                         \
    hipLaunchKernelGGL((k_scan_select<KK, false, UU, kHoistTerms, NW, NR>), dim3((unsigned)g), dim3(64 * NW), 0, \
                       s, L, lb, row_offset, ids, total, stamps, dbg, fs)
#define MBX_SCAN_SELECT(KK, UU)                  \
  if (nw != 16) {                                \
    MBX_SCAN_SELECT_NW(KK, UU, kWaves, kSelRegs); \
  } else if (nr == 1) {                          \
    MBX_SCAN_SELECT_NW(KK, UU, 16, 1);           \
  } else if (nr == 2) {                          \
    MBX_SCAN_SELECT_NW(KK, UU, 16, 2);           \
  } else if (nr == 4) {                          \
    MBX_SCAN_SELECT_NW(KK, UU, 16, 4);           \
  } else {                                       \
    MBX_SCAN_SELECT_NW(KK, UU, 16, kSelRegs);    \
  }
  // tiles in flight per wave as in the fast scan; one column at U = 8 (a C2
  // wave waits on two load batches instead of three) measured slower: the
  // scan part of C2 ends at 10.4 instead of 9.2 us (profiles/r03/lb)
  switch (L.fast_k) {
    case 1: MBX_SCAN_SELECT(1, 4); break;
    case 2: MBX_SCAN_SELECT(2, 2); break;
    case 3: MBX_SCAN_SELECT(3, 2); break;
    default: MBX_SCAN_SELECT(4, 2); break;
  }
#undef MBX_SCAN_SELECT
#undef MBX_SCAN_SELECT_NW
  return hipGetLastError();
}

hipError_t launch_index_build4(const KCol& col, int64_t nrows, const uint64_t* deleted, const uint32_t* values,
                               int32_t nvalues, uint64_t* const* outs, int64_t* const* segs, int64_t words_per_block,
                               hipStream_t s) {
  const int64_t nwords = (nrows + 63) >> 6;
  const int64_t g = nwords == 0 ? 1 : (nwords + words_per_block - 1) / words_per_block;
  for (int32_t v0 = 0; v0 < nvalues; v0 += 64) {
    IndexArgs4 A;
    const int32_t nv = nvalues - v0 < 64 ? nvalues - v0 : 64;
    for (int i = 0; i < nv; ++i) {
      A.out[i] = outs[v0 + i];
      A.segs[i] = segs[v0 + i];
    }
    hipLaunchKernelGGL(k_index_build4<2>, dim3((unsigned)g), dim3(kBlock), 0, s, (const int32_t*)col.base, col.kind,
                       nrows, deleted, values + v0, nv, A, words_per_block / kWordsPerTile);
  }
  return hipGetLastError();
}

hipError_t launch_index_build(const KCol& col, int64_t nrows, const uint64_t* deleted, const uint32_t* values,
                              int32_t nvalues, int32_t value_words, uint64_t* const* outs, int64_t words_per_block,
                              hipStream_t s) {
  const int64_t nwords = (nrows + 63) >> 6;
  const int64_t g = nwords == 0 ? 1 : (nwords + words_per_block - 1) / words_per_block;
  for (int32_t v0 = 0; v0 < nvalues; v0 += 64) {
    IndexArgs A;
    const int32_t nv = nvalues - v0 < 64 ? nvalues - v0 : 64;
    for (int i = 0; i < nv; ++i) A.out[i] = outs[v0 + i];
    hipLaunchKernelGGL(k_index_build, dim3((unsigned)g), dim3(kBlock), 0, s, col, nrows, deleted,
                       values + (int64_t)v0 * value_words, nv, value_words, A, words_per_block);
  }
  return hipGetLastError();
}

}  // namespace mbx
