// mbx_pages.hip -- CDNA4 kernels that turn Minibase DB pages (resident in
// HBM as they lie on disk) into the device column image (mbx_db_stage).
//
//   k_page_decode    one wave per data page of a column heapfile: reads the
//                    HFPage slot directory (R/heap/HFPage.java:31-40,543-573),
//                    byte-swaps each record (R/global/Convert.java:18-66) or
//                    turns its writeUTF image (Convert.java:108-126) into the
//                    device string encoding, and stores it at its reference
//                    position recsPerDataPage * pageIndex + slot
//                    (R/heap/Heapfile.java:262-289); the position's bit is set
//                    in the column's `present` BitSet.
//   k_present_merge  deleted = NOT present(column 0) OR cf.md, and a mismatch
//                    flag when another column's present set differs
//                    (Columnarfile.java:480-482 "Invalid position calculations").
//   k_distinct       distinct live values + first position (createBitMapIndex).
//   k_rows_fetch     a few rows of a column (the distinct values themselves).
//
// Byte/integer work, HBM bound: per page 1 KiB read + the decoded records
// written; no MFMA, no LDS.
#include "mbx_internal.hpp"

namespace mbx {

// One wave per data page: lane l handles slots l, l+64, l+128 (<= 143 records
// per page).  Slot entries are read as aligned big-endian words, 4-byte
// records as aligned words (every record of a column page has the same size,
// so offsets stay 4-aligned), outputs are written at consecutive positions;
// the `present` bits of each 64-slot group come from one ballot and go out
// with at most two atomicOr (page boundaries share words).
__device__ __forceinline__ uint32_t ld_be32a(const uint8_t* p) {
  return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(p));
}

__global__ __launch_bounds__(kBlock) void k_page_decode(PageDecodeArgs A) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * kWaves;
  int32_t err = 0;
  for (int64_t pi = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); pi < A.npages; pi += nwaves) {
    const int32_t pid = A.page_of[pi];
    if (pid < 0) continue;
    if ((int64_t)pid >= A.image_pages) {
      err |= 1;
      continue;
    }
    const uint8_t* pg = A.image + (int64_t)pid * kDbPage;
    int32_t slots = (int32_t)(int16_t)(ld_be32a(pg) >> 16);
    if (slots > A.recs_per_page || slots < 0) {
      err |= 2;
      slots = slots < 0 ? 0 : A.recs_per_page;
    }
    for (int32_t k0 = 0; k0 < slots; k0 += 64) {
      const int32_t k = k0 + lane;
      bool ok = false;
      if (k < slots) {
        const uint32_t se = ld_be32a(pg + kDbSlotBase + 4 * k);
        const int32_t len = (int32_t)(int16_t)(se >> 16);
        const int32_t off = (int32_t)(se & 0xFFFFu);
        const int64_t pos = (A.page_index0 + pi) * A.recs_per_page + k - A.pos_begin;  // output row
        if (len == -1) {
          // EMPTY_SLOT: no record at this position
        } else if (len != A.rec_len || off < kDbSlotBase || off + len > kDbPage) {
          err |= 4;
        } else if (pos < 0 || pos >= A.nrows) {
          if (!A.range) err |= 8;  // range staging: another shard's position
        } else {
          const uint8_t* rec = pg + off;
          ok = true;
          if (A.kind != kStr) {
            const uint32_t v = (off & 3) == 0 ? ld_be32a(rec)
                                              : ((uint32_t)rec[0] << 24) | ((uint32_t)rec[1] << 16) |
                                                    ((uint32_t)rec[2] << 8) | rec[3];
            reinterpret_cast<uint32_t*>(A.out)[pos] = v;
          } else {
            // writeUTF image: u16 length + modified UTF-8; device image rewrites
            // C0 80 (U+0000) as 00 01 and zero-pads to the stride
            int32_t L = (int32_t)(((uint32_t)rec[0] << 8) | rec[1]);
            if (L > A.size) {
              err |= 16;
              L = A.size;
            }
            uint32_t* dst = reinterpret_cast<uint32_t*>(A.out + pos * (int64_t)A.stride);
            uint32_t acc = 0;
            int32_t o = 0;
            auto put = [&](uint32_t byte) {
              acc |= byte << (8 * (o & 3));
              if ((o & 3) == 3) {
                dst[o >> 2] = acc;
                acc = 0;
              }
              ++o;
            };
            int32_t i = 0;
            while (i < L) {
              const uint32_t byte = rec[2 + i];
              if (byte == 0xC0u && i + 1 < L && rec[3 + i] == 0x80u) {
                put(0u);
                put(1u);
                i += 2;
              } else {
                put(byte);
                ++i;
              }
            }
            while (o < A.stride) put(0u);
          }
        }
      }
      const uint64_t m = __ballot(ok);
      if (lane == 0 && m) {
        const int64_t base = (A.page_index0 + pi) * A.recs_per_page + k0 - A.pos_begin;
        unsigned long long* w0 = reinterpret_cast<unsigned long long*>(A.present);
        if (base >= 0) {
          const int sh = (int)(base & 63);
          unsigned long long* w = w0 + (base >> 6);
          atomicOr(w, (unsigned long long)(m << sh));
          if (sh && (m >> (64 - sh))) atomicOr(w + 1, (unsigned long long)(m >> (64 - sh)));
        } else if (base > -64) {
          // the page starts before this shard (range staging): lanes below
          // -base hold another shard's positions and are not in m
          atomicOr(w0, (unsigned long long)(m >> (-base)));
        }
      }
    }
  }
  if (err) atomicOr(A.err, err);
}

__global__ __launch_bounds__(kBlock) void k_present_merge(const uint64_t* __restrict__ present0,
                                                          const uint64_t* __restrict__ other, int32_t nother,
                                                          int64_t nwords_each, const uint64_t* __restrict__ md,
                                                          int64_t md_words, int64_t nrows, uint64_t* __restrict__ del,
                                                          int32_t* flags) {
  const int64_t nwords = (nrows + 63) >> 6;
  for (int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * kBlock) {
    const uint64_t p = present0[w];
    for (int32_t j = 0; j < nother; ++j)
      if (other[j * nwords_each + w] != p) atomicOr(flags, 1);
    uint64_t d = ~p | (w < md_words ? md[w] : 0ull);
    if (w == nwords - 1 && (nrows & 63)) d &= (1ull << (nrows & 63)) - 1ull;
    del[w] = d;
    if (d) atomicOr(flags, 2);
  }
}

// ------------------------------------------------ distinct column values
//
// Columnarfile.createBitMapIndex registers one BitMapFile per distinct value
// of the live rows, in first-occurrence (ColumnScan) order
// (R/columnar/Columnarfile.java:698-753).  One pass over the column inserts
// every live row into an open-addressing table in HBM whose slots hold a
// representative row (the key: rows compare by column value) and the
// smallest position holding that value.  A row first READS the slot's
// minimum and only issues atomicMin when it is smaller, so a low-cardinality
// column (the bitmap-index case) costs reads of a few hot L2 lines, not
// same-address atomics per row.

__device__ __forceinline__ uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

__device__ __forceinline__ uint64_t row_hash(const KCol& c, int64_t row) {
  const uint32_t* p = (const uint32_t*)c.base + row * c.stride_w;
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < c.stride_w; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return mix64(h);
}

__device__ __forceinline__ bool rows_equal(const KCol& c, int64_t a, int64_t b) {
  const uint32_t* pa = (const uint32_t*)c.base + a * c.stride_w;
  const uint32_t* pb = (const uint32_t*)c.base + b * c.stride_w;
  for (int i = 0; i < c.stride_w; ++i)
    if (pa[i] != pb[i]) return false;
  return true;
}

// Global table insert of `row`: find or claim the slot of its value, lower
// the slot's first position to `row`.  keys / minpos are written only through
// atomics; plain (cached) reads may be stale but never wrong: a stale EMPTY
// only sends the row to the CAS, a stale minimum costs one more atomicMin.
__device__ __forceinline__ void distinct_insert(const DistinctArgs& A, int64_t row, uint64_t h) {
  const uint64_t mask = (uint64_t)A.cap - 1;
  h &= mask;
  for (int64_t probe = 0; probe < A.cap; ++probe, h = (h + 1) & mask) {
    unsigned long long k = A.keys[h];
    if (k == kEmptySlot) {
      k = atomicCAS(A.keys + h, kEmptySlot, (unsigned long long)row);
      if (k == kEmptySlot) k = (unsigned long long)row;
    }
    if (rows_equal(A.col, (int64_t)k, row)) {
      if ((unsigned long long)row < A.minpos[h]) atomicMin(A.minpos + h, (unsigned long long)row);
      return;
    }
  }
  atomicOr(A.overflow, 1);
}

// Two levels: each block first folds its rows into an LDS table (value ->
// smallest row of the block with it), so a low-cardinality column touches
// the global table once per value per block instead of once per row; rows
// whose value finds no LDS slot within kLdsProbes go to the global table
// directly (A.lds_probes, kLdsProbes by default).  4-byte columns keep the value itself as the LDS key (no column
// re-reads); wider ones keep a representative row.
constexpr int kLdsSlots = 2048;

template <bool V1>
__global__ __launch_bounds__(kBlock) void k_distinct(DistinctArgs A, int64_t rows_per_block) {
  __shared__ unsigned long long skey[kLdsSlots];
  __shared__ unsigned long long smin[kLdsSlots];
  for (int i = threadIdx.x; i < kLdsSlots; i += kBlock) {
    skey[i] = kEmptySlot;
    smin[i] = kEmptySlot;
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = min(r0 + rows_per_block, A.nrows);
  for (int64_t row = r0 + threadIdx.x; row < r1; row += kBlock) {
    if (A.del && ((A.del[row >> 6] >> (row & 63)) & 1ull)) continue;
    const uint64_t h = row_hash(A.col, row);
    const unsigned long long mine =
        V1 ? (unsigned long long)((const uint32_t*)A.col.base)[row] : (unsigned long long)row;
    uint32_t slot = (uint32_t)h & (kLdsSlots - 1);
    bool placed = false;
    for (int probe = 0; probe < A.lds_probes; ++probe, slot = (slot + 1) & (kLdsSlots - 1)) {
      unsigned long long k = skey[slot];
      if (k == kEmptySlot) {
        k = atomicCAS(skey + slot, kEmptySlot, mine);
        if (k == kEmptySlot) k = mine;
      }
      if (V1 ? k == mine : rows_equal(A.col, (int64_t)k, row)) {
        atomicMin(smin + slot, (unsigned long long)row);
        placed = true;
        break;
      }
    }
    if (!placed) distinct_insert(A, row, h);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLdsSlots; i += kBlock) {
    const unsigned long long row = smin[i];
    if (row != kEmptySlot) distinct_insert(A, (int64_t)row, row_hash(A.col, (int64_t)row));
  }
}

// rows[i] of a column -> out (stride_w words per row)
__global__ __launch_bounds__(kBlock) void k_rows_fetch(KCol c, const int64_t* __restrict__ rows, int64_t n,
                                                       uint32_t* __restrict__ out) {
  const int64_t total = n * c.stride_w;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / c.stride_w, w = i - r * c.stride_w;
    out[i] = ((const uint32_t*)c.base)[rows[r] * c.stride_w + w];
  }
}

hipError_t launch_distinct(const DistinctArgs& A, hipStream_t s) {
  if (A.nrows <= 0) return hipSuccess;
  // ~1024 blocks of contiguous row ranges (multiples of the block size)
  int64_t rpb = (A.nrows + 1023) / 1024;
  rpb = (rpb + kBlock - 1) / kBlock * kBlock;
  if (rpb < 4 * kBlock) rpb = 4 * kBlock;
  const int64_t g = (A.nrows + rpb - 1) / rpb;
  if (A.col.stride_w == 1)
    hipLaunchKernelGGL(k_distinct<true>, dim3((unsigned)g), dim3(kBlock), 0, s, A, rpb);
  else
    hipLaunchKernelGGL(k_distinct<false>, dim3((unsigned)g), dim3(kBlock), 0, s, A, rpb);
  return hipGetLastError();
}

hipError_t launch_rows_fetch(const KCol& c, const int64_t* rows, int64_t n, uint32_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  int64_t g = (n * c.stride_w + kBlock - 1) / kBlock;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(k_rows_fetch, dim3((unsigned)g), dim3(kBlock), 0, s, c, rows, n, out);
  return hipGetLastError();
}

hipError_t launch_page_decode(const PageDecodeArgs& A, hipStream_t s) {
  if (A.npages <= 0) return hipSuccess;
  int64_t g = (A.npages + kWaves - 1) / kWaves;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(k_page_decode, dim3((unsigned)g), dim3(kBlock), 0, s, A);
  return hipGetLastError();
}

hipError_t launch_present_merge(const uint64_t* present0, const uint64_t* other, int32_t nother, int64_t nwords_each,
                                const uint64_t* md, int64_t md_words, int64_t nrows, uint64_t* del, int32_t* flags,
                                hipStream_t s) {
  const int64_t nwords = (nrows + 63) >> 6;
  if (nwords == 0) return hipSuccess;
  int64_t g = (nwords + kBlock - 1) / kBlock;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(k_present_merge, dim3((unsigned)g), dim3(kBlock), 0, s, present0, other, nother, nwords_each, md,
                     md_words, nrows, del, flags);
  return hipGetLastError();
}

// Column group (mbx_table_group): out[r * ncols + k] = cols[k][r].  One
// thread per row; loads coalesce per column, the row's stores are adjacent.
template <int N>
__global__ __launch_bounds__(kBlock) void k_group_build(const uint32_t* __restrict__ c0,
                                                        const uint32_t* __restrict__ c1,
                                                        const uint32_t* __restrict__ c2,
                                                        const uint32_t* __restrict__ c3, int64_t nrows,
                                                        uint32_t* __restrict__ out) {
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * kBlock) {
    uint32_t* o = out + r * N;
    o[0] = c0[r];
    o[1] = c1[r];
    if constexpr (N > 2) o[2] = c2[r];
    if constexpr (N > 3) o[3] = c3[r];
  }
}

hipError_t launch_group_build(const uint32_t* const* cols, int32_t ncols, int64_t nrows, uint32_t* out,
                              hipStream_t s) {
  if (nrows <= 0) return hipSuccess;
  const int64_t want = (nrows + kBlock - 1) / kBlock;
  const unsigned g = (unsigned)(want < 8192 ? want : 8192);
  const uint32_t* c2 = ncols > 2 ? cols[2] : nullptr;
  const uint32_t* c3 = ncols > 3 ? cols[3] : nullptr;
  if (ncols == 2)
    hipLaunchKernelGGL(k_group_build<2>, dim3(g), dim3(kBlock), 0, s, cols[0], cols[1], c2, c3, nrows, out);
  else if (ncols == 3)
    hipLaunchKernelGGL(k_group_build<3>, dim3(g), dim3(kBlock), 0, s, cols[0], cols[1], c2, c3, nrows, out);
  else
    hipLaunchKernelGGL(k_group_build<4>, dim3(g), dim3(kBlock), 0, s, cols[0], cols[1], c2, c3, nrows, out);
  return hipGetLastError();
}

}  // namespace mbx
