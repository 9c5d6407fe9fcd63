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
//
// Byte/integer work, HBM bound: per page 1 KiB read + the decoded records
// written; no MFMA, no LDS.
#include "mbx_internal.hpp"

namespace mbx {

__device__ __forceinline__ uint32_t ld_be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | (uint32_t)p[1]; }

__global__ __launch_bounds__(kBlock) void k_page_decode(PageDecodeArgs A) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * kWaves;
  for (int64_t pi = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); pi < A.npages; pi += nwaves) {
    const int32_t pid = A.page_of[pi];
    if (pid < 0) continue;
    if ((int64_t)pid >= A.image_pages) {
      if (lane == 0) atomicOr(A.err, 1);
      continue;
    }
    const uint8_t* pg = A.image + (int64_t)pid * kDbPage;
    int32_t slots = (int32_t)(int16_t)ld_be16(pg);
    if (slots > A.recs_per_page || slots < 0) {
      if (lane == 0) atomicOr(A.err, 2);
      slots = slots < 0 ? 0 : A.recs_per_page;
    }
    for (int32_t k = lane; k < slots; k += 64) {
      const uint8_t* sp = pg + kDbSlotBase + 4 * k;
      const int32_t len = (int32_t)(int16_t)ld_be16(sp);
      const int32_t off = (int32_t)ld_be16(sp + 2);
      if (len == -1) continue;  // EMPTY_SLOT
      if (len != A.rec_len || off < kDbSlotBase || off + len > kDbPage) {
        atomicOr(A.err, 4);
        continue;
      }
      const int64_t pos = pi * A.recs_per_page + k;
      if (pos >= A.nrows) {
        atomicOr(A.err, 8);
        continue;
      }
      const uint8_t* rec = pg + off;
      if (A.kind != kStr) {
        const uint32_t v = ((uint32_t)rec[0] << 24) | ((uint32_t)rec[1] << 16) | ((uint32_t)rec[2] << 8) | rec[3];
        reinterpret_cast<uint32_t*>(A.out)[pos] = v;
      } else {
        // writeUTF image: u16 length + modified UTF-8; device image rewrites
        // C0 80 (U+0000) as 00 01 and zero-pads to the stride
        int32_t L = (int32_t)ld_be16(rec);
        if (L > A.size) {
          atomicOr(A.err, 16);
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
      atomicOr(reinterpret_cast<unsigned long long*>(A.present) + (pos >> 6), 1ull << (pos & 63));
    }
  }
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

}  // namespace mbx
