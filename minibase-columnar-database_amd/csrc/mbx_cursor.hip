// mbx_cursor.hip -- the delivery side of Iterator.get_next()
// (R/iterator/Iterator.java:12-141; the caller's loop, R/input/Query.java:137-152).
//
//   k_cursor_pack   rows [from, from + n) of a cursor's device results --
//                   positions and every projected column -- packed into ONE
//                   contiguous staging region in the caller's host layout
//                   (int64 positions, 4-byte values, char(n) as n bytes of
//                   zero-padded modified UTF-8: the device string encoding's
//                   00 01 turned back into C0 80, Convert.java:254-275), so a
//                   batch crosses PCIe as a single device -> pinned copy and
//                   needs no host-side unpack.
//
// Byte work of a batch (n x (8 + sum widths) bytes read and written); it is
// launch-latency bound at the batch sizes the drop-ins use (64 Ki rows).
#include "mbx_internal.hpp"

namespace mbx {

__global__ __launch_bounds__(256) void k_cursor_pack(const int64_t* __restrict__ ids, int64_t from, int64_t n,
                                                     CursorPack P, uint8_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = from + i;
  reinterpret_cast<int64_t*>(dst)[i] = ids[r];
  for (int32_t j = 0; j < P.ncols; j++) {
    const CursorPackCol& c = P.col[j];
    const uint8_t* s = c.src + r * c.src_stride;
    uint8_t* d = dst + c.dst_off + i * c.width;
    if (!c.is_string) {
      *reinterpret_cast<uint32_t*>(d) = *reinterpret_cast<const uint32_t*>(s);
      continue;
    }
    // mbx::decode_device_string, per row: stop at the padding, 00 01 -> C0 80
    int32_t k = 0;
    bool end = false;
    while (k < c.width) {
      const uint8_t b = k < c.src_stride && !end ? s[k] : 0;
      if (b == 0 && !end) {
        if (k + 1 < c.src_stride && k + 1 < c.width && s[k + 1] == 0x01) {
          d[k] = 0xC0;
          d[k + 1] = 0x80;
          k += 2;
          continue;
        }
        end = true;
      }
      d[k++] = end ? 0 : b;
    }
  }
}

hipError_t launch_cursor_pack(const int64_t* ids, int64_t from, int64_t n, const CursorPack& P, uint8_t* dst,
                              hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_cursor_pack, dim3((unsigned)blocks), dim3(256), 0, s, ids, from, n, P, dst);
  return hipGetLastError();
}

}  // namespace mbx
