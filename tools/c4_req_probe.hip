// C4 traffic calibration: which read-request sizes does
// the L2 send to memory for C4's access pattern, and what does each counter
// mean in bytes on gfx950?
//
// Kernels with KNOWN byte footprints, each launched `reps` times so a
// rocprofv3 --pmc pass gets per-dispatch request counts to compare with:
//   k_stream   two 400 MB int32 columns, 16 B per lane, non-temporal (C3's
//              load shape): exactly 800 MB of 128-B lines
//   k_words    two 12.5 MB BitSets streamed with 8 B per lane (C4's operand
//              words, 100 M bits each): 25 MB
//   k_pair     ~1 % ascending positions of 100 M rows, one 8-byte load per
//              row from a (c0, c1) column group (C4's grouped gather)
//   k_col2     the same positions, one 4-byte load per row from each of two
//              column-major int32 columns (C4 without the group)
// For the gathers the host counts the distinct 32-B, 64-B and 128-B aligned
// pieces the loads touch, so each counter can be matched to a granularity.
// One JSON line per kernel: footprint, launch time.  Results are checked.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/c4_req_probe tools/c4_req_probe.hip
//   tools/c4_req_probe [rows] [per_mille] [reps]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_fill(int32_t* a, int32_t* b, int32_t* g, uint64_t* w0, uint64_t* w1, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    a[i] = (int32_t)i;
    b[i] = (int32_t)(i ^ 0x5a5a5a);
    g[2 * i] = (int32_t)i;
    g[2 * i + 1] = (int32_t)(i ^ 0x5a5a5a);
    if (i < (n + 63) / 64) {
      w0[i] = 0x9e3779b97f4a7c15ull * (uint64_t)(i + 1);
      w1[i] = 0xc2b2ae3d27d4eb4full * (uint64_t)(i + 7);
    }
  }
}

__global__ void k_stream(const v4i* __restrict__ a, const v4i* __restrict__ b, int64_t n4, int32_t* __restrict__ sink) {
  int32_t x = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const v4i u = __builtin_nontemporal_load(a + i);
    const v4i v = __builtin_nontemporal_load(b + i);
    x ^= u.x ^ u.y ^ u.z ^ u.w ^ v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x7fffffff) sink[blockIdx.x] = x;  // keeps the loads
}

__global__ void k_words(const uint64_t* __restrict__ w0, const uint64_t* __restrict__ w1, int64_t nw,
                        uint64_t* __restrict__ sink) {
  uint64_t x = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nw; i += stride) x += __popcll(w0[i] & w1[i]);
  if (x == 0x7fffffffffffull) sink[blockIdx.x] = x;
}

__global__ void k_pair(const uint2* __restrict__ g, const int32_t* __restrict__ pos, int32_t* __restrict__ oa,
                       int32_t* __restrict__ ob, int64_t m) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint2 v = g[pos[i]];
  oa[i] = (int32_t)v.x;
  ob[i] = (int32_t)v.y;
}

__global__ void k_col2(const int32_t* __restrict__ a, const int32_t* __restrict__ b, const int32_t* __restrict__ pos,
                       int32_t* __restrict__ oa, int32_t* __restrict__ ob, int64_t m) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int32_t p = pos[i];
  oa[i] = a[p];
  ob[i] = b[p];
}

// distinct aligned pieces of `piece` bytes touched by loads of `width` bytes at
// base + pos * stride (ascending positions)
static int64_t pieces(const std::vector<int32_t>& pos, int64_t stride, int64_t width, int64_t piece) {
  int64_t n = 0, prev = -1;
  for (int32_t p : pos) {
    const int64_t lo = (int64_t)p * stride / piece, hi = ((int64_t)p * stride + width - 1) / piece;
    for (int64_t q = lo; q <= hi; ++q)
      if (q != prev) ++n, prev = q;
  }
  return n;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
  const int per_mille = argc > 2 ? atoi(argv[2]) : 10;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  std::vector<int32_t> pos;
  pos.reserve((size_t)(n * per_mille / 1000 * 11 / 10 + 16));
  std::mt19937_64 rng(42);
  std::uniform_int_distribution<int> d(0, 999);
  for (int64_t i = 0; i < n; ++i)
    if (d(rng) < per_mille) pos.push_back((int32_t)i);
  const int64_t m = (int64_t)pos.size(), nw = (n + 63) / 64;
  int32_t *a, *b, *g, *dpos, *oa, *ob, *sink;
  uint64_t *w0, *w1;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMalloc(&g, n * 8));
  CK(hipMalloc(&w0, nw * 8));
  CK(hipMalloc(&w1, nw * 8));
  CK(hipMalloc(&dpos, m * 4));
  CK(hipMalloc(&oa, m * 4));
  CK(hipMalloc(&ob, m * 4));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemcpy(dpos, pos.data(), m * 4, hipMemcpyHostToDevice));
  k_fill<<<4096, 256>>>(a, b, g, w0, w1, n);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int gb = (int)((m + 255) / 256);
  auto timed = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
  };
  const double us_s = timed("stream", [&] { k_stream<<<1024, 256>>>((const v4i*)a, (const v4i*)b, n / 4, sink); });
  printf("{\"kernel\": \"k_stream\", \"bytes\": %lld, \"us\": %.2f, \"launches\": %d}\n", (long long)(8 * (n / 4) * 4),
         us_s, reps + 1);
  const double us_w = timed("words", [&] { k_words<<<1024, 256>>>(w0, w1, nw, (uint64_t*)sink); });
  printf("{\"kernel\": \"k_words\", \"bytes\": %lld, \"us\": %.2f, \"launches\": %d}\n", (long long)(16 * nw), us_w,
         reps + 1);
  const double us_p = timed("pair", [&] { k_pair<<<gb, 256>>>((const uint2*)g, dpos, oa, ob, m); });
  std::vector<int32_t> ha(m), hb(m);
  CK(hipMemcpy(ha.data(), oa, m * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), ob, m * 4, hipMemcpyDeviceToHost));
  int64_t bad = 0;
  for (int64_t i = 0; i < m; ++i) bad += (ha[i] != pos[i]) + (hb[i] != (pos[i] ^ 0x5a5a5a));
  printf("{\"kernel\": \"k_pair\", \"rows\": %lld, \"selected\": %lld, \"value_bytes\": %lld, \"pos_bytes\": %lld, "
         "\"out_bytes\": %lld, \"sectors32\": %lld, \"sectors64\": %lld, \"lines128\": %lld, \"us\": %.2f, "
         "\"launches\": %d, \"bad\": %lld}\n",
         (long long)n, (long long)m, (long long)(8 * m), (long long)(4 * m), (long long)(8 * m),
         (long long)pieces(pos, 8, 8, 32), (long long)pieces(pos, 8, 8, 64), (long long)pieces(pos, 8, 8, 128), us_p,
         reps + 1, (long long)bad);
  const double us_c = timed("col2", [&] { k_col2<<<gb, 256>>>(a, b, dpos, oa, ob, m); });
  CK(hipMemcpy(ha.data(), oa, m * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), ob, m * 4, hipMemcpyDeviceToHost));
  bad = 0;
  for (int64_t i = 0; i < m; ++i) bad += (ha[i] != pos[i]) + (hb[i] != (pos[i] ^ 0x5a5a5a));
  printf("{\"kernel\": \"k_col2\", \"rows\": %lld, \"selected\": %lld, \"value_bytes\": %lld, \"pos_bytes\": %lld, "
         "\"out_bytes\": %lld, \"sectors32\": %lld, \"sectors64\": %lld, \"lines128\": %lld, \"us\": %.2f, "
         "\"launches\": %d, \"bad\": %lld}\n",
         (long long)n, (long long)m, (long long)(8 * m), (long long)(4 * m), (long long)(8 * m),
         2 * (long long)pieces(pos, 4, 4, 32), 2 * (long long)pieces(pos, 4, 4, 64),
         2 * (long long)pieces(pos, 4, 4, 128), us_c, reps + 1, (long long)bad);
  fflush(stdout);
  return bad ? 1 : 0;
}
