// Probe: does the page's memory type change what a sparse gather fetches?
//
// C4's late materialisation (k_cnf_select) reads 4-byte values at ~1 %
// selectivity from two 100M-row int32 columns: every value costs a whole
// 128-B L2 line from HBM (PMC: 221 MB of lines for 8 MB of values,
// DESIGN.md §5).  Load flavours (nt / sc0 / sc1) did not change the line
// size.  This probe times the same gather (ascending 1 % positions, two
// columns) and a streaming read of the same columns over three allocations:
//   coarse   hipMalloc
//   fine     hipExtMallocWithFlags(hipDeviceMallocFinegrained)
//   uncached hipExtMallocWithFlags(hipDeviceMallocUncached)
// and prints one JSON line per (memory type, kernel).  Results are checked.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/gather_mtype_probe tools/gather_mtype_probe.hip
//   tools/gather_mtype_probe [rows] [per_mille]
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

__global__ void k_iota(int32_t* a, int32_t* b, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    a[i] = (int32_t)i;
    b[i] = (int32_t)(i ^ 0x5a5a5a);
  }
}

__global__ void k_gather2(const int32_t* __restrict__ a, const int32_t* __restrict__ b,
                          const int32_t* __restrict__ pos, int32_t* __restrict__ oa,
                          int32_t* __restrict__ ob, int64_t m) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int32_t p = pos[i];
  oa[i] = a[p];
  ob[i] = b[p];
}

// streaming read of both columns, 16 B per lane, grid-stride
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k_stream2(const v4i* __restrict__ a, const v4i* __restrict__ b, int64_t n4,
                          int32_t* __restrict__ out) {
  int32_t x = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const v4i u = __builtin_nontemporal_load(a + i);
    const v4i v = __builtin_nontemporal_load(b + i);
    x ^= u.x ^ u.y ^ u.z ^ u.w ^ v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x7fffffff) out[blockIdx.x] = x;  // keeps the loads
}

static void* alloc(int kind, size_t bytes) {
  void* p = nullptr;
  if (kind == 0)
    CK(hipMalloc(&p, bytes));
  else
    CK(hipExtMallocWithFlags(&p, bytes, kind == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
  return p;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
  const int per_mille = argc > 2 ? atoi(argv[2]) : 10;
  const int reps = 20;
  // ascending positions, each row kept with probability per_mille / 1000
  std::vector<int32_t> pos;
  pos.reserve((size_t)(n * per_mille / 1000 * 11 / 10 + 16));
  std::mt19937_64 rng(42);
  std::uniform_int_distribution<int> d(0, 999);
  for (int64_t i = 0; i < n; ++i)
    if (d(rng) < per_mille) pos.push_back((int32_t)i);
  const int64_t m = (int64_t)pos.size();
  int32_t *dpos, *oa, *ob, *sink;
  CK(hipMalloc(&dpos, m * 4));
  CK(hipMalloc(&oa, m * 4));
  CK(hipMalloc(&ob, m * 4));
  CK(hipMalloc(&sink, 1 << 16));
  CK(hipMemcpy(dpos, pos.data(), m * 4, hipMemcpyHostToDevice));
  // distinct 128-B lines touched per column
  int64_t lines = 0, prev = -1;
  for (int32_t p : pos) {
    const int64_t l = (int64_t)p >> 5;
    if (l != prev) ++lines, prev = l;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[3] = {"coarse", "fine", "uncached"};
  for (int kind = 0; kind < 3; ++kind) {
    int32_t* a = (int32_t*)alloc(kind, n * 4);
    int32_t* b = (int32_t*)alloc(kind, n * 4);
    k_iota<<<4096, 256>>>(a, b, n);
    CK(hipDeviceSynchronize());
    const int gb = (int)((m + 255) / 256);
    for (int w = 0; w < 3; ++w) k_gather2<<<gb, 256>>>(a, b, dpos, oa, ob, m);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) k_gather2<<<gb, 256>>>(a, b, dpos, oa, ob, m);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms_g = 0;
    CK(hipEventElapsedTime(&ms_g, e0, e1));
    std::vector<int32_t> ha(m), hb(m);
    CK(hipMemcpy(ha.data(), oa, m * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), ob, m * 4, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < m; ++i) bad += (ha[i] != pos[i]) + (hb[i] != (pos[i] ^ 0x5a5a5a));
    const int64_t n4 = n / 4;
    for (int w = 0; w < 3; ++w) k_stream2<<<1024, 256>>>((const v4i*)a, (const v4i*)b, n4, sink);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) k_stream2<<<1024, 256>>>((const v4i*)a, (const v4i*)b, n4, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms_s = 0;
    CK(hipEventElapsedTime(&ms_s, e0, e1));
    const double us_g = ms_g * 1e3 / reps, us_s = ms_s * 1e3 / reps;
    printf("{\"mem\": \"%s\", \"kernel\": \"gather2\", \"rows\": %lld, \"selected\": %lld, \"lines_per_col\": %lld, "
           "\"us\": %.2f, \"line_gbs\": %.1f, \"value_gbs\": %.1f, \"bad\": %lld}\n",
           names[kind], (long long)n, (long long)m, (long long)lines, us_g, 2.0 * lines * 128 / (us_g * 1e3),
           2.0 * m * 4 / (us_g * 1e3), (long long)bad);
    printf("{\"mem\": \"%s\", \"kernel\": \"stream2\", \"bytes\": %lld, \"us\": %.2f, \"gbs\": %.1f}\n", names[kind],
           (long long)(8 * n4 * 4), us_s, 8.0 * n4 * 4 / (us_s * 1e3));
    fflush(stdout);
    CK(hipFree(a));
    CK(hipFree(b));
  }
  return 0;
}
