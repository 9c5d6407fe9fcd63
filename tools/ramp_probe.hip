// C3 read-pattern probe: is the streaming scan's end set by its slowest
// blocks, and does any block-to-work mapping end it sooner?
//
// The C3 scan (k_scan_fast, 1024 four-wave blocks, one contiguous segment of
// 256-row tiles each, U = 2 tiles in flight per wave, nontemporal dwordx4
// loads from two 400 MB int32 columns) ends when its LAST block ends.  This
// probe times the same loads (XOR-folded, one word per block stored; the XOR
// of every variant is checked against the first's) under several mappings:
//   static  G x W : G blocks of W waves, equal contiguous segments
//   xcd     G x W : static, block b (XCD b % 8) streams segment
//                   (b % 8) G / 8 + b / 8 (one contiguous eighth per XCD)
//   ramp    G x W : static segments shrinking linearly with blockIdx by a
//                   fraction f (early-dispatched blocks take more)
//   dyn     G x W : chunks of C tiles per wave from 8 per-XCD counters
//   hybrid  G x W : a static head (fraction h), the tail in chunks from 8
//                   per-XCD counters
//   Steal   G x W : hybrid whose blocks move on to the other XCDs' counters
//                   when their own is drained (at most 8 failing takes)
//   u / plain / wseg : static with U tiles in flight / plain loads / one
//                   contiguous sub-range per wave
// and records per-block start / end stamps (wall_clock64, 100 MHz) of one
// launch of each: the spread of end times by XCD and by eighth of blockIdx.
// Findings (profiles/r05/t, 4 boxes): on an idle GPU all 1024 blocks start
// within 0.5-1.5 us; block ends spread from ~103 to ~118 us, partly by
// blockIdx (later segments end later) and by XCD (which XCDs lag differs run
// to run).  Static contiguous segments are the fastest mapping: hybrid
// 0.9 / 4 tiles flattens the blockIdx spread but wins <= 1 % on slow boxes
// and loses 2-3 % on fast ones; Steal flattens the XCD spread too and is
// 8-30 % slower (stolen chunks and per-take atomics cost more bandwidth than
// the tail they recover); dyn is 4-22 % slower.  Load shapes (ramp5): U = 3
// / 4 tiles in flight within +-1 % of U = 2, plain loads 13 % slower than
// nontemporal, one contiguous sub-range per wave (4 streams per block) 2-5 %
// slower, 768 / 1280 / 1536 blocks 2-6 % slower.  Standalone:
// hipcc -O3 --offload-arch=gfx950 -o tools/ramp_probe tools/ramp_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                          \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

typedef int32_t v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4i gv4i;

constexpr int kTileRows = 256;
constexpr int kU = 2;

__device__ __forceinline__ v4i ld(const int32_t* p) { return __builtin_nontemporal_load((gv4i*)p); }

struct Args {
  const int32_t* c0;
  const int32_t* c1;
  int64_t ntiles;      // full tiles
  int64_t tpb;         // static: tiles per block
  int64_t chunk;       // dyn: tiles per wave per chunk
  int64_t nchunks;     // dyn
  float ramp;          // ramp: fraction; hybrid: static head fraction
  int64_t head_tiles;  // hybrid: tiles in the static head
  unsigned long long* ctr;  // dyn: 8 counters, 16 words apart
  uint32_t* sink;
  int64_t* stamps;     // 2 per block or null
};

// one wave's tiles t0 + wave + i * NW (i >= 0, t < t1), kU in flight
template <int NW>
__device__ __forceinline__ v4i wave_range(const Args& A, int64_t t0, int64_t t1, int wave, int lane, v4i acc) {
  for (int64_t base = t0 + wave; base < t1; base += NW * kU) {
    v4i q[kU][2];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      int64_t t = base + (int64_t)u * NW;
      const bool ok = t < t1;
      t = ok ? t : base;
      q[u][0] = ld(A.c0 + t * kTileRows + lane * 4);
      q[u][1] = ld(A.c1 + t * kTileRows + lane * 4);
      if (!ok) q[u][0] = q[u][1] = v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) acc ^= q[u][0] ^ q[u][1];
  }
  return acc;
}

template <int NW>
__device__ __forceinline__ void finish(const Args& A, v4i acc, int lane, int wave) {
  int32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  for (int off = 32; off > 0; off >>= 1) x ^= __shfl_xor(x, off);
  __shared__ int32_t red[NW];
  if (lane == 0) red[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t r = 0;
    for (int k = 0; k < NW; ++k) r ^= red[k];
    A.sink[blockIdx.x] = (uint32_t)r;
    if (A.stamps) A.stamps[2 * blockIdx.x + 1] = wall_clock64();
  }
}

// tiles first, first + stride, ... (< t1), U in flight; NT: nontemporal
template <int U, bool NT>
__device__ __forceinline__ v4i stream(const Args& A, int64_t first, int64_t t1, int64_t stride, int lane, v4i acc) {
  for (int64_t base = first; base < t1; base += stride * U) {
    v4i q[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t t = base + (int64_t)u * stride;
      const bool ok = t < t1;
      t = ok ? t : base;
      const int32_t* p0 = A.c0 + t * kTileRows + lane * 4;
      const int32_t* p1 = A.c1 + t * kTileRows + lane * 4;
      q[u][0] = NT ? ld(p0) : *(gv4i*)p0;
      q[u][1] = NT ? ld(p1) : *(gv4i*)p1;
      if (!ok) q[u][0] = q[u][1] = v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= q[u][0] ^ q[u][1];
  }
  return acc;
}

// static segments, U tiles in flight (kind "u"), plain loads (kind "p"), or
// one contiguous sub-range per wave (kind "w": 4 streams per block)
template <int NW, int U, bool NT, bool WSEG>
__global__ __launch_bounds__(64 * NW) void k_var(Args A) {
  if (A.stamps && threadIdx.x == 0) A.stamps[2 * blockIdx.x] = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * A.tpb;
  const int64_t t1 = min(t0 + A.tpb, A.ntiles);
  v4i acc;
  if (WSEG) {
    const int64_t per = (A.tpb + NW - 1) / NW;
    const int64_t w0 = min(t0 + wave * per, t1);
    acc = stream<U, NT>(A, w0, min(w0 + per, t1), 1, lane, v4i{0, 0, 0, 0});
  } else {
    acc = stream<U, NT>(A, t0 + wave, t1, NW, lane, v4i{0, 0, 0, 0});
  }
  finish<NW>(A, acc, lane, wave);
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_static(Args A) {
  if (A.stamps && threadIdx.x == 0) A.stamps[2 * blockIdx.x] = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * A.tpb;
  const int64_t t1 = min(t0 + A.tpb, A.ntiles);
  finish<NW>(A, wave_range<NW>(A, t0, t1, wave, lane, v4i{0, 0, 0, 0}), lane, wave);
}

// segment of block b: [start(b), start(b+1)), sizes proportional to
// 1 - ramp * b / G (integer tile boundaries from the closed form)
__device__ __forceinline__ int64_t ramp_start(int64_t b, int64_t G, float ramp, int64_t ntiles) {
  // cumulative weight W(b) = b - ramp * b (b - 1) / (2G), total W(G)
  const double w = (double)b - (double)ramp * (double)b * (double)(b - 1) / (2.0 * (double)G);
  const double W = (double)G - (double)ramp * (double)G * (double)(G - 1) / (2.0 * (double)G);
  int64_t s = (int64_t)((double)ntiles * w / W);
  return b >= G ? ntiles : min(s, ntiles);
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_ramp(Args A) {
  if (A.stamps && threadIdx.x == 0) A.stamps[2 * blockIdx.x] = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t t0 = ramp_start(blockIdx.x, gridDim.x, A.ramp, A.ntiles);
  const int64_t t1 = ramp_start(blockIdx.x + 1, gridDim.x, A.ramp, A.ntiles);
  finish<NW>(A, wave_range<NW>(A, t0, t1, wave, lane, v4i{0, 0, 0, 0}), lane, wave);
}

// static segments, XCD-major: block b (on XCD b % 8) streams segment
// (b % 8) * G / 8 + b / 8, so each XCD reads one contiguous eighth
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_xcd(Args A) {
  if (A.stamps && threadIdx.x == 0) A.stamps[2 * blockIdx.x] = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t seg = (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const int64_t t0 = seg * A.tpb;
  const int64_t t1 = min(t0 + A.tpb, A.ntiles);
  finish<NW>(A, wave_range<NW>(A, t0, t1, wave, lane, v4i{0, 0, 0, 0}), lane, wave);
}

// static head (tpb tiles per block over the first head_tiles), then chunks
// of the tail [head_tiles, ntiles) taken from 8 per-XCD counters
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_hybrid(Args A) {
  if (A.stamps && threadIdx.x == 0) A.stamps[2 * blockIdx.x] = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int x = blockIdx.x & 7;
  unsigned long long* ctr = A.ctr + 16 * x;
  __shared__ int64_t nxt[2];
  const int64_t h0 = (int64_t)blockIdx.x * A.tpb;
  const int64_t h1 = min(h0 + A.tpb, A.head_tiles);
  v4i acc = wave_range<NW>(A, h0, h1, wave, lane, v4i{0, 0, 0, 0});
  if (threadIdx.x == 0) nxt[0] = (int64_t)__hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 8 + x;
  __syncthreads();
  int64_t c = nxt[0];
  int par = 0;
  const int64_t per_chunk = A.chunk * NW;
  while (c < A.nchunks) {
    if (threadIdx.x == 0)
      nxt[par ^ 1] = (int64_t)__hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 8 + x;
    const int64_t t0 = A.head_tiles + c * per_chunk;
    const int64_t t1 = min(t0 + per_chunk, A.ntiles);
    acc = wave_range<NW>(A, t0, t1, wave, lane, acc);
    __syncthreads();
    par ^= 1;
    c = nxt[par];
  }
  finish<NW>(A, acc, lane, wave);
}

// hybrid with stealing: the tail's chunks are dealt to 8 counters (chunk
// 8k + x to counter x); a block drains its own XCD's counter, then the next
// ones whose bit in the exhausted mask (ctr[8 * 16]) is clear; a failing
// take sets its counter's bit.  ramp < 0 in the variant table: one global
// counter (no per-XCD split).
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_steal(Args A) {
  if (A.stamps && threadIdx.x == 0) A.stamps[2 * blockIdx.x] = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long* mask = A.ctr + 8 * 16;
  __shared__ int64_t nxt[2];
  __shared__ int cur_sh[2];
  const int64_t h0 = (int64_t)blockIdx.x * A.tpb;
  const int64_t h1 = min(h0 + A.tpb, A.head_tiles);
  v4i acc = wave_range<NW>(A, h0, h1, wave, lane, v4i{0, 0, 0, 0});
  // thread 0: the next chunk id (or -1: nothing left anywhere)
  // no shared mask: a failing take moves on to the next counter for good
  // (at most 8 failing takes per block, none on a counter with work left)
  auto take = [&](int& x, int& left) -> int64_t {
    while (left > 0) {
      const int64_t c =
          (int64_t)__hip_atomic_fetch_add(A.ctr + 16 * x, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 8 + x;
      if (c < A.nchunks) return c;
      x = (x + 1) & 7;
      --left;
    }
    return -1;
  };
  int x = blockIdx.x & 7, left = 8;
  if (threadIdx.x == 0) {
    nxt[0] = take(x, left);
    cur_sh[0] = x;
  }
  __syncthreads();
  int64_t c = nxt[0];
  int par = 0;
  const int64_t per_chunk = A.chunk * NW;
  while (c >= 0) {
    if (threadIdx.x == 0) nxt[par ^ 1] = take(x, left);
    const int64_t t0 = A.head_tiles + c * per_chunk;
    const int64_t t1 = min(t0 + per_chunk, A.ntiles);
    acc = wave_range<NW>(A, t0, t1, wave, lane, acc);
    __syncthreads();
    par ^= 1;
    c = nxt[par];
  }
  finish<NW>(A, acc, lane, wave);
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_dyn(Args A) {
  if (A.stamps && threadIdx.x == 0) A.stamps[2 * blockIdx.x] = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int x = blockIdx.x & 7;
  unsigned long long* ctr = A.ctr + 16 * x;
  __shared__ int64_t nxt[2];
  if (threadIdx.x == 0) nxt[0] = (int64_t)__hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 8 + x;
  __syncthreads();
  int64_t c = nxt[0];
  int par = 0;
  v4i acc = {0, 0, 0, 0};
  const int64_t per_chunk = A.chunk * NW;
  while (c < A.nchunks) {
    if (threadIdx.x == 0)
      nxt[par ^ 1] = (int64_t)__hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 8 + x;
    const int64_t t0 = c * per_chunk;
    const int64_t t1 = min(t0 + per_chunk, A.ntiles);
    acc = wave_range<NW>(A, t0, t1, wave, lane, acc);
    __syncthreads();
    par ^= 1;
    c = nxt[par];
  }
  finish<NW>(A, acc, lane, wave);
}

struct Variant {
  const char* kind;
  int G, NW;
  int64_t chunk;
  float ramp;
};

static void launch(const Variant& v, Args A, hipStream_t s) {
  dim3 g(v.G), b(64 * v.NW);
#define L3(K)                                                        \
  do {                                                               \
    if (v.NW == 4) hipLaunchKernelGGL(K<4>, g, b, 0, s, A);          \
    else if (v.NW == 8) hipLaunchKernelGGL(K<8>, g, b, 0, s, A);     \
    else hipLaunchKernelGGL(K<16>, g, b, 0, s, A);                   \
  } while (0)
  if (v.kind[0] == 's') L3(k_static);
  else if (v.kind[0] == 'r') L3(k_ramp);
  else if (v.kind[0] == 'x') L3(k_xcd);
  else if (v.kind[0] == 'h') L3(k_hybrid);
  else if (v.kind[0] == 'S') L3(k_steal);
  else if (v.kind[0] == 'u' && v.chunk == 3) hipLaunchKernelGGL((k_var<4, 3, true, false>), g, b, 0, s, A);
  else if (v.kind[0] == 'u' && v.chunk == 4) hipLaunchKernelGGL((k_var<4, 4, true, false>), g, b, 0, s, A);
  else if (v.kind[0] == 'u') hipLaunchKernelGGL((k_var<4, 2, true, false>), g, b, 0, s, A);
  else if (v.kind[0] == 'p') hipLaunchKernelGGL((k_var<4, 2, false, false>), g, b, 0, s, A);
  else if (v.kind[0] == 'w' && v.chunk == 4) hipLaunchKernelGGL((k_var<4, 4, true, true>), g, b, 0, s, A);
  else if (v.kind[0] == 'w') hipLaunchKernelGGL((k_var<4, 2, true, true>), g, b, 0, s, A);
  else L3(k_dyn);
  CHK(hipGetLastError());
}

__global__ void k_fill(int32_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (int32_t)((uint32_t)i * 2654435761u ^ seed);
}

int main(int argc, char** argv) {
  const int64_t nrows = argc > 1 ? atoll(argv[1]) : 100000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int64_t ntiles = nrows / kTileRows;
  int32_t *c0, *c1;
  CHK(hipMalloc(&c0, nrows * 4));
  CHK(hipMalloc(&c1, nrows * 4));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, c0, nrows, 1u);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, c1, nrows, 7u);
  uint32_t* sink;
  CHK(hipMalloc(&sink, 1 << 20));
  const int kMaxLaunch = 64;
  unsigned long long* ctr;
  CHK(hipMalloc(&ctr, kMaxLaunch * 256 * 8));
  int64_t* stamps;
  CHK(hipMalloc(&stamps, 2 * 65536 * 8));
  hipStream_t s;
  CHK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));

  // reference XOR of everything, from the static baseline
  std::vector<Variant> vs = {
      {"static", 1024, 4, 0, 0.f}, {"u", 1024, 4, 2, 0.f},    {"u", 1024, 4, 3, 0.f},   {"u", 1024, 4, 4, 0.f},
      {"plain", 1024, 4, 2, 0.f},  {"wseg", 1024, 4, 2, 0.f}, {"wseg", 1024, 4, 4, 0.f}, {"wseg", 512, 4, 2, 0.f},
      {"wseg", 2048, 4, 2, 0.f},   {"u", 768, 4, 2, 0.f},     {"u", 1280, 4, 2, 0.f},   {"u", 1536, 4, 2, 0.f},
      {"static", 1024, 4, 0, 0.f}, {"wseg", 1024, 4, 2, 0.f}, {"u", 1024, 4, 3, 0.f},
  };
  uint32_t want = 0;
  bool have_want = false;
  for (const Variant& v : vs) {
    Args A{c0, c1, ntiles, 0, v.chunk, 0, v.ramp, 0, ctr, sink, nullptr};
    A.tpb = (ntiles + v.G - 1) / v.G;
    if (v.kind[0] == 'd') A.nchunks = (ntiles + v.chunk * v.NW - 1) / (v.chunk * v.NW);
    if (v.kind[0] == 'h' || v.kind[0] == 'S') {
      A.head_tiles = (int64_t)((double)ntiles * v.ramp) / v.G * v.G;
      A.tpb = A.head_tiles / v.G;
      A.nchunks = (ntiles - A.head_tiles + v.chunk * v.NW - 1) / (v.chunk * v.NW);
    }
    // check: XOR over the blocks' words equals the static baseline's
    CHK(hipMemset(ctr, 0, kMaxLaunch * 256 * 8));
    CHK(hipMemset(sink, 0, 1 << 20));
    launch(v, A, s);
    CHK(hipStreamSynchronize(s));
    std::vector<uint32_t> hs(v.G);
    CHK(hipMemcpy(hs.data(), sink, v.G * 4, hipMemcpyDeviceToHost));
    uint32_t x = 0;
    for (uint32_t w : hs) x ^= w;
    if (!have_want) {
      want = x;
      have_want = true;
    }
    // timed: reps launches, each with its own zeroed counters
    float best = 1e30f, sum = 0.f;
    const int rounds = 3;
    for (int r = 0; r < rounds; ++r) {
      CHK(hipMemsetAsync(ctr, 0, kMaxLaunch * 256 * 8, s));
      CHK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) {
        Args B = A;
        B.ctr = ctr + (i % kMaxLaunch) * 256;
        launch(v, B, s);
      }
      CHK(hipEventRecord(e1, s));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms / reps);
      sum += ms / reps;
    }
    // one stamped launch
    CHK(hipMemsetAsync(ctr, 0, 256 * 8, s));
    Args S = A;
    S.stamps = stamps;
    launch(v, S, s);
    CHK(hipStreamSynchronize(s));
    std::vector<int64_t> st(2 * v.G);
    CHK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
    int64_t t0 = INT64_MAX, smax = 0, emin = INT64_MAX, emax = 0;
    for (int b = 0; b < v.G; ++b) t0 = std::min(t0, st[2 * b]);
    std::vector<double> ends;
    for (int b = 0; b < v.G; ++b) {
      smax = std::max(smax, st[2 * b] - t0);
      emin = std::min(emin, st[2 * b + 1] - t0);
      emax = std::max(emax, st[2 * b + 1] - t0);
      ends.push_back((st[2 * b + 1] - t0) * 0.01);
    }
    double xe[8] = {0}, xn[8] = {0}, de[8] = {0}, dn[8] = {0};
    for (int b = 0; b < v.G; ++b) {
      xe[b & 7] += ends[b];
      xn[b & 7] += 1;
      de[b * 8 / v.G] += ends[b];
      dn[b * 8 / v.G] += 1;
    }
    char xs[256], ds[256];
    int o1 = 0, o2 = 0;
    for (int k = 0; k < 8; ++k) {
      o1 += snprintf(xs + o1, sizeof(xs) - o1, "%s%.1f", k ? ", " : "", xe[k] / xn[k]);
      o2 += snprintf(ds + o2, sizeof(ds) - o2, "%s%.1f", k ? ", " : "", de[k] / dn[k]);
    }
    std::sort(ends.begin(), ends.end());
    const double bytes = 2.0 * 4.0 * (double)ntiles * kTileRows;
    printf("{\"kind\": \"%s\", \"blocks\": %d, \"waves\": %d, \"chunk\": %lld, \"ramp\": %.3f, \"ok\": %s, "
           "\"us_best\": %.2f, \"us_avg\": %.2f, \"gbs_best\": %.1f, \"last_start_us\": %.2f, "
           "\"first_end_us\": %.2f, \"end_p50_us\": %.2f, \"end_p99_us\": %.2f, \"last_end_us\": %.2f, "
           "\"end_by_xcd\": [%s], \"end_by_eighth\": [%s]}\n",
           v.kind, v.G, v.NW, (long long)v.chunk, v.ramp, x == want ? "true" : "false", best * 1e3,
           sum / rounds * 1e3, bytes / (best * 1e-3) / 1e9, smax * 0.01, emin * 0.01, ends[ends.size() / 2],
           ends[ends.size() * 99 / 100], emax * 0.01, xs, ds);
    fflush(stdout);
  }
  return 0;
}
