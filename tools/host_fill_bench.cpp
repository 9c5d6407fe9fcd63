// host_fill_bench.cpp -- the host half of get_next() delivery with no GPU:
// a Jtuple filled row by row from a batch of 4 int columns (the C2 shape), as
// CursorBatches::fill does, timed per row.  Separates the Jtuple / loop cost
// from the PCIe copies bench_delivery measures.
//   g++ -O2 -std=c++17 -I.. tools/host_fill_bench.cpp minibase-columnar-database_amd/host/minibase.o
//       -Lminibase-columnar-database_amd -lmbx -o /tmp/host_fill_bench
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../minibase-columnar-database_amd/host/minibase.hpp"

using namespace minibase;

int main() {
  const int64_t n = 1 << 20, ncols = 4;
  std::vector<std::vector<int32_t>> cols(ncols, std::vector<int32_t>(n));
  for (int c = 0; c < ncols; c++)
    for (int64_t i = 0; i < n; i++) cols[c][i] = (int32_t)(i * 7 + c);
  heap::Tuple J;
  J.setHdr(std::vector<global::AttrType>(ncols, global::AttrType(global::AttrType::attrInteger)), {});
  for (int rep = 0; rep < 5; rep++) {
    int64_t sum = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int64_t i = 0; i < n; i++) {
      for (int c = 0; c < ncols; c++) {
        int32_t v;
        memcpy(&v, cols[c].data() + i, 4);
        J.setIntFld(c + 1, v);
      }
      sum += J.getIntFld(1);
    }
    const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"form\": \"setIntFld\", \"rows\": %lld, \"ns_per_row\": %.2f, \"checksum\": %lld}\n", (long long)n,
           ns / n, (long long)sum);
  }
  const int32_t* cp[ncols];
  for (int c = 0; c < ncols; c++) cp[c] = cols[c].data();
  for (int rep = 0; rep < 5; rep++) {
    int64_t sum = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int64_t i = 0; i < n; i++) {
      J.setIntFlds(cp, i, ncols);
      sum += J.getIntFld(1);
    }
    const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"form\": \"setIntFlds\", \"rows\": %lld, \"ns_per_row\": %.2f, \"checksum\": %lld}\n", (long long)n,
           ns / n, (long long)sum);
  }
  return 0;
}
