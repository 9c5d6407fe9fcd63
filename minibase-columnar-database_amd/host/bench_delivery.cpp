// bench_delivery.cpp -- rows handed to the CALLER through the C++ drop-ins'
// get_next() (Iterator.get_next, R/iterator/Iterator.java:12-141; the
// Query driver's loop, R/input/Query.java:137-152), next to the time the
// device needs for the same query.  Every headline elsewhere stops in HBM;
// this one ends in the caller's Jtuple.
//
//   C2  ColumnarFileScan over a 10M-row 4 x int32 Columnarfile, c0 < 104858
//       (~1M rows), all 4 columns projected
//   C4  ColumnarIndexScan over a 100M-row file, bm(c2 = 3) AND bm(c3 = 7)
//       (~1M rows) from BitMapFiles, c0 and c1 projected (one k_cnf_select
//       launch into the cursor)
//
// Both tables are written as Minibase DB files (include/mbx_db.h) and
// staged by the GPU page decoder, as the CLI does.  Per query and per cursor
// mode (double-buffered delivery on / off: knob cursor_prefetch) it prints
// one JSON line: constructor time (predicate / CNF kernels + materialise),
// delivery loop time, rows/s handed out, ns per row, and the split of the
// loop between the cursor's batch copies (mbx_cursor_next) and the
// row-by-row Jtuple fill.
//
//   bench_delivery DIR [c2_rows] [c4_rows] [reps]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "minibase.hpp"

using namespace minibase;
using global::AttrOperator;
using global::AttrType;
using global::IndexType;
using iterator::CondExpr;
using iterator::FldSpec;
using iterator::RelSpec;

namespace {

double now_ms() {
  using C = std::chrono::steady_clock;
  return std::chrono::duration<double, std::milli>(C::now().time_since_epoch()).count();
}

// the columns of bench_configs.py's shapes, from a fixed 64-bit LCG
std::vector<int32_t> column(int64_t n, int32_t hi, uint64_t seed) {
  std::vector<int32_t> v((size_t)n);
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  for (int64_t i = 0; i < n; i++) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    v[(size_t)i] = (int32_t)((x >> 33) % (uint64_t)hi);
  }
  return v;
}

columnar::Columnarfile make_file(mbx_db* db, const std::string& name, int64_t n, int32_t hi23) {
  std::vector<std::string> names{"c0", "c1", "c2", "c3"};
  std::vector<AttrType> types(4, AttrType(AttrType::attrInteger));
  std::vector<short> sizes(4, 4);
  columnar::Columnarfile cf(db, name, 4, names, types, sizes);
  std::vector<std::vector<int32_t>> ints{column(n, 1 << 20, 42), column(n, 1 << 20, 43), column(n, hi23, 44),
                                         column(n, hi23, 45)};
  cf.insertColumns(ints, {}, {}, n);
  return cf;
}

struct Loop {
  int64_t rows = 0;
  double ms = 0;
  int64_t checksum = 0;
};

template <class It>
Loop drain(It& it) {
  Loop r;
  const double t0 = now_ms();
  heap::Tuple* t;
  while ((t = it.get_next()) != nullptr) {
    r.checksum += t->getIntFld(1);
    r.rows++;
  }
  r.ms = now_ms() - t0;
  return r;
}

struct Batches {
  int64_t rows;
  double ms;
  int64_t bytes;
};

void emit(const char* cfg, const char* mode, int64_t nrows, double ctor_ms, const Loop& l,
          const std::vector<Batches>& bo) {
  printf("{\"config\": \"%s\", \"cursor\": \"%s\", \"table_rows\": %lld, \"rows_delivered\": %lld, "
         "\"ctor_ms\": %.3f, \"get_next_loop_ms\": %.3f, \"delivered_rows_per_s\": %.4g, \"ns_per_row\": %.2f, "
         "\"checksum\": %lld, \"cursor_batches_only\": [",
         cfg, mode, (long long)nrows, (long long)l.rows, ctor_ms, l.ms, l.rows / (l.ms * 1e-3),
         l.ms * 1e6 / (double)(l.rows > 0 ? l.rows : 1), (long long)l.checksum);
  for (size_t i = 0; i < bo.size(); i++)
    printf("%s{\"batch_rows\": %lld, \"ms\": %.3f, \"d2h_bytes\": %lld, \"gbs\": %.2f}", i ? ", " : "",
           (long long)bo[i].rows, bo[i].ms, (long long)bo[i].bytes, bo[i].bytes / (bo[i].ms * 1e-3) / 1e9);
  printf("]}\n");
  fflush(stdout);
}

// the cursor's batches alone (mbx_cursor_next_view, rows left in the pinned
// buffer, no Jtuple fill): the part of the loop that is device -> host
// delivery, at a few batch sizes; bytes = what crossed PCIe
std::vector<Batches> batches_only(mbx_cursor* c) {
  std::vector<Batches> out;
  const void* cols[16];
  for (int64_t rows : {8192, 65536, 65536, 262144, 262144}) {  // the first pass at a new size allocates
    const int64_t* ids = nullptr;
    int64_t n = 0, b0 = 0, b1 = 0, d = 0;
    mbx_cursor_restart(c);
    mbx_cursor_stats(c, &d, &b0);
    const double t0 = now_ms();
    do {
      if (mbx_cursor_next_view(c, rows, &ids, cols, &n) < 0) {
        fprintf(stderr, "cursor_next_view: %s\n", mbx_last_error());
        exit(1);
      }
    } while (n > 0);
    const double ms = now_ms() - t0;
    mbx_cursor_stats(c, &d, &b1);
    out.push_back({rows, ms, b1 - b0});
  }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: bench_delivery DIR [c2_rows] [c4_rows] [reps]\n");
    return 2;
  }
  const std::string dir = argv[1];
  const int64_t n2 = argc > 2 ? atoll(argv[2]) : 10000000;
  const int64_t n4 = argc > 3 ? atoll(argv[3]) : 100000000;
  const int reps = argc > 4 ? atoi(argv[4]) : 3;
  try {
    // pages: 4 columns x n / 125 data pages + directories + 20 BitMapFiles
    const int64_t pages = (n2 + n4) * 4 / 120 + 20 * (n4 / 8000 + 2) + (1 << 16);
    mbx_db* db = global::SystemDefs::open(dir + "/db", (int)pages);
    mbx_ctx* ctx = global::SystemDefs::ctx();
    double t0 = now_ms();
    columnar::Columnarfile f2 = make_file(db, "c2", n2, 1 << 20);
    columnar::Columnarfile f4 = make_file(db, "c4", n4, 10);
    fprintf(stderr, "files written: %.0f ms\n", now_ms() - t0);
    t0 = now_ms();
    f4.createBitMapIndex(2);
    f4.createBitMapIndex(3);
    fprintf(stderr, "bitmap indexes built + persisted: %.0f ms\n", now_ms() - t0);

    const std::vector<AttrType> types(4, AttrType(AttrType::attrInteger));
    for (int prefetch = 1; prefetch >= 0; prefetch--) {
      mbx_set_tuning(ctx, "cursor_prefetch", prefetch);
      const char* mode = prefetch ? "double-buffered" : "on-demand";
      for (int r = 0; r < reps; r++) {
        // C2: query db c2 [c0,c1,c2,c3] {c0,<,104858} FILESCAN
        CondExpr e;
        e.op = AttrOperator(AttrOperator::aopLT);
        e.type1 = AttrType(AttrType::attrSymbol);
        e.type2 = AttrType(AttrType::attrInteger);
        e.operand1.symbol = FldSpec(RelSpec(RelSpec::outer), 1);
        e.operand2.integer = 104858;
        CondExpr* filt[2] = {&e, nullptr};
        std::vector<FldSpec> proj;
        for (int c = 0; c < 4; c++) proj.emplace_back(RelSpec(RelSpec::outer), c + 1);
        double c0 = now_ms();
        iterator::ColumnarFileScan fs("c2", types, {}, 4, 4, proj, filt);
        const double ctor2 = now_ms() - c0;
        Loop l2 = drain(fs);
        mbx_cursor* c2cur = nullptr;
        int32_t pc4[4] = {0, 1, 2, 3};
        if (mbx_cursor_open(ctx, f2.table(), fs.selection()->get(), pc4, 4, &c2cur) < 0) {
          fprintf(stderr, "cursor_open: %s\n", mbx_last_error());
          return 1;
        }
        const auto bo2 = batches_only(c2cur);
        mbx_cursor_close(c2cur);
        fs.close();
        emit("C2", mode, n2, ctor2, l2, bo2);

        // C4: indexes_query db c4 [c0,c1] {(c2,=,3,BM)}^{(c3,=,7,BM)}
        CondExpr a, b;
        for (CondExpr* x : {&a, &b}) {
          x->op = AttrOperator(AttrOperator::aopEQ);
          x->type1 = AttrType(AttrType::attrSymbol);
          x->type2 = AttrType(AttrType::attrInteger);
          x->indexType = IndexType(IndexType::Bitmap);
        }
        a.operand1.symbol = FldSpec(RelSpec(RelSpec::outer), 3);
        a.operand2.integer = 3;
        b.operand1.symbol = FldSpec(RelSpec(RelSpec::outer), 4);
        b.operand2.integer = 7;
        CondExpr* sel[3] = {&a, &b, nullptr};
        std::vector<FldSpec> proj4{FldSpec(RelSpec(RelSpec::outer), 1), FldSpec(RelSpec(RelSpec::outer), 2)};
        c0 = now_ms();
        index::ColumnarIndexScan is(&f4, {}, {IndexType(IndexType::Bitmap), IndexType(IndexType::Bitmap)},
                                    {"", ""}, types, {}, 4, 2, {0, 1}, proj4, sel, false);
        heap::Tuple* first = is.get_next();  // the one-launch CNF cursor opens at the first get_next
        const double ctor4 = now_ms() - c0;
        Loop l4 = drain(is);
        if (first) {
          l4.rows++;
          l4.checksum += first->getIntFld(1);
        }
        // the same cursor's batches alone
        std::vector<mbx_bitmap*> bms;
        auto v3 = index::ColumnIndexScan::valueBitmaps(f4, 2, a);
        auto v7 = index::ColumnIndexScan::valueBitmaps(f4, 3, b);
        bms.push_back(v3.at(0)->get());
        bms.push_back(v7.at(0)->get());
        int32_t offs[3] = {0, 1, 2}, pc[2] = {0, 1};
        mbx_cursor* cur = nullptr;
        if (mbx_cnf_cursor_open(ctx, f4.table(), bms.data(), offs, 2, nullptr, pc, 2, &cur) < 0) {
          fprintf(stderr, "cnf_cursor_open: %s\n", mbx_last_error());
          return 1;
        }
        const auto bo = batches_only(cur);
        mbx_cursor_close(cur);
        is.close();
        emit("C4", mode, n4, ctor4, l4, bo);
      }
    }
    global::SystemDefs::shutdown();
  } catch (const std::exception& e) {
    fprintf(stderr, "bench_delivery: %s\n", e.what());
    return 1;
  }
  return 0;
}
