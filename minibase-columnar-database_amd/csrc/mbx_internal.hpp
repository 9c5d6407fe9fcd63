// mbx_internal.hpp -- device-side plan layout and kernel launchers shared by
// the C-ABI layer (mbx_api.cpp) and the CDNA4 kernels (mbx_kernels.hip).
//
// HBM layout (DESIGN.md "Data layout"):
//   * int32 / float32 column: nrows contiguous 4-byte values, position order.
//   * char(n) column: nrows rows of `stride` bytes (n rounded up to 4), the
//     modified-UTF-8 payload with C0 80 (U+0000) rewritten to 00 01 and zero
//     padding, so that an unsigned big-endian word compare of two rows equals
//     the sign of Java String.compareTo (TupleUtils.java:79-82).
//   * bitmaps: java.util.BitSet words (bit p%64 of uint64 word p/64).
// Work decomposition: a "tile" is 256 rows = 4 bitmap words = one wave of 64
// lanes x 4 consecutive rows (one 16-byte load per lane per 4-byte column).
// A block (4 waves) owns a contiguous "segment" of tiles; per-segment counts
// feed the compaction scan, so every producer of a bitmap also reports them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mbx {

constexpr int64_t kResidentBlocks = 1024;  // 256-thread blocks the chip holds at once (4 per CU)
constexpr int kHoistTerms = 4;        // literal terms the fast scan hoists into registers
constexpr int kTileRows = 256;       // rows per wave tile
constexpr int kWordsPerTile = 4;     // bitmap words per tile
constexpr int kBlock = 256;          // threads per block (4 waves)
constexpr int kWaves = kBlock / 64;
constexpr int kMaxTerms = 32;
constexpr int kMaxCols = 8;
constexpr int kMaxStrWords = 64;     // 256-byte strings
constexpr int kMaxPoolWords = 512;
constexpr int kMaxBitmaps = 64;      // bitmaps in one CNF launch
constexpr int kMaxProj = 16;
// select_dbg kernel bits that exist only for A/B measurements: skip the
// prefix loads / the look-back wait (wrong output by design), skip the
// emission (64), the staging (16), the BitSet words (256), everything after
// the count (128), nontemporal positions stores (512), the back-off and
// plain-load poll forms.  A production build
// compiles them out (the kernels mask dbg with kDiagDbg); -DMBX_DIAG keeps
// them.  Stamps, the write-through flip and the every-predecessor look-back
// (tables of >= 2^32 rows take it) stay in every build.
#ifdef MBX_DIAG
constexpr int32_t kDiagDbg = ~0;
#else
constexpr int32_t kDiagDbg = ~(1 | 2 | 4 | 16 | 64 | 128 | 256 | 512);
#endif

enum ColKind : int32_t { kInt = 0, kReal = 1, kStr = 2 };

// normalized comparison: the kernel evaluates `lhs_col OP rhs` where rhs is a
// literal or another column; literal-on-left terms are flipped on the host.
// kNever: aopNOP / opRANGE, never true (PredEval.java:137-162 has no case for
// them) -- kept as a term only where reaching it can raise (a float compare).
enum CmpOp : int32_t { kLT = 0, kLE = 1, kGT = 2, kGE = 3, kEQ = 4, kNE = 5, kNever = 6 };

struct KCol {
  const void* base;
  int32_t kind;      // ColKind
  int32_t stride_w;  // 32-bit words per row (1 for int/real)
};

struct KTerm {
  int32_t kind;      // comparison type (ColKind)
  int32_t op;        // CmpOp
  int32_t lhs;       // column slot
  int32_t rhs;       // column slot, or -1 for a literal
  uint32_t conj_bit; // 1u << conjunct
  int32_t ilit;
  float flit;
  int32_t soff;      // string literal: word offset in the pool
  int32_t swords;    // string literal: words
  // PredEval's evaluation order (R/iterator/PredEval.java:164-175): this term
  // is evaluated for a row only if every required conjunct before it held
  // ((cb & req_below) == req_below) and no earlier term of its own conjunct
  // held (!(cb & conj_bit)).  A float compare reached with a NaN operand
  // raises (TupleUtils.java:61-69 falls through to the string branch).
  uint32_t req_below;  // all_conj & (conj_bit - 1)
  int32_t nan_lit;     // the literal is NaN (or a literal-vs-literal NaN term): raises whenever reached
  // `column OP literal` as one unsigned range test over a signed-ordered key
  // (the scan's branch-free term body): holds iff ((uint32)(x - rlo) <= rspan)
  // != rneg, x = the int value; a float's bits with the low 31 bits flipped
  // when negative (x = a ^ ((a >> 31) & rm31), rm31 = 0x7fffffff: -0.0 and
  // +0.0 become the adjacent keys -1 and 0, NaNs fall outside [-inf, +inf]);
  // a string's compareTo sign against the literal (-1 / 0 / 1)
  int32_t rlo;
  uint32_t rspan;
  int32_t rneg;
  uint32_t rm31;
};

// The compiled predicate (PredEval over one CNF) + optional aggregate column.
// Lives in device memory; kernels read it with uniform (scalar) loads.
struct KPlan {
  int32_t ncols;
  int32_t nterms;
  uint32_t all_conj;  // every conjunct bit that must be set (0: no filter)
  int32_t agg_slot;   // -1: none
  int32_t has_real;   // any float comparison (NaN detection)
  int32_t pad_;
  KCol cols[kMaxCols];
  KTerm terms[kMaxTerms];
  uint32_t pool[kMaxPoolWords];
};

// per-block partial result of a scan (deterministic finalize, no atomics)
struct Partial {
  int64_t count;
  int64_t isum;
  double fsum;
  int32_t imin, imax;
  float fmin, fmax;
  int32_t nan_seen;
  int32_t pad_;
};

// mirrors mbx_agg (include/mbx.h) field for field
struct AggOut {
  int64_t count;
  int32_t agg_type;
  int32_t pad_;
  int64_t isum;
  int32_t imin, imax;
  double fsum;
  float fmin, fmax;
};

// COUNT / BitSet finalize partials store only these words of a Partial
constexpr int kSegStride = (int)(sizeof(Partial) / sizeof(int64_t));

enum ScanMode : int32_t { kModeCount = 0, kModeBitmap = 1, kModeAgg = 2 };

struct ScanLaunch {
  const KPlan* plan;          // device
  int64_t nrows;
  int64_t tiles_per_block;    // segment = tiles_per_block tiles
  const uint64_t* deleted;    // device or null
  uint64_t* out_words;        // device or null
  Partial* partials;          // device, one per block
  int32_t mode;
  int32_t fast_k;             // fast kernel: 4-byte slots 0..K-1 (fast_k + fast_ks == 0: generic)
  int32_t fast_ks;            // fast kernel: 16-byte string slots K..K+KS-1
  int32_t agg_kind;           // kInt / kReal when mode == kModeAgg
  // in-launch finalize: the last block to arrive on `ticket` reduces all
  // partials in block order (release/acquire hand-off, zeroed by that block)
  uint32_t* ticket;           // device, kTicketWords zeros before the launch; null: no finalize
  int32_t ticket_groups;      // 0: one flat ticket; G: G group tickets + one top ticket
  int64_t* count_out;         // device or null
  AggOut* agg_out;            // device or null
  int32_t* nan_out;           // device or null
  int32_t nterms_host;        // the plan's term count, for launch-time kernel choice
  int32_t hoist_terms;        // 1..kHoistTerms literal terms: hoisted into registers
  int32_t fin_mode;           // FinMode (MBX_FIN_MODE): how the last block sees the partials
  int32_t ri;                 // 1: row-interleaved tile layout (register j of lane l = row 64j + l)
  int32_t sink_lds;           // 1: BitSet words of the block's full tiles staged in dynamic LDS
                              //    (tiles_per_block x 32 B) and stored in one burst at the block's end
  int64_t* seg_counts;        // BitSet scans: the output bitmap's per-segment counts (one per block)
  int32_t words_wt;           // BitSet words stored write-through (sc1) instead of plain
  int32_t int_range;          // branch-free range-test term body: 1 every term an int literal
                              // compare, 2 literal compares of any type (int / float / char(16))
};

// dynamic LDS per block for the staged BitSet (4 blocks per CU: <= 128 KB of
// the CU's 160 KB)
constexpr int64_t kSinkLdsMaxBytes = 32 * 1024;

// Arrival tickets of the in-launch finalize.  Blocks arrive on the ticket of
// their group (blockIdx % G, so a group lives on one XCD -- blocks are dealt
// to the 8 XCDs round-robin); the last arriver of a group then arrives on the
// top ticket.  Same-address device atomics serialize (~12 ns each measured on
// MI355X), so one flat ticket costs ~12 us per 1000 blocks when they finish
// together; G groups cut the chain to nblocks/G + G.  Each ticket owns a
// 128-byte line.
constexpr int kTicketStride = 32;                 // uint32 per ticket line
constexpr int kMaxTicketGroups = 64;
constexpr int kTicketWords = (kMaxTicketGroups + 1) * kTicketStride;
constexpr int kDefaultTicketGroups = 32;

enum FinMode : int32_t {
  kFinWriteThrough = 0,  // sc1 partial stores + ticket, sc1 loads by the last block
  kFinFences = 1,        // plain stores + agent release / acquire fences
  kFinSeparate = 2,      // no ticket: a separate k_finalize launch
  kFinPackedCount = 3,   // COUNT: each block adds (count, nan, 1) packed in one
                         // 64-bit word to its group's ticket; the last arriver
                         // of the top ticket holds the total -- no partials
  kFinSegOnly = 4,       // BitSet scans whose caller reads only the segment
                         // counts (async BitSet / select with no float term:
                         // no NaN to report): no ticket, no count.  Forced on
                         // a COUNT scan (MBX_FIN_MODE=4) it is a diagnostic:
                         // the count is not produced -- what the finalize costs
  kFinFrame = 5,         // COUNT into a caller-zeroed count frame: each block adds
                         // its packed (count, nan, 1) word to slot blockIdx % 32
                         // with a no-return atomic -- no ticket, no last arriver,
                         // no dependent round trip at the end of the launch; the
                         // reader adds the 32 slots (mbx_count_frame_decode)
};

// count frame (mbx_scan_count_frame_async): MBX_COUNT_FRAME_SLOTS packed words,
// one per 128-byte line so the slots' atomics do not share a line
constexpr int kFrameSlots = 32;
constexpr int kFrameSlotStride = 16;  // int64 words per slot line

struct ProjCol {
  const void* base;
  int32_t stride_w;
  int32_t gstride = 0;           // > 0: a 4-byte column also in a column group (mbx_table_group):
  const void* gbase = nullptr;   // its value of row r at ((const uint32_t*)gbase)[r * gstride]
};

struct BitmapCnf {
  const uint64_t* bms[kMaxBitmaps];
  int32_t conj_off[33];
  int32_t nconj;
};

// ---- Minibase DB pages (mbx_pages.hip, include/mbx_db.h)
constexpr int kDbPage = 1024;      // GlobalConst.MINIBASE_PAGESIZE
constexpr int kDbSlotBase = 20;    // HFPage.DPFIXED: slot directory start

struct PageDecodeArgs {
  const uint8_t* image;      // device copy of DB pages 0..image_pages-1
  int64_t image_pages;
  const int32_t* page_of;    // page index -> pid (-1: none), npages entries
  int64_t npages;
  int32_t rec_len;           // record bytes (4, or n + 2 for char(n))
  int32_t recs_per_page;     // (1024 - 20) / (4 + rec_len)
  int32_t kind;              // ColKind
  int32_t size;              // char(n): n
  int32_t stride;            // output bytes per row
  int32_t pad_;
  uint8_t* out;              // column image, nrows rows
  uint64_t* present;         // BitSet of positions that hold a record
  int64_t nrows;
  int32_t* err;              // bit flags of malformed pages
  // row-range staging (mbx_db_stage_range): page_of[i] is page index
  // page_index0 + i, output row r is position pos_begin + r; positions
  // outside [pos_begin, pos_begin + nrows) are another shard's (range = 1:
  // skipped, not an error)
  int64_t page_index0;
  int64_t pos_begin;
  int32_t range;
  int32_t pad2_;
};

hipError_t launch_page_decode(const PageDecodeArgs& A, hipStream_t s);
hipError_t launch_present_merge(const uint64_t* present0, const uint64_t* other, int32_t nother, int64_t nwords_each,
                                const uint64_t* md, int64_t md_words, int64_t nrows, uint64_t* del, int32_t* flags,
                                hipStream_t s);

constexpr unsigned long long kEmptySlot = ~0ull;

constexpr int kLdsProbes = 16;   // k_distinct's default LDS probe bound
struct DistinctArgs {
  KCol col;
  int64_t nrows;
  const uint64_t* del;          // deleted positions are skipped (ColumnScan)
  unsigned long long* keys;     // cap slots, kEmptySlot = free; else a representative row
  unsigned long long* minpos;   // cap slots, kEmptySlot initially; smallest row with the value
  int64_t cap;                  // power of two
  int32_t* overflow;
  int32_t lds_probes;           // LDS pre-fold probe bound (0: every row goes to the global table)
};

hipError_t launch_distinct(const DistinctArgs& A, hipStream_t s);
hipError_t launch_rows_fetch(const KCol& c, const int64_t* rows, int64_t n, uint32_t* out, hipStream_t s);

// ---- joins (mbx_join.hip, include/mbx_join.h)
constexpr int kMaxJoinTerms = 16;

struct JoinTerm {
  int32_t kind;        // ColKind of both columns
  int32_t op;          // CmpOp; -1: never true (aopNOP / opRANGE)
  const void* ocol;    // outer column (table-local rows)
  const void* icol;    // inner column
  int32_t ostride_w, istride_w;
  uint32_t conj_bit;
  uint32_t req_below;  // all_conj & (conj_bit - 1): PredEval's reach rule (KTerm.req_below)
};

struct JoinArgs {
  JoinTerm terms[kMaxJoinTerms];
  int32_t nterms;
  uint32_t all_conj;
  int32_t mode;                 // 0 BMJ, 1 NLJ
  int32_t pad_;
  const int64_t* opos;          // outer selection: table-local rows, ascending
  int64_t no;
  const int64_t* ipos;          // inner selection
  int64_t ni;
  int64_t block;                // NLJ outer block (tuples per pass)
  int64_t row0, nrows;          // matrix rows of this launch
  int64_t words_per_row;
  uint64_t* out;                // nrows * words_per_row words
  int32_t* nan;
  int32_t plain;                // 1: k_join_matrix even where the fast form applies (A/B)
  int32_t pad2_;
};

struct JoinDecode {
  int32_t mode;
  int32_t pad_;
  const int64_t* opos;
  const int64_t* ipos;
  int64_t ni, block, row0, words_per_row;
  int64_t outer_offset, inner_offset;  // tables' row_offset (global positions)
  int64_t base;                         // output index of the first pair of this chunk
  int64_t* out_outer;
  int64_t* out_inner;
  int32_t* out_pass;
};

hipError_t launch_join_matrix(const JoinArgs& A, hipStream_t s);
hipError_t launch_join_decode(const int64_t* ids, const int64_t* n, int64_t max_n, const JoinDecode& D,
                              hipStream_t s);
hipError_t launch_gather_pos(const int64_t* pos, int64_t n, int64_t row_offset, const void* col, int32_t stride_w,
                             void* out, hipStream_t s);

// read-bandwidth probe (k_read_probe): the scan's loads without a predicate
constexpr int kMaxProbeCols = 4;
struct ProbeArgs {
  const int32_t* cols[kMaxProbeCols];
  int32_t ncols;
  int32_t interleave;       // 0: segments of tiles_per_block tiles; 1: grid-stride over `grid` blocks
  int64_t nrows;
  int64_t tiles_per_block;
  int64_t grid;
  uint32_t* sink;           // one word per block
};
hipError_t launch_read_probe(const ProbeArgs& A, hipStream_t s);

int64_t grid_blocks(int64_t nrows, int64_t tiles_per_block);
int64_t choose_tiles_per_block(int64_t nrows);

hipError_t launch_scan(const ScanLaunch& L, hipStream_t s);
hipError_t launch_finalize(const Partial* partials, int64_t nblocks, int32_t agg_kind, AggOut* out,
                           int64_t* count_out, int32_t* nan_flag, hipStream_t s);
// one launch: words of the CNF (never stored) -> positions (ids may be null)
// + <= 4 projected 4-byte columns; lb = kLookbackWords int64 look-back words,
// zeroed once at allocation (k_cnf_select)
// k_cnf_select's A/B knobs (MbxTuning cnf_*): grid (0: 1024 blocks), polled
// flag stride (1 or kFlagStride), look-back form (0 auto, 1 chained, 2
// polled), output stores (0 default, 1 plain, 2 write-through, 3 nontemporal)
struct CnfTune {
  int32_t blocks = 0, flag_stride = 1, lookback = 0, store = 0, gather_pair = 1;
};
hipError_t launch_cnf_materialize(const BitmapCnf& c, const uint64_t* deleted, int64_t nwords, int64_t nbits,
                                  int64_t* lb, int64_t row_offset, int64_t* ids, const ProjCol* proj,
                                  void* const* out, int32_t nproj, int64_t* total, hipStream_t s,
                                  int64_t* stamps = nullptr, int32_t dbg = 0,
                                  int64_t cap = INT64_MAX, const struct CnfTune* tune = nullptr);
// epoch, per-block counts, per-block inclusive prefixes; the polling form's
// counts may sit one per 128-byte line (kFlagStride words apart)
constexpr int32_t kFlagStride = 16;
constexpr int64_t kLookbackWords = 1 + kFlagStride * 1024;
// BitSet + positions + COUNT of a plan in one launch (k_scan_select): plans of
// 1..4 int literal terms on 4-byte columns, tables whose segments fit the
// one-launch form (scan_select_fusable); L as for a kModeBitmap scan (its
// out_words / seg_counts: the BitSet and its segment counts)
bool scan_select_fusable(int64_t nrows, int64_t tiles_per_block, int32_t fast_k, int32_t fast_ks, int32_t nterms,
                         int32_t has_real, int32_t waves);
hipError_t launch_scan_select(const ScanLaunch& L, int64_t* lb, int64_t row_offset, int64_t* ids, int64_t* total,
                              hipStream_t s, int64_t* stamps, int32_t dbg, int32_t waves, int32_t flag_stride);
hipError_t launch_bitmap_cnf(const BitmapCnf& c, const uint64_t* deleted, int64_t nwords, int64_t nbits,
                             int64_t words_per_block, uint64_t* out, int64_t* segc, hipStream_t s);
hipError_t launch_bitmap_combine(int32_t op, const uint64_t* a, const uint64_t* b, int64_t nwords,
                                 int64_t nbits, int64_t words_per_block, uint64_t* out, int64_t* segc,
                                 hipStream_t s);
// per-segment counts of a BitSet (segments of words_per_block words): a
// compact int64 array, one per segment
hipError_t launch_seg_popcount(const uint64_t* words, int64_t nwords, int64_t words_per_block,
                               int64_t* segc, hipStream_t s);
hipError_t launch_count_sum(const int64_t* segc, int64_t n, int64_t* out, hipStream_t s);
// positions (ascending) of the set bits + gather of the projected columns;
// *total = the number of set bits (written on the stream)
hipError_t launch_materialize(const uint64_t* words, int64_t nwords, int64_t words_per_block,
                              const int64_t* segc, int64_t row_offset, int64_t* ids,
                              const ProjCol* proj, void* const* out, int32_t nproj, int64_t* total,
                              hipStream_t s, int32_t dbg = 0, int64_t* stamps = nullptr, bool fuse_gather = true,
                              int64_t max_blocks = 1024, bool gather_pair = true);
// 4-byte columns (int / float): also writes every output's segment counts
hipError_t launch_index_build4(const KCol& col, int64_t nrows, const uint64_t* deleted, const uint32_t* values,
                               int32_t nvalues, uint64_t* const* outs, int64_t* const* segs, int64_t words_per_block,
                               hipStream_t s);
hipError_t launch_index_build(const KCol& col, int64_t nrows, const uint64_t* deleted, const uint32_t* values,
                              int32_t nvalues,
                              int32_t value_words, uint64_t* const* outs, int64_t words_per_block, hipStream_t s);

// cursor delivery (mbx_cursor.hip): rows [from, from + n) of a cursor's
// positions + projected columns packed into one staging region in the host
// layout; column j at dst + col[j].dst_off, width bytes per row
struct CursorPackCol {
  const uint8_t* src;
  int64_t dst_off;
  int32_t src_stride;  // bytes per device row
  int32_t width;       // bytes per host row (4, or n for char(n))
  int32_t is_string;
  int32_t pad_;
};
struct CursorPack {
  CursorPackCol col[kMaxProj];
  int32_t ncols;
  int32_t pad_;
};
// column group (mbx_table_group): out[r * ncols + k] = cols[k][r]
hipError_t launch_group_build(const uint32_t* const* cols, int32_t ncols, int64_t nrows, uint32_t* out,
                              hipStream_t s);
hipError_t launch_cursor_pack(const int64_t* ids, int64_t from, int64_t n, const CursorPack& P, uint8_t* dst,
                              hipStream_t s);

}  // namespace mbx
