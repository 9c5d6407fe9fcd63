// mbx_objects.hpp -- host-side objects behind the opaque handles of
// include/mbx.h and include/mbx_db.h, shared by mbx_api.cpp (scans, bitmaps,
// cursors) and mbx_db.cpp (Minibase DB files).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <deque>
#include <string>
#include <vector>

#include "../../include/mbx.h"
#include "mbx_internal.hpp"

namespace mbx {

// ------------------------------------------------------------------ errors

// sets the thread-local message mbx_last_error() returns; returns `code`
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess) return fail(MBX_E_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

#define NOTNULL(p) \
  do {             \
    if (!(p)) return fail(MBX_E_INVALID, "%s: null argument `%s`", __func__, #p); \
  } while (0)

}  // namespace mbx

// ----------------------------------------------------------------- objects

using mbx::AggOut;
using mbx::KPlan;
using mbx::Partial;

// A/B tuning knobs of the scan path.  Read from the
// MBX_* environment once in mbx_init and changed only by mbx_set_tuning, so
// no launch reads the environment.  -1 = the built-in default.
// The knobs' defaults are the production forms.  Names in comments are the
// environment variables a -DMBX_DIAG build reads at mbx_init (the default
// library reads none: mbx_set_tuning only).
struct MbxTuning {
  int64_t tiles_per_block = -1;   // MBX_TILES_PER_BLOCK: segment size of every scan / BitSet
  int32_t force_generic = 0;      // MBX_FORCE_GENERIC: plans compiled after this use k_scan_generic
  int32_t scan_hoist = 1;         // MBX_SCAN_HOIST: 0 reads terms from the plan per tile
  int32_t scan_int_range = 2;     // MBX_SCAN_INT_RANGE: literal terms as branch-free range tests --
                                  // 0 off, 1 int-only plans, 2 (default) also float / char(16) terms
  int32_t scan_ri = 1;            // MBX_SCAN_RI: 0 never, 1 BitSet output only, 2 always
  int32_t sink_lds = 1;           // MBX_SINK_LDS: 0 never, 1 segments >= 128 tiles, 2 whenever it fits
  int32_t ticket_groups = -1;     // MBX_TICKET_GROUPS
  int32_t fin_mode = -1;          // MBX_FIN_MODE (FinMode)
  int32_t join_plain = 0;         // MBX_JOIN_PLAIN: k_join_matrix instead of the fast form
  int32_t distinct_lds_probes = -1;  // MBX_DISTINCT_LDS_PROBES
  int32_t gather_fused = 1;       // MBX_GATHER_FUSED: 0 = compaction, then k_gather (two launches)
  int32_t gather_pair = 1;        // MBX_GATHER_PAIR: 0 = two 4-byte loads per grouped pair row instead of one 8-byte
  int32_t cnf_store = 0;          // MBX_CNF_STORE: k_cnf_select outputs 0 default, 1 plain, 2 write-through, 3 nontemporal
  int32_t cnf_lookback = 0;       // MBX_CNF_LOOKBACK: k_cnf_select look-back 0 auto, 1 chained, 2 polled
  int32_t cnf_flag_stride = 1;    // MBX_CNF_FLAG_STRIDE: k_cnf_select's polled count flags 16 words apart, or 1
  int32_t cnf_blocks = 0;         // MBX_CNF_BLOCKS: k_cnf_select blocks (0: 1024; chained look-back: up to 8192)
  int32_t select_blocks = 1024;   // MBX_SELECT_BLOCKS: compaction blocks at most (segments per block = nseg / this)
  int32_t cursor_prefetch = 1;    // MBX_CURSOR_PREFETCH: 0 = mbx_cursor_next copies each batch on demand
  int32_t scan_select_fused = 1;  // MBX_SCAN_SELECT_FUSED: 1 = BitSet + positions in one launch (k_scan_select)
  int32_t scan_select_waves = 16; // MBX_SCAN_SELECT_WAVES: waves per k_scan_select block (4 or 16)
  int32_t select_flag_stride = 16; // MBX_SELECT_FLAG_STRIDE: 16 = k_scan_select's polled flags one per line, or 1
  int32_t scan_words_wt = 1;      // MBX_SCAN_WORDS_WT: BitSet scan words stored write-through
  int32_t comm_same_stream = 1;   // MBX_COMM_SAME_STREAM: collectives on the context stream (0: the exchange stream)
  int32_t select_dbg = 0;         // MBX_SELECT_DBG: bit 3 per-block stamps, 128 every-predecessor poll
                                  // instead of the chained look-back, 512 write-through flip; -DMBX_DIAG
                                  // builds only: k_select_ids bit 0 no prefix / bit 1 no emission, the
                                  // one-launch selections' 16 back-off / 32 no wait / 64 plain-load polls
};
constexpr int64_t kMaxStampBlocks = 65536;

struct mbx_ctx {
  int32_t device = 0;
  MbxTuning tune;
  hipStream_t stream = nullptr;
  Partial* partials = nullptr;  // scratch, one per block of the largest scan so far
  int64_t partials_cap = 0;
  AggOut* dagg = nullptr;
  int64_t* dcount = nullptr;
  int32_t* dnan = nullptr;       // async scans: [0] last, [1] sticky until mbx_sync; sync scans: [2]
  uint32_t* ticket = nullptr;   // in-launch finalize ticket (always 0 between launches)
  int64_t* ids_scratch = nullptr;  // positions for a gather whose caller wants no positions
  int64_t ids_cap = 0;
  int64_t* stamps = nullptr;    // diagnostic per-block stamps (select_dbg bit 3)
  int64_t* lookback = nullptr;  // k_cnf_select's epoch + per-block counts (kLookbackWords, zeroed once)
  void* pinned = nullptr;       // 256 bytes of pinned host scratch
  mbx_comm* comm = nullptr;     // multi-GPU exchange (mbx_comm.cpp), owned
  bool capturing = false;       // mbx_graph_begin .. mbx_graph_end
};

struct TCol {
  int32_t attr_type = 0;
  int32_t size = 0;
  int32_t stride_w = 1;  // device words per row
  void* dev = nullptr;
  bool owned = false;
};

// a column group (mbx_table_group): row r of column cols[k] at dev[r * cols.size() + k]
struct TGroup {
  std::vector<int32_t> cols;
  uint32_t* dev = nullptr;
};

struct mbx_table {
  mbx_ctx* ctx = nullptr;
  int64_t nrows = 0;
  int64_t row_offset = 0;
  std::vector<TCol> cols;
  std::vector<TGroup> groups;  // owned
  uint64_t* deleted = nullptr;
  bool owns_deleted = false;
  bool aligned16 = true;
};

struct PlanVariant {
  int32_t agg_col = -1;  // -1: filter only
  KPlan* dev = nullptr;
  int32_t fast_k = 0;
  int32_t fast_ks = 0;
  int32_t agg_kind = mbx::kInt;
};

struct mbx_plan {
  mbx_ctx* ctx = nullptr;
  const mbx_table* t = nullptr;
  KPlan host{};
  std::vector<int32_t> slot_col;  // table column of each slot
  bool all_literal = true;        // every term is `column OP literal`
  bool str_lit_fits16 = true;     // every string literal is <= 16 bytes
  std::deque<PlanVariant> variants;
};

struct mbx_bitmap {
  mbx_ctx* ctx = nullptr;
  int64_t nbits = 0;
  int64_t nwords = 0;
  uint64_t* words = nullptr;
  int64_t wpb = 4;        // words per segment
  int64_t nseg = 1;
  int64_t* segc = nullptr;  // per-segment counts, compact (one int64 per segment of wpb words)
  int64_t count = -1;     // host copy of the cardinality, -1 = unknown
};

struct mbx_cursor {
  mbx_ctx* ctx = nullptr;
  int64_t count = 0;
  int64_t next = 0;
  const mbx_table* t = nullptr;
  int64_t* ids = nullptr;  // device
  std::vector<void*> outs; // device, one per projected column
  std::vector<int32_t> proj;
  // double-buffered delivery (mbx_cursor_next): while the caller consumes
  // batch k, batch k+1 is already on its way into the other pinned buffer.
  // A batch is packed on the device (k_cursor_pack into `stage`) in the host
  // layout -- positions, then each projected column, 16-byte aligned -- and
  // crosses PCIe as ONE copy into pin[b].
  uint8_t* pin[2] = {nullptr, nullptr};
  uint8_t* stage = nullptr;  // device staging region of one batch
  hipEvent_t ev[2] = {nullptr, nullptr};
  int64_t batch_rows = 0;   // rows a pinned buffer holds
  int64_t pf_start = -1;    // first row of the batch in flight into pin[pf_buf] (-1: none)
  int64_t pf_n = 0;
  int pf_buf = 0;
  int64_t d2h_bytes = 0;    // statistics: bytes copied device -> pinned
  // mbx_cnf_cursor_launch: the count is still on the device (in dcount)
  // until the first mbx_cursor_count / mbx_cursor_next reads it
  int64_t* dcount = nullptr;
  int64_t bound = 0;        // capacity of ids / outs (rows)
  bool count_pending = false;
};

namespace mbx {

int set_device(mbx_ctx* c);
int32_t stride_words(const mbx_col_desc& d);
int check_cols(const mbx_col_desc* cols, int32_t ncols);
int64_t words_for(int64_t nbits);
// a table whose device columns (and, with_deleted, deleted words) are
// allocated but not filled; the caller writes them on the context stream
int table_alloc(mbx_ctx* c, const mbx_col_desc* cols, int32_t ncols, int64_t nrows, int64_t row_offset,
                bool with_deleted, mbx_table** out);
int bitmap_new(mbx_ctx* c, int64_t nbits, mbx_bitmap** out);
// one BitSet per value of column `col` (values in the device image: 1 word
// for int/float, stride_w words for char(n)); out[nvalues]
int index_build_encoded(mbx_ctx* c, const mbx_table* t, int32_t col, const uint32_t* host_vals, int32_t nvalues,
                        mbx_bitmap** out);
// host modified UTF-8 (zero padded to len) <-> device string image (stride bytes)
void encode_device_string(const uint8_t* src, int32_t len, uint8_t* dst, int32_t stride);
void decode_device_string(const uint8_t* src, int32_t stride, uint8_t* dst, int32_t size);
// device column image rows -> caller layout (char(n): n bytes modified UTF-8)
void unpack_rows(const TCol& tc, const uint8_t* dev_img, int64_t n, void* host_out);
// b->count on the host (one finalize + sync when unknown)
int ensure_count(mbx_ctx* c, mbx_bitmap* b);
// recount per-segment popcounts of a bitmap written on the device, sync, and
// set b->count
int bitmap_recount(mbx_ctx* c, mbx_bitmap* b);
// a COUNT scan that leaves one count per block in dev_parts (no finalize,
// no count): *nparts = the blocks; MBX_E_INVALID for a plan with a float
// term (its NaN needs the finalize) or more blocks than cap
int scan_count_parts(mbx_ctx* c, const mbx_plan* p, int64_t* dev_parts, int64_t cap, int64_t* nparts);
bool plan_has_real(const mbx_plan* p);
// mbx_comm.cpp: mbx_sync / mbx_free of a context with a communicator
int comm_sync(mbx_ctx* c);
void comm_release_of(mbx_ctx* c);

}  // namespace mbx
