// mbx_api.cpp -- the C-ABI (include/mbx.h) over the CDNA4 kernels.
//
// Host-side responsibilities, each restating a piece of the reference:
//   * staging (TupleScan / Columnarfile open, R/columnar/TupleScan.java:29-47):
//     host column arrays -> HBM column chunks, char(n) into the device string
//     image (mbx_internal.hpp);
//   * plan compilation (PredEval.Eval type rules, R/iterator/PredEval.java:54-135):
//     operand types, FldSpec ranges, literal-on-left orientation, constant
//     terms, NOT == NE, NOP / RANGE never true;
//   * result plumbing for get_next()/get_next_tid() (cursors, BitSets).
// Nothing here computes a query result on the CPU: every row-level operation
// is a kernel launch on the context stream.
#include "../../include/mbx.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <deque>
#include <vector>

#include "mbx_internal.hpp"
#include "mbx_objects.hpp"

using namespace mbx;

// ------------------------------------------------------------------ errors

static thread_local std::string g_err;

int mbx::fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// ----------------------------------------------------------------- helpers

// A bitmap's segment = the BitSet scan's block and the unit of its compact
// segment counts (~1024 segments).  Capping segments at 48 tiles (one column,
// 100M rows) speeds the BitSet scan 78.1 -> 71.2 us but slows the AND over
// such bitmaps 7.2 -> 10.2 us and the compaction 20.9 -> 24.4 us, both of
// which want ~1024 blocks (profiles/r02/anatomy/segment_cap_48.jsonl): not kept.
static int64_t tiles_per_block_for(const mbx_ctx* c, int64_t nrows) {
  if (c->tune.tiles_per_block > 0) return c->tune.tiles_per_block;
  return choose_tiles_per_block(nrows);
}

// COUNT / aggregate scans choose their own grid (BitSet scans follow the
// output bitmap's segments).  Plans with 16-byte string slots do more work per
// byte and run best with ~4096 blocks (C5, 125M rows: 483 -> 470 us; 1B rows:
// 3908 -> 3729 us, profiles/r01/round_e); 4-byte-only plans with ~1024.
static int64_t scan_tiles_per_block(const mbx_ctx* c, int64_t nrows, const PlanVariant& v) {
  if (c->tune.tiles_per_block > 0) return c->tune.tiles_per_block;
  if (v.fast_ks > 0) {
    const int64_t ntiles = (nrows + kTileRows - 1) / kTileRows;
    const int64_t tpb = (ntiles + 4095) / 4096;
    return tpb < 4 ? 4 : tpb;
  }
  return choose_tiles_per_block(nrows);
}

#ifdef MBX_DIAG
static int64_t env_knob(const char* name, int64_t dflt) {
  const char* e = getenv(name);
  return e && *e ? atoll(e) : dflt;
}
#endif

// The context's tuning at mbx_init and after mbx_set_tuning("reset"): the
// production defaults.  A -DMBX_DIAG build (tools/build_diag.sh,
// tools/build_variant.sh) also reads the MBX_* A/B knobs from the environment;
// the default library reads no environment at all -- tests and tools drive the
// same knobs through mbx_set_tuning.
static void tuning_defaults(MbxTuning& t) {
  t = MbxTuning();
#ifdef MBX_DIAG
  t.tiles_per_block = env_knob("MBX_TILES_PER_BLOCK", -1);
  t.force_generic = (int32_t)env_knob("MBX_FORCE_GENERIC", 0);
  t.scan_hoist = (int32_t)env_knob("MBX_SCAN_HOIST", 1);
  t.scan_int_range = (int32_t)env_knob("MBX_SCAN_INT_RANGE", 2);
  if (t.scan_int_range < 0 || t.scan_int_range > 2) t.scan_int_range = 2;
  t.scan_ri = (int32_t)env_knob("MBX_SCAN_RI", 1);
  t.sink_lds = (int32_t)env_knob("MBX_SINK_LDS", 1);
  t.ticket_groups = (int32_t)env_knob("MBX_TICKET_GROUPS", -1);
  t.fin_mode = (int32_t)env_knob("MBX_FIN_MODE", -1);
  t.join_plain = (int32_t)env_knob("MBX_JOIN_PLAIN", 0);
  t.distinct_lds_probes = (int32_t)env_knob("MBX_DISTINCT_LDS_PROBES", -1);
  t.select_dbg = (int32_t)env_knob("MBX_SELECT_DBG", 0);
  t.gather_fused = (int32_t)env_knob("MBX_GATHER_FUSED", 1);
  t.gather_pair = env_knob("MBX_GATHER_PAIR", 1) != 0;
  t.cursor_prefetch = (int32_t)env_knob("MBX_CURSOR_PREFETCH", 1);
  t.scan_select_fused = (int32_t)env_knob("MBX_SCAN_SELECT_FUSED", 1);
  t.scan_select_waves = (int32_t)env_knob("MBX_SCAN_SELECT_WAVES", 16);
  t.select_flag_stride = (int32_t)env_knob("MBX_SELECT_FLAG_STRIDE", kFlagStride);
  t.scan_words_wt = (int32_t)env_knob("MBX_SCAN_WORDS_WT", 1);
  t.comm_same_stream = (int32_t)env_knob("MBX_COMM_SAME_STREAM", 1);
  t.cnf_blocks = (int32_t)env_knob("MBX_CNF_BLOCKS", 0);
  t.cnf_flag_stride = env_knob("MBX_CNF_FLAG_STRIDE", 1) == kFlagStride ? kFlagStride : 1;
  t.cnf_lookback = (int32_t)env_knob("MBX_CNF_LOOKBACK", 0);
  t.cnf_store = (int32_t)env_knob("MBX_CNF_STORE", 0) & 3;
  if (t.cnf_lookback < 0 || t.cnf_lookback > 2) t.cnf_lookback = 0;
  t.select_blocks = (int32_t)env_knob("MBX_SELECT_BLOCKS", 1024);
  if (t.select_blocks < 1) t.select_blocks = 1024;  // as mbx_set_tuning: never a zero / negative grid divisor
#endif
}

static int ensure_partials(mbx_ctx* c, int64_t n) {
  if (n <= c->partials_cap) return MBX_OK;
  if (c->partials) HIPCHK(hipFree(c->partials));
  c->partials = nullptr;
  const int64_t cap = n < 4096 ? 4096 : n;
  HIPCHK(hipMalloc(&c->partials, sizeof(Partial) * cap));
  c->partials_cap = cap;
  return MBX_OK;
}

int mbx::set_device(mbx_ctx* c) {
  HIPCHK(hipSetDevice(c->device));
  return MBX_OK;
}

// device string image: modified UTF-8, C0 80 -> 00 01, zero padded to stride
void mbx::encode_device_string(const uint8_t* src, int32_t len, uint8_t* dst, int32_t stride) {
  int32_t n = len < stride ? len : stride;
  // the payload ends at the first 0x00 (zero padding never occurs inside modified UTF-8)
  int32_t m = 0;
  while (m < n && src[m] != 0) m++;
  memset(dst, 0, (size_t)stride);
  for (int32_t i = 0; i < m; i++) {
    if (src[i] == 0xC0 && i + 1 < m && src[i + 1] == 0x80) {
      dst[i] = 0x00;
      dst[i + 1] = 0x01;
      i++;
    } else {
      dst[i] = src[i];
    }
  }
}

void mbx::decode_device_string(const uint8_t* src, int32_t stride, uint8_t* dst, int32_t size) {
  memset(dst, 0, (size_t)size);
  for (int32_t i = 0; i < stride && i < size; i++) {
    if (src[i] == 0x00) {
      if (i + 1 < stride && src[i + 1] == 0x01 && i + 1 < size) {
        dst[i] = 0xC0;
        dst[i + 1] = 0x80;
        i++;
        continue;
      }
      break;
    }
    dst[i] = src[i];
  }
}

int64_t mbx::words_for(int64_t nbits) { return (nbits + 63) / 64; }

int mbx::bitmap_new(mbx_ctx* c, int64_t nbits, mbx_bitmap** out) {
  mbx_bitmap* b = new (std::nothrow) mbx_bitmap();
  if (!b) return fail(MBX_E_NOMEM, "bitmap: host allocation");
  b->ctx = c;
  b->nbits = nbits;
  b->nwords = words_for(nbits);
  b->wpb = tiles_per_block_for(c, nbits) * kWordsPerTile;
  b->nseg = b->nwords == 0 ? 1 : (b->nwords + b->wpb - 1) / b->wpb;
  hipError_t e = hipMalloc(&b->words, sizeof(uint64_t) * (size_t)(b->nwords > 0 ? b->nwords : 1));
  if (e == hipSuccess) e = hipMalloc(&b->segc, sizeof(int64_t) * (size_t)b->nseg);
  if (e != hipSuccess) {
    hipFree(b->words);
    hipFree(b->segc);
    delete b;
    return fail(MBX_E_NOMEM, "bitmap of %lld bits: %s", (long long)nbits, hipGetErrorString(e));
  }
  if (b->nwords == 0) hipMemsetAsync(b->segc, 0, sizeof(int64_t), c->stream);
  *out = b;
  return MBX_OK;
}

// ----------------------------------------------------------------- library

extern "C" int mbx_abi_version(void) { return MBX_ABI_VERSION; }

extern "C" const char* mbx_last_error(void) { return g_err.c_str(); }

extern "C" int mbx_device_count(int32_t* n) {
  NOTNULL(n);
  int k = 0;
  hipError_t e = hipGetDeviceCount(&k);
  if (e != hipSuccess) {
    *n = 0;
    return fail(MBX_E_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *n = k;
  return MBX_OK;
}

extern "C" int mbx_init(int32_t device, mbx_ctx** out) {
  NOTNULL(out);
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(MBX_E_DEVICE, "mbx_init: no HIP device visible (the executor has no CPU fallback)");
  if (device < 0 || device >= n) return fail(MBX_E_INVALID, "mbx_init: device %d of %d", device, n);
  mbx_ctx* c = new (std::nothrow) mbx_ctx();
  if (!c) return fail(MBX_E_NOMEM, "mbx_init: host allocation");
  c->device = device;
  tuning_defaults(c->tune);
  int rc = MBX_OK;
  do {
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&c->dagg, sizeof(AggOut));
    if (e == hipSuccess) e = hipMalloc(&c->dcount, sizeof(int64_t) * 2);
    if (e == hipSuccess) e = hipMalloc(&c->dnan, sizeof(int32_t) * 4);
    if (e == hipSuccess) e = hipMemset(c->dnan, 0, sizeof(int32_t) * 4);
    if (e == hipSuccess) e = hipMalloc(&c->ticket, sizeof(uint32_t) * kTicketWords);
    if (e == hipSuccess) e = hipMemset(c->ticket, 0, sizeof(uint32_t) * kTicketWords);
    if (e == hipSuccess) e = hipHostMalloc(&c->pinned, 256, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(&c->lookback, sizeof(int64_t) * kLookbackWords);
    if (e == hipSuccess) e = hipMemset(c->lookback, 0, sizeof(int64_t) * kLookbackWords);
    if (e != hipSuccess) {
      rc = fail(MBX_E_DEVICE, "mbx_init: %s", hipGetErrorString(e));
      break;
    }
    rc = ensure_partials(c, 4096);
  } while (0);
  if (rc != MBX_OK) {
    mbx_free(c);
    return rc;
  }
  *out = c;
  return MBX_OK;
}

extern "C" int mbx_free(mbx_ctx* c) {
  if (!c) return MBX_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  comm_release_of(c);
  hipFree(c->partials);
  hipFree(c->dagg);
  hipFree(c->dcount);
  hipFree(c->dnan);
  hipFree(c->ticket);
  hipFree(c->ids_scratch);
  hipFree(c->stamps);
  hipFree(c->lookback);
  if (c->pinned) hipHostFree(c->pinned);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return MBX_OK;
}

// Waits for the context stream and reports what the *_async scans enqueued
// since the last mbx_sync raised: a NaN reached by a float compare sets the
// sticky word dnan[1] (the kernels' last block), read and cleared here.
extern "C" int mbx_sync(mbx_ctx* c) {
  NOTNULL(c);
  if (c->capturing) return fail(MBX_E_INVALID, "mbx_sync inside a graph capture");
  HIPCHK(hipSetDevice(c->device));
  if (int rc = comm_sync(c)) return rc;
  int32_t* h = (int32_t*)c->pinned + 24;
  HIPCHK(hipMemcpyAsync(h, c->dnan + 1, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (*h) {
    HIPCHK(hipMemsetAsync(c->dnan + 1, 0, sizeof(int32_t), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return fail(MBX_E_TYPE,
                "NaN in a float comparison in an asynchronous scan (TupleUtils falls through to the string compare "
                "and raises)");
  }
  return MBX_OK;
}

extern "C" int mbx_set_tuning(mbx_ctx* c, const char* knob, int64_t value) {
  NOTNULL(c);
  NOTNULL(knob);
  MbxTuning& t = c->tune;
  if (!strcmp(knob, "reset")) {
    tuning_defaults(t);
    return MBX_OK;
  }
  const int32_t v = (int32_t)value;
  if (!strcmp(knob, "tiles_per_block")) t.tiles_per_block = value;
  else if (!strcmp(knob, "force_generic")) t.force_generic = v;
  else if (!strcmp(knob, "scan_hoist")) t.scan_hoist = v;
  else if (!strcmp(knob, "scan_int_range")) {
    if (v < 0 || v > 2) return fail(MBX_E_INVALID, "mbx_set_tuning: scan_int_range %d (0, 1 or 2)", v);
    t.scan_int_range = v;
  }
  else if (!strcmp(knob, "scan_ri")) t.scan_ri = v;
  else if (!strcmp(knob, "sink_lds")) t.sink_lds = v;
  else if (!strcmp(knob, "ticket_groups")) t.ticket_groups = v;
  else if (!strcmp(knob, "fin_mode")) {
#ifndef MBX_DIAG
    // kFinFences (plain stores + fences) and kFinSegOnly forced on a COUNT
    // scan (no count) exist for A/B measurements only
    if (v == kFinFences || v == kFinSegOnly)
      return fail(MBX_E_UNSUPPORTED, "mbx_set_tuning: fin_mode %d needs a -DMBX_DIAG build", v);
#endif
    t.fin_mode = v;
  }
  else if (!strcmp(knob, "join_plain")) t.join_plain = v;
  else if (!strcmp(knob, "distinct_lds_probes")) t.distinct_lds_probes = v;
  else if (!strcmp(knob, "select_dbg")) {
    // k_select_ids takes bits 0-1, the one-launch selections bits 4-6: A/B
    // forms a production build compiles out (kDiagDbg)
    if (((v & 3) | ((v >> 4) & 983)) & ~kDiagDbg)
      return fail(MBX_E_UNSUPPORTED, "mbx_set_tuning: select_dbg %d needs a -DMBX_DIAG build", v);
    t.select_dbg = v;
  }
  else if (!strcmp(knob, "gather_fused")) t.gather_fused = v;
  else if (!strcmp(knob, "gather_pair")) t.gather_pair = v != 0;
  else if (!strcmp(knob, "select_blocks")) t.select_blocks = v < 1 ? 1024 : (int32_t)v;
  else if (!strcmp(knob, "cnf_blocks")) t.cnf_blocks = v < 0 ? 0 : (int32_t)v;
  else if (!strcmp(knob, "cnf_flag_stride")) t.cnf_flag_stride = v == kFlagStride ? kFlagStride : 1;
  else if (!strcmp(knob, "cnf_lookback")) t.cnf_lookback = v >= 0 && v <= 2 ? (int32_t)v : 0;
  else if (!strcmp(knob, "cnf_store")) t.cnf_store = v >= 0 && v <= 3 ? (int32_t)v : 0;
  else if (!strcmp(knob, "cursor_prefetch")) t.cursor_prefetch = v;
  else if (!strcmp(knob, "scan_select_fused")) t.scan_select_fused = v;
  else if (!strcmp(knob, "scan_select_waves")) t.scan_select_waves = v == 4 ? 4 : 16;
  else if (!strcmp(knob, "select_flag_stride")) t.select_flag_stride = v == 1 ? 1 : kFlagStride;
  else if (!strcmp(knob, "scan_words_wt")) t.scan_words_wt = v != 0;
  else if (!strcmp(knob, "comm_same_stream")) t.comm_same_stream = v != 0;
  else return fail(MBX_E_INVALID, "mbx_set_tuning: unknown knob `%s`", knob);
  return MBX_OK;
}

extern "C" void* mbx_stream(mbx_ctx* c) { return c ? (void*)c->stream : nullptr; }

extern "C" int mbx_dev_alloc(mbx_ctx* c, int64_t bytes, void** dev) {
  NOTNULL(c);
  NOTNULL(dev);
  *dev = nullptr;
  if (bytes <= 0) return fail(MBX_E_INVALID, "dev_alloc: %lld bytes", (long long)bytes);
  if (c->capturing) return fail(MBX_E_INVALID, "dev_alloc inside a graph capture");
  HIPCHK(hipSetDevice(c->device));
  void* p = nullptr;
  if (hipMalloc(&p, (size_t)bytes) != hipSuccess) return fail(MBX_E_NOMEM, "dev_alloc: %lld bytes", (long long)bytes);
  hipError_t e = hipMemsetAsync(p, 0, (size_t)bytes, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    hipFree(p);
    return fail(MBX_E_DEVICE, "dev_alloc: %s", hipGetErrorString(e));
  }
  *dev = p;
  return MBX_OK;
}

extern "C" int mbx_dev_free(mbx_ctx* c, void* dev) {
  NOTNULL(c);
  if (!dev) return MBX_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipFree(dev));
  return MBX_OK;
}

extern "C" int mbx_dev_download(mbx_ctx* c, const void* dev, void* host, int64_t bytes) {
  NOTNULL(c);
  NOTNULL(dev);
  NOTNULL(host);
  if (bytes < 0) return fail(MBX_E_INVALID, "dev_download: %lld bytes", (long long)bytes);
  if (c->capturing) return fail(MBX_E_INVALID, "dev_download inside a graph capture");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(host, dev, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MBX_OK;
}

extern "C" int mbx_probe_read(mbx_ctx* c, const mbx_table* t, const int32_t* cols, int32_t ncols,
                              int64_t tiles_per_block, int32_t interleave, int64_t grid) {
  NOTNULL(c);
  NOTNULL(t);
  NOTNULL(cols);
  if (ncols < 1 || ncols > kMaxProbeCols) return fail(MBX_E_INVALID, "probe: ncols %d not in 1..%d", ncols, kMaxProbeCols);
  ProbeArgs A{};
  for (int i = 0; i < ncols; ++i) {
    if (cols[i] < 0 || cols[i] >= (int32_t)t->cols.size() || t->cols[cols[i]].stride_w != 1)
      return fail(MBX_E_INVALID, "probe: column %d is not a 4-byte column of the table", cols[i]);
    A.cols[i] = (const int32_t*)t->cols[cols[i]].dev;
  }
  A.ncols = ncols;
  A.interleave = interleave ? 1 : 0;
  A.nrows = t->nrows;
  A.tiles_per_block = tiles_per_block > 0 ? tiles_per_block : tiles_per_block_for(c, t->nrows);
  const int64_t ntiles = t->nrows / kTileRows;
  A.grid = interleave ? (grid > 0 ? grid : 1024) : (ntiles + A.tiles_per_block - 1) / A.tiles_per_block;
  if (A.grid < 1) A.grid = 1;
  if (A.grid > (1 << 20)) return fail(MBX_E_INVALID, "probe: grid %lld too large", (long long)A.grid);
  if (int rc = ensure_partials(c, A.grid)) return rc;
  A.sink = (uint32_t*)c->partials;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_read_probe(A, c->stream));
  return MBX_OK;
}

// ------------------------------------------------------------------ tables

int mbx::check_cols(const mbx_col_desc* cols, int32_t ncols) {
  if (ncols <= 0) return fail(MBX_E_INVALID, "table: ncols = %d", ncols);
  for (int32_t j = 0; j < ncols; j++) {
    const int32_t t = cols[j].attr_type;
    if (t != MBX_ATTR_INTEGER && t != MBX_ATTR_REAL && t != MBX_ATTR_STRING)
      return fail(MBX_E_TYPE, "table: column %d has AttrType %d (only attrInteger/attrReal/attrString are stored)",
                  j, t);
    if (t == MBX_ATTR_STRING && (cols[j].size <= 0 || cols[j].size > MBX_MAX_STR_BYTES))
      return fail(MBX_E_UNSUPPORTED, "table: column %d char(%d) outside 1..%d", j, cols[j].size,
                  MBX_MAX_STR_BYTES);
  }
  return MBX_OK;
}

int32_t mbx::stride_words(const mbx_col_desc& d) {
  return d.attr_type == MBX_ATTR_STRING ? (d.size + 3) / 4 : 1;
}

extern "C" int mbx_table_free(mbx_table* t) {
  if (!t) return MBX_OK;
  hipSetDevice(t->ctx->device);
  hipStreamSynchronize(t->ctx->stream);
  for (auto& c : t->cols)
    if (c.owned) hipFree(c.dev);
  for (auto& g : t->groups) hipFree(g.dev);
  if (t->owns_deleted) hipFree(t->deleted);
  delete t;
  return MBX_OK;
}

// Column group: a row-interleaved copy of 2..4 four-byte columns (row r's
// values side by side), built on the device and owned by the table.  The
// narrow gathers of a late materialisation (k_select_ids<4>, k_cnf_select)
// read a grouped column from the group, so the projected values of one row
// share a 128-byte line: a sparse gather (1 % of rows) touches ~15 % of the
// group's lines instead of ~28 % of every column's.
extern "C" int mbx_table_group(mbx_ctx* c, mbx_table* t, const int32_t* cols, int32_t ncols) {
  NOTNULL(c);
  NOTNULL(t);
  if (c->capturing) return fail(MBX_E_INVALID, "table_group: inside a graph capture (it allocates)");
  if (ncols == 0) {  // drop every group (a wrapped table's columns were rewritten: drop, then group again)
    int rc = set_device(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));  // no launch in flight still reads a group
    for (TGroup& g : t->groups) hipFree(g.dev);
    t->groups.clear();
    return MBX_OK;
  }
  NOTNULL(cols);
  if (ncols < 2 || ncols > 4) return fail(MBX_E_INVALID, "table_group: %d columns (2..4)", ncols);
  const uint32_t* src[4];
  for (int32_t k = 0; k < ncols; k++) {
    if (cols[k] < 0 || cols[k] >= (int32_t)t->cols.size())
      return fail(MBX_E_RANGE, "table_group: column %d outside 0..%zu", cols[k], t->cols.size() - 1);
    if (t->cols[(size_t)cols[k]].stride_w != 1)
      return fail(MBX_E_INVALID, "table_group: column %d is not a 4-byte column", cols[k]);
    for (int32_t j = 0; j < k; j++)
      if (cols[j] == cols[k]) return fail(MBX_E_INVALID, "table_group: column %d twice", cols[k]);
    for (const TGroup& g : t->groups)
      for (int32_t gc : g.cols)
        if (gc == cols[k]) return fail(MBX_E_INVALID, "table_group: column %d is already grouped", cols[k]);
    src[k] = (const uint32_t*)t->cols[(size_t)cols[k]].dev;
  }
  int rc = set_device(c);
  if (rc) return rc;
  TGroup g;
  g.cols.assign(cols, cols + ncols);
  const size_t bytes = sizeof(uint32_t) * (size_t)ncols * (size_t)(t->nrows > 0 ? t->nrows : 1);
  if (hipMalloc(&g.dev, bytes) != hipSuccess) return fail(MBX_E_NOMEM, "table_group: %zu bytes", bytes);
  hipError_t e = launch_group_build(src, ncols, t->nrows, g.dev, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    hipFree(g.dev);
    return fail(MBX_E_DEVICE, "table_group: %s", hipGetErrorString(e));
  }
  t->groups.push_back(g);
  return MBX_OK;
}

int mbx::table_alloc(mbx_ctx* c, const mbx_col_desc* cols, int32_t ncols, int64_t nrows, int64_t row_offset,
                     bool with_deleted, mbx_table** out) {
  *out = nullptr;
  int rc = check_cols(cols, ncols);
  if (rc) return rc;
  if (nrows < 0) return fail(MBX_E_INVALID, "table: nrows = %lld", (long long)nrows);
  if (row_offset < 0 || (row_offset & 63)) return fail(MBX_E_INVALID, "table: row_offset %lld not a multiple of 64",
                                                      (long long)row_offset);
  if ((rc = set_device(c))) return rc;
  mbx_table* t = new (std::nothrow) mbx_table();
  if (!t) return fail(MBX_E_NOMEM, "table: host allocation");
  t->ctx = c;
  t->nrows = nrows;
  t->row_offset = row_offset;
  const size_t n = (size_t)(nrows > 0 ? nrows : 1);
  for (int32_t j = 0; j < ncols; j++) {
    TCol col;
    col.attr_type = cols[j].attr_type;
    col.size = cols[j].attr_type == MBX_ATTR_STRING ? cols[j].size : 4;
    col.stride_w = stride_words(cols[j]);
    col.owned = true;
    const size_t bytes = n * (size_t)col.stride_w * 4;
    hipError_t e = hipMalloc(&col.dev, bytes);
    if (e != hipSuccess) {
      mbx_table_free(t);
      return fail(MBX_E_NOMEM, "table: column %d (%zu bytes): %s", j, bytes, hipGetErrorString(e));
    }
    t->cols.push_back(col);
  }
  if (with_deleted && nrows > 0) {
    const int64_t nw = words_for(nrows);
    hipError_t e = hipMalloc(&t->deleted, sizeof(uint64_t) * (size_t)nw);
    if (e != hipSuccess) {
      mbx_table_free(t);
      return fail(MBX_E_NOMEM, "table: deleted bitmap: %s", hipGetErrorString(e));
    }
    t->owns_deleted = true;
  }
  *out = t;
  return MBX_OK;
}

extern "C" int mbx_table_stage(mbx_ctx* c, const mbx_col_desc* cols, int32_t ncols, int64_t nrows,
                               const void* const* host_cols, const uint64_t* deleted_words, int64_t row_offset,
                               mbx_table** out) {
  NOTNULL(c);
  NOTNULL(cols);
  NOTNULL(host_cols);
  NOTNULL(out);
  *out = nullptr;
  mbx_table* t = nullptr;
  int rc = table_alloc(c, cols, ncols, nrows, row_offset, deleted_words != nullptr, &t);
  if (rc) return rc;
  for (int32_t j = 0; j < ncols && nrows > 0; j++) {
    const TCol& col = t->cols[j];
    if (!host_cols[j]) {
      mbx_table_free(t);
      return fail(MBX_E_INVALID, "table: host_cols[%d] is null", j);
    }
    hipError_t e;
    if (col.attr_type != MBX_ATTR_STRING) {
      e = hipMemcpy(col.dev, host_cols[j], (size_t)nrows * 4, hipMemcpyHostToDevice);
    } else {
      const int32_t stride = col.stride_w * 4;
      std::vector<uint8_t> img((size_t)nrows * (size_t)stride);
      const uint8_t* src = (const uint8_t*)host_cols[j];
      for (int64_t r = 0; r < nrows; r++)
        encode_device_string(src + (size_t)r * (size_t)col.size, col.size, img.data() + (size_t)r * (size_t)stride,
                             stride);
      e = hipMemcpy(col.dev, img.data(), img.size(), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
      mbx_table_free(t);
      return fail(MBX_E_DEVICE, "table: staging column %d: %s", j, hipGetErrorString(e));
    }
  }
  if (t->deleted) {
    const int64_t nw = words_for(nrows);
    std::vector<uint64_t> d(deleted_words, deleted_words + nw);
    if (nrows & 63) d[nw - 1] &= (1ull << (nrows & 63)) - 1ull;
    hipError_t e = hipMemcpy(t->deleted, d.data(), sizeof(uint64_t) * (size_t)nw, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      mbx_table_free(t);
      return fail(MBX_E_DEVICE, "table: staging deleted bitmap: %s", hipGetErrorString(e));
    }
  }
  *out = t;
  return MBX_OK;
}

extern "C" int mbx_table_wrap(mbx_ctx* c, const mbx_col_desc* cols, int32_t ncols, int64_t nrows,
                              const void* const* dev_cols, const uint64_t* dev_deleted_words, int64_t row_offset,
                              mbx_table** out) {
  NOTNULL(c);
  NOTNULL(cols);
  NOTNULL(dev_cols);
  NOTNULL(out);
  *out = nullptr;
  int rc = check_cols(cols, ncols);
  if (rc) return rc;
  if (nrows < 0 || row_offset < 0 || (row_offset & 63))
    return fail(MBX_E_INVALID, "table_wrap: nrows %lld row_offset %lld", (long long)nrows, (long long)row_offset);
  mbx_table* t = new (std::nothrow) mbx_table();
  if (!t) return fail(MBX_E_NOMEM, "table: host allocation");
  t->ctx = c;
  t->nrows = nrows;
  t->row_offset = row_offset;
  for (int32_t j = 0; j < ncols; j++) {
    if (!dev_cols[j] && nrows > 0) {
      delete t;
      return fail(MBX_E_INVALID, "table_wrap: dev_cols[%d] is null", j);
    }
    TCol col;
    col.attr_type = cols[j].attr_type;
    col.size = cols[j].attr_type == MBX_ATTR_STRING ? cols[j].size : 4;
    col.stride_w = stride_words(cols[j]);
    col.dev = const_cast<void*>(dev_cols[j]);
    col.owned = false;
    if (((uintptr_t)col.dev) & 15) t->aligned16 = false;
    t->cols.push_back(col);
  }
  t->deleted = const_cast<uint64_t*>(dev_deleted_words);
  t->owns_deleted = false;
  *out = t;
  return MBX_OK;
}

extern "C" int mbx_table_info(const mbx_table* t, int64_t* nrows, int64_t* row_offset, int32_t* ncols) {
  NOTNULL(t);
  if (nrows) *nrows = t->nrows;
  if (row_offset) *row_offset = t->row_offset;
  if (ncols) *ncols = (int32_t)t->cols.size();
  return MBX_OK;
}

// ------------------------------------------------------------------- plans

static int col_kind(int32_t attr) { return attr == MBX_ATTR_INTEGER ? kInt : (attr == MBX_ATTR_REAL ? kReal : kStr); }

static int slot_for(mbx_plan* p, int32_t col) {
  for (size_t s = 0; s < p->slot_col.size(); s++)
    if (p->slot_col[s] == col) return (int)s;
  if ((int)p->slot_col.size() >= kMaxCols) return -1;
  const TCol& tc = p->t->cols[(size_t)col];
  const int s = (int)p->slot_col.size();
  p->slot_col.push_back(col);
  p->host.cols[s].base = tc.dev;
  p->host.cols[s].kind = col_kind(tc.attr_type);
  p->host.cols[s].stride_w = tc.stride_w;
  p->host.ncols = s + 1;
  return s;
}

// PredEval's op table (R/iterator/PredEval.java:137-162) applied to a constant
// comparison result.
static bool op_on(int32_t op, int comp) {
  switch (op) {
    case MBX_OP_EQ: return comp == 0;
    case MBX_OP_LT: return comp < 0;
    case MBX_OP_GT: return comp > 0;
    case MBX_OP_NE:
    case MBX_OP_NOT: return comp != 0;
    case MBX_OP_LE: return comp <= 0;
    case MBX_OP_GE: return comp >= 0;
    default: return false;
  }
}

static int32_t cmp_op_of(int32_t op) {
  switch (op) {
    case MBX_OP_LT: return kLT;
    case MBX_OP_LE: return kLE;
    case MBX_OP_GT: return kGT;
    case MBX_OP_GE: return kGE;
    case MBX_OP_EQ: return kEQ;
    default: return kNE;  // aopNE, aopNOT
  }
}

// comp(lit, col) = -comp(col, lit): mirror the operator
static void int_range_of(KTerm& kt);
static void float_range_of(KTerm& kt);
static void str_range_of(KTerm& kt);

static int32_t flip(int32_t op) {
  switch (op) {
    case kLT: return kGT;
    case kLE: return kGE;
    case kGT: return kLT;
    case kGE: return kLE;
    default: return op;
  }
}

static int literal_type_ok(int32_t type) {
  return type == MBX_ATTR_INTEGER || type == MBX_ATTR_REAL || type == MBX_ATTR_STRING;
}

static int add_pool_string(mbx_plan* p, const mbx_operand& o, int32_t& words_used, KTerm& kt) {
  if (o.string_len < 0 || o.string_len > MBX_MAX_STR_BYTES || (o.string_len > 0 && !o.string))
    return fail(MBX_E_UNSUPPORTED, "plan: string literal of %d bytes (max %d)", o.string_len, MBX_MAX_STR_BYTES);
  const int32_t w = (o.string_len + 3) / 4;
  if (words_used + (w > 0 ? w : 1) > kMaxPoolWords)
    return fail(MBX_E_UNSUPPORTED, "plan: string literals exceed %d bytes", kMaxPoolWords * 4);
  uint8_t tmp[MBX_MAX_STR_BYTES + 4];
  encode_device_string((const uint8_t*)o.string, o.string_len, tmp, w * 4);
  memcpy(&p->host.pool[words_used], tmp, (size_t)w * 4);
  kt.soff = words_used;
  kt.swords = w;
  words_used += w > 0 ? w : 1;
  return MBX_OK;
}

static int compile_into(mbx_ctx* c, const mbx_table* t, const mbx_cnf* cnf, mbx_plan* p) {
  p->ctx = c;
  p->t = t;
  memset(&p->host, 0, sizeof(KPlan));
  p->host.agg_slot = -1;
  const int32_t ncols = (int32_t)t->cols.size();
  int32_t nconj = cnf ? cnf->nconj : 0;
  if (nconj < 0) return fail(MBX_E_INVALID, "plan: nconj = %d", nconj);
  if (nconj > MBX_MAX_CONJ) return fail(MBX_E_UNSUPPORTED, "plan: %d conjuncts (max %d)", nconj, MBX_MAX_CONJ);
  if (nconj > 0 && (!cnf->conds || !cnf->conj_offsets)) return fail(MBX_E_INVALID, "plan: null conds/conj_offsets");
  uint32_t all = 0;
  int32_t nterms = 0, pool_used = 0;
  for (int32_t ci = 0; ci < nconj; ci++) {
    const int32_t k0 = cnf->conj_offsets[ci], k1 = cnf->conj_offsets[ci + 1];
    if (k0 < 0 || k1 < k0) return fail(MBX_E_INVALID, "plan: conj_offsets not ascending at %d", ci);
    // always_true: a literal-vs-literal term that holds ends the conjunct's OR
    // list (PredEval.java:164-166); later terms are never evaluated
    bool always_true = false;
    const int32_t first_term = nterms;
    for (int32_t k = k0; k < k1; k++) {
      const mbx_condexpr& e = cnf->conds[k];
      const mbx_operand& o1 = e.operand1;
      const mbx_operand& o2 = e.operand2;
      if (e.op < MBX_OP_EQ || e.op > MBX_OP_RANGE) return fail(MBX_E_INVALID, "plan: AttrOperator %d", e.op);
      // comparison type from operand 1 (PredEval.java:54-91)
      int32_t ctype;
      if (o1.type == MBX_ATTR_SYMBOL) {
        if (o1.fld < 1 || o1.fld > ncols)
          return fail(MBX_E_RANGE, "plan: FldSpec offset %d outside 1..%d", o1.fld, ncols);
        ctype = t->cols[(size_t)o1.fld - 1].attr_type;
      } else if (literal_type_ok(o1.type)) {
        ctype = o1.type;
      } else {
        return fail(MBX_E_TYPE, "plan: operand1 AttrType %d", o1.type);
      }
      int32_t t2;
      if (o2.type == MBX_ATTR_SYMBOL) {
        if (o2.fld < 1 || o2.fld > ncols)
          return fail(MBX_E_RANGE, "plan: FldSpec offset %d outside 1..%d", o2.fld, ncols);
        t2 = t->cols[(size_t)o2.fld - 1].attr_type;
      } else if (literal_type_ok(o2.type)) {
        t2 = o2.type;
      } else {
        return fail(MBX_E_TYPE, "plan: operand2 AttrType %d", o2.type);
      }
      if (t2 != ctype)
        return fail(MBX_E_TYPE, "plan: term %d compares AttrType %d with %d (reference misreads the field)", k,
                    ctype, t2);
      if (always_true) continue;  // never reached; still type-checked above
      const bool real = ctype == MBX_ATTR_REAL;
      const bool never = e.op == MBX_OP_NOP || e.op == MBX_OP_RANGE;  // no case in the op switch: false
      const mbx_operand* lit = o2.type == MBX_ATTR_SYMBOL ? (o1.type == MBX_ATTR_SYMBOL ? nullptr : &o1) : &o2;
      // TupleUtils compares first and maps the operator after
      // (PredEval.java:131-162): a float compare with a NaN operand raises
      // whenever it is reached, whatever the operator.
      const bool nan_lit = lit && real && std::isnan(lit->real);
      KTerm kt;
      memset(&kt, 0, sizeof(kt));
      kt.conj_bit = 1u << ci;
      kt.rhs = -1;
      if (o1.type != MBX_ATTR_SYMBOL && o2.type != MBX_ATTR_SYMBOL) {
        // two literals share PredEval's `value` tuple: operand 2 vs itself
        if (real && std::isnan(o2.real)) {
          // raises wherever reached: a never-true float term that reads no
          // column (its slot is any one the plan streams anyway)
          const int s0 = p->slot_col.empty() ? slot_for(p, 0) : 0;
          if (s0 < 0) return fail(MBX_E_UNSUPPORTED, "plan: more than %d distinct columns", kMaxCols);
          if (nterms >= kMaxTerms) return fail(MBX_E_UNSUPPORTED, "plan: more than %d terms", kMaxTerms);
          kt.kind = kReal;
          kt.op = kNever;
          kt.lhs = s0;
          kt.nan_lit = 1;
          float_range_of(kt);  // empty: never true (it raises wherever reached)
          p->host.has_real = 1;
          p->host.terms[nterms++] = kt;
        } else if (!never && op_on(e.op, 0)) {
          always_true = true;
        }
        continue;
      }
      if (never && !real) continue;  // never true and cannot raise: dropped
      if (nterms >= kMaxTerms) return fail(MBX_E_UNSUPPORTED, "plan: more than %d terms", kMaxTerms);
      kt.kind = col_kind(ctype);
      int32_t op = never ? kNever : cmp_op_of(e.op);
      const mbx_operand* coln;
      if (o1.type == MBX_ATTR_SYMBOL) {
        coln = &o1;
        if (o2.type == MBX_ATTR_SYMBOL) {
          const int s2 = slot_for(p, o2.fld - 1);
          if (s2 < 0) return fail(MBX_E_UNSUPPORTED, "plan: more than %d distinct columns", kMaxCols);
          kt.rhs = s2;
          p->all_literal = false;
        }
      } else {
        coln = &o2;  // literal on the left: compare column with literal, operator mirrored
        op = flip(op);
      }
      const int s1 = slot_for(p, coln->fld - 1);
      if (s1 < 0) return fail(MBX_E_UNSUPPORTED, "plan: more than %d distinct columns", kMaxCols);
      kt.lhs = s1;
      kt.op = op;
      kt.nan_lit = nan_lit ? 1 : 0;
      if (kt.rhs < 0) {
        if (ctype == MBX_ATTR_INTEGER) {
          kt.ilit = lit->integer;
          int_range_of(kt);
        } else if (real) {
          kt.flit = lit->real;
          float_range_of(kt);
        } else {
          int rc = add_pool_string(p, *lit, pool_used, kt);
          if (rc) return rc;
          str_range_of(kt);
        }
      }
      if (ctype == MBX_ATTR_STRING && kt.rhs < 0 && kt.swords > 4) p->str_lit_fits16 = false;
      if (real) p->host.has_real = 1;
      p->host.terms[nterms++] = kt;
    }
    if (always_true) {
      // the conjunct holds for every row: it is not required, but the float
      // compares before the folding term still run for their NaN reach
      bool can_raise = false;
      for (int32_t i = first_term; i < nterms; i++) can_raise = can_raise || p->host.terms[i].kind == kReal;
      if (!can_raise) nterms = first_term;
      continue;
    }
    all |= 1u << ci;  // an empty conjunct stays required and is never satisfied
  }
  for (int32_t i = 0; i < nterms; i++) p->host.terms[i].req_below = all & (p->host.terms[i].conj_bit - 1u);
  p->host.nterms = nterms;
  p->host.all_conj = all;
  return MBX_OK;
}

// kt.op against kt.ilit as one unsigned range test: a OP lit holds iff
// ((uint32)a - (uint32)rlo <= rspan) != rneg -- the same truth table as the
// kernels' cmp4 for every int32 a (empty ranges: the full range negated)
static void int_range_of(KTerm& kt) {
  const int64_t lit = kt.ilit, mn = INT32_MIN, mx = INT32_MAX;
  int64_t lo = mn, hi = mx;
  bool neg = false, empty = false;
  switch (kt.op) {
    case kLT: empty = lit == mn; hi = lit - 1; break;
    case kLE: hi = lit; break;
    case kGT: empty = lit == mx; lo = lit + 1; break;
    case kGE: lo = lit; break;
    case kEQ: lo = hi = lit; break;
    case kNE: lo = hi = lit; neg = true; break;
    default: empty = true; break;  // kNever
  }
  if (empty) lo = mn, hi = mx, neg = true;
  kt.rlo = (int32_t)lo;
  kt.rspan = (uint32_t)hi - (uint32_t)(int32_t)lo;
  kt.rneg = neg ? 1 : 0;
  kt.rm31 = 0;
}

static void set_key_range(KTerm& kt, int64_t lo, int64_t hi, bool neg, uint32_t rm31) {
  if (lo > hi) lo = INT32_MIN, hi = INT32_MAX, neg = true;  // empty
  kt.rlo = (int32_t)lo;
  kt.rspan = (uint32_t)(int32_t)hi - (uint32_t)(int32_t)lo;
  kt.rneg = neg ? 1 : 0;
  kt.rm31 = rm31;
}

// float `a OP lit` over the signed-ordered key of a (KTerm.rm31): the kernels'
// cmp4<float> IEEE truth table for every non-NaN a (-0.0 == +0.0); a NaN row
// that reaches the term raises whatever the range says (nan_lit: empty)
static int32_t float_key(float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  return (int32_t)(b ^ ((uint32_t)((int32_t)b >> 31) & 0x7fffffffu));
}

static void float_range_of(KTerm& kt) {
  const int64_t ninf = float_key(-INFINITY), pinf = float_key(INFINITY);
  const float lit = kt.flit;
  if (kt.nan_lit || std::isnan(lit) || kt.op == kNever) return set_key_range(kt, 1, 0, false, 0x7fffffffu);
  const int64_t elo = lit == 0.0f ? float_key(-0.0f) : float_key(lit);
  const int64_t ehi = lit == 0.0f ? float_key(0.0f) : float_key(lit);
  switch (kt.op) {
    case kLT: return set_key_range(kt, ninf, elo - 1, false, 0x7fffffffu);
    case kLE: return set_key_range(kt, ninf, ehi, false, 0x7fffffffu);
    case kGT: return set_key_range(kt, ehi + 1, pinf, false, 0x7fffffffu);
    case kGE: return set_key_range(kt, elo, pinf, false, 0x7fffffffu);
    case kEQ: return set_key_range(kt, elo, ehi, false, 0x7fffffffu);
    default: return set_key_range(kt, elo, ehi, true, 0x7fffffffu);  // kNE
  }
}

// char(n) `s OP lit`: the compareTo sign c in {-1, 0, 1} against 0
static void str_range_of(KTerm& kt) {
  switch (kt.op) {
    case kLT: return set_key_range(kt, -1, -1, false, 0);
    case kLE: return set_key_range(kt, -1, 0, false, 0);
    case kGT: return set_key_range(kt, 1, 1, false, 0);
    case kGE: return set_key_range(kt, 0, 1, false, 0);
    case kEQ: return set_key_range(kt, 0, 0, false, 0);
    case kNE: return set_key_range(kt, 0, 0, true, 0);
    default: return set_key_range(kt, 1, 0, false, 0);  // kNever
  }
}

static int plan_variant(mbx_plan* p, int32_t agg_col, PlanVariant** out) {
  for (auto& v : p->variants)
    if (v.agg_col == agg_col) {
      *out = &v;
      return MBX_OK;
    }
  PlanVariant v;
  v.agg_col = agg_col;
  KPlan kp = p->host;
  std::vector<int32_t> slots = p->slot_col;
  if (agg_col >= 0) {
    const int32_t at = p->t->cols[(size_t)agg_col].attr_type;
    if (at != MBX_ATTR_INTEGER && at != MBX_ATTR_REAL)
      return fail(MBX_E_TYPE, "aggregate: column %d is not attrInteger/attrReal", agg_col);
    v.agg_kind = at == MBX_ATTR_REAL ? kReal : kInt;
    int s = -1;
    for (size_t i = 0; i < slots.size(); i++)
      if (slots[i] == agg_col) s = (int)i;
    if (s < 0) {
      if ((int)slots.size() >= kMaxCols) return fail(MBX_E_UNSUPPORTED, "aggregate: too many columns");
      s = (int)slots.size();
      slots.push_back(agg_col);
      const TCol& tc = p->t->cols[(size_t)agg_col];
      kp.cols[s].base = tc.dev;
      kp.cols[s].kind = col_kind(tc.attr_type);
      kp.cols[s].stride_w = tc.stride_w;
      kp.ncols = s + 1;
    }
    kp.agg_slot = s;
  }
  // Fast kernel eligibility: every term `column OP literal`, 16-byte aligned
  // columns, <= 4 four-byte slots and <= 2 char(13..16) slots whose literals
  // fit 16 bytes.  Slots are renumbered 4-byte first, strings after.
  bool fast = p->all_literal && p->str_lit_fits16 && p->t->aligned16 && !p->ctx->tune.force_generic;
  std::vector<int> four, wide;
  for (size_t i = 0; i < slots.size(); i++) {
    const TCol& tc = p->t->cols[slots[i]];
    if (tc.attr_type != MBX_ATTR_STRING) four.push_back((int)i);
    else if (tc.stride_w == 4) wide.push_back((int)i);
    else fast = false;
  }
  if (four.size() > 4 || wide.size() > 2 || four.size() + wide.size() > 4) fast = false;
  if (fast && !slots.empty()) {
    std::vector<int> order(four);
    order.insert(order.end(), wide.begin(), wide.end());
    std::vector<int> newpos(slots.size());
    KPlan q = kp;
    for (size_t k = 0; k < order.size(); k++) {
      newpos[(size_t)order[k]] = (int)k;
      q.cols[k] = kp.cols[order[k]];
    }
    for (int ti = 0; ti < kp.nterms; ti++) q.terms[ti].lhs = newpos[(size_t)kp.terms[ti].lhs];
    if (kp.agg_slot >= 0) q.agg_slot = newpos[(size_t)kp.agg_slot];
    kp = q;
    v.fast_k = (int32_t)four.size();
    v.fast_ks = (int32_t)wide.size();
  }
  const bool all4 = fast && wide.empty();
  if (all4 && slots.empty()) {
    // no column referenced (no filter, or only constant terms): slot 0 is
    // any 4-byte column so the fast kernel has something to stream
    for (size_t j = 0; j < p->t->cols.size(); j++)
      if (p->t->cols[j].attr_type != MBX_ATTR_STRING) {
        kp.cols[0].base = p->t->cols[j].dev;
        kp.cols[0].kind = col_kind(p->t->cols[j].attr_type);
        kp.cols[0].stride_w = 1;
        kp.ncols = 1;
        v.fast_k = 1;
        break;
      }
  }
  hipError_t e = hipMalloc(&v.dev, sizeof(KPlan));
  if (e == hipSuccess) e = hipMemcpy(v.dev, &kp, sizeof(KPlan), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    hipFree(v.dev);
    return fail(MBX_E_DEVICE, "plan upload: %s", hipGetErrorString(e));
  }
  p->variants.push_back(v);  // std::deque: earlier PlanVariant pointers stay valid
  *out = &p->variants.back();
  return MBX_OK;
}

extern "C" int mbx_plan_compile(mbx_ctx* c, const mbx_table* t, const mbx_cnf* cnf, mbx_plan** out) {
  NOTNULL(c);
  NOTNULL(t);
  NOTNULL(out);
  *out = nullptr;
  int rc = set_device(c);
  if (rc) return rc;
  mbx_plan* p = new (std::nothrow) mbx_plan();
  if (!p) return fail(MBX_E_NOMEM, "plan: host allocation");
  rc = compile_into(c, t, cnf, p);
  PlanVariant* v = nullptr;
  if (!rc) rc = plan_variant(p, -1, &v);
  if (rc) {
    mbx_plan_free(p);
    return rc;
  }
  *out = p;
  return MBX_OK;
}

extern "C" int mbx_plan_free(mbx_plan* p) {
  if (!p) return MBX_OK;
  hipSetDevice(p->ctx->device);
  hipStreamSynchronize(p->ctx->stream);
  for (auto& v : p->variants) hipFree(v.dev);
  delete p;
  return MBX_OK;
}

// ------------------------------------------------------------------- scans

// kFinPackedCount's 64-bit ticket words hold < 4096 arrivals and NaN blocks
// per word and a 40-bit count (mbx_kernels.hip, packed_count_finalize).
static bool packed_count_fits(int64_t nrows, int64_t nb, int32_t groups) {
  const int64_t per_word = (groups > 1 && nb > groups) ? std::max<int64_t>((nb + groups - 1) / groups, groups) : nb;
  return per_word < 4096 && nrows < (int64_t(1) << 40);
}

// One launch per scan: the kernel's last block finalizes (count / aggregate /
// NaN flag) through the context's ticket.
static int32_t ticket_groups_of(const mbx_ctx* c) {
  const int32_t g = c->tune.ticket_groups >= 0 ? c->tune.ticket_groups : kDefaultTicketGroups;
  return g > kMaxTicketGroups ? kDefaultTicketGroups : g;
}

// k_scan_select's extra arguments (a BitSet scan that also writes the positions)
struct FusedSelect {
  int64_t* ids;
  int64_t* total;
};

static int enqueue_scan(mbx_ctx* c, const mbx_plan* p, const PlanVariant& v, int32_t mode, uint64_t* out_words,
                        Partial* parts, int64_t tpb, int64_t* count_out, AggOut* agg_out, int32_t* nan_out,
                        int64_t* seg_counts = nullptr, const FusedSelect* fused = nullptr,
                        bool need_count = true, bool frame = false) {
  ScanLaunch L;
  L.plan = v.dev;
  L.nrows = p->t->nrows;
  L.tiles_per_block = tpb;
  L.deleted = p->t->deleted;
  L.out_words = out_words;
  L.partials = parts;
  L.mode = mode;
  L.fast_k = v.fast_k;
  L.fast_ks = v.fast_ks;
  L.agg_kind = v.agg_kind;
  L.ticket = c->ticket;
  L.count_out = count_out;
  L.agg_out = agg_out;
  L.nan_out = nan_out;
  const MbxTuning& tu = c->tune;
  L.nterms_host = p->host.nterms;
  L.hoist_terms = p->host.nterms >= 1 && p->host.nterms <= kHoistTerms && tu.scan_hoist != 0;
  // tile layout: row-interleaved for BitSet output (the ballots are the words)
  L.ri = tu.scan_ri == 2 || (tu.scan_ri == 1 && mode == kModeBitmap);
  // BitSet words staged in LDS per block when the segment fits; the fast
  // kernel's RI BitSet form only.  Measured: 100 M rows (382 tiles per block)
  // 79.1 -> 77.6 us; 10 M / 12.5 M rows (<= 48 tiles per block) +0.2 us, so
  // small segments keep the direct stores (profiles/r01/round_i/sink_lds)
  const bool sink_fits = mode == kModeBitmap && L.ri && v.fast_k + v.fast_ks > 0 &&
                         tpb * kWordsPerTile * (int64_t)sizeof(uint64_t) <= kSinkLdsMaxBytes;
  L.sink_lds = sink_fits && (tu.sink_lds == 2 || (tu.sink_lds == 1 && tpb >= 128));
  L.ticket_groups = ticket_groups_of(c);
  L.seg_counts = seg_counts;
  L.words_wt = tu.scan_words_wt;
  L.int_range = 0;
  if (tu.scan_int_range && p->host.nterms >= 1) {
    bool ints = true, lits = true;
    for (int32_t i = 0; i < p->host.nterms; i++) {
      ints = ints && p->host.terms[i].kind == kInt;
      lits = lits && p->host.terms[i].rhs < 0;
    }
    if (lits && ints && !p->host.has_real && v.fast_ks == 0)
      L.int_range = 1;
    // typed range tests (float / char(16) terms too): COUNT and aggregate scans
    // of up to kHoistTerms terms, knob value 2 or more
    else if (lits && tu.scan_int_range >= 2 && mode != kModeBitmap && p->host.nterms <= kHoistTerms)
      L.int_range = 2;
  }
  L.fin_mode = tu.fin_mode >= 0 ? tu.fin_mode : (mode != kModeAgg ? kFinPackedCount : kFinWriteThrough);
  // aggregates over more blocks than the chip holds at once (string-slot
  // plans, ~4096 blocks): each block's drained write-through partial and
  // ticket round trip hold its slot from the next block, four rounds per
  // slot -- plain partial stores and a separate fold launch instead (C5 125 M
  // rows: scan 472.7 -> 458.4 us + a 6 us fold, query 481 -> 471 us,
  // profiles/r03/c5fin)
  if (tu.fin_mode < 0 && mode == kModeAgg && grid_blocks(L.nrows, tpb) > kResidentBlocks) L.fin_mode = kFinSeparate;
  if (L.fin_mode == kFinPackedCount && !packed_count_fits(L.nrows, grid_blocks(L.nrows, tpb), L.ticket_groups))
    L.fin_mode = kFinWriteThrough;
  if ((L.fin_mode == kFinPackedCount || L.fin_mode == kFinSegOnly) && mode == kModeAgg) L.fin_mode = kFinWriteThrough;
  if (L.fin_mode > kFinSegOnly) L.fin_mode = kFinWriteThrough;
  // a BitSet whose count nobody reads from this launch (the async BitSet /
  // select entry points count it from its segment counts when asked) and a
  // plan with no float term (no NaN to report): no finalize at all -- its
  // ticket round trips are ~1 us at the end of every launch (10 M rows:
  // 10.7 -> 9.7 us, profiles/r03/fin)
  if (!need_count && (mode == kModeBitmap || mode == kModeCount) && seg_counts && !p->host.has_real &&
      tu.fin_mode < 0)
    L.fin_mode = kFinSegOnly;
  if (frame) {  // mbx_scan_count_frame_async: count_out is the frame
    L.fin_mode = kFinFrame;
    L.ticket = nullptr;
  }
  if (L.fin_mode == kFinSeparate) L.ticket = nullptr;
  if (fused) {
    int64_t* stamps = nullptr;
    if (c->tune.select_dbg & 8) {  // diagnostic stamps (mbx_diag_select_stamps)
      if (!c->stamps) HIPCHK(hipMalloc(&c->stamps, sizeof(int64_t) * 4 * kMaxStampBlocks));
      stamps = c->stamps;
    }
    HIPCHK(launch_scan_select(L, c->lookback, p->t->row_offset, fused->ids, fused->total, c->stream, stamps,
                              c->tune.select_dbg >> 4, c->tune.scan_select_waves, c->tune.select_flag_stride));
    return MBX_OK;
  }
  HIPCHK(launch_scan(L, c->stream));
  if (L.fin_mode == kFinSeparate)
    HIPCHK(launch_finalize(parts, grid_blocks(L.nrows, tpb), L.agg_kind, agg_out, count_out, nan_out, c->stream));
  return MBX_OK;
}

static int scan_to_count(mbx_ctx* c, mbx_plan* p, int64_t* dev_count, int32_t* dev_nan) {
  PlanVariant* v = nullptr;
  int rc = plan_variant(p, -1, &v);
  if (rc) return rc;
  const int64_t tpb = scan_tiles_per_block(c, p->t->nrows, *v);
  const int64_t nb = grid_blocks(p->t->nrows, tpb);
  if ((rc = ensure_partials(c, nb))) return rc;
  return enqueue_scan(c, p, *v, kModeCount, nullptr, c->partials, tpb, dev_count, nullptr, dev_nan);
}

// NaN words: the *_async entry points report through dnan[0..1] ([1] sticky
// until mbx_sync); the synchronous ones read their own flag, dnan[2], so a
// NaN they already raised is not reported again by mbx_sync
static int32_t* nan_sync(mbx_ctx* c) { return c->dnan + 2; }

static int check_nan(mbx_ctx* c) {
  const int32_t* h = (const int32_t*)c->pinned;
  if (h[8]) return fail(MBX_E_TYPE, "NaN in a float comparison (TupleUtils falls through to the string compare and raises)");
  return MBX_OK;
}

extern "C" int mbx_scan_count(mbx_ctx* c, const mbx_plan* pc, int64_t* count) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(count);
  mbx_plan* p = const_cast<mbx_plan*>(pc);
  int rc = set_device(c);
  if (rc) return rc;
  if ((rc = scan_to_count(c, p, c->dcount, nan_sync(c)))) return rc;
  int64_t* h = (int64_t*)c->pinned;
  HIPCHK(hipMemcpyAsync(h, c->dcount, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync((int32_t*)c->pinned + 8, nan_sync(c), sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *count = h[0];
  return check_nan(c);
}

bool mbx::plan_has_real(const mbx_plan* p) { return p->host.has_real != 0; }

int mbx::scan_count_parts(mbx_ctx* c, const mbx_plan* pc, int64_t* dev_parts, int64_t cap, int64_t* nparts) {
  mbx_plan* p = const_cast<mbx_plan*>(pc);
  if (p->host.has_real)
    return fail(MBX_E_INVALID, "scan_count_parts: a plan with a float term needs the in-launch finalize (NaN)");
  PlanVariant* v = nullptr;
  int rc = plan_variant(p, -1, &v);
  if (rc) return rc;
  const int64_t tpb = scan_tiles_per_block(c, p->t->nrows, *v);
  const int64_t nb = grid_blocks(p->t->nrows, tpb);
  if (nb > cap) return fail(MBX_E_INVALID, "scan_count_parts: %lld blocks, capacity %lld", (long long)nb, (long long)cap);
  if ((rc = ensure_partials(c, nb))) return rc;
  *nparts = nb;
  return enqueue_scan(c, p, *v, kModeCount, nullptr, c->partials, tpb, nullptr, nullptr, c->dnan, dev_parts, nullptr,
                      false);
}

extern "C" int mbx_scan_count_async(mbx_ctx* c, const mbx_plan* pc, int64_t* dev_count) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(dev_count);
  return scan_to_count(c, const_cast<mbx_plan*>(pc), dev_count, c->dnan);
}

// a frame slot holds < 4096 arrivals (and NaN blocks) summed over every rank
// that adds into it: ceil(blocks / 32) <= 255 keeps 16 ranks' frames exact
constexpr int64_t kFrameMaxArrivalsPerSlot = 255;

extern "C" int mbx_scan_count_frame_async(mbx_ctx* c, const mbx_plan* pc, int64_t* dev_frame) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(dev_frame);
  static_assert(kFrameSlots * kFrameSlotStride == MBX_COUNT_FRAME_WORDS, "count frame layout");
  mbx_plan* p = const_cast<mbx_plan*>(pc);
  if ((reinterpret_cast<uintptr_t>(dev_frame) & 127) != 0)
    return fail(MBX_E_INVALID, "scan_count_frame: the frame must be 128-byte aligned");
  int rc = set_device(c);
  if (rc) return rc;
  PlanVariant* v = nullptr;
  if ((rc = plan_variant(p, -1, &v))) return rc;
  const int64_t tpb = scan_tiles_per_block(c, p->t->nrows, *v);
  const int64_t nb = grid_blocks(p->t->nrows, tpb);
  if ((nb + kFrameSlots - 1) / kFrameSlots > kFrameMaxArrivalsPerSlot || p->t->nrows >= (int64_t(1) << 36))
    return fail(MBX_E_INVALID, "scan_count_frame: %lld rows in %lld blocks do not fit a count frame",
                (long long)p->t->nrows, (long long)nb);
  if ((rc = ensure_partials(c, nb))) return rc;
  return enqueue_scan(c, p, *v, kModeCount, nullptr, c->partials, tpb, dev_frame, nullptr, c->dnan, nullptr, nullptr,
                      true, true);
}

extern "C" int mbx_count_frame_fits(int64_t nblocks, int32_t nranks) {
  if (nblocks < 0 || nranks <= 0) return 0;
  const int64_t per_slot = (nblocks + kFrameSlots - 1) / kFrameSlots;
  return per_slot <= kFrameMaxArrivalsPerSlot && per_slot * nranks < 4096 ? 1 : 0;
}

extern "C" int mbx_count_frame_decode(const int64_t* frame, int64_t* count, int64_t* nan_blocks, int64_t* arrivals) {
  NOTNULL(frame);
  NOTNULL(count);
  int64_t n = 0, nan = 0, arr = 0;
  for (int s = 0; s < kFrameSlots; ++s) {
    const uint64_t w = (uint64_t)frame[(size_t)s * kFrameSlotStride];
    n += (int64_t)(w >> 24);
    nan += (int64_t)((w >> 12) & 0xfff);
    arr += (int64_t)(w & 0xfff);
  }
  *count = n;
  if (nan_blocks) *nan_blocks = nan;
  if (arrivals) *arrivals = arr;
  return MBX_OK;
}

extern "C" int mbx_scan_blocks(mbx_ctx* c, const mbx_plan* pc, int64_t* blocks) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(blocks);
  mbx_plan* p = const_cast<mbx_plan*>(pc);
  PlanVariant* v = nullptr;
  int rc = plan_variant(p, -1, &v);
  if (rc) return rc;
  *blocks = grid_blocks(p->t->nrows, scan_tiles_per_block(c, p->t->nrows, *v));
  return MBX_OK;
}

static int scan_bitmap_into(mbx_ctx* c, mbx_plan* p, mbx_bitmap* b, int32_t* dev_nan, bool need_count = true) {
  if (b->nbits != p->t->nrows)
    return fail(MBX_E_INVALID, "scan_bitmap: bitmap has %lld bits, table %lld rows", (long long)b->nbits,
                (long long)p->t->nrows);
  PlanVariant* v = nullptr;
  int rc = plan_variant(p, -1, &v);
  if (rc) return rc;
  const int64_t tpb = b->wpb / kWordsPerTile;
  if (grid_blocks(p->t->nrows, tpb) != b->nseg) return fail(MBX_E_INVALID, "scan_bitmap: segment mismatch");
  if ((rc = ensure_partials(c, b->nseg))) return rc;
  return enqueue_scan(c, p, *v, kModeBitmap, b->words, c->partials, tpb, c->dcount, nullptr, dev_nan, b->segc,
                      nullptr, need_count);
}

// read back the count + NaN flag the last scan's final block wrote
static int scan_result_sync(mbx_ctx* c, int64_t* count) {
  int64_t* h = (int64_t*)c->pinned;
  HIPCHK(hipMemcpyAsync(h, c->dcount, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync((int32_t*)c->pinned + 8, nan_sync(c), sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *count = h[0];
  return MBX_OK;
}

extern "C" int mbx_scan_bitmap_async(mbx_ctx* c, const mbx_plan* pc, mbx_bitmap* out) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(out);
  out->count = -1;
  return scan_bitmap_into(c, const_cast<mbx_plan*>(pc), out, c->dnan, false);
}

static int materialize_dev(mbx_ctx* c, const mbx_table* t, const mbx_bitmap* sel, const int32_t* proj,
                           int32_t nproj, int64_t row_offset, int64_t* dev_ids, void* const* dev_out,
                           int64_t* dev_total);

// BitSet + ascending positions.  Default (tuning scan_select_fused = 1): ONE
// launch, k_scan_select -- the scan writes the BitSet words and each block
// finds its output offset by decoupled look-back, then emits its positions --
// for plans of 1..4 int literal terms on 4-byte columns whose segments fit
// (scan_select_fusable).  Every other plan (float / string terms, symbol-vs-
// symbol terms, scan_select_fused = 0) takes the two-launch form: the BitSet
// scan, then k_select_ids over its segment counts.  dev_ids holds every row's
// position.
static int scan_select_into(mbx_ctx* c, mbx_plan* p, mbx_bitmap* b, int64_t* dev_ids, int64_t* dev_count,
                            int32_t* dev_nan) {
  if (c->tune.scan_select_fused && b->nbits == p->t->nrows) {
    // one launch (k_scan_select): int literal terms on <= 4 four-byte columns
    PlanVariant* v = nullptr;
    int rc = plan_variant(p, -1, &v);
    if (rc) return rc;
    const int64_t tpb = b->wpb / kWordsPerTile;
    if (c->tune.scan_ri != 0 && p->all_literal &&
        scan_select_fusable(p->t->nrows, tpb, v->fast_k, v->fast_ks, p->host.nterms, p->host.has_real,
                            c->tune.scan_select_waves) &&
        grid_blocks(p->t->nrows, tpb) == b->nseg) {
      const FusedSelect f{dev_ids, dev_count};
      return enqueue_scan(c, p, *v, kModeBitmap, b->words, c->partials, tpb, dev_count, nullptr, dev_nan, b->segc, &f);
    }
  }
  int rc = scan_bitmap_into(c, p, b, dev_nan, false);
  if (rc) return rc;
  return materialize_dev(c, p->t, b, nullptr, 0, p->t->row_offset, dev_ids, nullptr, dev_count);
}

extern "C" int mbx_scan_select_async(mbx_ctx* c, const mbx_plan* pc, mbx_bitmap* out, int64_t* dev_ids,
                                     int64_t* dev_count) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(out);
  NOTNULL(dev_ids);
  NOTNULL(dev_count);
  int rc = set_device(c);
  if (rc) return rc;
  out->count = -1;
  return scan_select_into(c, const_cast<mbx_plan*>(pc), out, dev_ids, dev_count, c->dnan);
}

extern "C" int mbx_scan_select(mbx_ctx* c, const mbx_plan* pc, int64_t* host_ids, int64_t cap, int64_t* n) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(n);
  *n = 0;
  if (cap < 0) return fail(MBX_E_INVALID, "scan_select: capacity %lld", (long long)cap);
  mbx_plan* p = const_cast<mbx_plan*>(pc);
  int rc = set_device(c);
  if (rc) return rc;
  const int64_t nrows = p->t->nrows;
  mbx_bitmap* b = nullptr;
  if ((rc = bitmap_new(c, nrows, &b))) return rc;
  // device positions: the count, once the BitSet scan has it (at most the
  // caller's capacity), allocated for this call only
  int64_t* d = nullptr;
  int64_t count = 0;
  if (!(rc = scan_bitmap_into(c, p, b, nan_sync(c))) && !(rc = scan_result_sync(c, &count)) &&
      !(rc = check_nan(c)) && count > 0 && count <= cap) {
    if (hipMalloc(&d, sizeof(int64_t) * (size_t)count) != hipSuccess)
      rc = fail(MBX_E_NOMEM, "scan_select: %lld positions of device scratch", (long long)count);
    else
      rc = materialize_dev(c, p->t, b, nullptr, 0, p->t->row_offset, d, nullptr, c->dcount);
  }
  if (!rc && count > cap)
    rc = fail(MBX_E_INVALID, "scan_select: %lld positions, capacity %lld", (long long)count, (long long)cap);
  if (!rc && count > 0) {
    if (!host_ids) rc = fail(MBX_E_INVALID, "scan_select: null host_ids");
    else {
      hipError_t e = hipMemcpyAsync(host_ids, d, (size_t)count * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
      if (e != hipSuccess) rc = fail(MBX_E_DEVICE, "scan_select: %s", hipGetErrorString(e));
    }
  }
  hipStreamSynchronize(c->stream);
  if (d) hipFree(d);
  mbx_bitmap_free(b);
  if (rc) return rc;
  *n = count;
  return MBX_OK;
}

static int bitmap_count_sync(mbx_ctx* c, mbx_bitmap* b, bool with_nan) {
  (void)with_nan;  // segment counts carry no NaN flag: scans report theirs through their own finalize
  HIPCHK(launch_count_sum(b->segc, b->nseg, c->dcount, c->stream));
  int64_t* h = (int64_t*)c->pinned;
  HIPCHK(hipMemcpyAsync(h, c->dcount, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  b->count = h[0];
  return MBX_OK;
}

int mbx::bitmap_recount(mbx_ctx* c, mbx_bitmap* b) {
  HIPCHK(launch_seg_popcount(b->words, b->nwords, b->wpb, b->segc, c->stream));
  return bitmap_count_sync(c, b, false);
}

extern "C" int mbx_scan_bitmap(mbx_ctx* c, const mbx_plan* pc, mbx_bitmap** out, int64_t* count) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(out);
  *out = nullptr;
  mbx_plan* p = const_cast<mbx_plan*>(pc);
  int rc = set_device(c);
  if (rc) return rc;
  mbx_bitmap* b = nullptr;
  if ((rc = bitmap_new(c, p->t->nrows, &b))) return rc;
  if (!(rc = scan_bitmap_into(c, p, b, nan_sync(c))) && !(rc = scan_result_sync(c, &b->count))) rc = check_nan(c);
  if (rc) {
    mbx_bitmap_free(b);
    return rc;
  }
  if (count) *count = b->count;
  *out = b;
  return MBX_OK;
}

static int scan_agg(mbx_ctx* c, mbx_plan* p, int32_t agg_col, AggOut* dev_out, int32_t* dev_nan) {
  if (agg_col < 0 || agg_col >= (int32_t)p->t->cols.size())
    return fail(MBX_E_RANGE, "aggregate: column %d outside 0..%zu", agg_col, p->t->cols.size() - 1);
  PlanVariant* v = nullptr;
  int rc = plan_variant(p, agg_col, &v);
  if (rc) return rc;
  const int64_t tpb = scan_tiles_per_block(c, p->t->nrows, *v);
  const int64_t nb = grid_blocks(p->t->nrows, tpb);
  if ((rc = ensure_partials(c, nb))) return rc;
  return enqueue_scan(c, p, *v, kModeAgg, nullptr, c->partials, tpb, nullptr, dev_out, dev_nan);
}

extern "C" int mbx_scan_aggregate(mbx_ctx* c, const mbx_plan* pc, int32_t agg_col, mbx_agg* out) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(out);
  static_assert(sizeof(mbx_agg) == sizeof(AggOut), "mbx_agg layout");
  int rc = set_device(c);
  if (rc) return rc;
  if ((rc = scan_agg(c, const_cast<mbx_plan*>(pc), agg_col, c->dagg, nan_sync(c)))) return rc;
  HIPCHK(hipMemcpyAsync(c->pinned, c->dagg, sizeof(AggOut), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync((int32_t*)c->pinned + 16, nan_sync(c), sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  memcpy(out, c->pinned, sizeof(mbx_agg));
  if (((const int32_t*)c->pinned)[16])
    return fail(MBX_E_TYPE, "NaN in a float comparison (TupleUtils falls through to the string compare and raises)");
  return MBX_OK;
}

extern "C" int mbx_scan_aggregate_async(mbx_ctx* c, const mbx_plan* pc, int32_t agg_col, mbx_agg* dev_out) {
  NOTNULL(c);
  NOTNULL(pc);
  NOTNULL(dev_out);
  return scan_agg(c, const_cast<mbx_plan*>(pc), agg_col, (AggOut*)dev_out, c->dnan);
}

// ----------------------------------------------------------------- bitmaps

extern "C" int mbx_bitmap_alloc(mbx_ctx* c, int64_t nbits, mbx_bitmap** out) {
  NOTNULL(c);
  NOTNULL(out);
  *out = nullptr;
  if (nbits < 0) return fail(MBX_E_INVALID, "bitmap: nbits %lld", (long long)nbits);
  int rc = set_device(c);
  if (rc) return rc;
  return bitmap_new(c, nbits, out);
}

extern "C" int mbx_bitmap_free(mbx_bitmap* b) {
  if (!b) return MBX_OK;
  hipSetDevice(b->ctx->device);
  hipStreamSynchronize(b->ctx->stream);
  hipFree(b->words);
  hipFree(b->segc);
  delete b;
  return MBX_OK;
}

extern "C" int mbx_bitmap_upload(mbx_ctx* c, int64_t nbits, const uint64_t* host_words, mbx_bitmap** out) {
  NOTNULL(c);
  NOTNULL(out);
  *out = nullptr;
  if (nbits < 0) return fail(MBX_E_INVALID, "bitmap: nbits %lld", (long long)nbits);
  if (nbits > 0 && !host_words) return fail(MBX_E_INVALID, "bitmap_upload: null words");
  int rc = set_device(c);
  if (rc) return rc;
  mbx_bitmap* b = nullptr;
  if ((rc = bitmap_new(c, nbits, &b))) return rc;
  if (b->nwords > 0) {
    hipError_t e = hipMemcpy(b->words, host_words, sizeof(uint64_t) * (size_t)b->nwords, hipMemcpyHostToDevice);
    if (e == hipSuccess && (nbits & 63)) {
      const uint64_t last = host_words[b->nwords - 1] & ((1ull << (nbits & 63)) - 1ull);
      e = hipMemcpy(b->words + b->nwords - 1, &last, sizeof(uint64_t), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
      mbx_bitmap_free(b);
      return fail(MBX_E_DEVICE, "bitmap_upload: %s", hipGetErrorString(e));
    }
  }
  hipError_t e = launch_seg_popcount(b->words, b->nwords, b->wpb, b->segc, c->stream);
  if (e != hipSuccess || (rc = bitmap_count_sync(c, b, false))) {
    mbx_bitmap_free(b);
    return rc ? rc : fail(MBX_E_DEVICE, "bitmap_upload: %s", hipGetErrorString(e));
  }
  *out = b;
  return MBX_OK;
}

extern "C" int mbx_bitmap_download(mbx_ctx* c, const mbx_bitmap* b, uint64_t* host_words, int64_t nwords) {
  NOTNULL(c);
  NOTNULL(b);
  if (nwords < b->nwords) return fail(MBX_E_INVALID, "bitmap_download: need %lld words", (long long)b->nwords);
  if (b->nwords == 0) return MBX_OK;
  NOTNULL(host_words);
  int rc = set_device(c);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(host_words, b->words, sizeof(uint64_t) * (size_t)b->nwords, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MBX_OK;
}

extern "C" int mbx_bitmap_info(const mbx_bitmap* b, int64_t* nbits, int64_t* nwords, int64_t* count) {
  NOTNULL(b);
  if (nbits) *nbits = b->nbits;
  if (nwords) *nwords = b->nwords;
  if (count) *count = b->count;
  return MBX_OK;
}

extern "C" int mbx_bitmap_combine(mbx_ctx* c, int32_t op, const mbx_bitmap* a, const mbx_bitmap* b,
                                  mbx_bitmap** out, int64_t* count) {
  NOTNULL(c);
  NOTNULL(a);
  NOTNULL(b);
  NOTNULL(out);
  *out = nullptr;
  if (op < MBX_BM_AND || op > MBX_BM_ANDNOT) return fail(MBX_E_INVALID, "bitmap_combine: op %d", op);
  if (a->nbits != b->nbits) return fail(MBX_E_INVALID, "bitmap_combine: %lld vs %lld bits", (long long)a->nbits,
                                        (long long)b->nbits);
  int rc = set_device(c);
  if (rc) return rc;
  mbx_bitmap* r = nullptr;
  if ((rc = bitmap_new(c, a->nbits, &r))) return rc;
  hipError_t e = launch_bitmap_combine(op, a->words, b->words, r->nwords, r->nbits, r->wpb, r->words, r->segc,
                                       c->stream);
  if (e != hipSuccess) {
    mbx_bitmap_free(r);
    return fail(MBX_E_DEVICE, "bitmap_combine: %s", hipGetErrorString(e));
  }
  if ((rc = bitmap_count_sync(c, r, false))) {
    mbx_bitmap_free(r);
    return rc;
  }
  if (count) *count = r->count;
  *out = r;
  return MBX_OK;
}

static int cnf_args(int64_t nbits, const mbx_bitmap* const* bms, const int32_t* conj_offsets, int32_t nconj,
                    const mbx_bitmap* deleted, BitmapCnf* C) {
  if (nconj < 1 || nconj > 32) return fail(MBX_E_UNSUPPORTED, "bitmap_cnf: %d conjuncts (1..32)", nconj);
  NOTNULL(conj_offsets);
  const int32_t nb = conj_offsets[nconj];
  if (nb < 0 || nb > kMaxBitmaps) return fail(MBX_E_UNSUPPORTED, "bitmap_cnf: %d bitmaps (max %d)", nb, kMaxBitmaps);
  if (nb > 0) NOTNULL(bms);
  memset(C, 0, sizeof(*C));
  C->nconj = nconj;
  for (int32_t i = 0; i <= nconj; i++) {
    if (conj_offsets[i] < 0 || conj_offsets[i] > nb || (i > 0 && conj_offsets[i] < conj_offsets[i - 1]))
      return fail(MBX_E_INVALID, "bitmap_cnf: conj_offsets not ascending");
    C->conj_off[i] = conj_offsets[i];
  }
  for (int32_t k = 0; k < nb; k++) {
    if (!bms[k]) return fail(MBX_E_INVALID, "bitmap_cnf: bms[%d] null", k);
    if (bms[k]->nbits != nbits) return fail(MBX_E_INVALID, "bitmap_cnf: bms[%d] has %lld bits, want %lld", k,
                                            (long long)bms[k]->nbits, (long long)nbits);
    C->bms[k] = bms[k]->words;
  }
  if (deleted && deleted->nbits != nbits) return fail(MBX_E_INVALID, "bitmap_cnf: deleted bitmap size");
  return MBX_OK;
}

extern "C" int mbx_bitmap_cnf(mbx_ctx* c, int64_t nbits, const mbx_bitmap* const* bms, const int32_t* conj_offsets,
                              int32_t nconj, const mbx_bitmap* deleted, mbx_bitmap** out, int64_t* count) {
  NOTNULL(c);
  NOTNULL(out);
  *out = nullptr;
  BitmapCnf C;
  int rc = cnf_args(nbits, bms, conj_offsets, nconj, deleted, &C);
  if (rc) return rc;
  if ((rc = set_device(c))) return rc;
  mbx_bitmap* r = nullptr;
  if ((rc = bitmap_new(c, nbits, &r))) return rc;
  hipError_t e = launch_bitmap_cnf(C, deleted ? deleted->words : nullptr, r->nwords, r->nbits, r->wpb, r->words,
                                   r->segc, c->stream);
  if (e != hipSuccess) {
    mbx_bitmap_free(r);
    return fail(MBX_E_DEVICE, "bitmap_cnf: %s", hipGetErrorString(e));
  }
  if ((rc = bitmap_count_sync(c, r, false))) {
    mbx_bitmap_free(r);
    return rc;
  }
  if (count) *count = r->count;
  *out = r;
  return MBX_OK;
}

extern "C" int mbx_bitmap_cnf_async(mbx_ctx* c, const mbx_bitmap* const* bms, const int32_t* conj_offsets,
                                    int32_t nconj, const mbx_bitmap* deleted, mbx_bitmap* out) {
  NOTNULL(c);
  NOTNULL(out);
  BitmapCnf C;
  int rc = cnf_args(out->nbits, bms, conj_offsets, nconj, deleted, &C);
  if (rc) return rc;
  out->count = -1;
  HIPCHK(launch_bitmap_cnf(C, deleted ? deleted->words : nullptr, out->nwords, out->nbits, out->wpb, out->words,
                           out->segc, c->stream));
  return MBX_OK;
}

extern "C" int mbx_bitmap_index_build(mbx_ctx* c, const mbx_table* t, int32_t col, const mbx_operand* values,
                                      int32_t nvalues, mbx_bitmap** out) {
  NOTNULL(c);
  NOTNULL(t);
  NOTNULL(out);
  if (nvalues <= 0) return fail(MBX_E_INVALID, "index_build: nvalues %d", nvalues);
  NOTNULL(values);
  if (col < 0 || col >= (int32_t)t->cols.size()) return fail(MBX_E_RANGE, "index_build: column %d", col);
  const TCol& tc = t->cols[(size_t)col];
  int rc = set_device(c);
  if (rc) return rc;
  const int32_t vw = tc.attr_type == MBX_ATTR_STRING ? tc.stride_w : 1;
  std::vector<uint32_t> vals((size_t)nvalues * (size_t)vw, 0u);
  for (int32_t v = 0; v < nvalues; v++) {
    const mbx_operand& o = values[v];
    if (o.type != tc.attr_type) return fail(MBX_E_TYPE, "index_build: value %d has AttrType %d, column %d", v, o.type,
                                            tc.attr_type);
    if (o.type == MBX_ATTR_INTEGER) {
      memcpy(&vals[(size_t)v], &o.integer, 4);
    } else if (o.type == MBX_ATTR_REAL) {
      memcpy(&vals[(size_t)v], &o.real, 4);
    } else {
      if (o.string_len > tc.size) {
        // longer than any value the column can hold: the bitmap stays empty
        vals[(size_t)v * vw] = 0xFFFFFFFFu;  // never equal: 0xFF is not valid modified UTF-8
        continue;
      }
      encode_device_string((const uint8_t*)o.string, o.string_len, (uint8_t*)&vals[(size_t)v * vw], vw * 4);
    }
  }
  return index_build_encoded(c, t, col, vals.data(), nvalues, out);
}

int mbx::index_build_encoded(mbx_ctx* c, const mbx_table* t, int32_t col, const uint32_t* host_vals,
                             int32_t nvalues, mbx_bitmap** out) {
  const TCol& tc = t->cols[(size_t)col];
  const int32_t vw = tc.attr_type == MBX_ATTR_STRING ? tc.stride_w : 1;
  int rc = MBX_OK;
  std::vector<uint32_t> vals(host_vals, host_vals + (size_t)nvalues * (size_t)vw);
  for (int32_t v = 0; v < nvalues; v++) out[v] = nullptr;
  uint32_t* dvals = nullptr;
  HIPCHK(hipMalloc(&dvals, vals.size() * 4));
  hipError_t e = hipMemcpy(dvals, vals.data(), vals.size() * 4, hipMemcpyHostToDevice);
  std::vector<uint64_t*> outs((size_t)nvalues);
  for (int32_t v = 0; v < nvalues && e == hipSuccess && !rc; v++) {
    rc = bitmap_new(c, t->nrows, &out[v]);
    if (!rc) outs[(size_t)v] = out[v]->words;
  }
  if (!rc && e == hipSuccess && t->nrows > 0) {
    KCol kc;
    kc.base = tc.dev;
    kc.kind = col_kind(tc.attr_type);
    kc.stride_w = tc.stride_w;
    if (kc.kind != kStr && tc.stride_w == 1 && !(reinterpret_cast<uintptr_t>(tc.dev) & 15)) {
      std::vector<int64_t*> segs((size_t)nvalues);
      for (int32_t v = 0; v < nvalues; v++) segs[(size_t)v] = out[v]->segc;
      e = launch_index_build4(kc, t->nrows, t->deleted, dvals, nvalues, outs.data(), segs.data(), out[0]->wpb,
                              c->stream);
    } else {
      e = launch_index_build(kc, t->nrows, t->deleted, dvals, nvalues, vw, outs.data(), out[0]->wpb, c->stream);
      for (int32_t v = 0; v < nvalues && e == hipSuccess; v++)
        e = launch_seg_popcount(out[v]->words, out[v]->nwords, out[v]->wpb, out[v]->segc, c->stream);
    }
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(dvals);
  if (!rc && e != hipSuccess) rc = fail(MBX_E_DEVICE, "index_build: %s", hipGetErrorString(e));
  for (int32_t v = 0; v < nvalues && !rc; v++) rc = bitmap_count_sync(c, out[v], false);
  if (rc) {
    for (int32_t v = 0; v < nvalues; v++) {
      mbx_bitmap_free(out[v]);
      out[v] = nullptr;
    }
  }
  return rc;
}

// ---------------------------------------------------- late materialisation

// a projected column as the gathers read it: its device rows, plus the
// column group holding it (mbx_table_group) for the narrow 4-byte gathers
static ProjCol proj_col(const mbx_table* t, int32_t col) {
  ProjCol p;
  const TCol& tc = t->cols[(size_t)col];
  p.base = tc.dev;
  p.stride_w = tc.stride_w;
  for (const TGroup& g : t->groups)
    for (size_t k = 0; k < g.cols.size(); k++)
      if (g.cols[k] == col) {
        p.gbase = g.dev + k;
        p.gstride = (int32_t)g.cols.size();
        return p;
      }
  return p;
}

static int materialize_dev(mbx_ctx* c, const mbx_table* t, const mbx_bitmap* sel, const int32_t* proj,
                           int32_t nproj, int64_t row_offset, int64_t* dev_ids, void* const* dev_out,
                           int64_t* dev_total) {
  if (nproj < 0 || nproj > kMaxProj) return fail(MBX_E_UNSUPPORTED, "materialize: %d columns (max %d)", nproj,
                                                 kMaxProj);
  ProjCol pc[kMaxProj];
  for (int32_t j = 0; j < nproj; j++) {
    if (!t) return fail(MBX_E_INVALID, "materialize: projection without a table");
    if (proj[j] < 0 || proj[j] >= (int32_t)t->cols.size())
      return fail(MBX_E_RANGE, "materialize: column %d outside 0..%zu", proj[j], t->cols.size() - 1);
    pc[j] = proj_col(t, proj[j]);
  }
  if (t && sel->nbits != t->nrows) return fail(MBX_E_INVALID, "materialize: bitmap/table size mismatch");
  if (!dev_total) dev_total = c->dcount + 1;
  if (!dev_ids) {
    // positions are the gather's input: keep them in context scratch
    if (c->ids_cap < sel->nbits) {
      if (c->ids_scratch) HIPCHK(hipFree(c->ids_scratch));
      c->ids_scratch = nullptr;
      c->ids_cap = 0;
      HIPCHK(hipMalloc(&c->ids_scratch, sizeof(int64_t) * (size_t)(sel->nbits > 0 ? sel->nbits : 1)));
      c->ids_cap = sel->nbits;
    }
    dev_ids = c->ids_scratch;
  }
  int64_t* stamps = nullptr;
  if (c->tune.select_dbg & 8) {  // diagnostic stamps (mbx_diag_select_stamps)
    if (!c->stamps) HIPCHK(hipMalloc(&c->stamps, sizeof(int64_t) * 4 * kMaxStampBlocks));
    if (sel->nseg <= kMaxStampBlocks) stamps = c->stamps;
  }
  HIPCHK(launch_materialize(sel->words, sel->nwords, sel->wpb, sel->segc, row_offset, dev_ids, pc, dev_out, nproj,
                            dev_total, c->stream, (c->tune.select_dbg & 3) | ((c->tune.select_dbg >> 4) & 32), stamps,
                            c->tune.gather_fused != 0,
                            c->tune.select_blocks, c->tune.gather_pair != 0));
  return MBX_OK;
}

// the projection of a one-launch ColumnarIndexScan: any columns (<= kMaxProj)
// in their device row layout (4 bytes; char(n): stride_w words)
static int cnf_proj_args(const mbx_table* t, const int32_t* proj, int32_t nproj, void* const* dev_out, ProjCol* pc) {
  if (nproj < 0 || nproj > kMaxProj)
    return fail(MBX_E_UNSUPPORTED, "cnf_materialize: %d columns (max %d)", nproj, kMaxProj);
  if (nproj > 0) {
    NOTNULL(proj);
    NOTNULL(dev_out);
  }
  for (int32_t j = 0; j < nproj; j++) {
    if (proj[j] < 0 || proj[j] >= (int32_t)t->cols.size())
      return fail(MBX_E_RANGE, "cnf_materialize: column %d outside 0..%zu", proj[j], t->cols.size() - 1);
    const TCol& tc = t->cols[(size_t)proj[j]];
    if (!dev_out[j]) return fail(MBX_E_INVALID, "cnf_materialize: dev_out[%d] null", j);
    (void)tc;
    pc[j] = proj_col(t, proj[j]);
  }
  return MBX_OK;
}

static CnfTune cnf_tune(const mbx_ctx* c) {
  CnfTune k;
  k.blocks = c->tune.cnf_blocks;
  k.flag_stride = c->tune.cnf_flag_stride;
  k.lookback = c->tune.cnf_lookback;
  k.store = c->tune.cnf_store;
  k.gather_pair = c->tune.gather_pair;
  return k;
}

extern "C" int mbx_cnf_materialize_async(mbx_ctx* c, const mbx_table* t, const mbx_bitmap* const* bms,
                                         const int32_t* conj_offsets, int32_t nconj, const mbx_bitmap* deleted,
                                         const int32_t* proj, int32_t nproj, int64_t* dev_ids,
                                         void* const* dev_out, int64_t* dev_count) {
  NOTNULL(c);
  NOTNULL(t);
  NOTNULL(dev_count);
  BitmapCnf C;
  int rc = cnf_args(t->nrows, bms, conj_offsets, nconj, deleted, &C);
  if (rc) return rc;
  ProjCol pc[kMaxProj];
  if ((rc = cnf_proj_args(t, proj, nproj, dev_out, pc))) return rc;
  if ((rc = set_device(c))) return rc;
  const int64_t nwords = (t->nrows + 63) >> 6;
  int64_t* stamps = nullptr;
  if (c->tune.select_dbg & 8) {  // diagnostic stamps (mbx_diag_select_stamps), <= 1024 blocks
    if (!c->stamps) HIPCHK(hipMalloc(&c->stamps, sizeof(int64_t) * 4 * kMaxStampBlocks));
    stamps = c->stamps;
  }
  CnfTune ct = cnf_tune(c);
  if (stamps) ct.blocks = 0;  // the stamps buffer holds <= 1024 blocks
  HIPCHK(launch_cnf_materialize(C, deleted ? deleted->words : nullptr, nwords, t->nrows, c->lookback,
                                t->row_offset, dev_ids, pc, dev_out, nproj, dev_count, c->stream, stamps,
                                c->tune.select_dbg >> 4, INT64_MAX, &ct));
  return MBX_OK;
}

extern "C" int mbx_diag_select_stamps(mbx_ctx* c, int64_t* host, int64_t nblocks) {
  NOTNULL(c);
  NOTNULL(host);
  if (!c->stamps) return fail(MBX_E_INVALID, "diag_select_stamps: no stamped launch (select_dbg bit 3)");
  if (nblocks < 0 || nblocks > kMaxStampBlocks) return fail(MBX_E_INVALID, "diag_select_stamps: %lld blocks",
                                                            (long long)nblocks);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(host, c->stamps, sizeof(int64_t) * 4 * (size_t)nblocks, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MBX_OK;
}

extern "C" int mbx_diag_lookback_epoch(mbx_ctx* c, int64_t epoch) {
  NOTNULL(c);
  if (epoch < 0 || epoch > 0x7fffffff) return fail(MBX_E_INVALID, "diag_lookback_epoch: %lld", (long long)epoch);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(c->lookback, &epoch, sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MBX_OK;
}

static int64_t col_bytes(const mbx_table* t, int32_t j) {
  const TCol& tc = t->cols[(size_t)j];
  return (int64_t)tc.stride_w * 4;
}

int mbx::ensure_count(mbx_ctx* c, mbx_bitmap* b) {
  if (b->count >= 0) return MBX_OK;
  return bitmap_count_sync(c, b, false);
}

// device rows (stride) -> caller layout (size bytes, modified UTF-8)
void mbx::unpack_rows(const TCol& tc, const uint8_t* dev_img, int64_t n, void* host_out) {
  if (tc.attr_type != MBX_ATTR_STRING) {
    memcpy(host_out, dev_img, (size_t)n * 4);
    return;
  }
  const int32_t stride = tc.stride_w * 4;
  for (int64_t r = 0; r < n; r++)
    decode_device_string(dev_img + (size_t)r * stride, stride, (uint8_t*)host_out + (size_t)r * tc.size, tc.size);
}

extern "C" int mbx_cursor_open(mbx_ctx* c, const mbx_table* t, const mbx_bitmap* selc, const int32_t* proj,
                               int32_t nproj, mbx_cursor** out) {
  NOTNULL(c);
  NOTNULL(selc);
  NOTNULL(out);
  *out = nullptr;
  if (nproj > 0) {
    NOTNULL(t);
    NOTNULL(proj);
  }
  mbx_bitmap* sel = const_cast<mbx_bitmap*>(selc);
  int rc = set_device(c);
  if (rc) return rc;
  if ((rc = ensure_count(c, sel))) return rc;
  mbx_cursor* k = new (std::nothrow) mbx_cursor();
  if (!k) return fail(MBX_E_NOMEM, "cursor: host allocation");
  k->ctx = c;
  k->t = t;
  k->count = sel->count;
  const size_t n = (size_t)(k->count > 0 ? k->count : 1);
  hipError_t e = hipMalloc(&k->ids, n * sizeof(int64_t));
  for (int32_t j = 0; j < nproj && e == hipSuccess; j++) {
    if (proj[j] < 0 || proj[j] >= (int32_t)t->cols.size()) {
      mbx_cursor_close(k);
      return fail(MBX_E_RANGE, "cursor: column %d", proj[j]);
    }
    void* d = nullptr;
    e = hipMalloc(&d, n * (size_t)col_bytes(t, proj[j]));
    k->outs.push_back(d);
    k->proj.push_back(proj[j]);
  }
  if (e != hipSuccess) {
    mbx_cursor_close(k);
    return fail(MBX_E_NOMEM, "cursor: %s", hipGetErrorString(e));
  }
  rc = materialize_dev(c, t, sel, proj, nproj, t ? t->row_offset : 0, k->ids, k->outs.data(), c->dcount);
  if (!rc) {
    hipError_t e2 = hipStreamSynchronize(c->stream);
    if (e2 != hipSuccess) rc = fail(MBX_E_DEVICE, "cursor: %s", hipGetErrorString(e2));
  }
  if (rc) {
    mbx_cursor_close(k);
    return rc;
  }
  *out = k;
  return MBX_OK;
}

// a launched CNF cursor: wait for its launch and read the count
static int cursor_resolve(mbx_cursor* k) {
  if (!k->count_pending) return MBX_OK;
  mbx_ctx* c = k->ctx;
  int rc = set_device(c);
  if (rc) return rc;
  int64_t* h = (int64_t*)c->pinned + 20;
  HIPCHK(hipMemcpyAsync(h, k->dcount, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  k->count_pending = false;
  k->count = *h;
  if (k->count < 0 || k->count > k->bound)  // cannot happen: the bound holds for any CNF
    return fail(MBX_E_DEVICE, "cnf_cursor: %lld rows outside the bound %lld", (long long)k->count,
                (long long)k->bound);
  return MBX_OK;
}

extern "C" int mbx_cursor_count(const mbx_cursor* kc, int64_t* count) {
  NOTNULL(kc);
  NOTNULL(count);
  mbx_cursor* k = const_cast<mbx_cursor*>(kc);
  if (int rc = cursor_resolve(k)) return rc;
  *count = k->count;
  return MBX_OK;
}

// bytes per row of projected column j in the host layout (mbx_materialize's)
static int64_t host_width(const mbx_cursor* k, size_t j) {
  const TCol& tc = k->t->cols[(size_t)k->proj[j]];
  return tc.attr_type == MBX_ATTR_STRING ? (int64_t)tc.size : 4;
}

static int64_t align16(int64_t v) { return (v + 15) & ~int64_t(15); }

// host / staging layout of an n-row batch: n positions, then each projected
// column's n rows, every part 16-byte aligned; returns the batch's bytes
// the largest cursor batch buffer (256 Ki rows of 16 x char(256)
// would pin ~1 GiB per buffer)
constexpr int64_t kCursorBatchBytes = int64_t(64) << 20;

static int64_t batch_layout(const mbx_cursor* k, int64_t n, int64_t* off) {
  int64_t o = align16(n * (int64_t)sizeof(int64_t));
  for (size_t j = 0; j < k->outs.size(); j++) {
    off[j] = o;
    o = align16(o + n * host_width(k, j));
  }
  return o;
}

// enqueue rows [from, from + n) into pin[b]: one pack kernel into the device
// staging region, one device -> pinned copy, one event
static int cursor_fetch(mbx_cursor* k, int b, int64_t from, int64_t n) {
  mbx_ctx* c = k->ctx;
  int64_t off[kMaxProj];
  const int64_t bytes = batch_layout(k, n, off);
  CursorPack P;
  memset(&P, 0, sizeof(P));
  P.ncols = (int32_t)k->outs.size();
  for (size_t j = 0; j < k->outs.size(); j++) {
    const TCol& tc = k->t->cols[(size_t)k->proj[j]];
    P.col[j].src = (const uint8_t*)k->outs[j];
    P.col[j].src_stride = tc.stride_w * 4;
    P.col[j].width = (int32_t)host_width(k, j);
    P.col[j].is_string = tc.attr_type == MBX_ATTR_STRING;
    P.col[j].dst_off = off[j];
  }
  HIPCHK(launch_cursor_pack(k->ids, from, n, P, k->stage, c->stream));
  HIPCHK(hipMemcpyAsync(k->pin[b], k->stage, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipEventRecord(k->ev[b], c->stream));
  k->d2h_bytes += bytes;
  return MBX_OK;
}

// wait for (and forget) a batch still in flight
static int cursor_drain(mbx_cursor* k) {
  if (k->pf_start < 0) return MBX_OK;
  k->pf_start = -1;
  HIPCHK(hipEventSynchronize(k->ev[k->pf_buf]));
  return MBX_OK;
}

static void cursor_release_pinned(mbx_cursor* k) {
  for (int b = 0; b < 2; b++) {
    if (k->ev[b]) hipEventDestroy(k->ev[b]);
    if (k->pin[b]) hipHostFree(k->pin[b]);
    k->ev[b] = nullptr;
    k->pin[b] = nullptr;
  }
  if (k->stage) hipFree(k->stage);
  k->stage = nullptr;
  k->batch_rows = 0;
}

// the next <= max_rows rows as pointers into the pinned batch buffer
static int cursor_next_view(mbx_cursor* k, int64_t max_rows, const int64_t** ids, const void** cols, int64_t* n) {
  NOTNULL(k);
  NOTNULL(n);
  *n = 0;
  if (max_rows <= 0) return fail(MBX_E_INVALID, "cursor_next: max_rows %lld", (long long)max_rows);
  {
    // a batch's buffers (2 pinned + 1 device) are sized by bytes, not rows:
    // at most kCursorBatchBytes each, however wide the projected row --
    // batch_layout rounds each of its 1 + nproj parts up to 16 bytes, so
    // that padding is set aside first
    int64_t row_bytes = (int64_t)sizeof(int64_t);
    for (size_t j = 0; j < k->outs.size(); j++) row_bytes += host_width(k, j);
    const int64_t cap = (kCursorBatchBytes - 16 * (int64_t)(k->outs.size() + 1)) / row_bytes;
    if (max_rows > cap) max_rows = cap > 0 ? cap : 1;
  }
  if (int rc0 = cursor_resolve(k)) return rc0;
  const int64_t take = k->count - k->next < max_rows ? k->count - k->next : max_rows;
  if (take <= 0) return MBX_OK;  // end of stream: get_next() returns null
  mbx_ctx* c = k->ctx;
  int rc = set_device(c);
  if (rc) return rc;
  // pinned batch buffers + the device staging region, sized to the largest
  // batch asked for so far
  const int64_t rows = max_rows < k->count ? max_rows : k->count;
  if (k->batch_rows < rows) {
    if ((rc = cursor_drain(k))) return rc;
    cursor_release_pinned(k);
    int64_t off[kMaxProj];
    const int64_t bytes = batch_layout(k, rows, off);
    for (int b = 0; b < 2; b++) {
      HIPCHK(hipHostMalloc((void**)&k->pin[b], (size_t)bytes, hipHostMallocDefault));
      HIPCHK(hipEventCreateWithFlags(&k->ev[b], hipEventDisableTiming));
    }
    HIPCHK(hipMalloc((void**)&k->stage, (size_t)bytes));
    k->batch_rows = rows;
  }
  int b;
  int64_t laid = take;  // rows the buffer's layout was packed for
  if (k->pf_start == k->next && k->pf_n >= take) {
    b = k->pf_buf;  // this batch is already on its way (perhaps with more rows)
    laid = k->pf_n;
    k->pf_start = -1;
  } else {
    if ((rc = cursor_drain(k))) return rc;
    b = k->pf_buf ^ 1;
    if ((rc = cursor_fetch(k, b, k->next, take))) return rc;
  }
  // the following batch into the other buffer, before this one is consumed
  const int64_t nxt = k->next + take;
  const int64_t m = k->count - nxt < max_rows ? k->count - nxt : max_rows;
  HIPCHK(hipEventSynchronize(k->ev[b]));
  if (m > 0 && c->tune.cursor_prefetch) {
    if ((rc = cursor_fetch(k, b ^ 1, nxt, m))) return rc;
    k->pf_start = nxt;
    k->pf_n = m;
    k->pf_buf = b ^ 1;
  }
  int64_t off[kMaxProj];
  batch_layout(k, laid, off);
  if (ids) *ids = (const int64_t*)k->pin[b];
  for (size_t j = 0; cols && j < k->outs.size(); j++) cols[j] = k->pin[b] + off[j];
  k->next += take;
  *n = take;
  return MBX_OK;
}

extern "C" int mbx_cursor_next_view(mbx_cursor* k, int64_t max_rows, const int64_t** ids, const void** cols,
                                    int64_t* n) {
  return cursor_next_view(k, max_rows, ids, cols, n);
}

extern "C" int mbx_cursor_next(mbx_cursor* k, int64_t max_rows, int64_t* host_ids, void* const* host_out,
                               int64_t* n) {
  NOTNULL(k);
  const int64_t* vids = nullptr;
  const void* vcols[kMaxProj];
  if (k->outs.size() > (size_t)kMaxProj) return fail(MBX_E_UNSUPPORTED, "cursor_next: %zu columns", k->outs.size());
  int rc = cursor_next_view(k, max_rows, &vids, vcols, n);
  if (rc || *n == 0) return rc;
  if (host_ids) memcpy(host_ids, vids, (size_t)*n * sizeof(int64_t));
  for (size_t j = 0; host_out && j < k->outs.size(); j++)
    if (host_out[j]) memcpy(host_out[j], vcols[j], (size_t)(*n * host_width(k, j)));
  return MBX_OK;
}

extern "C" int mbx_cursor_restart(mbx_cursor* k) {
  NOTNULL(k);
  int rc = cursor_drain(k);
  k->next = 0;
  return rc;
}

extern "C" int mbx_cursor_close(mbx_cursor* k) {
  if (!k) return MBX_OK;
  hipSetDevice(k->ctx->device);
  hipStreamSynchronize(k->ctx->stream);
  cursor_release_pinned(k);
  hipFree(k->dcount);
  hipFree(k->ids);
  for (void* d : k->outs) hipFree(d);
  delete k;
  return MBX_OK;
}

extern "C" int mbx_cursor_stats(const mbx_cursor* k, int64_t* delivered, int64_t* d2h_bytes) {
  NOTNULL(k);
  if (delivered) *delivered = k->next;
  if (d2h_bytes) *d2h_bytes = k->d2h_bytes;
  return MBX_OK;
}

// ColumnarIndexScan end to end into a cursor: one k_cnf_select launch writes
// the positions and projected rows of the CNF's selection into the cursor's
// device buffers (no BitSet stored, no second launch), then get_next()
// batches come out of mbx_cursor_next.  The buffers are sized by an upper
// bound of the count: min over conjuncts of the sum of their bitmaps'
// cardinalities (OR <= sum, AND <= min), at most the table's rows.
extern "C" int mbx_cnf_cursor_launch(mbx_ctx* c, const mbx_table* t, const mbx_bitmap* const* bms,
                                     const int32_t* conj_offsets, int32_t nconj, const mbx_bitmap* deleted,
                                     const int32_t* proj, int32_t nproj, mbx_cursor** out, int64_t** dev_count) {
  NOTNULL(c);
  NOTNULL(t);
  NOTNULL(out);
  *out = nullptr;
  if (dev_count) *dev_count = nullptr;
  if (c->capturing) return fail(MBX_E_INVALID, "cnf_cursor: inside a graph capture (it allocates)");
  BitmapCnf C;
  int rc = cnf_args(t->nrows, bms, conj_offsets, nconj, deleted, &C);
  if (rc) return rc;
  if (nproj < 0 || nproj > kMaxProj) return fail(MBX_E_UNSUPPORTED, "cnf_cursor: %d columns (max %d)", nproj, kMaxProj);
  if (nproj > 0) NOTNULL(proj);
  for (int32_t j = 0; j < nproj; j++)
    if (proj[j] < 0 || proj[j] >= (int32_t)t->cols.size())
      return fail(MBX_E_RANGE, "cnf_cursor: column %d outside 0..%zu", proj[j], t->cols.size() - 1);
  if ((rc = set_device(c))) return rc;
  int64_t bound = t->nrows;
  for (int32_t cj = 0; cj < nconj; cj++) {
    int64_t s = 0;
    for (int32_t k = conj_offsets[cj]; k < conj_offsets[cj + 1] && s < bound; k++) {
      mbx_bitmap* b = const_cast<mbx_bitmap*>(bms[k]);
      if ((rc = ensure_count(c, b))) return rc;
      s += b->count;
    }
    if (s < bound) bound = s;
  }
  mbx_cursor* k = new (std::nothrow) mbx_cursor();
  if (!k) return fail(MBX_E_NOMEM, "cnf_cursor: host allocation");
  k->ctx = c;
  k->t = t;
  k->bound = bound;
  const size_t cap = (size_t)(bound > 0 ? bound : 1);
  hipError_t e = hipMalloc(&k->dcount, sizeof(int64_t));
  if (e == hipSuccess) e = hipMalloc(&k->ids, cap * sizeof(int64_t));
  for (int32_t j = 0; j < nproj && e == hipSuccess; j++) {
    void* d = nullptr;
    e = hipMalloc(&d, cap * (size_t)col_bytes(t, proj[j]));
    k->outs.push_back(d);
    k->proj.push_back(proj[j]);
  }
  if (e != hipSuccess) {
    mbx_cursor_close(k);
    return fail(MBX_E_NOMEM, "cnf_cursor: %s", hipGetErrorString(e));
  }
  ProjCol pc[kMaxProj];
  for (int32_t j = 0; j < nproj; j++) {
    pc[j] = proj_col(t, proj[j]);
  }
  const CnfTune ct = cnf_tune(c);
  e = launch_cnf_materialize(C, deleted ? deleted->words : nullptr, (t->nrows + 63) >> 6, t->nrows, c->lookback,
                             t->row_offset, k->ids, pc, k->outs.data(), nproj, k->dcount, c->stream, nullptr,
                             c->tune.select_dbg >> 4, bound, &ct);
  if (e != hipSuccess) {
    mbx_cursor_close(k);
    return fail(MBX_E_DEVICE, "cnf_cursor: %s", hipGetErrorString(e));
  }
  k->count_pending = true;
  if (dev_count) *dev_count = k->dcount;
  *out = k;
  return MBX_OK;
}

extern "C" int mbx_cnf_cursor_open(mbx_ctx* c, const mbx_table* t, const mbx_bitmap* const* bms,
                                   const int32_t* conj_offsets, int32_t nconj, const mbx_bitmap* deleted,
                                   const int32_t* proj, int32_t nproj, mbx_cursor** out) {
  int rc = mbx_cnf_cursor_launch(c, t, bms, conj_offsets, nconj, deleted, proj, nproj, out, nullptr);
  if (rc) return rc;
  if ((rc = cursor_resolve(*out))) {
    mbx_cursor_close(*out);
    *out = nullptr;
  }
  return rc;
}

extern "C" int mbx_bitmap_select(mbx_ctx* c, const mbx_bitmap* b, int64_t row_offset, int64_t* host_ids, int64_t cap,
                                 int64_t* n) {
  NOTNULL(c);
  NOTNULL(b);
  NOTNULL(n);
  *n = 0;
  mbx_bitmap* sel = const_cast<mbx_bitmap*>(b);
  int rc = set_device(c);
  if (rc) return rc;
  if ((rc = ensure_count(c, sel))) return rc;
  if (sel->count > cap) return fail(MBX_E_INVALID, "bitmap_select: %lld ids, capacity %lld", (long long)sel->count,
                                    (long long)cap);
  if (sel->count == 0) return MBX_OK;
  NOTNULL(host_ids);
  int64_t* d = nullptr;
  HIPCHK(hipMalloc(&d, (size_t)sel->count * sizeof(int64_t)));
  rc = materialize_dev(c, nullptr, sel, nullptr, 0, row_offset, d, nullptr, c->dcount);
  hipError_t e = hipSuccess;
  if (!rc) e = hipMemcpyAsync(host_ids, d, (size_t)sel->count * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream);
  if (!rc && e == hipSuccess) e = hipStreamSynchronize(c->stream);
  hipFree(d);
  if (rc) return rc;
  if (e != hipSuccess) return fail(MBX_E_DEVICE, "bitmap_select: %s", hipGetErrorString(e));
  *n = sel->count;
  return MBX_OK;
}

extern "C" int mbx_materialize(mbx_ctx* c, const mbx_table* t, const mbx_bitmap* sel, const int32_t* proj,
                               int32_t nproj, int64_t* host_ids, void* const* host_out, int64_t cap, int64_t* n) {
  NOTNULL(c);
  NOTNULL(t);
  NOTNULL(sel);
  NOTNULL(n);
  *n = 0;
  mbx_cursor* k = nullptr;
  int rc = mbx_cursor_open(c, t, sel, proj, nproj, &k);
  if (rc) return rc;
  if (k->count > cap) {
    mbx_cursor_close(k);
    return fail(MBX_E_INVALID, "materialize: %lld rows, capacity %lld", (long long)k->count, (long long)cap);
  }
  // batch after batch (a cursor batch holds at most kCursorBatchBytes), each
  // copied to its rows' offset in the caller's arrays
  int64_t done = 0;
  while (rc == MBX_OK && done < k->count) {
    const int64_t* vids = nullptr;
    const void* vcols[kMaxProj];
    int64_t got = 0;
    rc = cursor_next_view(k, k->count - done, &vids, vcols, &got);
    if (rc || got == 0) break;
    if (host_ids) memcpy(host_ids + done, vids, (size_t)got * sizeof(int64_t));
    for (size_t j = 0; host_out && j < k->outs.size(); j++) {
      const int64_t w = host_width(k, j);
      if (host_out[j]) memcpy((uint8_t*)host_out[j] + done * w, vcols[j], (size_t)(got * w));
    }
    done += got;
  }
  if (rc == MBX_OK && done != k->count)
    rc = fail(MBX_E_DEVICE, "materialize: %lld of %lld rows delivered", (long long)done, (long long)k->count);
  if (rc == MBX_OK) *n = done;
  mbx_cursor_close(k);
  return rc;
}

extern "C" int mbx_materialize_async(mbx_ctx* c, const mbx_table* t, const mbx_bitmap* sel, const int32_t* proj,
                                     int32_t nproj, int64_t* dev_ids, void* const* dev_out, int64_t* dev_count) {
  NOTNULL(c);
  NOTNULL(t);
  NOTNULL(sel);
  if (nproj > 0) {
    NOTNULL(proj);
    NOTNULL(dev_out);
  }
  return materialize_dev(c, t, sel, proj, nproj, t->row_offset, dev_ids, dev_out, dev_count);
}
