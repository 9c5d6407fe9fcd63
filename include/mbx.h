/*
 * mbx.h -- C-ABI of the MI355X columnar scan/filter/aggregate executor for
 * the Minibase-Columnar engine (drop-in for the ColumnarFileScan /
 * ColumnIndexScan / ColumnarIndexScan / BitMapFile hot path).
 *
 * Plain C: no C++ or HIP types cross this boundary.  Every entry point names
 * the reference interface it replaces; R/ = minijava/src of
 * Neehaarika/MiniBase-Columnar-Database.  INTEGRATION.md shows the JNI glue a
 * Java maintainer would add on top (GpuColumnarFileScan etc.).
 *
 * Conventions
 *   - Every function returns MBX_OK (0) or a negative MBX_E_* code; the
 *     message of the last failure on the calling thread is mbx_last_error().
 *     Codes map onto the reference's checked exceptions (see below).
 *   - One mbx_ctx per GPU; a context owns one HIP stream and is used by one
 *     thread at a time (the reference engine is single threaded,
 *     R/global/SystemDefs.java:6-9).  Multi-GPU = one process (or one
 *     context) per GPU, rows sharded by range.
 *   - Synchronous calls return with their results on the host.  *_async calls
 *     only enqueue on the context stream; mbx_sync() waits and returns
 *     MBX_E_TYPE if a scan enqueued since the previous mbx_sync reached a
 *     float compare on a NaN (the exception PredEval would have thrown).
 *   - Positions: a table holds rows [row_offset, row_offset + nrows) of a
 *     Columnarfile in position order (position == row index of a dense file,
 *     R/heap/Heapfile.java:262-289).  row_offset must be a multiple of 64 so
 *     bitmap words never straddle shards.  Bitmaps are table-local
 *     java.util.BitSet images (bit p%64 of uint64 word p/64, local p);
 *     row ids returned to the host are global positions (row_offset + p).
 */
#ifndef MBX_H
#define MBX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MBX_ABI_VERSION 1

/* ---- status codes (reference exception each one stands for) ------------ */
#define MBX_OK 0
#define MBX_E_INVALID (-1)     /* bad argument: FileScanException / IndexException / InvalidRelation */
#define MBX_E_TYPE (-2)        /* UnknowAttrType / PredEvalException (operand type mismatch) */
#define MBX_E_RANGE (-3)       /* FieldNumberOutOfBoundException (FldSpec offset out of range) */
#define MBX_E_DEVICE (-4)      /* HIP runtime failure */
#define MBX_E_NOMEM (-5)       /* device or host allocation failed */
#define MBX_E_UNSUPPORTED (-6) /* outside the GPU path's envelope (limits below) */

/* ---- global.AttrType (R/global/AttrType.java:45-49) ----------------------- */
#define MBX_ATTR_STRING 0
#define MBX_ATTR_INTEGER 1
#define MBX_ATTR_REAL 2
#define MBX_ATTR_SYMBOL 3
#define MBX_ATTR_NULL 4

/* ---- global.AttrOperator (R/global/AttrOperator.java:98-106) -------------- */
#define MBX_OP_EQ 0
#define MBX_OP_LT 1
#define MBX_OP_GT 2
#define MBX_OP_NE 3
#define MBX_OP_LE 4
#define MBX_OP_GE 5
#define MBX_OP_NOT 6
#define MBX_OP_NOP 7
#define MBX_OP_RANGE 8

/* ---- global.IndexType (R/global/IndexType.java:10-13) --------------------- */
#define MBX_INDEX_NONE 0
#define MBX_INDEX_BTREE 1
#define MBX_INDEX_HASH 2
#define MBX_INDEX_BITMAP 3

/* ---- bitmap combine ops (java.util.BitSet and / or / andNot) ------------- */
#define MBX_BM_AND 0
#define MBX_BM_OR 1
#define MBX_BM_ANDNOT 2

/* ---- limits of one compiled predicate (checked, MBX_E_UNSUPPORTED) ------ */
#define MBX_MAX_TERMS 32        /* CondExprs in one CNF */
#define MBX_MAX_CONJ 32         /* conjuncts */
#define MBX_MAX_PRED_COLS 8     /* distinct columns a CNF (+ aggregate) touches */
#define MBX_MAX_STR_BYTES 256   /* char(n) size and string literal bytes */

typedef struct mbx_ctx mbx_ctx;
typedef struct mbx_table mbx_table;
typedef struct mbx_plan mbx_plan;
typedef struct mbx_bitmap mbx_bitmap;
typedef struct mbx_cursor mbx_cursor;

/* One column of a Columnarfile (Columnarfile.getAttributeTypes /
 * getStringSizes, R/columnar/Columnarfile.java:239-359). */
typedef struct {
  int32_t attr_type; /* MBX_ATTR_INTEGER / _REAL / _STRING */
  int32_t size;      /* char(n): n payload bytes; ignored (4) for int/real */
} mbx_col_desc;

/* iterator.Operand + CondExpr.typeN (R/iterator/Operand.java, CondExpr.java:12-57). */
typedef struct {
  int32_t type;        /* MBX_ATTR_SYMBOL: column reference; else the literal's AttrType */
  int32_t fld;         /* FldSpec.offset, 1-based (RelSpec.outer) when type == SYMBOL */
  int32_t integer;     /* Operand.integer */
  float real;          /* Operand.real */
  const char *string;  /* Operand.string as modified UTF-8 (JNI GetStringUTFChars), not NUL-terminated */
  int32_t string_len;  /* bytes */
} mbx_operand;

/* iterator.CondExpr: `operand1 op operand2` (R/iterator/CondExpr.java:12-57). */
typedef struct {
  int32_t op;          /* MBX_OP_* */
  mbx_operand operand1;
  mbx_operand operand2;
  int32_t index_type;  /* CondExpr.indexType (only ColumnarIndexScan reads it) */
} mbx_condexpr;

/* CondExpr[] in CNF, flattened: conjunct c is the OR-list
 * conds[conj_offsets[c] .. conj_offsets[c+1]) (the .next chain), conjuncts
 * are AND-ed (the null-terminated array).  nconj == 0 is `p == null` (true),
 * R/iterator/PredEval.java:46-49. */
typedef struct {
  const mbx_condexpr *conds;
  const int32_t *conj_offsets; /* nconj + 1 entries */
  int32_t nconj;
} mbx_cnf;

/* COUNT / SUM / MIN / MAX of one column over the selected rows (no
 * reference equivalent; COUNT == Query's resultCount, R/input/Query.java:147). */
typedef struct {
  int64_t count;
  int32_t agg_type;   /* AttrType of the aggregated column */
  int32_t pad_;
  int64_t isum;       /* attrInteger: exact */
  int32_t imin, imax; /* attrInteger (INT32_MAX / INT32_MIN when count == 0) */
  double fsum;        /* attrReal: double accumulation, deterministic order */
  float fmin, fmax;   /* attrReal (+inf / -inf when count == 0) */
} mbx_agg;

/* ---- library ------------------------------------------------------------- */
int mbx_abi_version(void);
const char *mbx_last_error(void);
int mbx_device_count(int32_t *n);

/* ---- context: SystemDefs (R/global/SystemDefs.java:19-95) minus the disk;
 * one HIP stream on `device` -------------------------------------------- */
int mbx_init(int32_t device, mbx_ctx **out);
int mbx_free(mbx_ctx *ctx);
int mbx_sync(mbx_ctx *ctx);
/* the hipStream_t every launch of this context goes to (for event timing) */
void *mbx_stream(mbx_ctx *ctx);

/* ---- tables: the HBM image of a Columnarfile ------------------------------
 * Replaces opening one heap.Scan per column (TupleScan, R/columnar/TupleScan.java:29-47)
 * and reading `cf.md` (Columnarfile.getMarkedDeleted): columns are staged once
 * as contiguous chunks.  host_cols[j]: nrows values in position order --
 * int32 / float32 host order, or `size` bytes of zero-padded modified UTF-8
 * per row for char(n).  deleted_words: the markedDeleted BitSet image
 * (ceil(nrows/64) words) or NULL.  The library copies; the caller keeps
 * ownership of its buffers. */
int mbx_table_stage(mbx_ctx *ctx, const mbx_col_desc *cols, int32_t ncols, int64_t nrows,
                    const void *const *host_cols, const uint64_t *deleted_words,
                    int64_t row_offset, mbx_table **out);
/* Same, over device buffers the caller already holds in the table's device
 * layout (int32/float32 arrays; strings padded to a multiple of 4 bytes per
 * row in the device string encoding).  No copy; buffers must
 * outlive the table. */
int mbx_table_wrap(mbx_ctx *ctx, const mbx_col_desc *cols, int32_t ncols, int64_t nrows,
                   const void *const *dev_cols, const uint64_t *dev_deleted_words,
                   int64_t row_offset, mbx_table **out);
int mbx_table_free(mbx_table *t);
int mbx_table_info(const mbx_table *t, int64_t *nrows, int64_t *row_offset, int32_t *ncols);
/* Column group (no reference counterpart; a physical layout choice of the
 * executor): a device-built, table-owned row-interleaved copy of 2..4 of the
 * table's 4-byte columns (cols, 0-based; each column in at most one group).
 * Late materialisation that projects grouped columns (mbx_cursor_open,
 * mbx_materialize*, mbx_cnf_cursor_open, mbx_cnf_materialize_async with
 * <= 4 four-byte columns) gathers them from the group, so one row's values
 * share a line: fewer HBM lines for a sparse selection.  Results are
 * identical; scans keep reading the columns.  Costs ncols x 4 bytes x nrows
 * of HBM.  A group is a snapshot taken at this call: for a table over caller
 * memory (mbx_table_wrap) whose columns the caller rewrites, drop the groups
 * (ncols = 0, cols may be NULL) and group again after the rewrite -- until
 * then gathers of grouped columns return the snapshot's values (and a HIP
 * graph captured before a drop must not be replayed after it). */
int mbx_table_group(mbx_ctx *ctx, mbx_table *t, const int32_t *cols, int32_t ncols);

/* ---- predicates: PredEval.Eval over one tuple (R/iterator/PredEval.java:25-183),
 * compiled once for one table.  Type rules follow the reference: the
 * comparison type is operand1's, both operands must carry it (else
 * MBX_E_TYPE); FldSpec offsets are checked (MBX_E_RANGE). ----------------- */
int mbx_plan_compile(mbx_ctx *ctx, const mbx_table *t, const mbx_cnf *cnf, mbx_plan **out);
int mbx_plan_free(mbx_plan *p);

/* ---- ColumnarFileScan (R/iterator/ColumnarFileScan.java:156-188) --------- */
/* COUNT of get_next() results: Query.executeFileScan's resultCount. */
int mbx_scan_count(mbx_ctx *ctx, const mbx_plan *p, int64_t *count);
/* enqueue only; *dev_count (device memory) receives the count */
int mbx_scan_count_async(mbx_ctx *ctx, const mbx_plan *p, int64_t *dev_count);
/* Count frame: the same COUNT (Query.executeFileScan's resultCount,
 * R/input/Query.java:137-152) enqueued with no in-launch finalize -- every
 * block adds its packed (count, NaN block, arrival) word to one of 32 slots
 * of a caller-zeroed, 128-byte-aligned frame of MBX_COUNT_FRAME_WORDS int64
 * words (slot s at word 16 s) with a no-return atomic, so the launch ends
 * without the last-arriver round trips.  Frames are additive: an in-place
 * int64 sum all-reduce of whole frames (mbx_comm_allreduce_count_async with
 * n = MBX_COUNT_FRAME_WORDS) combines ranks, and mbx_count_frame_decode
 * reads the total from a host copy.  A NaN in a float comparison is counted
 * per block in the frame and also raised at the next mbx_sync, like every
 * async scan.  Tables up to 2^36 rows per rank and 16 ranks per frame. */
#define MBX_COUNT_FRAME_WORDS 512
int mbx_scan_count_frame_async(mbx_ctx *ctx, const mbx_plan *p, int64_t *dev_frame);
int mbx_count_frame_decode(const int64_t *host_frame, int64_t *count, int64_t *nan_blocks, int64_t *arrivals);
/* 1 when the frames of nranks ranks whose scans have at most nblocks blocks
 * each sum exactly (every slot's summed arrivals and NaN blocks < 4096),
 * else 0 (then combine in-launch-finalized counts instead) */
int mbx_count_frame_fits(int64_t nblocks, int32_t nranks);
/* blocks of this plan's COUNT launch (= the arrivals one frame records) */
int mbx_scan_blocks(mbx_ctx *ctx, const mbx_plan *p, int64_t *blocks);
/* the selection as a device BitSet (the get_next_tid() stream as positions) */
int mbx_scan_bitmap(mbx_ctx *ctx, const mbx_plan *p, mbx_bitmap **out, int64_t *count);
int mbx_scan_bitmap_async(mbx_ctx *ctx, const mbx_plan *p, mbx_bitmap *out);
/* the get_next_tid() stream as ascending positions (TID.position, global:
 * row_offset added; SURVEY 8(b) mbx_scan_select): ONE launch (k_scan_select:
 * BitSet scan, decoupled look-back, positions) for plans of 1-4 int literal
 * terms on <= 4 four-byte columns (knob scan_select_fused), else two
 * launches, the BitSet scan and the compaction over its segment counts
 * (DESIGN.md section 3).  host_ids holds up to cap positions; their device
 * scratch is sized to the count and released before the call returns. */
int mbx_scan_select(mbx_ctx *ctx, const mbx_plan *p, int64_t *host_ids, int64_t cap, int64_t *n);
/* enqueue only: BitSet into `out` (nbits = the table's rows), positions into
 * dev_ids (capacity: the selected rows, at most the table's rows), the count
 * into *dev_count (device memory) */
int mbx_scan_select_async(mbx_ctx *ctx, const mbx_plan *p, mbx_bitmap *out, int64_t *dev_ids,
                          int64_t *dev_count);
/* COUNT/SUM/MIN/MAX of column `agg_col` (0-based) over the selection */
int mbx_scan_aggregate(mbx_ctx *ctx, const mbx_plan *p, int32_t agg_col, mbx_agg *out);
int mbx_scan_aggregate_async(mbx_ctx *ctx, const mbx_plan *p, int32_t agg_col, mbx_agg *dev_out);

/* ---- device BitSets (BitMapFile.getBitSet / java.util.BitSet, R/bitmap/BitMapFile.java:478,
 * R/bitmap/BM.java:179-215: bit p%64 of word p/64) ------------------------ */
int mbx_bitmap_alloc(mbx_ctx *ctx, int64_t nbits, mbx_bitmap **out);
int mbx_bitmap_upload(mbx_ctx *ctx, int64_t nbits, const uint64_t *host_words, mbx_bitmap **out);
int mbx_bitmap_download(mbx_ctx *ctx, const mbx_bitmap *b, uint64_t *host_words, int64_t nwords);
int mbx_bitmap_info(const mbx_bitmap *b, int64_t *nbits, int64_t *nwords, int64_t *count);
int mbx_bitmap_free(mbx_bitmap *b);
/* BitSet.and / or / andNot into a new bitmap (+ cardinality) */
int mbx_bitmap_combine(mbx_ctx *ctx, int32_t op, const mbx_bitmap *a, const mbx_bitmap *b,
                       mbx_bitmap **out, int64_t *count);
/* ColumnarIndexScan's CNF over index BitSets (R/index/ColumnarIndexScan.java:130-181) and
 * ColumnIndexScan.getBitSet's value-set OR (R/index/ColumnIndexScan.java:656-740):
 * result = AND_c ( OR_{k in conj c} bms[k] ) AND NOT deleted, in one pass.
 * conj_offsets has nconj + 1 entries; an empty conjunct is all-zero.
 * deleted may be NULL. */
int mbx_bitmap_cnf(mbx_ctx *ctx, int64_t nbits, const mbx_bitmap *const *bms,
                   const int32_t *conj_offsets, int32_t nconj, const mbx_bitmap *deleted,
                   mbx_bitmap **out, int64_t *count);
int mbx_bitmap_cnf_async(mbx_ctx *ctx, const mbx_bitmap *const *bms, const int32_t *conj_offsets,
                         int32_t nconj, const mbx_bitmap *deleted, mbx_bitmap *out);
/* Columnarfile.createBitMapIndex (R/columnar/Columnarfile.java:698-753): one
 * BitMapFile per value, bit p set where column `col` (0-based) equals
 * values[v]; deleted positions stay clear (the reference builds the index
 * from a ColumnScan, which skips them).  One pass over the column for all
 * values. */
int mbx_bitmap_index_build(mbx_ctx *ctx, const mbx_table *t, int32_t col, const mbx_operand *values,
                           int32_t nvalues, mbx_bitmap **out);

/* ColumnarIndexScan end to end in ONE kernel launch (R/index/ColumnarIndexScan.java:130-181, then the
 * nextSetBit + getRecord loop :287-308): the CNF of index BitSets exactly as mbx_bitmap_cnf (the CNF's
 * BitSet itself is never stored), then the positions (dev_ids, may be NULL) and the rows of the
 * projected columns (proj: 0-based, at most 16; dev_out[j] receives column proj[j] in the table's
 * device row layout -- 4 bytes for int / float, the padded device string image for char(n), as
 * mbx_materialize_async) of every selected row, and the count in *dev_count.  Each block publishes its
 * count and takes its output offset from its predecessors' counts (decoupled look-back) -- the
 * one-launch form of mbx_bitmap_cnf_async + mbx_materialize_async.  Up to 4 four-byte columns are
 * loaded into registers before the look-back resolves; other projections copy rows. */
int mbx_cnf_materialize_async(mbx_ctx *ctx, const mbx_table *t, const mbx_bitmap *const *bms,
                              const int32_t *conj_offsets, int32_t nconj, const mbx_bitmap *deleted,
                              const int32_t *proj, int32_t nproj, int64_t *dev_ids,
                              void *const *dev_out, int64_t *dev_count);

/* ---- late materialisation: the nextSetBit loops + Heapfile.findRID/getRecord
 * per output column (R/index/ColumnarIndexScan.java:287-308,
 * R/iterator/ColumnarColumnScan.java:151-176, R/iterator/Projection.java:103-146) */
/* ascending global positions of the set bits (BitSet.nextSetBit order) */
int mbx_bitmap_select(mbx_ctx *ctx, const mbx_bitmap *b, int64_t row_offset, int64_t *host_ids,
                      int64_t cap, int64_t *n);
/* positions + projected column values of every selected row, column-major
 * into host buffers (proj: 0-based columns; value layout as in
 * mbx_table_stage; ids may be NULL).  All *n rows, however large: the rows
 * cross PCIe in cursor batches of <= 64 MiB, each copied to its offset. */
int mbx_materialize(mbx_ctx *ctx, const mbx_table *t, const mbx_bitmap *sel, const int32_t *proj,
                    int32_t nproj, int64_t *host_ids, void *const *host_out, int64_t cap, int64_t *n);
/* device-side variant (outputs stay in HBM: dev_ids / dev_out[j] of `cap` rows) */
int mbx_materialize_async(mbx_ctx *ctx, const mbx_table *t, const mbx_bitmap *sel,
                          const int32_t *proj, int32_t nproj, int64_t *dev_ids,
                          void *const *dev_out, int64_t *dev_count);

/* ---- iterator.Iterator get_next() batching (R/iterator/Iterator.java:12-141):
 * a cursor holds the materialised selection in HBM and hands it out in
 * batches; get_next() of a Java/C++ Iterator walks one batch at a time. */
int mbx_cursor_open(mbx_ctx *ctx, const mbx_table *t, const mbx_bitmap *sel, const int32_t *proj,
                    int32_t nproj, mbx_cursor **out);
int mbx_cursor_count(const mbx_cursor *c, int64_t *count);
/* At most max_rows rows per call, fewer when max_rows rows of the projection
 * (8 + its host widths per row) would exceed 64 MiB of batch buffer: *n <
 * max_rows is not the end of the stream, *n == 0 is. */
int mbx_cursor_next(mbx_cursor *c, int64_t max_rows, int64_t *host_ids, void *const *host_out,
                    int64_t *n);
/* The same batch without a copy: *ids and cols[j] (an array of nproj
 * pointers the caller provides) point into the cursor's pinned batch buffer
 * -- positions, then each projected column in the mbx_materialize host
 * layout -- valid until the next mbx_cursor_next / _next_view / _restart /
 * _close on this cursor.  A batch crosses PCIe as one copy (packed on the
 * device), so a caller that consumes rows in place (Iterator.get_next filling
 * its Jtuple, the JNI glue filling int[] / String[]) touches each byte once. */
int mbx_cursor_next_view(mbx_cursor *c, int64_t max_rows, const int64_t **ids, const void **cols, int64_t *n);
int mbx_cursor_restart(mbx_cursor *c); /* Iterator.restart() */
int mbx_cursor_close(mbx_cursor *c);   /* Iterator.close(), idempotent via free */
/* Delivery is double buffered: mbx_cursor_next returns batch k from pinned
 * host memory and has already enqueued the device -> host copy of batch k+1
 * (same max_rows) into a second pinned buffer, so the caller's consumption of
 * batch k overlaps the copy.  Statistics: rows handed out so far, bytes copied
 * device -> host (no reference counterpart). */
int mbx_cursor_stats(const mbx_cursor *c, int64_t *delivered, int64_t *d2h_bytes);
/* ColumnarIndexScan (R/index/ColumnarIndexScan.java:79-182 + get_next :287-308) as a cursor in ONE
 * kernel launch: the CNF of index BitSets (as mbx_bitmap_cnf) straight into the cursor's positions and
 * projected rows (k_cnf_select, as mbx_cnf_materialize_async, any projection); mbx_cursor_next then
 * hands out get_next() batches in nextSetBit order. */
int mbx_cnf_cursor_open(mbx_ctx *ctx, const mbx_table *t, const mbx_bitmap *const *bms,
                        const int32_t *conj_offsets, int32_t nconj, const mbx_bitmap *deleted,
                        const int32_t *proj, int32_t nproj, mbx_cursor **out);
/* The same, launch only: the cursor's rows are written on the context
 * stream, the count lands in the cursor's device slot *dev_count (may be
 * NULL) -- e.g. for mbx_comm_allgather_count_async, whose result gives every
 * shard its offset in the concatenated stream; the first mbx_cursor_count or
 * mbx_cursor_next waits for it.  One launch per GPU, all GPUs in flight. */
int mbx_cnf_cursor_launch(mbx_ctx *ctx, const mbx_table *t, const mbx_bitmap *const *bms,
                          const int32_t *conj_offsets, int32_t nconj, const mbx_bitmap *deleted,
                          const int32_t *proj, int32_t nproj, mbx_cursor **out, int64_t **dev_count);

/* ---- multi-GPU: row-range shards + one RCCL combine over xGMI ------------
 * SURVEY.md 8(e), DESIGN.md section 6.  The reference engine is one process
 * (R/global/SystemDefs.java:6-9); a drop-in caller either drives every GPU
 * of the node from that process (mbx_comm_init_all: one context per GPU, one
 * RCCL clique, the *_all collectives in one RCCL group) or runs one process
 * per GPU (mbx_comm_init_rank with an id from mbx_comm_unique_id, shared by
 * the launcher).  Rows are independent, so scans never communicate; a
 * shard's table is staged with row_offset = its first position, and the one
 * exchange step combines per-shard results:
 *   COUNT             -> in-place int64 all-reduce (SUM), exact in any order
 *   COUNT/SUM/MIN/MAX -> all-gather of every rank's 48-byte mbx_agg, folded
 *                        in rank order on the device (int64 sums exact, the
 *                        double SUM of the per-rank partials in rank order,
 *                        MIN/MAX over the per-rank values)
 *   positions         -> all-gather of the per-rank counts (the concatenation
 *                        offsets; shard order = ascending global positions)
 * Stream order: a collective runs after everything already enqueued on the
 * context stream -- on the context stream itself (the default), or with the
 * tuning knob comm_same_stream = 0 (mbx_set_tuning) on the
 * communicator's exchange stream, which the context stream does not wait for
 * (the next scans may overlap it; inside a captured HIP graph on this ROCm
 * they do not, and the fork costs more than it hides).  mbx_sync waits for
 * both; mbx_comm_wait makes later context work (device side) wait for it. */
typedef struct mbx_comm mbx_comm;
#define MBX_COMM_ID_BYTES 128

/* [begin, end) of shard `shard` of `nshards` over nrows positions: begins are
 * multiples of 64 (BitSet words never straddle shards); non-empty ranges tile
 * [0, nrows) in shard order */
int mbx_shard_bounds(int64_t nrows, int32_t nshards, int32_t shard, int64_t *begin, int64_t *end);
int mbx_comm_unique_id(void *id /* MBX_COMM_ID_BYTES */);
int mbx_comm_init_rank(mbx_ctx *ctx, int32_t nranks, int32_t rank, const void *id, mbx_comm **out);
/* one process: ctxs[i] (distinct devices) becomes rank i of one clique */
int mbx_comm_init_all(mbx_ctx *const *ctxs, int32_t n, mbx_comm **outs);
int mbx_comm_free(mbx_comm *comm);
int mbx_comm_info(const mbx_comm *comm, int32_t *nranks, int32_t *rank);
/* the context stream waits (on the device) for the collectives enqueued so far */
int mbx_comm_wait(mbx_comm *comm);
int mbx_comm_allreduce_count_async(mbx_comm *comm, int64_t *dev_counts, int64_t n);
int mbx_comm_allreduce_agg_async(mbx_comm *comm, mbx_agg *dev_rec);
/* One COUNT query of this rank's shard combined over all ranks into
 * *dev_count (Query.executeFileScan's resultCount, R/input/Query.java:121-155,
 * for the whole row-range-sharded table): the scan launch leaves one count
 * per block in dev_parts (parts_cap int64 slots, device memory, caller-owned;
 * ~1024 suffice, one buffer per query in flight) and does no finalize; the
 * exchange stream sums them into *dev_count and all-reduces it -- the sum and
 * the collective overlap the context stream's next scan.  A plan with a float
 * term keeps the scan's own finalize (its NaN check): scan, then the
 * all-reduce, dev_parts unused. */
int mbx_comm_scan_count_async(mbx_comm *comm, const mbx_plan *plan, int64_t *dev_parts, int64_t parts_cap,
                              int64_t *dev_count);
/* dev_all[r] = rank r's *dev_count (device memory, nranks entries) */
int mbx_comm_allgather_count_async(mbx_comm *comm, const int64_t *dev_count, int64_t *dev_all);
/* The aggregate combine's fold alone: *dev_out = the rank-ordered fold of
 * dev_recs[0..n) (device memory; dev_out may alias dev_recs[0]) on the context
 * stream -- exactly what mbx_comm_allreduce_agg_async runs after its
 * all-gather (dist.fold_aggregates restated on the device: COUNT and int SUM
 * exact, the double SUM added in record order, MIN / MAX over the records,
 * whose empty shards carry the identities). */
int mbx_agg_fold_async(mbx_ctx *ctx, const mbx_agg *dev_recs, int32_t n, mbx_agg *dev_out);
/* one process, n communicators of one mbx_comm_init_all clique (rank order) */
int mbx_comm_allreduce_count_all(mbx_comm *const *comms, int32_t n, int64_t *const *dev_counts, int64_t count);
int mbx_comm_allreduce_agg_all(mbx_comm *const *comms, int32_t n, mbx_agg *const *dev_recs);
/* dev_alls[i][r] = rank r's *dev_counts[r], for every rank i (one grouped all-gather) */
int mbx_comm_allgather_count_all(mbx_comm *const *comms, int32_t n, const int64_t *const *dev_counts,
                                 int64_t *const *dev_alls);

/* ---- HIP graphs: a repeated query (scan + exchange) captured once and
 * replayed with one launch.  Between begin and end the context's *_async
 * calls and its communicator's collectives are recorded, not run; scratch
 * must already be sized by one uncaptured call of the same query (a capture
 * allocates nothing).  Replays run on the context stream. */
typedef struct mbx_graph mbx_graph;
int mbx_graph_begin(mbx_ctx *ctx);
int mbx_graph_end(mbx_ctx *ctx, mbx_graph **out);
int mbx_graph_launch(mbx_graph *g);
int mbx_graph_free(mbx_graph *g);

/* ---- device result slots for callers without a HIP allocator of their own
 * (the JNI glue: *_async results and the collectives' buffers live in device
 * memory).  No reference counterpart.  mbx_dev_alloc zero-fills; download
 * waits for the context stream first. */
int mbx_dev_alloc(mbx_ctx *ctx, int64_t bytes, void **dev);
int mbx_dev_free(mbx_ctx *ctx, void *dev);
int mbx_dev_download(mbx_ctx *ctx, const void *dev, void *host, int64_t bytes);

/* ---- diagnostics (no reference counterpart): the scan's load pattern with
 * the predicate removed, over the 4-byte columns cols[0..ncols) (ncols <= 4)
 * of t's full 256-row tiles, enqueued on mbx_stream(ctx).  Timed by the
 * caller; it is the measured read ceiling the scan's roofline is set beside.
 * tiles_per_block <= 0: the scan's own segment size; interleave != 0:
 * grid-stride over `grid` blocks instead of segments. */
int mbx_probe_read(mbx_ctx *ctx, const mbx_table *t, const int32_t *cols, int32_t ncols,
                   int64_t tiles_per_block, int32_t interleave, int64_t grid);
/* A/B tuning knobs of this context, no reference
 * counterpart.  Every context starts on the production defaults: the library
 * reads no environment (a -DMBX_DIAG build, tools/build_diag.sh, also takes
 * MBX_<KNOB> environment values at mbx_init).  knob: "tiles_per_block", "force_generic",
 * "scan_hoist", "scan_ri", "sink_lds", "ticket_groups", "fin_mode",
 * "join_plain", "distinct_lds_probes", "gather_fused", "gather_pair" (0: two 4-byte loads per grouped pair row),
 * "select_blocks", "select_dbg", "cursor_prefetch", "scan_select_fused", "scan_select_waves", "select_flag_stride",
 * "comm_same_stream", "scan_words_wt", and the one-launch ColumnarIndexScan's (k_cnf_select) "cnf_lookback" (0 auto,
 * 1 chained, 2 polled), "cnf_flag_stride" (1 or 16), "cnf_blocks" (0: 1024), "cnf_store" (0 default, 1 plain,
 * 2 write-through, 3 nontemporal); "reset" restores the defaults. */
int mbx_set_tuning(mbx_ctx *ctx, const char *knob, int64_t value);
/* per-block wall_clock64() stamps (start, loads in, after the block barrier,
 * end) of the last compaction launched with select_dbg bit 3: 4 * nblocks
 * int64 into host (diagnostic of DESIGN.md section 5) */
int mbx_diag_select_stamps(mbx_ctx *ctx, int64_t *host, int64_t nblocks);
/* the epoch the next one-launch selection (k_scan_select / k_cnf_select)
 * counts from (the look-back words' lb[0], 0 .. 2^31 - 1): lets a test run
 * launches across the epoch wrap (diagnostic of DESIGN.md section 3) */
int mbx_diag_lookback_epoch(mbx_ctx *ctx, int64_t epoch);

#ifdef __cplusplus
}
#endif
#endif /* MBX_H */
