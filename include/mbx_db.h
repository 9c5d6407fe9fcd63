/*
 * mbx_db.h -- Minibase DB files on the MI355X path.
 *
 * Reads and writes the reference's on-disk format so the GPU executor can
 * stage a Columnarfile straight from a Minibase DB file (no JVM) and so
 * large DBs can be produced for the Java CPU baseline (BatchInsert only
 * knows the 1M-page default DB).  R/ = minijava/src of the reference.
 *
 * Format restated (big-endian throughout, R/global/Convert.java:18-126):
 *   - DB file = num_pages pages of 1024 bytes (GlobalConst.MINIBASE_PAGESIZE).
 *     Page 0 = DBFirstPage: next header page @0, entry count @4, file entries
 *     of 56 bytes from @8 {first page i32, name writeUTF}, numDBPages @1020
 *     (R/diskmgr/DB.java:866-1080).  Pages 1..ceil(num_pages/8192) = space map,
 *     one bit per page, LSB first within a byte (DB.java:245-330).
 *   - Heapfile = chain of directory HFPages whose records are DataPageInfo
 *     {availspace i16, recct i16, pid i32} (R/heap/DataPageInfo.java:29-70)
 *     + data HFPages: header slotCnt@0 usedPtr@2 freeSpace@4 type@6 prev@8
 *     next@12 cur@16, slots {len i16, off i16} from @20, records packed from
 *     the end (R/heap/HFPage.java:31-40,337-396).  Empty slot: len -1.
 *   - Columnarfile `cf` (R/columnar/Columnarfile.java:60-192): heapfile
 *     cf.hdr {ncols; types; sizes; names (writeUTF in 17-byte cells);
 *     bTreeExist; bitmapExist; "col.value" registry ...}, one heapfile cf.<i>
 *     per column (record = 4 bytes, or n+2 bytes writeUTF for char(n)),
 *     BitMapFile cf.md (deleted positions), heapfile cf.dtid.
 *   - Position of a record = recsPerDataPage * (dirPageIndex * 83 + dirSlot)
 *     + slot (R/heap/Heapfile.java:262-289,349-417).
 *   - BitMapFile = HFPage chain, one record of 1000 bytes per page =
 *     java.util.BitSet.toByteArray() chunk (R/bitmap/BM.java:60-215).
 *
 * Writer page allocation follows DB.allocate_page (first fit over the space
 * map) in the reference's call order, so a BatchInsert of the same rows
 * produces the same page numbers (tests/test_dbfile.py pins this against the
 * reference transcript, R/phase3_output:19-22,3172).
 */
#ifndef MBX_DB_H
#define MBX_DB_H

#include <stdint.h>

#include "mbx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mbx_db mbx_db;

#define MBX_DB_PAGE_SIZE 1024
#define MBX_DB_MAX_NAME 50        /* GlobalConst.MAX_NAME: file entry names */
#define MBX_DB_MAX_ATTR_NAME 15   /* GlobalConst.MAXATTRNAME */
#define MBX_DB_MAX_CF_NAME 15     /* GlobalConst.MAXFILENAME: Columnarfile names */

/* DB.openDB(name, num_pgs) (R/diskmgr/DB.java:64-110): create (truncate) a DB
 * file of max(num_pages, 2) zero pages with page 0 and the space map set up.
 * The file is sparse; pages are mapped, not read, until touched. */
int mbx_db_create(const char* path, int32_t num_pages, mbx_db** out);

/* DB.openDB(name) (R/diskmgr/DB.java:25-50): open an existing DB file. */
int mbx_db_open(const char* path, mbx_db** out);

/* Flush dirty pages (msync) and close.  Null is a no-op. */
int mbx_db_close(mbx_db* db);

/* DB.db_num_pages and the number of pages set in the space map. */
int mbx_db_info(const mbx_db* db, int32_t* num_pages, int32_t* allocated_pages);

/* DB.allocate_page(start, run_size) (R/diskmgr/DB.java:212-290): the first
 * run of free pages (first fit over the space map), marked in use; and
 * DB.add_file_entry (DB.java:420-500).  For files this library does not model
 * (B+-tree index files) so page numbering stays the reference's. */
int mbx_db_allocate_pages(mbx_db* db, int32_t run_size, int32_t* start);
int mbx_db_add_file_entry(mbx_db* db, const char* name, int32_t start);

/* DB.get_file_entry (R/diskmgr/DB.java:520-590): *first_page = the file's
 * first page, or -1 when no entry has that name (not an error). */
int mbx_db_file_entry(mbx_db* db, const char* name, int32_t* first_page);

/* Columnarfile(name, numColumns, attrNames, attrTypes, attrSizes)
 * (R/columnar/Columnarfile.java:60-192): creates cf.hdr (+ its 6 header
 * records), cf.0 .. cf.<n-1>, cf.md, cf.dtid.  cols[i].size is 4 for
 * int/float, n for char(n).  MBX_E_INVALID when it already exists. */
int mbx_db_columnar_create(mbx_db* db, const char* name, int32_t ncols, const mbx_col_desc* cols,
                           const char* const* attr_names);

/* Columnarfile.insertTuple for nrows rows in order (the BatchInsert loop,
 * R/input/BatchInsert.java:84-104; R/columnar/Columnarfile.java:400-470).
 * host_cols use the mbx_table_stage layout (int32 / float32 per row; char(n)
 * = n bytes of modified UTF-8, zero padded).  Appends after existing rows. */
int mbx_db_columnar_insert(mbx_db* db, const char* name, int64_t nrows, const void* const* host_cols);

/* Columnarfile(name) (R/columnar/Columnarfile.java:194-300): schema from
 * cf.hdr.  cols / attr_names (16-byte cells, NUL terminated) may be null;
 * they hold max_cols entries.  *nrows = highest position + 1 (the table size
 * mbx_db_stage produces), *live = records in cf.0 minus deleted positions
 * (Columnarfile.getTupleCnt counts cf.dtid records instead). */
int mbx_db_columnar_info(mbx_db* db, const char* name, int32_t max_cols, int32_t* ncols, mbx_col_desc* cols,
                         char* attr_names, int64_t* nrows, int64_t* live);

/* Columnarfile.markTupleDeleted (R/columnar/Columnarfile.java:812-835): sets
 * the position in cf.md and appends the TID record to cf.dtid. */
int mbx_db_mark_deleted(mbx_db* db, const char* name, int64_t position);

/* markTupleDeleted for n positions in order (one header read for the batch:
 * DeleteQuery marks every position its scan returns, R/input/DeleteQuery.java:105-180). */
int mbx_db_mark_deleted_many(mbx_db* db, const char* name, const int64_t* positions, int64_t n);

/* Columnarfile.purgeAllDeletedTuples (R/columnar/Columnarfile.java:837-925):
 * removes the record of every cf.dtid TID from every column heapfile
 * (HFPage compaction; emptied data pages freed, emptied directory pages
 * unlinked and freed -- which shifts the positions after them), clears the
 * deleted positions from every bitmap index and drops the shifted position
 * ranges (BitMapFile.purgeDelete), clears cf.md and recreates cf.dtid.
 * Positions of the surviving rows are otherwise unchanged (holes stay holes,
 * mbx_db_stage marks them deleted).  Not for files with B+-tree indexes. */
int mbx_db_purge(mbx_db* db, const char* name);

/* BitMapFile images (R/bitmap/BitMapFile.java:60-120, R/bitmap/BM.java:60-215).
 * write: creates `filename` (BMHEAD header page + one 1000-byte chunk page per
 * 8000 bits of BitSet.toByteArray(); MBX_E_INVALID if it exists or the
 * BitSet is empty -- BM.insertBitSet cannot store one).  read: *nwords_out =
 * words of the stored image (ceil(bytes/8)); words[] gets min(cap, that). */
int mbx_db_bitmap_write(mbx_db* db, const char* filename, const uint64_t* words, int64_t nwords);
int mbx_db_bitmap_read(mbx_db* db, const char* filename, uint64_t* words, int64_t nwords_cap, int64_t* nwords_out);

/* Columnarfile.createBitMapIndex(col) (R/columnar/Columnarfile.java:698-753)
 * on the GPU: distinct live values in first-occurrence order (k_distinct),
 * one BitSet per value (k_index_build4 / k_index_build) over `t` -- the
 * table mbx_db_stage produced for `name` -- then, in the reference's order,
 * one BitMapFile cf.bm.<col>.<value> header + hdr registry record "col.value"
 * per value, the BitSet chunks (BM.insertBitSet, values in java.util.HashMap
 * iteration order) and bitmapExist[col] = 1.  Int and char(n) columns, as in
 * the reference; at most 65536 distinct values.  *nvalues = values indexed
 * (0 when the column already had a bitmap index: the reference is a no-op). */
int mbx_db_create_bitmap_index(mbx_ctx* ctx, mbx_db* db, const char* name, const mbx_table* t, int32_t col,
                               int32_t* nvalues);

/* The bitmap-index registry of column col ("col.value" records of cf.hdr,
 * Columnarfile.java:150-162): *count values, written NUL-separated (modified
 * UTF-8 text of the value) into buf when it is large enough; *bytes = the
 * size needed. */
int mbx_db_bitmap_values(mbx_db* db, const char* name, int32_t col, char* buf, int64_t cap, int32_t* count,
                         int64_t* bytes);

/* BitMapFile `filename` -> a device bitmap of nbits bits (BM.readBitSet; bits
 * past nbits are dropped, missing words are zero), ready for
 * mbx_bitmap_cnf / mbx_materialize. */
int mbx_db_bitmap_stage(mbx_ctx* ctx, mbx_db* db, const char* filename, int64_t nbits, mbx_bitmap** out);

/* Stage a Columnarfile from the DB file into HBM: the used pages of the file
 * are copied to the device as they lie on disk and one k_page_decode launch
 * per column walks the slot directories, byte-swaps the records and rewrites
 * char(n) into the device string image.  The table keeps reference positions
 * (row p = position p); positions with no record (holes) and positions set in
 * cf.md become deleted rows, so every scan skips them exactly as TupleScan /
 * ColumnScan do.  MBX_E_INVALID if the column heapfiles disagree on
 * positions (Columnarfile.java:480-482 raises the same). */
int mbx_db_stage(mbx_ctx* ctx, mbx_db* db, const char* name, mbx_table** out);

/* One shard of a Columnarfile: positions [row_begin, row_end) (row_begin a
 * multiple of 64, row_end clipped to the file's positions) staged exactly as
 * mbx_db_stage stages the whole file -- same decode, same deleted rows -- into
 * a table with row_offset = row_begin.  Only the directory pages and this
 * range's data pages are read and copied: the shards of one file can be
 * staged by one process per GPU, or one process driving every GPU, without
 * any of them holding the others' rows (TupleScan / heap.Scan over a
 * position range, R/columnar/TupleScan.java:29-89, R/heap/Heapfile.java:262-289). */
int mbx_db_stage_range(mbx_ctx* ctx, mbx_db* db, const char* name, int64_t row_begin, int64_t row_end,
                       mbx_table** out);

/* Bits [bit_begin, bit_begin + nbits) of BitMapFile `filename` (bit_begin a
 * multiple of 64) as a device bitmap of nbits bits: one shard's slice of
 * BitMapFile.getBitSet() (BM.readBitSet, R/bitmap/BM.java:179-215) for a
 * table staged with mbx_db_stage_range. */
int mbx_db_bitmap_stage_range(mbx_ctx* ctx, mbx_db* db, const char* filename, int64_t bit_begin, int64_t nbits,
                              mbx_bitmap** out);

#ifdef __cplusplus
}
#endif

#endif /* MBX_DB_H */
