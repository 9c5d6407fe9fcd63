package global;

import java.nio.ByteBuffer;

import iterator.CondExpr;

/**
 * The MI355X executor's C-ABI (include/mbx.h, include/mbx_db.h) as seen from
 * the engine: jni/mbx_jni.c implements every method.  Handles are the C-ABI's
 * opaque pointers.  Errors arrive as the reference's checked exceptions
 * (PredEvalException, FileScanException, IndexException,
 * heap.FieldNumberOutOfBoundException, ChainException) carrying
 * mbx_last_error().  Not compiled in this image (no JDK): see jni/Makefile.
 */
public final class Native {
  static { System.loadLibrary("mbx_jni"); }          // libmbx_jni.so -> libmbx.so

  private Native() {}

  public static final int BM_AND = 0, BM_OR = 1, BM_ANDNOT = 2;   // MBX_BM_*
  public static final int AGG_RECORD_BYTES = 48;                   // sizeof(mbx_agg)

  // context: one per GPU (SystemDefs' singletons, R/global/SystemDefs.java:6-9)
  public static native int deviceCount();
  public static native long init(int device) throws Exception;
  public static native void free(long ctx);
  public static native void sync(long ctx) throws Exception;

  // tables: the HBM image of a Columnarfile
  public static native long tableStage(long ctx, int[] attrTypes, short[] sizes, long nrows, ByteBuffer[] cols,
                                       long[] deleted, long rowOffset) throws Exception;
  public static native void tableFree(long table);
  /** positions of the staged table (the bits of its BitSets) */
  public static native long tableRows(long table) throws Exception;
  public static native long dbOpen(String path) throws Exception;
  public static native void dbClose(long db);
  public static native long dbStage(long ctx, long db, String columnarFile) throws Exception;
  public static native long dbBitmapStage(long ctx, long db, String bitMapFile, long nbits) throws Exception;
  /** positions [rowBegin, rowEnd) of a Columnarfile (rowBegin % 64 == 0): one shard, only its pages read */
  public static native long dbStageRange(long ctx, long db, String columnarFile, long rowBegin, long rowEnd)
      throws Exception;
  /** bits [bitBegin, bitBegin + nbits) of a BitMapFile (bitBegin % 64 == 0): a shard's slice */
  public static native long dbBitmapStageRange(long ctx, long db, String bitMapFile, long bitBegin, long nbits)
      throws Exception;
  public static native long tableRowOffset(long table) throws Exception;
  /** a row-interleaved copy of 2..4 four-byte columns the sparse gathers read (mbx_table_group) */
  public static native void tableGroup(long ctx, long table, int[] cols) throws Exception;
  /** the Columnarfile's positions (highest position + 1) from its directory (mbx_db_columnar_info) */
  public static native long dbColumnarRows(long db, String columnarFile) throws Exception;

  // PredEval over a table (R/iterator/PredEval.java:25-183)
  public static native long planCompile(long ctx, long table, CondExpr[] filter) throws Exception;
  public static native void planFree(long plan);
  public static native long scanCount(long ctx, long plan) throws Exception;
  public static native long scanBitmap(long ctx, long plan) throws Exception;
  public static native long[] scanSelect(long ctx, long plan, long cap) throws Exception;
  /** {count, aggType, isum, imin, imax, doubleBits(fsum), floatBits(fmin), floatBits(fmax)} */
  public static native long[] scanAggregate(long ctx, long plan, int col) throws Exception;
  public static native void scanCountAsync(long ctx, long plan, long devCount) throws Exception;
  public static native void scanAggregateAsync(long ctx, long plan, int col, long devRec) throws Exception;

  // device BitSets (java.util.BitSet long[] images)
  public static native long bitmapUpload(long ctx, long nbits, long[] words) throws Exception;
  public static native long[] bitmapDownload(long ctx, long bitmap) throws Exception;
  public static native long bitmapCardinality(long bitmap) throws Exception;
  public static native long bitmapCnf(long ctx, long nbits, long[] bitmaps, int[] conjOffsets, long deleted)
      throws Exception;
  public static native long bitmapCombine(long ctx, int op, long a, long b) throws Exception;
  /** ColumnarIndexScan in one launch: CNF + positions (devIds 0: none) + the projected columns' rows into
   *  device slots (devAlloc; char(n) in the device row layout); returns the selected row count
   *  (mbx_cnf_materialize_async; waits for the launch only -- an earlier async scan's NaN is not raised here) */
  public static native long cnfMaterialize(long ctx, long table, long[] bitmaps, int[] conjOffsets, long deleted,
                                           int[] proj, long devIds, long[] devOut, long devCount) throws Exception;
  public static native void bitmapFree(long bitmap);

  // late materialisation in batches (Iterator.get_next)
  public static native long cursorOpen(long ctx, long table, long selection, int[] proj) throws Exception;
  /** ColumnarIndexScan (CNF of index BitSets minus deleted) + positions + projection in ONE launch, as a
   *  cursor (mbx_cnf_cursor_open); deleted 0: none */
  public static native long cnfCursorOpen(long ctx, long table, long[] bitmaps, int[] conjOffsets, long deleted,
                                          int[] proj) throws Exception;
  /** the same, launch only (mbx_cnf_cursor_launch): {cursor, device pointer of its count} */
  public static native long[] cnfCursorLaunch(long ctx, long table, long[] bitmaps, int[] conjOffsets, long deleted,
                                              int[] proj) throws Exception;
  public static native long cursorCount(long cursor) throws Exception;
  /** {long[] positions, Object[] columns (int[] / float[] / String[])}, or null at the end */
  public static native Object[] cursorNext(long cursor, int maxRows, int[] types, short[] sizes) throws Exception;
  public static native void cursorRestart(long cursor) throws Exception;
  public static native void cursorClose(long cursor);

  // device result slots + the multi-GPU exchange (RCCL over xGMI)
  public static native long devAlloc(long ctx, long bytes) throws Exception;
  public static native void devFree(long ctx, long dev);
  public static native long countDownload(long ctx, long devCount) throws Exception;
  public static native long[] aggDownload(long ctx, long devRec) throws Exception;
  public static native long[] shardBounds(long nrows, int nshards, int shard) throws Exception;
  public static native byte[] commUniqueId() throws Exception;
  public static native long commInitRank(long ctx, int nranks, int rank, byte[] id) throws Exception;
  public static native long[] commInitAll(long[] ctxs) throws Exception;
  public static native void commFree(long comm);
  public static native void commAllreduceCount(long comm, long devCount) throws Exception;
  public static native void commAllreduceAgg(long comm, long devRec) throws Exception;
  public static native void commAllreduceCountAll(long[] comms, long[] devCounts) throws Exception;
  public static native void commAllreduceAggAll(long[] comms, long[] devRecs) throws Exception;
  /** devAlls[i] (nranks longs, devAlloc) receives every rank's devCounts[r]: one grouped all-gather */
  public static native void commAllgatherCountAll(long[] comms, long[] devCounts, long[] devAlls) throws Exception;
  public static native void commWait(long comm) throws Exception;
  public static native long[] longsDownload(long ctx, long dev, int n) throws Exception;

  // joins (include/mbx_join.h): nlj / bmj pairs on the GPU in the reference's order
  public static final int JOIN_BMJ = 0, JOIN_NLJ = 1;
  /** terms: {op, outerCol, innerCol} triples (0-based file columns); returns the join result handle */
  public static native long join(long ctx, long outerTable, long outerSel, long innerTable, long innerSel,
                                 int[] terms, int[] conjOffsets, int order, long outerBlock) throws Exception;
  /** {pairs, passes} */
  public static native long[] joinInfo(long result) throws Exception;
  /** pairs [start, start + n): {long[] outer positions, long[] inner positions, int[] pass} */
  public static native Object[] joinFetch(long ctx, long result, long start, int n) throws Exception;
  public static native void joinFree(long result);
  /** late materialisation by positions (mbx_gather): one int[] / float[] / String[] per projected column */
  public static native Object[] gather(long ctx, long table, long[] positions, int[] proj, int[] types,
                                       short[] sizes) throws Exception;
}
