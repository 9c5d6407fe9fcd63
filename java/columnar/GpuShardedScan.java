package columnar;

import global.GpuContext;
import global.Native;
import iterator.CondExpr;

/**
 * One JVM driving every GPU of the node (SURVEY.md 8(e), DESIGN.md section 6).
 * A Columnarfile of the DB file is split into one 64-aligned row range per
 * GPU (Native.shardBounds, positions as long), and each range is staged
 * straight from the DB file onto its GPU (Native.dbStageRange ->
 * mbx_db_stage_range: only that range's pages are read; no column passes
 * through the JVM, so no 2 GB ByteBuffer limit -- C5's 16 GB char(16)
 * column included).  A query runs one scan per GPU and ONE RCCL exchange
 * over xGMI combines the per-shard results on the devices (COUNT: int64
 * all-reduce; COUNT/SUM/MIN/MAX: all-gather of the 48-byte records folded in
 * rank order, so the double SUM is reproducible for a given GPU count).  The
 * clique is GpuContext's, shared by every sharded scan of the JVM.  The
 * reference engine is one process (R/global/SystemDefs.java:6-9); so is
 * this.  Sharded index scans: {@link #indexScan}.
 */
public final class GpuShardedScan implements AutoCloseable {
  final long[] ctxs, tables, begins, ends;
  private final long[] slots, comms;
  final long db, nrows;
  final String name;
  private boolean closed;

  /** the Columnarfile `columnarFile` of the DB file GpuTables.open(...) named */
  public GpuShardedScan(String columnarFile) throws Exception {
    final int n = GpuContext.devices();
    name = columnarFile;
    db = GpuTables.dbHandle();                    // dirty unpinned frames flushed first
    nrows = Native.dbColumnarRows(db, columnarFile);
    ctxs = new long[n];
    tables = new long[n];
    slots = new long[n];
    begins = new long[n];
    ends = new long[n];
    try {
      for (int g = 0; g < n; g++) {
        ctxs[g] = GpuContext.ctx(g);
        long[] be = Native.shardBounds(nrows, n, g);
        begins[g] = be[0];
        ends[g] = be[1];
        tables[g] = Native.dbStageRange(ctxs[g], db, columnarFile, be[0], be[1]);
        slots[g] = Native.devAlloc(ctxs[g], Native.AGG_RECORD_BYTES);
      }
      comms = GpuContext.comms();                  // one RCCL clique, rank g = GPU g
    } catch (Exception e) {
      release();
      throw e;
    }
  }

  private long[] compile(CondExpr[] filter) throws Exception {
    long[] plans = new long[ctxs.length];
    try {
      for (int g = 0; g < ctxs.length; g++) plans[g] = Native.planCompile(ctxs[g], tables[g], filter);
    } catch (Exception e) {
      free(plans);
      throw e;
    }
    return plans;
  }

  private static void free(long[] plans) {
    for (long p : plans) if (p != 0) Native.planFree(p);
  }

  /**
   * Waits for every GPU.  Every context is synced even when one raises (a NaN
   * an async scan reached raises at the sync, PredEval's exception): each
   * context's sticky flag is read and cleared and its exchange stream
   * drained; the first exception is rethrown after the loop.
   */
  static void syncAll(long[] ctxs) throws Exception {
    Exception first = null;
    for (long c : ctxs) {
      try {
        Native.sync(c);
      } catch (Exception e) {
        if (first == null) first = e;
      }
    }
    if (first != null) throw first;
  }

  /** Query.executeFileScan's resultCount over all shards: one scan per GPU + one all-reduce */
  public long count(CondExpr[] filter) throws Exception {
    long[] plans = compile(filter);
    try {
      for (int g = 0; g < ctxs.length; g++) Native.scanCountAsync(ctxs[g], plans[g], slots[g]);
      Native.commAllreduceCountAll(comms, slots);
      syncAll(ctxs);
      return Native.countDownload(ctxs[0], slots[0]);
    } finally {
      free(plans);
    }
  }

  /** COUNT/SUM/MIN/MAX of column col (0-based): the Native.scanAggregate record, whole table */
  public long[] aggregate(CondExpr[] filter, int col) throws Exception {
    long[] plans = compile(filter);
    try {
      for (int g = 0; g < ctxs.length; g++) Native.scanAggregateAsync(ctxs[g], plans[g], col, slots[g]);
      Native.commAllreduceAggAll(comms, slots);
      syncAll(ctxs);
      return Native.aggDownload(ctxs[0], slots[0]);
    } finally {
      free(plans);
    }
  }

  /**
   * ColumnarIndexScan over the shards (index.GpuShardedColumnarIndexScan):
   * same arguments as the reference constructor minus the Columnarfile.
   */
  public index.GpuShardedColumnarIndexScan indexScan(Columnarfile cf, global.AttrType[] types, short[] str_sizes,
                                                    int noInFlds, int noOutFlds, int[] out_indexes,
                                                    iterator.FldSpec[] outFlds, CondExpr[] selects)
      throws Exception {
    return new index.GpuShardedColumnarIndexScan(this, cf, types, str_sizes, noInFlds, noOutFlds, out_indexes,
                                                 outFlds, selects);
  }

  public long rows() {
    return nrows;
  }

  public int shards() {
    return ctxs.length;
  }

  public long context(int g) {
    return ctxs[g];
  }

  public long table(int g) {
    return tables[g];
  }

  public long rowBegin(int g) {
    return begins[g];
  }

  public long rowEnd(int g) {
    return ends[g];
  }

  /** the DB file the shards were staged from (their BitMapFile slices come from it too) */
  public long db() {
    return db;
  }

  /** the clique over the shards' GPUs (rank g = shard g) */
  public long[] comms() {
    return comms;
  }

  public String fileName() {
    return name;
  }

  private void release() {
    for (int g = 0; g < ctxs.length; g++) {
      if (slots[g] != 0) Native.devFree(ctxs[g], slots[g]);
      if (tables[g] != 0) Native.tableFree(tables[g]);
      slots[g] = tables[g] = 0;
    }
  }

  /** frees the shards; the clique stays with GpuContext */
  public void close() {
    if (closed) return;
    release();
    closed = true;
  }
}
