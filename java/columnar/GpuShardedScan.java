package columnar;

import java.nio.ByteBuffer;

import global.GpuContext;
import global.Native;
import iterator.CondExpr;

/**
 * One JVM driving every GPU of the node (SURVEY.md 8(e), DESIGN.md section 6):
 * the table's rows are split into 64-aligned row ranges (Native.shardBounds),
 * each staged on its own GPU with row_offset = the range's first position;
 * a query runs one scan per GPU and ONE RCCL exchange over xGMI combines the
 * per-shard results on the devices (COUNT: int64 all-reduce; COUNT/SUM/MIN/MAX:
 * all-gather of the 48-byte records folded in rank order, so the double SUM
 * is reproducible for a given GPU count).  The reference engine is one
 * process (R/global/SystemDefs.java:6-9); so is this.
 */
public final class GpuShardedScan implements AutoCloseable {
  private final long[] ctxs, comms, tables, slots;
  private final long nrows;

  /**
   * cols: one direct ByteBuffer per column in host order (char(n): n bytes of
   * zero-padded modified UTF-8 per row); deleted: cf.md's BitSet.toLongArray()
   * or null.
   */
  public GpuShardedScan(int[] attrTypes, short[] sizes, long nrows, ByteBuffer[] cols, long[] deleted)
      throws Exception {
    final int n = GpuContext.devices();
    this.nrows = nrows;
    ctxs = new long[n];
    tables = new long[n];
    slots = new long[n];
    for (int g = 0; g < n; g++) {
      ctxs[g] = GpuContext.ctx(g);
      long[] be = Native.shardBounds(nrows, n, g);
      ByteBuffer[] part = new ByteBuffer[cols.length];
      for (int j = 0; j < cols.length; j++) {
        int w = attrTypes[j] == global.AttrType.attrString ? sizes[j] : 4;
        ByteBuffer d = cols[j].duplicate();
        d.position((int) (be[0] * w)).limit((int) (be[1] * w));
        part[j] = d.slice().order(cols[j].order());
      }
      long[] del = null;
      if (deleted != null) {                         // be[0] is a multiple of 64: whole words
        int w0 = (int) (be[0] / 64), w1 = (int) Math.min(deleted.length, (be[1] + 63) / 64);
        del = new long[Math.max(0, w1 - w0)];
        if (w1 > w0) System.arraycopy(deleted, w0, del, 0, w1 - w0);
      }
      tables[g] = Native.tableStage(ctxs[g], attrTypes, sizes, be[1] - be[0], part, del, be[0]);
      slots[g] = Native.devAlloc(ctxs[g], Native.AGG_RECORD_BYTES);
    }
    comms = Native.commInitAll(ctxs);                 // one RCCL clique, rank g = GPU g
  }

  private long[] compile(CondExpr[] filter) throws Exception {
    long[] plans = new long[ctxs.length];
    for (int g = 0; g < ctxs.length; g++) plans[g] = Native.planCompile(ctxs[g], tables[g], filter);
    return plans;
  }

  private void free(long[] plans) {
    for (long p : plans) if (p != 0) Native.planFree(p);
  }

  /** Query.executeFileScan's resultCount over all shards: one scan per GPU + one all-reduce */
  public long count(CondExpr[] filter) throws Exception {
    long[] plans = compile(filter);
    try {
      for (int g = 0; g < ctxs.length; g++) Native.scanCountAsync(ctxs[g], plans[g], slots[g]);
      Native.commAllreduceCountAll(comms, slots);
      for (long c : ctxs) Native.sync(c);             // a NaN reached by a float compare raises here
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
      for (long c : ctxs) Native.sync(c);
      return Native.aggDownload(ctxs[0], slots[0]);
    } finally {
      free(plans);
    }
  }

  public long rows() {
    return nrows;
  }

  public void close() {
    for (long c : comms) Native.commFree(c);
    for (int g = 0; g < ctxs.length; g++) {
      Native.devFree(ctxs[g], slots[g]);
      Native.tableFree(tables[g]);
    }
  }
}
