package index;

import java.util.ArrayList;
import java.util.HashSet;
import java.util.List;
import java.util.Set;

import columnar.Columnarfile;
import columnar.GpuShardedScan;
import global.AttrType;
import global.IndexType;
import global.Native;
import heap.Tuple;
import iterator.CondExpr;
import iterator.FldSpec;
import iterator.Iterator;
import iterator.TupleUtils;

/**
 * ColumnarIndexScan (R/index/ColumnarIndexScan.java:79-182, get_next
 * :287-308) over the row-range shards of a GpuShardedScan, one per GPU.  Each
 * shard takes its slice of every BitMapFile the CNF names and of cf.md
 * straight from the DB file (Native.dbBitmapStageRange) and runs the
 * one-launch CNF + positions + projection (Native.cnfCursorLaunch, all GPUs
 * in flight together); ONE grouped RCCL all-gather of the shard counts
 * (Native.commAllgatherCountAll) gives every shard its offset in the output,
 * and get_next() walks the shards in order -- ascending positions, the
 * reference's nextSetBit order.  Bitmap terms only, no repeated constraint
 * (the reference's mutable duplicate cache, :147-172): anything else throws
 * IndexException -- use GpuColumnarIndexScan.
 */
public class GpuShardedColumnarIndexScan extends Iterator {
  static final int BATCH = 262144;  // rows per cursor batch: one packed copy each, 42 vs 24 GB/s at 64 Ki (profiles/r04/b)

  private final GpuShardedScan s;
  private final Tuple Jtuple = new Tuple();
  private final int[] outIdx, projTypes;
  private final short[] projSizes;
  private final long[] cursors;
  private final List<List<Long>> staged = new ArrayList<>();   // per shard: bitmap slices to free
  private final long[] offsets;                                // nshards + 1
  private int shard;
  private long[] ids;
  private Object[] batch;
  private int n, i;

  public GpuShardedColumnarIndexScan(GpuShardedScan shards, Columnarfile cf, AttrType[] types, short[] str_sizes,
                                     int noInFlds, int noOutFlds, int[] out_indexes, FldSpec[] outFlds,
                                     CondExpr[] selects) throws Exception {
    s = shards;
    AttrType[] outTypes = new AttrType[noOutFlds];
    TupleUtils.setup_op_tuple(Jtuple, outTypes, types, noInFlds, str_sizes, outFlds, noOutFlds);
    outIdx = out_indexes == null ? new int[0] : out_indexes.clone();
    projTypes = new int[outIdx.length];
    projSizes = new short[outIdx.length];
    for (int k = 0; k < outIdx.length; k++) {
      projTypes[k] = cf.getAttributeType(outIdx[k]).attrType;
      projSizes[k] = projTypes[k] == AttrType.attrString ? cf.getAttrSizes()[outIdx[k]] : 4;
    }
    // the CNF as lists of BitMapFile names (value selection of ColumnIndexScan.getBitSet)
    List<List<String>> conj = new ArrayList<>();
    Set<String> keys = new HashSet<>();
    for (int c = 0; selects[c] != null; c++) {
      List<String> files = new ArrayList<>();
      for (CondExpr e = selects[c]; e != null; e = e.next) {
        if (e.type1.attrType != AttrType.attrSymbol || e.type2.attrType == AttrType.attrSymbol)
          throw new IndexException(null, "IndexScan.java: invalid constraint");
        if (e.indexType == null || e.indexType.indexType != IndexType.Bitmap)
          throw new IndexException(null, "sharded index scan: Bitmap terms only (use GpuColumnarIndexScan)");
        final int col = e.operand1.symbol.offset - 1;
        String key = cf.indexToColName(col).concat(e.op.toString())
            .concat(e.type2.attrType == AttrType.attrInteger ? Integer.toString(e.operand2.integer) : e.operand2.string)
            .concat(e.indexType.toString());
        if (!keys.add(key))
          throw new IndexException(null, "sharded index scan: repeated constraint (use GpuColumnarIndexScan)");
        for (Object v : GpuBitmapValues.values(cf, col, e))
          files.add(cf.get_fileName() + ".bm." + col + "." + v);
      }
      conj.add(files);
    }
    final int ns = s.shards();
    cursors = new long[ns];
    long[] dcounts = new long[ns];
    long[] alls = new long[ns];
    offsets = new long[ns + 1];
    try {
      for (int g = 0; g < ns; g++) {
        final long ctx = s.context(g), b = s.rowBegin(g), nb = s.rowEnd(g) - s.rowBegin(g);
        List<Long> mine = new ArrayList<>();
        staged.add(mine);
        List<Long> bms = new ArrayList<>();
        int[] offs = new int[conj.size() + 1];
        for (int c = 0; c < conj.size(); c++) {
          for (String f : conj.get(c)) {
            long h = Native.dbBitmapStageRange(ctx, s.db(), f, b, nb);
            mine.add(h);
            bms.add(h);
          }
          offs[c + 1] = bms.size();
        }
        long del = Native.dbBitmapStageRange(ctx, s.db(), cf.get_fileName() + ".md", b, nb);
        mine.add(del);
        long[] h = new long[bms.size()];
        for (int k = 0; k < h.length; k++) h[k] = bms.get(k);
        // launch only: the cursor's capacity bound comes from the slices' counts,
        // which Native.dbBitmapStageRange fixed at staging (mbx_bitmap_upload
        // counts every upload), so no shard waits for its launch before the
        // next shard's is enqueued -- all GPUs in flight
        long[] r = Native.cnfCursorLaunch(ctx, s.table(g), h, offs, del, outIdx);
        cursors[g] = r[0];
        dcounts[g] = r[1];
      }
      for (int g = 0; g < ns; g++) alls[g] = Native.devAlloc(s.context(g), 8L * ns);
      Native.commAllgatherCountAll(s.comms(), dcounts, alls);          // the one exchange
      Native.commWait(s.comms()[0]);
      long[] counts = Native.longsDownload(s.context(0), alls[0], ns);
      for (int g = 0; g < ns; g++) offsets[g + 1] = offsets[g] + counts[g];
    } catch (Exception e) {
      close();
      throw e;
    } finally {
      for (int g = 0; g < ns; g++) if (alls[g] != 0) Native.devFree(s.context(g), alls[g]);
    }
  }

  /** selected rows over all shards (the concatenation's length) */
  public long count() {
    return offsets[offsets.length - 1];
  }

  /** shard g's rows are get_next() results [offset(g), offset(g + 1)) */
  public long offset(int g) {
    return offsets[g];
  }

  private boolean fill() throws Exception {
    while (i == n) {
      if (shard >= cursors.length) return false;
      Object[] r = Native.cursorNext(cursors[shard], BATCH, projTypes, projSizes);
      if (r == null) {
        shard++;
        continue;
      }
      ids = (long[]) r[0];
      batch = (Object[]) r[1];
      n = ids.length;
      i = 0;
    }
    return true;
  }

  public Tuple get_next() throws Exception {
    if (!fill()) return null;
    for (int k = 0; k < outIdx.length; k++) {
      switch (projTypes[k]) {
        case AttrType.attrInteger: Jtuple.setIntFld(k + 1, ((int[]) batch[k])[i]); break;
        case AttrType.attrReal: Jtuple.setFloFld(k + 1, ((float[]) batch[k])[i]); break;
        default: Jtuple.setStrFld(k + 1, ((String[]) batch[k])[i]);
      }
    }
    i++;
    return Jtuple;
  }

  /** the next selected position (global), -1 at the end */
  public long get_next_position() throws Exception {
    if (!fill()) return -1;
    return ids[i++];
  }

  public void close() {
    if (!closeFlag) {
      for (long c : cursors) if (c != 0) Native.cursorClose(c);
      for (List<Long> l : staged) for (long b : l) Native.bitmapFree(b);
      staged.clear();
      closeFlag = true;
    }
  }

  public void restart() throws iterator.FileScanException {
    try {
      for (long c : cursors) Native.cursorRestart(c);
    } catch (Exception e) {
      throw new iterator.FileScanException(e, "restart failed");
    }
    shard = 0;
    n = i = 0;
  }

  public int getTupleSize() {
    return Jtuple.size();
  }
}
