package index;

import java.util.BitSet;
import java.util.List;

import columnar.Columnarfile;
import columnar.GpuTables;
import global.AttrType;
import global.GpuContext;
import global.IndexType;
import global.Native;
import global.TID;
import heap.Tuple;
import iterator.CondExpr;
import iterator.FldSpec;
import iterator.Iterator;
import iterator.TupleUtils;

/**
 * Drop-in for ColumnIndexScan's Bitmap branch (R/index/ColumnIndexScan.java:76-272,
 * 647-740): `column op literal` over the column's bitmap indexes -- the value
 * BitSets' OR minus cf.md in one k_bitmap_cnf launch -- and the rows of
 * out_indexes materialised on the GPU, in position order.  A B_Index scan
 * keeps the reference's ColumnIndexScan for its positions (B-tree access is
 * out of scope for the GPU path).
 */
public class GpuColumnIndexScan extends Iterator {
  private final long ctx, table;
  private long positions, cursor;
  private final Tuple Jtuple = new Tuple();
  private final int[] outIdx, projTypes;
  private final short[] projSizes;
  private final int numFields;
  private long[] ids;
  private Object[] batch;
  private int n, i;

  public GpuColumnIndexScan(IndexType index, Columnarfile columnarfile, final String indName, AttrType[] types,
                            short[] str_sizes, int noInFlds, int noOutFlds, int[] out_indexes, FldSpec[] outFlds,
                            CondExpr[] selects, final int fldNum, final boolean indexOnly) throws Exception {
    AttrType[] Jtypes = new AttrType[noOutFlds];
    TupleUtils.setup_op_tuple(Jtuple, Jtypes, types, noInFlds, str_sizes, outFlds, noOutFlds);
    ctx = GpuContext.ctx();
    table = GpuTables.get(columnarfile.get_fileName());
    numFields = columnarfile.getFieldCount();
    final long nbits = Native.tableRows(table);
    outIdx = out_indexes == null ? new int[0] : out_indexes.clone();
    projTypes = new int[outIdx.length];
    projSizes = new short[outIdx.length];
    for (int k = 0; k < outIdx.length; k++) {
      projTypes[k] = columnarfile.getAttributeType(outIdx[k]).attrType;
      projSizes[k] = projTypes[k] == AttrType.attrString ? columnarfile.getAttrSizes()[outIdx[k]] : 4;
    }
    if (index.indexType == IndexType.Bitmap) {
      List<Long> bms = GpuBitmapValues.of(columnarfile, fldNum - 1, selects[0], nbits);
      long[] h = new long[bms.size()];
      for (int k = 0; k < h.length; k++) h[k] = bms.get(k);
      long deleted = Native.bitmapUpload(ctx, nbits, columnarfile.getMarkedDeleted().getBitSet().toLongArray());
      try {
        positions = Native.bitmapCnf(ctx, nbits, h, new int[] {0, h.length}, deleted);
      } finally {
        Native.bitmapFree(deleted);
      }
    } else {
      ColumnIndexScan ref = new ColumnIndexScan(index, columnarfile, indName, types, str_sizes, noInFlds, noOutFlds,
                                                out_indexes, outFlds, selects, fldNum, indexOnly);
      positions = Native.bitmapUpload(ctx, nbits, ref.getPositionsOfIndexScan().toLongArray());
      ref.close();
    }
    cursor = Native.cursorOpen(ctx, table, positions, outIdx);
  }

  private boolean fill() throws Exception {
    if (i < n) return true;
    Object[] r = Native.cursorNext(cursor, 65536, projTypes, projSizes);
    if (r == null) return false;
    ids = (long[]) r[0];
    batch = (Object[]) r[1];
    n = ids.length;
    i = 0;
    return n > 0;
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

  public TID get_next_tid() throws Exception {
    if (!fill()) return null;
    return new TID(numFields, (int) ids[i++]);
  }

  public BitSet getPositionsOfIndexScan() throws Exception {
    return BitSet.valueOf(Native.bitmapDownload(ctx, positions));
  }

  public void close() {
    if (!closeFlag) {
      if (cursor != 0) Native.cursorClose(cursor);
      if (positions != 0) Native.bitmapFree(positions);
      cursor = positions = 0;
      closeFlag = true;
    }
  }

  public void restart() throws iterator.FileScanException {
    try {
      Native.cursorRestart(cursor);
    } catch (Exception e) {
      throw new iterator.FileScanException(e, "restart failed");
    }
    n = i = 0;
  }

  public int getTupleSize() {
    return Jtuple.size();
  }
}
