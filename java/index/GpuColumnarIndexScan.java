package index;

import java.util.ArrayList;
import java.util.BitSet;
import java.util.HashSet;
import java.util.List;
import java.util.Set;

import columnar.Columnarfile;
import columnar.GpuTables;
import global.AttrType;
import global.GpuContext;
import global.IndexType;
import global.Native;
import heap.Tuple;
import iterator.CondExpr;
import iterator.FldSpec;
import iterator.Iterator;
import iterator.TupleUtils;

/**
 * Drop-in for ColumnarIndexScan (R/index/ColumnarIndexScan.java:79-330): same
 * constructors (the projecting one, :79-182, and the bitmap-only one BitMapQuery
 * uses, :185-268), getOutputPositions(), get_next() in nextSetBit order.
 * Bitmap-index CNFs run as ONE kernel launch (Native.cnfCursorOpen,
 * k_cnf_select) over the value BitSets of every term -- OR within a
 * conjunct, AND across, AND NOT cf.md -- that also writes the positions and
 * the projected out_indexes rows (char(n) included) for get_next(); the
 * CNF's BitSet is formed only if getOutputPositions() asks for it.  Two
 * cases keep the reference's own ColumnarIndexScan for the positions, so its
 * results stay identical: a B-tree term (B-tree access is out of scope for
 * the GPU path) and a repeated identical constraint (its duplicateConstraints
 * cache ORs in a BitSet that a later AND mutates, :147-172); their
 * projection is still materialised on the GPU.
 */
public class GpuColumnarIndexScan extends Iterator implements iterator.GpuSelection {
  private final long ctx, table, nbits;
  private long output, cursor, deleted;
  private long[] cnfBitmaps;
  private int[] cnfOffsets;
  private final Tuple Jtuple = new Tuple();
  private final AttrType[] outTypes;
  private final int[] outIdx, projTypes;
  private final short[] projSizes;
  private final boolean fused, projecting;
  public FldSpec[] perm_mat;
  private BitSet positions;                // getOutputPositions()'s BitSet, formed on first use
  private long[] ids;
  private Object[] batch;
  private int n, i;

  public GpuColumnarIndexScan(Columnarfile columnarFile, final int[] fldNums, IndexType[] indexTypes,
                              final String[] indNames, AttrType[] types, short[] str_sizes, int noInFlds,
                              int noOutFlds, int[] out_indexes, FldSpec[] outFlds, CondExpr[] selects,
                              final boolean indexOnly) throws Exception {
    this(true, columnarFile, fldNums, indexTypes, indNames, types, str_sizes, noInFlds, noOutFlds, out_indexes,
         outFlds, selects, indexOnly);
  }

  /**
   * The bitmap-only form (:185-268) BitMapQuery uses for getOutputPositions()
   * (R/input/BitMapQuery.java:244,339): the CNF's BitSet, no projection.  As
   * in the reference, get_next() fails on a selected row (its out_indexes is
   * null, :292) with IndexException, and getTupleSize() with the
   * NullPointerException of its null Jtuple.
   */
  public GpuColumnarIndexScan(Columnarfile columnarFile, final int[] fldNums, IndexType[] indexTypes,
                              final String[] indNames, AttrType[] types, short[] str_sizes, int noInFlds,
                              CondExpr[] selects) throws Exception {
    this(false, columnarFile, fldNums, indexTypes, indNames, types, str_sizes, noInFlds, 0, null, null, selects,
         false);
  }

  private GpuColumnarIndexScan(boolean projecting, Columnarfile columnarFile, int[] fldNums, IndexType[] indexTypes,
                               String[] indNames, AttrType[] types, short[] str_sizes, int noInFlds, int noOutFlds,
                               int[] out_indexes, FldSpec[] outFlds, CondExpr[] selects, boolean indexOnly)
      throws Exception {
    this.projecting = projecting;
    outTypes = new AttrType[noOutFlds];
    if (projecting) TupleUtils.setup_op_tuple(Jtuple, outTypes, types, noInFlds, str_sizes, outFlds, noOutFlds);
    perm_mat = outFlds;
    ctx = GpuContext.ctx();
    table = GpuTables.get(columnarFile.get_fileName());
    nbits = tableRows(table);
    outIdx = out_indexes == null ? new int[0] : out_indexes.clone();
    projTypes = new int[outIdx.length];
    projSizes = new short[outIdx.length];
    for (int k = 0; k < outIdx.length; k++) {
      projTypes[k] = columnarFile.getAttributeType(outIdx[k]).attrType;
      projSizes[k] = projTypes[k] == AttrType.attrString ? columnarFile.getAttrSizes()[outIdx[k]] : 4;
    }
    fused = bitmapOnlyWithoutRepeats(columnarFile, selects);
    if (fused) {
      List<Long> bms = new ArrayList<>();
      List<Integer> offs = new ArrayList<>();
      offs.add(0);
      for (int c = 0; selects[c] != null; c++) {
        for (CondExpr e = selects[c]; e != null; e = e.next)
          bms.addAll(GpuBitmapValues.of(columnarFile, fieldOf(e) - 1, e, nbits));
        offs.add(bms.size());
      }
      cnfBitmaps = new long[bms.size()];
      for (int k = 0; k < cnfBitmaps.length; k++) cnfBitmaps[k] = bms.get(k);
      cnfOffsets = new int[offs.size()];
      for (int k = 0; k < cnfOffsets.length; k++) cnfOffsets[k] = offs.get(k);
      deleted = Native.bitmapUpload(ctx, nbits, columnarFile.getMarkedDeleted().getBitSet().toLongArray());
      try {
        if (projecting)   // CNF + positions + projected rows: one kernel, any CNF shape
          cursor = Native.cnfCursorOpen(ctx, table, cnfBitmaps, cnfOffsets, deleted, outIdx);
        else              // the BitSet alone: one k_bitmap_cnf launch
          output = Native.bitmapCnf(ctx, nbits, cnfBitmaps, cnfOffsets, deleted);
      } catch (Exception e) {
        close();
        throw e;
      }
    } else {
      ColumnarIndexScan ref = projecting
          ? new ColumnarIndexScan(columnarFile, fldNums, indexTypes, indNames, types, str_sizes, noInFlds, noOutFlds,
                                  out_indexes, outFlds, selects, indexOnly)
          : new ColumnarIndexScan(columnarFile, fldNums, indexTypes, indNames, types, str_sizes, noInFlds, selects);
      output = Native.bitmapUpload(ctx, nbits, ref.getOutputPositions().toLongArray());
      ref.close();
      if (projecting) cursor = Native.cursorOpen(ctx, table, output, outIdx);
    }
  }

  private static long tableRows(long table) throws Exception {
    return Native.tableRows(table);
  }

  private static int fieldOf(CondExpr e) throws IndexException {
    if (e.type1.attrType == AttrType.attrSymbol && e.type2.attrType != AttrType.attrSymbol)
      return e.operand1.symbol.offset;
    if (e.type2.attrType == AttrType.attrSymbol && e.type1.attrType != AttrType.attrSymbol)
      return e.operand2.symbol.offset;
    throw new IndexException("IndexScan.java: invalid constraint");          // :135-141
  }

  /** every term a Bitmap term and no constraint string repeated (:142-146) */
  private static boolean bitmapOnlyWithoutRepeats(Columnarfile f, CondExpr[] selects) throws Exception {
    Set<String> seen = new HashSet<>();
    for (int c = 0; selects[c] != null; c++)
      for (CondExpr e = selects[c]; e != null; e = e.next) {
        fieldOf(e);
        if (e.indexType == null || e.indexType.indexType != IndexType.Bitmap) return false;
        String key = f.indexToColName(e.operand1.symbol.offset - 1).concat(e.op.toString())
            .concat(e.type2.attrType == AttrType.attrInteger ? Integer.toString(e.operand2.integer) : e.operand2.string)
            .concat(e.indexType.toString());
        if (!seen.add(key)) return false;
      }
    return true;
  }

  /** the CNF's BitSet (:270-272): the same object on every call, as the reference's outputPositions */
  public BitSet getOutputPositions() {
    if (positions == null) {
      try {
        positions = BitSet.valueOf(Native.bitmapDownload(ctx, gpuSelection()));
      } catch (Exception e) {
        // the reference's getOutputPositions() declares no checked exception: a
        // device failure here surfaces unchecked, carrying mbx_last_error()
        throw new IllegalStateException("GPU ColumnarIndexScan: " + e.getMessage(), e);
      }
    }
    return positions;
  }

  public long gpuSelection() throws Exception {
    if (output == 0) output = Native.bitmapCnf(ctx, nbits, cnfBitmaps, cnfOffsets, deleted);
    return output;
  }

  public long gpuTable() {
    return table;
  }

  public int[] fileColumns() {
    return outIdx.clone();
  }

  public Tuple get_next() throws Exception {
    if (!projecting) {
      // the reference's bitmap-only form walks a null out_indexes at the
      // first remaining position (:287-307); a scan with none returns null
      if (cursor == 0) cursor = Native.cursorOpen(ctx, table, gpuSelection(), outIdx);
      if (Native.cursorCount(cursor) > 0)
        throw new IndexException(new NullPointerException("outIndexes"), "IndexScan.java: Heapfile error");
      return null;
    }
    if (i == n) {
      Object[] r = Native.cursorNext(cursor, 262144, projTypes, projSizes);
      if (r == null) return null;
      ids = (long[]) r[0];
      batch = (Object[]) r[1];
      n = ids.length;
      i = 0;
      if (n == 0) return null;
    }
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

  /** true where the CNF, positions and projection ran as one GPU launch (false: the reference's positions) */
  public boolean usedFusedCnf() {
    return fused;
  }

  public void close() {
    if (!closeFlag) {
      if (cursor != 0) Native.cursorClose(cursor);
      if (output != 0) Native.bitmapFree(output);
      if (deleted != 0) Native.bitmapFree(deleted);
      cursor = output = deleted = 0;
      closeFlag = true;
    }
  }

  public void restart() throws iterator.FileScanException {
    try {
      if (cursor != 0) Native.cursorRestart(cursor);                    // currentBitMapPos = 0 (:321-323)
    } catch (Exception e) {
      throw new iterator.FileScanException(e, "restart failed");
    }
    n = i = 0;
  }

  public int getTupleSize() {
    if (!projecting) throw new NullPointerException("ColumnarIndexScan: the bitmap-only form has no Jtuple");
    return Jtuple.size();
  }
}
