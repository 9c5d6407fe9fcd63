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
 * 497-740): both constructors -- the projecting one (:76-183) and the
 * bitmap-only one ColumnarIndexScan builds per term (:185-272) -- and
 * `column op literal` over the column's bitmap indexes: the value BitSets'
 * OR minus cf.md in one k_bitmap_cnf launch, and the rows of out_indexes
 * materialised on the GPU, in position order.  A B_Index scan keeps the
 * reference's ColumnIndexScan for its positions (B-tree access is out of
 * scope for the GPU path).  Iterator contract as the reference's:
 * get_next_tid() carries TID(noInFlds, position) (:597); with indexOnly,
 * get_next() returns the literal key as a one-field tuple (:517-567);
 * getPositionsOfIndexScan() drains the scan (:647-654); restart() and
 * getTupleSize() are Iterator's own (no-op, -1; R/iterator/Iterator.java:134-140).
 */
public class GpuColumnIndexScan extends Iterator {
  private final long ctx, table;
  private long positions, cursor;
  private Tuple Jtuple;                   // null in the bitmap-only form, as the reference's
  private final Columnarfile f;
  private final IndexType index;
  private final CondExpr[] _selects;
  private final AttrType[] _types;
  private final short[] _s_sizes;
  private final int _fldNum, _noInFlds;
  private final boolean indexOnly, projecting;
  private final int[] outIdx, projTypes;
  private final short[] projSizes;
  public FldSpec[] perm_mat;
  private boolean started, drained, keyHeader;
  private long[] ids;
  private Object[] batch;
  private int n, i;

  public GpuColumnIndexScan(IndexType index, Columnarfile columnarfile, final String indName, AttrType[] types,
                            short[] str_sizes, int noInFlds, int noOutFlds, int[] out_indexes, FldSpec[] outFlds,
                            CondExpr[] selects, final int fldNum, final boolean indexOnly) throws Exception {
    this(true, index, columnarfile, indName, types, str_sizes, noInFlds, noOutFlds, out_indexes, outFlds, selects,
         fldNum, indexOnly);
  }

  /** the bitmap-only form (:185-272): positions, no projection (ColumnarIndexScan's per-term scan) */
  public GpuColumnIndexScan(IndexType index, Columnarfile columnarfile, final String indName, AttrType[] types,
                            short[] str_sizes, int noInFlds, CondExpr[] selects, final int fldNum) throws Exception {
    this(false, index, columnarfile, indName, types, str_sizes, noInFlds, 0, null, null, selects, fldNum, false);
  }

  private GpuColumnIndexScan(boolean projecting, IndexType index, Columnarfile columnarfile, String indName,
                             AttrType[] types, short[] str_sizes, int noInFlds, int noOutFlds, int[] out_indexes,
                             FldSpec[] outFlds, CondExpr[] selects, int fldNum, boolean indexOnly) throws Exception {
    this.projecting = projecting;
    this.index = index;
    this.f = columnarfile;
    this._selects = selects;
    this._types = types;
    this._s_sizes = str_sizes;
    this._fldNum = fldNum;
    this._noInFlds = noInFlds;
    this.indexOnly = indexOnly;
    if (projecting) {
      Jtuple = new Tuple();
      AttrType[] Jtypes = new AttrType[noOutFlds];
      try {
        TupleUtils.setup_op_tuple(Jtuple, Jtypes, types, noInFlds, str_sizes, outFlds, noOutFlds);   // :104-112
      } catch (iterator.TupleUtilsException e) {
        throw new IndexException(e, "IndexScan.java: TupleUtilsException caught from TupleUtils.setup_op_tuple()");
      } catch (iterator.InvalidRelation e) {
        throw new IndexException(e, "IndexScan.java: InvalidRelation caught from TupleUtils.setup_op_tuple()");
      }
      perm_mat = outFlds;
    }
    ctx = GpuContext.ctx();
    table = GpuTables.get(columnarfile.get_fileName());
    final long nbits = Native.tableRows(table);
    outIdx = out_indexes == null ? new int[0] : out_indexes.clone();
    projTypes = new int[outIdx.length];
    projSizes = new short[outIdx.length];
    for (int k = 0; k < outIdx.length; k++) {
      projTypes[k] = columnarfile.getAttributeType(outIdx[k]).attrType;
      projSizes[k] = projTypes[k] == AttrType.attrString ? columnarfile.getAttrSizes()[outIdx[k]] : 4;
    }
    switch (index.indexType) {
      case IndexType.Bitmap:
        try {
          positions = bitmapPositions(nbits);
        } catch (Exception e) {
          throw new IndexException(e, "ColumnIndexScan.java: BitMapFile exceptions.");          // :172-173
        }
        break;
      case IndexType.B_Index: {
        ColumnIndexScan ref = projecting
            ? new ColumnIndexScan(index, columnarfile, indName, types, str_sizes, noInFlds, noOutFlds, out_indexes,
                                  outFlds, selects, fldNum, indexOnly)
            : new ColumnIndexScan(index, columnarfile, indName, types, str_sizes, noInFlds, selects, fldNum);
        positions = Native.bitmapUpload(ctx, nbits, ref.getPositionsOfIndexScan().toLongArray());
        ref.close();
        break;
      }
      default:
        throw new UnknownIndexTypeException("Only BTree and Bitmap index is supported so far");  // :177-179
    }
    cursor = Native.cursorOpen(ctx, table, positions, outIdx);
  }

  /** getBitSet's value BitSets (:656-740) OR-ed, AND NOT cf.md (get_bm_next's skip, :503-513): one launch */
  private long bitmapPositions(long nbits) throws Exception {
    List<Long> bms = GpuBitmapValues.of(f, _fldNum - 1, _selects[0], nbits);
    long[] h = new long[bms.size()];
    for (int k = 0; k < h.length; k++) h[k] = bms.get(k);
    long deleted = Native.bitmapUpload(ctx, nbits, f.getMarkedDeleted().getBitSet().toLongArray());
    try {
      return Native.bitmapCnf(ctx, nbits, h, new int[] {0, h.length}, deleted);
    } finally {
      Native.bitmapFree(deleted);
    }
  }

  private boolean fill() throws Exception {
    if (i < n) return true;
    if (drained) return false;
    started = true;
    Object[] r = Native.cursorNext(cursor, 262144, projTypes, projSizes);
    if (r == null) return false;
    ids = (long[]) r[0];
    batch = (Object[]) r[1];
    n = ids.length;
    i = 0;
    return n > 0;
  }

  public Tuple get_next() throws Exception {
    if (!fill()) return null;
    if (indexOnly) {
      setKeyHeader();
      i++;
      return Jtuple;
    }
    if (!projecting) {
      // the reference walks a null out_indexes here (:571-579), before advancing
      throw new IndexException(new NullPointerException("out_indexes"), "IndexScan.java: Heapfile error");
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

  /** index_only: the key -- the select's literal -- as a one-field tuple (:517-567) */
  private void setKeyHeader() throws Exception {
    if (keyHeader) return;
    AttrType[] attrType = new AttrType[1];
    short[] s_sizes = new short[1];
    int t = _types[_fldNum - 1].attrType;
    try {
      if (t == AttrType.attrInteger) {
        attrType[0] = new AttrType(AttrType.attrInteger);
        Jtuple.setHdr((short) 1, attrType, s_sizes);
        Jtuple.setIntFld(1, _selects[0].operand2.integer);
      } else if (t == AttrType.attrString) {
        int count = 0;
        for (int k = 0; k < _fldNum; k++)
          if (_types[k].attrType == AttrType.attrString) count++;
        attrType[0] = new AttrType(AttrType.attrString);
        s_sizes[0] = _s_sizes[count - 1];
        Jtuple.setHdr((short) 1, attrType, s_sizes);
        Jtuple.setStrFld(1, _selects[0].operand2.string);
      }
    } catch (Exception e) {
      throw new IndexException(e, "IndexScan.java: Heapfile error");
    }
    if (t != AttrType.attrInteger && t != AttrType.attrString)
      throw new iterator.UnknownKeyTypeException("Only Integer and String keys are supported so far");
    keyHeader = true;
  }

  public TID get_next_tid() throws Exception {
    if (!fill()) return null;
    return new TID(_noInFlds, (int) ids[i++]);                                   // :597
  }

  /** the positions the scan has not returned yet; the scan is then exhausted (:647-654) */
  public BitSet getPositionsOfIndexScan() throws Exception {
    BitSet out;
    if (!started) {
      out = BitSet.valueOf(Native.bitmapDownload(ctx, positions));   // nothing consumed: the whole device BitSet
    } else {
      out = new BitSet();
      TID tid;
      while ((tid = get_next_tid()) != null) out.set(tid.position);
    }
    started = drained = true;
    n = i = 0;
    return out;
  }

  /**
   * Re-derives the scan's BitSet from the column's bitmap indexes (:656-740),
   * raising the reference's errors for a column without them.  The files
   * cannot change under an open scan (GpuTables invalidates on writes), so the
   * result equals the device BitSet the scan already iterates.
   */
  public void getBitSet() throws Exception {
    long b = bitmapPositions(Native.tableRows(table));
    Native.bitmapFree(b);
  }

  public void close() {
    if (!closeFlag) {
      if (cursor != 0) Native.cursorClose(cursor);
      if (positions != 0) Native.bitmapFree(positions);
      cursor = positions = 0;
      closeFlag = true;
    }
  }
}
