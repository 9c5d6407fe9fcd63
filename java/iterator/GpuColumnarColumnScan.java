package iterator;

import java.io.IOException;

import columnar.Columnarfile;
import columnar.GpuTables;
import global.AttrType;
import global.GpuContext;
import global.Native;
import global.TID;
import heap.Tuple;

/**
 * Drop-in for ColumnarColumnScan (R/iterator/ColumnarColumnScan.java:39-211):
 * same constructors (projecting and delete-query), get_next / get_next_tid / close contract.  The CondExpr's
 * field 1 is column colNo (the reference evaluates PredEval on a one-field
 * tuple of that column, :55-77), so the CNF is compiled against the staged
 * table with field 1 renumbered to colNo + 1; the predicate, the deleted-row
 * skip (ColumnScan, R/columnar/ColumnScan.java:49-65) and the late
 * materialisation of out_indexes (Heapfile.findRID + getRecord per output
 * column, :166-171) run as MI355X kernels, rows in position order.  Jtuple's
 * types come from proj_list, its values from out_indexes, as in the
 * reference (:55-60, :166-171).
 */
public class GpuColumnarColumnScan extends Iterator implements GpuSelection {
  static final int BATCH = 262144;  // rows per cursor batch: one packed copy each, 42 vs 24 GB/s at 64 Ki (profiles/r04/b)

  private final long ctx, table, plan;
  private long selection, cursor;
  private final Tuple Jtuple = new Tuple();
  private final int fieldCount;
  private final boolean deleteQuery;
  public FldSpec[] perm_mat;
  private final int[] outIdx, projTypes;
  private final short[] projSizes;
  private long[] ids;
  private Object[] batch;
  private int n, i;

  public GpuColumnarColumnScan(Columnarfile columnarfile, int colNo, int n_out_flds, int[] out_indexes,
                               FldSpec[] proj_list, CondExpr[] outFilter)
      throws IOException, FileScanException, TupleUtilsException, InvalidRelation {
    this(false, columnarfile, colNo, n_out_flds, out_indexes, proj_list, outFilter);
  }

  /**
   * The delete-query form (:91-132): no projection, for get_next_tid()
   * (DeleteQuery -> markTupleDeleted).  Its get_next() on a selected row
   * fails with the NullPointerException the reference's null outIndexes
   * raises (:166).
   */
  public GpuColumnarColumnScan(Columnarfile columnarfile, int colNo, CondExpr[] outFilter)
      throws IOException, FileScanException, TupleUtilsException, InvalidRelation {
    this(true, columnarfile, colNo, 0, null, null, outFilter);
  }

  private GpuColumnarColumnScan(boolean deleteQuery, Columnarfile columnarfile, int colNo, int n_out_flds,
                                int[] out_indexes, FldSpec[] proj_list, CondExpr[] outFilter)
      throws IOException, FileScanException, TupleUtilsException, InvalidRelation {
    // the reference's checked exceptions only (R/iterator/ColumnarColumnScan.java:39,91): a device or plan
    // failure (PredEvalException on operand types included) is a FileScanException
    try {
      this.deleteQuery = deleteQuery;
      AttrType[] in1 = columnarfile.getAttributeTypes();
      fieldCount = columnarfile.getFieldCount();
      if (!deleteQuery) {
        AttrType[] jtypes = new AttrType[n_out_flds];
        TupleUtils.setup_op_tuple(Jtuple, jtypes, in1, (short) fieldCount, columnarfile.getStringSizes(), proj_list,
                                  n_out_flds);
      }
      perm_mat = proj_list;
      ctx = GpuContext.ctx();
      table = GpuTables.get(columnarfile.get_fileName());
      outIdx = new int[n_out_flds];
      projTypes = new int[n_out_flds];
      projSizes = new short[n_out_flds];
      for (int k = 0; k < n_out_flds; k++) {
        outIdx[k] = out_indexes[k];
        projTypes[k] = in1[outIdx[k]].attrType;
        projSizes[k] = projTypes[k] == AttrType.attrString ? columnarfile.getAttrSizes()[outIdx[k]] : 4;
      }
      plan = Native.planCompile(ctx, table, onColumn(outFilter, colNo));   // PredEvalException on type errors
      try {
        selection = Native.scanBitmap(ctx, plan);
        cursor = Native.cursorOpen(ctx, table, selection, outIdx);
      } catch (Exception e) {
        close();
        throw new FileScanException(e, "GPU column scan failed");
      }
    } catch (IOException | FileScanException | TupleUtilsException | InvalidRelation | RuntimeException e) {
      close();
      throw e;
    } catch (Exception e) {
      close();
      throw new FileScanException(e, "GPU scan setup failed");
    }
  }

  /** shows what input fields go where in the output tuple (:134-137) */
  public FldSpec[] show() {
    return perm_mat;
  }

  /** a copy of the CNF whose field-1 symbols name column colNo of the file */
  static CondExpr[] onColumn(CondExpr[] filter, int colNo) {
    return GpuCondExprs.remap(filter, new int[] {colNo});
  }

  public long gpuTable() {
    return table;
  }

  public long gpuSelection() {
    return selection;
  }

  public int[] fileColumns() {
    return outIdx.clone();
  }

  private boolean fill() throws Exception {
    if (i < n) return true;
    Object[] r = Native.cursorNext(cursor, BATCH, projTypes, projSizes);
    if (r == null) return false;
    ids = (long[]) r[0];
    batch = (Object[]) r[1];
    n = ids.length;
    i = 0;
    return n > 0;
  }

  public Tuple get_next() throws Exception {
    if (!fill()) return null;
    if (deleteQuery) throw new NullPointerException("ColumnarColumnScan: the delete-query form has no out_indexes");
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

  /** the TID of the next selected position (:188-205), null at the end */
  public TID get_next_tid() throws Exception {
    if (!fill()) return null;
    return new TID(fieldCount, (int) ids[i++]);
  }

  public void close() {
    if (!closeFlag) {
      if (cursor != 0) Native.cursorClose(cursor);
      if (selection != 0) Native.bitmapFree(selection);
      if (plan != 0) Native.planFree(plan);
      cursor = selection = 0;
      closeFlag = true;
    }
  }

  /** ColumnarColumnScan does not override Iterator.restart() (R/iterator/Iterator.java:134-136): a no-op */
  public void restart() throws FileScanException {
  }

  /** nor Iterator.getTupleSize() (:138-140): -1 */
  public int getTupleSize() {
    return -1;
  }
}
