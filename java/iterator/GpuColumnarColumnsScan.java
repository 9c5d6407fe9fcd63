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
 * Drop-in for ColumnarColumnsScan (R/iterator/ColumnarColumnsScan.java:39-257),
 * the predicate scan NljQuery hands ColumnarNestedLoopJoins (NljQuery.java:269):
 * same constructors (projecting and delete-query), get_next / get_next_tid /
 * close / restart / getTupleSize contract.  PredEval runs over a tuple of the
 * colNos columns (:86, :190), so field k of the CondExpr[] is file column
 * colNos[k - 1]: the CNF is compiled against the staged table with its fields
 * renumbered, and the predicate, the deleted-row skip (the lockstep
 * ColumnScans) and the late materialisation of out_indexes (:195-200) run as
 * MI355X kernels, rows in position order.  The reference's quirks are kept:
 * dest_s_sizes is indexed by the colNos index (:80), so a string column
 * after the first nstr entries of colNos raises its
 * ArrayIndexOutOfBoundsException; get_next_tid() looks the last column's RID
 * up in colNos[0]'s heapfile (:219), which is an "Invalid RID" whenever those
 * two columns differ.
 */
public class GpuColumnarColumnsScan extends Iterator implements GpuSelection {
  static final int BATCH = 262144;  // rows per cursor batch (profiles/r04/b)

  private final long ctx, table, plan;
  private long selection, cursor;
  private final Tuple Jtuple = new Tuple();
  private final int fieldCount;
  private final int[] colNos, outIdx, projTypes;
  private final short[] projSizes;
  private final boolean deleteQuery;
  public FldSpec[] perm_mat;
  private long[] ids;
  private Object[] batch;
  private int n, i;

  public GpuColumnarColumnsScan(Columnarfile columnarfile, int[] colNos, int n_out_flds, int[] out_indexes,
                                FldSpec[] proj_list, CondExpr[] outFilter)
      throws IOException, FileScanException, TupleUtilsException, InvalidRelation {
    this(false, columnarfile, colNos, n_out_flds, out_indexes, proj_list, outFilter);
  }

  /** the delete-query form (:104-157): no projection, for get_next_tid() */
  public GpuColumnarColumnsScan(Columnarfile columnarfile, int[] colNos, CondExpr[] outFilter)
      throws IOException, FileScanException, TupleUtilsException, InvalidRelation {
    this(true, columnarfile, colNos, 0, null, null, outFilter);
  }

  private GpuColumnarColumnsScan(boolean deleteQuery, Columnarfile columnarfile, int[] colNos, int n_out_flds,
                                 int[] out_indexes, FldSpec[] proj_list, CondExpr[] outFilter)
      throws IOException, FileScanException, TupleUtilsException, InvalidRelation {
    // the reference's checked exceptions only (R/iterator/ColumnarColumnsScan.java:39,104): a device or plan
    // failure (PredEvalException on operand types included) is a FileScanException
    try {
      this.deleteQuery = deleteQuery;
      this.colNos = colNos.clone();
      AttrType[] in1 = columnarfile.getAttributeTypes();
      fieldCount = columnarfile.getFieldCount();
      if (!deleteQuery) {
        AttrType[] jtypes = new AttrType[n_out_flds];
        TupleUtils.setup_op_tuple(Jtuple, jtypes, in1, (short) fieldCount, columnarfile.getStringSizes(), proj_list,
                                  n_out_flds);                                                   // :57-60
      }
      perm_mat = proj_list;
      // destType / dest_s_sizes exactly as :68-82 (its index quirk included)
      int nstr = 0;
      for (int c : colNos)
        if (in1[c].attrType == AttrType.attrString) nstr++;
      short[] destSizes = new short[nstr];
      for (int k = 0; k < colNos.length; k++)
        if (in1[colNos[k]].attrType == AttrType.attrString) destSizes[k] = columnarfile.getAttrSizes()[colNos[k]];
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
      plan = Native.planCompile(ctx, table, GpuCondExprs.remap(outFilter, this.colNos));
      try {
        selection = Native.scanBitmap(ctx, plan);
        cursor = Native.cursorOpen(ctx, table, selection, outIdx);
      } catch (Exception e) {
        close();
        throw new FileScanException(e, "GPU columns scan failed");
      }
    } catch (IOException | FileScanException | TupleUtilsException | InvalidRelation | RuntimeException e) {
      close();
      throw e;
    } catch (Exception e) {
      close();
      throw new FileScanException(e, "GPU scan setup failed");
    }
  }

  /** shows what input fields go where in the output tuple (:159-162) */
  public FldSpec[] show() {
    return perm_mat;
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
    if (deleteQuery) throw new NullPointerException("ColumnarColumnsScan: the delete-query form has no out_indexes");
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
    if (colNos.length > 1 && colNos[0] != colNos[colNos.length - 1]) throw new Exception("Invalid RID");  // :219
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

  public void restart() throws FileScanException {
    try {
      Native.cursorRestart(cursor);
    } catch (Exception e) {
      throw new FileScanException(e, "restart ColumnsScan() failed");
    }
    n = i = 0;
  }

  public int getTupleSize() {
    if (deleteQuery) throw new NullPointerException("ColumnarColumnsScan: the delete-query form has no output tuple");
    return Jtuple.size();
  }
}
