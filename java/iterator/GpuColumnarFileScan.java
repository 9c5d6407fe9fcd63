package iterator;

import java.io.IOException;

import columnar.GpuTables;
import global.AttrType;
import global.GpuContext;
import global.Native;
import global.TID;
import heap.Tuple;

/**
 * Drop-in for ColumnarFileScan (R/iterator/ColumnarFileScan.java:51-216): same
 * constructors (the projecting one and the delete-query one), same get_next / get_next_tid / close / restart contract and
 * the same shared Jtuple.  The predicate (PredEval over the CondExpr[]), the
 * deleted-row skip and the projection run as MI355X kernels; rows come back
 * in batches of BATCH through a device cursor, in position order.
 * get_next_tid's TID carries the position (numRIDs = len_in1); its recordIDs
 * are left unset -- the reference's callers (DeleteQuery -> markTupleDeleted,
 * R/columnar/Columnarfile.java:812-830) read only the position.
 */
public class GpuColumnarFileScan extends Iterator implements GpuSelection {
  static final int BATCH = 262144;  // rows per cursor batch: one packed copy each, 42 vs 24 GB/s at 64 Ki (profiles/r04/b)

  private final long ctx, table, plan;
  private long selection, cursor;
  private final Tuple Jtuple = new Tuple();
  private final AttrType[] outTypes;
  private final int[] proj, projTypes;
  private final short[] projSizes;
  private final short len_in1;
  private final boolean deleteQuery;
  public FldSpec[] perm_mat;
  private long[] ids;
  private Object[] batch;
  private int n, i;

  public GpuColumnarFileScan(String file_name, AttrType[] in1, short[] s1_sizes, short len_in1, int n_out_flds,
                             FldSpec[] proj_list, CondExpr[] outFilter)
      throws IOException, FileScanException, TupleUtilsException, InvalidRelation {
    this(false, file_name, in1, s1_sizes, len_in1, n_out_flds, proj_list, outFilter);
  }

  /**
   * The delete-query form (:101-135): no projection, for get_next_tid()
   * (DeleteQuery -> markTupleDeleted).  As in the reference, it has no output
   * tuple: get_next() on a selected row and getTupleSize() fail with the
   * NullPointerException the reference's null Jtuple raises (:167, :214).
   */
  public GpuColumnarFileScan(String file_name, AttrType[] in1, short[] s1_sizes, short len_in1,
                             CondExpr[] outFilter)
      throws IOException, FileScanException, TupleUtilsException, InvalidRelation {
    this(true, file_name, in1, s1_sizes, len_in1, 0, null, outFilter);
  }

  private GpuColumnarFileScan(boolean deleteQuery, String file_name, AttrType[] in1, short[] s1_sizes,
                              short len_in1, int n_out_flds, FldSpec[] proj_list, CondExpr[] outFilter)
      throws IOException, FileScanException, TupleUtilsException, InvalidRelation {
    // the reference's checked exceptions only (R/iterator/ColumnarFileScan.java:51-62): a device or plan
    // failure (PredEvalException on operand types included) is a FileScanException
    try {
      this.deleteQuery = deleteQuery;
      this.len_in1 = len_in1;
      outTypes = new AttrType[n_out_flds];
      if (!deleteQuery)
        TupleUtils.setup_op_tuple(Jtuple, outTypes, in1, len_in1, s1_sizes, proj_list, n_out_flds);  // :66-71
      perm_mat = proj_list;
      ctx = GpuContext.ctx();
      table = GpuTables.get(file_name);
      // per-column char(n) sizes: s1_sizes lists the string columns' sizes in order
      short[] colSize = new short[len_in1];
      for (int c = 0, k = 0; c < len_in1; c++)
        colSize[c] = in1[c].attrType == AttrType.attrString ? s1_sizes[k++] : 4;
      proj = new int[n_out_flds];
      projTypes = new int[n_out_flds];
      projSizes = new short[n_out_flds];
      for (int k = 0; k < n_out_flds; k++) {
        if (proj_list[k].relation.key != RelSpec.outer) throw new InvalidRelation("Invalid relation -innerRel");
        proj[k] = proj_list[k].offset - 1;
        projTypes[k] = in1[proj[k]].attrType;
        projSizes[k] = colSize[proj[k]];
      }
      plan = Native.planCompile(ctx, table, outFilter);                    // PredEvalException on type errors
      try {
        selection = Native.scanBitmap(ctx, plan);                         // one kernel launch
        cursor = Native.cursorOpen(ctx, table, selection, proj);          // positions + projected values in HBM
      } catch (Exception e) {
        close();
        throw new FileScanException(e, "GPU scan failed");
      }
    } catch (IOException | FileScanException | TupleUtilsException | InvalidRelation | RuntimeException e) {
      close();
      throw e;
    } catch (Exception e) {
      close();
      throw new FileScanException(e, "GPU scan setup failed");
    }
  }

  /** shows what input fields go where in the output tuple (:139-142) */
  public FldSpec[] show() {
    return perm_mat;
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
    if (deleteQuery) throw new NullPointerException("ColumnarFileScan: the delete-query form has no output tuple");
    for (int k = 0; k < outTypes.length; k++) {
      switch (outTypes[k].attrType) {
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
    return new TID(len_in1, (int) ids[i++]);
  }

  public long gpuTable() {
    return table;
  }

  public long gpuSelection() {
    return selection;
  }

  public int[] fileColumns() {
    return proj.clone();
  }

  /** the whole selection's size (Query's resultCount) without materialising it */
  public long resultCount() throws Exception {
    return Native.cursorCount(cursor);
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
      throw new FileScanException(e, "restart failed");
    }
    n = i = 0;
  }

  public int getTupleSize() {
    if (deleteQuery) throw new NullPointerException("ColumnarFileScan: the delete-query form has no output tuple");
    return Jtuple.size();
  }
}
