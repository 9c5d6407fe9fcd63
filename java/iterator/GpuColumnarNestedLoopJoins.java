package iterator;

import java.io.IOException;
import java.util.ArrayList;
import java.util.List;

import columnar.Columnarfile;
import global.AttrType;
import global.GlobalConst;
import global.GpuContext;
import global.Native;
import heap.HFBufMgrException;
import heap.HFDiskMgrException;
import heap.HFException;
import heap.InvalidTupleSizeException;
import heap.InvalidTypeException;
import heap.Tuple;

/**
 * Drop-in for ColumnarNestedLoopJoins (R/iterator/ColumnarNestedLoopJoins.java:48-220):
 * same constructor, same get_next() rows in the same order, the same "Next
 * Pass Over Inner Table" and statistics lines.  The pair loop runs on the
 * GPU (Native.join -> mbx_join, MBX_JOIN_NLJ): the outer rows in blocks of
 * (amt_of_mem - 1) * (1024 / outer tuple size) -- one pass over the inner
 * relation per block -- and within a pass inner ascending, then outer
 * ascending, exactly as fillOuterBuffer / fillInnerBuffer / get_next walk
 * them (:120-200).  The pending filters (OuterFilter / RightFilter, PredEval
 * over the iterators' tuples) are scans AND-ed into the iterators' device
 * selections; Projection.Join is a gather by position of the projected
 * columns (Native.gather).  outerItr and innerItr must be GPU scans
 * (GpuSelection): their rows stay on the device.
 */
public class GpuColumnarNestedLoopJoins extends Iterator implements GlobalConst {
  static final int BATCH = 262144;  // rows per cursor batch: one packed copy each, 42 vs 24 GB/s at 64 Ki (profiles/r04/b)

  private final long ctx, res, outerTable, innerTable;
  private final List<Long> owned = new ArrayList<>();    // bitmaps this operator made
  private final Tuple Jtuple = new Tuple();
  private final AttrType[] Jtypes;
  private final FldSpec[] perm_mat;
  private final Columnarfile outerFile, innerFile;
  private final int[] ocols, icols;
  private final long npairs, passes, block, fullCount, iterCount;
  private final int tupleSize;
  private long fetched;
  private int k, batchN;
  private long curPass;
  private boolean done;
  private int[] pass;
  private Object[] outerVals, innerVals;   // per perm_mat entry of that side (null for the other side)

  public GpuColumnarNestedLoopJoins(Columnarfile outerColumnarFile, Columnarfile innerColumnarFile, AttrType in1[],
                                    int in1_len, short[] t1_str_sizes, AttrType in2[], int in2_len,
                                    short[] t2_str_sizes, Iterator outerItr, Iterator innerItr, CondExpr[] outFilter,
                                    CondExpr[] rightFilter, CondExpr[] joinFilter, FldSpec[] proj_list,
                                    int n_out_flds, int amt_of_mem)
      throws IOException, NestedLoopException, InvalidTypeException, InvalidTupleSizeException, JoinsException,
      HFException, HFBufMgrException, HFDiskMgrException {
    // the reference constructor's checked exceptions only (R/iterator/ColumnarNestedLoopJoins.java:47-61):
    // TupleUtilsException and device / plan failures become a NestedLoopException, as the reference wraps
    // setup_op_tuple's (:88-94)
    try {
      if (!(outerItr instanceof GpuSelection) || !(innerItr instanceof GpuSelection))
        throw new NestedLoopException("GpuColumnarNestedLoopJoins: outerItr / innerItr must be GPU scans "
                                      + "(GpuColumnarFileScan, GpuColumnarColumnScan, GpuColumnarColumnsScan, "
                                      + "GpuColumnarIndexScan)");
      outerFile = outerColumnarFile;
      innerFile = innerColumnarFile;
      Jtypes = new AttrType[n_out_flds];
      perm_mat = proj_list;
      TupleUtils.setup_op_tuple(Jtuple, Jtypes, in1, in1_len, in2, in2_len, t1_str_sizes, t2_str_sizes, proj_list,
                                n_out_flds);                                                          // :88-94
      ctx = GpuContext.ctx();
      GpuSelection o = (GpuSelection) outerItr, in = (GpuSelection) innerItr;
      outerTable = o.gpuTable();
      innerTable = in.gpuTable();
      ocols = o.fileColumns();
      icols = in.fileColumns();
      long osel = filtered(outerTable, o.gpuSelection(), outFilter, ocols);
      long isel = filtered(innerTable, in.gpuSelection(), rightFilter, icols);
      iterCount = Native.bitmapCardinality(o.gpuSelection());      // "Total Outer Tuples By Iterator"
      fullCount = Native.bitmapCardinality(osel);                  // "... By Full Constraint"
      // the join CNF: outer field OP inner field (NljQuery.buildCNFJoinCondExpr)
      List<int[]> terms = new ArrayList<>();
      List<Integer> offs = new ArrayList<>();
      offs.add(0);
      for (int c = 0; joinFilter != null && c < joinFilter.length && joinFilter[c] != null; c++) {
        for (CondExpr e = joinFilter[c]; e != null; e = e.next) {
          if (e.type1.attrType != AttrType.attrSymbol || e.type2.attrType != AttrType.attrSymbol)
            throw new NestedLoopException("GpuColumnarNestedLoopJoins: join terms compare an outer and an inner field");
          terms.add(new int[] {e.op.attrOperator, ocols[e.operand1.symbol.offset - 1], icols[e.operand2.symbol.offset - 1]});
        }
        offs.add(terms.size());
      }
      int[] t3 = new int[3 * terms.size()];
      for (int j = 0; j < terms.size(); j++) System.arraycopy(terms.get(j), 0, t3, 3 * j, 3);
      int[] o1 = new int[offs.size()];
      for (int j = 0; j < o1.length; j++) o1[j] = offs.get(j);
      tupleSize = outerItr.getTupleSize();
      block = (long) (amt_of_mem - 1) * (MINIBASE_PAGESIZE / tupleSize);                             // :122
      res = Native.join(ctx, outerTable, osel, innerTable, isel, t3, o1, Native.JOIN_NLJ, block);
      long[] info = Native.joinInfo(res);
      npairs = info[0];
      passes = info[1];
      passHeader(0);                                                                                 // :103-107
    } catch (IOException | NestedLoopException | InvalidTypeException | InvalidTupleSizeException | JoinsException
             | HFException | HFBufMgrException | HFDiskMgrException | RuntimeException e) {
      close();
      throw e;
    } catch (Exception e) {
      close();
      throw new NestedLoopException(e, "GpuColumnarNestedLoopJoins: GPU join setup failed");
    }
  }

  /** the iterator's selection AND the pending filter's scan (a new bitmap), or the selection itself */
  private long filtered(long table, long sel, CondExpr[] filter, int[] cols) throws Exception {
    if (filter == null || filter.length == 0 || filter[0] == null) return sel;
    long plan = Native.planCompile(ctx, table, GpuCondExprs.remap(filter, cols));
    try {
      long scan = Native.scanBitmap(ctx, plan);
      try {
        long both = Native.bitmapCombine(ctx, Native.BM_AND, sel, scan);
        owned.add(both);
        return both;
      } finally {
        Native.bitmapFree(scan);
      }
    } finally {
      Native.planFree(plan);
    }
  }

  private static void passHeader(long p) {
    System.out.println();
    System.out.println("************************************************************************");
    System.out.println("Next Pass Over Inner Table: " + p);
    System.out.println("************************************************************************");
    System.out.println();
  }

  private void statistics() {
    System.out.println();
    System.out.println("************************************************************************");
    System.out.println("Tuple Size: " + tupleSize);
    System.out.println("Number of Tuples Buffer Can Hold: " + block);
    System.out.println("Total Outer Tuples By Full Constraint: " + fullCount);
    System.out.println("Total Outer Tuples By Iterator: " + iterCount);
    System.out.println("************************************************************************");
    System.out.println();
  }

  /** the next batch of pairs and the projected values of both sides */
  private void fetch() throws Exception {
    final int m = (int) Math.min(BATCH, npairs - fetched);
    Object[] r = Native.joinFetch(ctx, res, fetched, m);
    long[] op = (long[]) r[0], ip = (long[]) r[1];
    pass = (int[]) r[2];
    outerVals = side(op, outerFile, ocols, outerTable, RelSpec.outer);
    innerVals = side(ip, innerFile, icols, innerTable, RelSpec.innerRel);
    fetched += m;
    batchN = m;
    k = 0;
  }

  private Object[] side(long[] pos, Columnarfile f, int[] cols, long table, int rel) throws Exception {
    int cnt = 0;
    for (FldSpec p : perm_mat) if (p.relation.key == rel) cnt++;
    int[] proj = new int[cnt], types = new int[cnt];
    short[] sizes = new short[cnt];
    int j = 0;
    for (FldSpec p : perm_mat) {
      if (p.relation.key != rel) continue;
      proj[j] = cols[p.offset - 1];
      types[j] = f.getAttributeType(proj[j]).attrType;
      sizes[j] = types[j] == AttrType.attrString ? f.getAttrSizes()[proj[j]] : 4;
      j++;
    }
    Object[] g = cnt > 0 ? Native.gather(ctx, table, pos, proj, types, sizes) : new Object[0];
    Object[] byPerm = new Object[perm_mat.length];
    j = 0;
    for (int q = 0; q < perm_mat.length; q++) if (perm_mat[q].relation.key == rel) byPerm[q] = g[j++];
    return byPerm;
  }

  public Tuple get_next() throws InvalidTupleSizeException, IOException, InvalidTypeException {
    // get_next's checked exceptions as the reference declares them (:157); a device failure while
    // fetching pairs or rows is an IOException (the pairs' I/O), its cause attached
    try {
      while (true) {
        if (k < batchN) {
          for (; curPass < pass[k]; ) passHeader(++curPass);
          for (int q = 0; q < perm_mat.length; q++) {                                  // Projection.Join
            Object col = perm_mat[q].relation.key == RelSpec.outer ? outerVals[q] : innerVals[q];
            switch (Jtypes[q].attrType) {
              case AttrType.attrInteger: Jtuple.setIntFld(q + 1, ((int[]) col)[k]); break;
              case AttrType.attrReal: Jtuple.setFloFld(q + 1, ((float[]) col)[k]); break;
              default: Jtuple.setStrFld(q + 1, ((String[]) col)[k]);
            }
          }
          k++;
          return Jtuple;
        }
        if (fetched < npairs) {
          fetch();
          continue;
        }
        if (!done) {                            // the passes without a pair, then the statistics (:178-190)
          for (; curPass < passes - 1; ) passHeader(++curPass);
          statistics();
          done = true;
        }
        return null;
      }
    } catch (InvalidTupleSizeException | IOException | InvalidTypeException | RuntimeException e) {
      throw e;
    } catch (Exception e) {
      throw new IOException("GpuColumnarNestedLoopJoins: GPU pair fetch failed", e);
    }
  }

  public void close() {
    if (!closeFlag) {
      if (res != 0) Native.joinFree(res);
      for (long b : owned) Native.bitmapFree(b);
      owned.clear();
      closeFlag = true;
    }
  }

  public int getTupleSize() {
    return Jtuple.size();
  }
}
