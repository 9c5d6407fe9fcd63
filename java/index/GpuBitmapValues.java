package index;

import java.util.ArrayList;
import java.util.List;
import java.util.Set;

import bitmap.BitMapFile;
import columnar.Columnarfile;
import columnar.GpuTables;
import global.AttrOperator;
import global.AttrType;
import global.IntegerValue;
import global.StringValue;
import iterator.CondExpr;

/**
 * ColumnIndexScan.getBitSet's value selection (R/index/ColumnIndexScan.java:656-740),
 * kept on the host exactly as the reference does it -- it walks the column's
 * registered bitmap values, not rows -- returning the device handles of the
 * BitMapFiles whose value v satisfies `v op literal`; their OR (and the
 * AND across conjuncts, and NOT deleted) is one kernel (Native.bitmapCnf).
 * A value that is not registered contributes the empty BitSet the reference
 * ORs in (getBitmapIndex returns `new BitMapFile()`), i.e. nothing.
 * aopNOT / aopNOP / opRANGE select nothing (getBitSet has no branch for them).
 */
final class GpuBitmapValues {
  private GpuBitmapValues() {}

  static List<Long> of(Columnarfile f, int colNo, CondExpr e, long nbits) throws Exception {
    final boolean str = f.getAttributeType(colNo).attrType == AttrType.attrString;
    final List<Long> out = new ArrayList<>();
    for (Object v : values(f, colNo, e)) out.add(handle(f, colNo, v, str, nbits));
    return out;
  }

  /** the registered values v with `v op literal` (String or Integer), in getBitSet's order */
  static List<Object> values(Columnarfile f, int colNo, CondExpr e) throws Exception {
    final int op = e.op.attrOperator;
    final boolean str = f.getAttributeType(colNo).attrType == AttrType.attrString;
    final Set<?> all = f.getBitmapValues(colNo);
    final List<Object> out = new ArrayList<>();
    final Object lit = str ? (Object) e.operand2.string : (Object) Integer.valueOf(e.operand2.integer);
    if ((op == AttrOperator.aopEQ || op == AttrOperator.aopLE || op == AttrOperator.aopGE) && all.contains(lit))
      out.add(lit);
    for (Object v : all) {
      final int c = str ? ((String) lit).compareTo((String) v) : Integer.compare((Integer) lit, (Integer) v);
      final boolean take = ((op == AttrOperator.aopLT || op == AttrOperator.aopLE) && c > 0)
          || ((op == AttrOperator.aopGT || op == AttrOperator.aopGE) && c < 0)
          || (op == AttrOperator.aopNE && c != 0);
      if (take) out.add(v);
    }
    return out;
  }

  private static long handle(Columnarfile f, int colNo, Object v, boolean str, long nbits) throws Exception {
    BitMapFile bm = f.getBitmapIndex(colNo, str ? new StringValue((String) v) : new IntegerValue((Integer) v));
    return GpuTables.bitmap(bm, nbits);
  }
}
