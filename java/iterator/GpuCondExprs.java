package iterator;

import global.AttrType;

/**
 * CondExpr[] copies whose symbol operands are renumbered from an iterator's
 * tuple fields to file columns, so a CNF written against a projected tuple
 * (ColumnarColumnScan's one-field tuple, :55-77; a join's pending filters
 * over its iterators' tuples, ColumnarNestedLoopJoins.java:120-158) compiles
 * against the staged Columnarfile.  A field outside the map keeps its number
 * and fails the plan compile (FieldNumberOutOfBoundException).
 */
final class GpuCondExprs {
  private GpuCondExprs() {}

  /** field k (1-based) -> file column cols[k - 1] + 1 */
  static CondExpr[] remap(CondExpr[] filter, int[] cols) {
    if (filter == null) return null;
    CondExpr[] out = new CondExpr[filter.length];
    for (int c = 0; c < filter.length && filter[c] != null; c++) {
      CondExpr head = null, tail = null;
      for (CondExpr e = filter[c]; e != null; e = e.next) {
        CondExpr x = new CondExpr();
        x.op = e.op;
        x.type1 = e.type1;
        x.type2 = e.type2;
        x.indexType = e.indexType;
        x.operand1 = operand(e.type1, e.operand1, cols);
        x.operand2 = operand(e.type2, e.operand2, cols);
        if (head == null) head = x;
        else tail.next = x;
        tail = x;
      }
      out[c] = head;
    }
    return out;
  }

  private static Operand operand(AttrType t, Operand o, int[] cols) {
    Operand x = new Operand();
    x.string = o.string;
    x.integer = o.integer;
    x.real = o.real;
    x.symbol = o.symbol;
    if (t != null && t.attrType == AttrType.attrSymbol && o.symbol != null && o.symbol.offset >= 1
        && o.symbol.offset <= cols.length)
      x.symbol = new FldSpec(o.symbol.relation, cols[o.symbol.offset - 1] + 1);
    return x;
  }
}
