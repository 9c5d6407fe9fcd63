package iterator;

/**
 * What the GPU join operators need from the iterator they are handed (the
 * outerItr / innerItr of ColumnarNestedLoopJoins,
 * R/iterator/ColumnarNestedLoopJoins.java:48-66): the iterator's rows as a
 * device BitSet over its staged table, and which file column each field of
 * its output tuple holds.  Implemented by GpuColumnarFileScan,
 * GpuColumnarColumnScan, GpuColumnarColumnsScan and GpuColumnarIndexScan.
 */
public interface GpuSelection {
  /** the staged table (mbx_table handle) the selection's positions index */
  long gpuTable() throws Exception;

  /** the rows get_next() returns, as a device BitSet (mbx_bitmap handle, owned by the iterator) */
  long gpuSelection() throws Exception;

  /** field k + 1 of the output tuple is file column fileColumns()[k] (0-based) */
  int[] fileColumns();
}
