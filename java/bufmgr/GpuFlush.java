package bufmgr;

import global.GlobalConst;
import global.PageId;

/**
 * Brings the DB file up to date for the GPU's reader without
 * BufMgr.flushAllPages().  flushAllPages (privFlushPages with all_pages,
 * R/bufmgr/BufMgr.java:349-400,785-796) writes and evicts every dirty frame,
 * pinned ones included, and then throws PagePinnedException if ANY frame is
 * pinned -- so a GPU drop-in constructed while a reference iterator holds a
 * pin (a ColumnarFileScan outer of a join mid-scan) would fail, and the
 * iterator's pinned frame would have been evicted under it.  Here each dirty,
 * unpinned frame is flushed on its own (flushPage, :765-773, which leaves
 * every other frame alone) and the dirty pinned frames are only counted: their
 * bytes are not on disk yet, so the caller lifts the columns through the
 * buffer pool instead (columnar.GpuTables).  In package bufmgr because the
 * frame table's element class FrameDesc is package-private (:16); the table
 * itself is public (frameTable(), :815).
 */
public final class GpuFlush implements GlobalConst {
  private GpuFlush() {}

  /** flushes every dirty unpinned frame; returns how many dirty frames are pinned */
  public static int flushUnpinned(BufMgr bm) throws Exception {
    int dirtyPinned = 0;
    FrameDesc[] frames = bm.frameTable();
    for (int i = 0; i < frames.length; i++) {
      FrameDesc f = frames[i];
      if (!f.dirty || f.pageNo.pid == INVALID_PAGE) continue;
      if (f.pin_count() != 0) {
        dirtyPinned++;
        continue;
      }
      bm.flushPage(new PageId(f.pageNo.pid));   // a fresh PageId: privFlushPages writes into its argument
    }
    return dirtyPinned;
  }
}
