package columnar;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.BitSet;
import java.util.HashMap;
import java.util.IdentityHashMap;
import java.util.Map;

import bitmap.BitMapFile;
import bufmgr.GpuFlush;
import global.AttrType;
import global.Convert;
import global.GpuContext;
import global.Native;
import global.RID;
import global.SystemDefs;
import heap.Heapfile;
import heap.Scan;
import heap.Tuple;

/**
 * HBM images of Columnarfiles and BitMapFiles, staged once per file and kept
 * until the file changes (tables are scanned many times, DESIGN.md section 2).
 * A Columnarfile is staged straight from the DB file (mbx_db_stage: pages ->
 * HBM -> GPU page decoder, the reference's positions kept, cf.md and holes
 * as deleted rows) after the dirty UNPINNED frames of the buffer pool were
 * flushed one by one (bufmgr.GpuFlush; never flushAllPages, which throws
 * PagePinnedException when a reference iterator holds a pin,
 * R/bufmgr/BufMgr.java:349-400).  If a dirty frame is pinned, its bytes are not
 * on disk yet: the Columnarfile is then lifted through the buffer pool
 * instead (heap.Scan per column, decoded into direct ByteBuffers,
 * Native.tableStage) -- the JVM's own view, pinned pages included.
 */
public final class GpuTables {
  private static String dbPath;
  private static long db;
  private static final Map<String, Long> tables = new HashMap<>();
  private static final Map<BitMapFile, Long> bitmaps = new IdentityHashMap<>();

  private GpuTables() {}

  /** the DB file SystemDefs opened (its path, as passed to new SystemDefs(...)) */
  public static synchronized void open(String path) throws Exception {
    if (path.equals(dbPath)) return;
    invalidateAll();
    if (db != 0) Native.dbClose(db);
    db = 0;
    dbPath = path;
  }

  private static int dirtyPinned;   // dirty frames the last flush had to leave in the pool

  private static long db() throws Exception {
    if (dbPath == null) throw new IllegalStateException("GpuTables.open(dbPath) first");
    dirtyPinned = GpuFlush.flushUnpinned(SystemDefs.JavabaseBM);
    if (db == 0) db = Native.dbOpen(dbPath);
    return db;
  }

  /**
   * The DB file handle (dirty unpinned frames flushed first): sharded scans
   * stage their row ranges straight from it, so a dirty frame still pinned
   * (an insert in progress) makes the file stale for them: FileScanException.
   */
  public static synchronized long dbHandle() throws Exception {
    long d = db();
    if (dirtyPinned != 0)
      throw new iterator.FileScanException(null, "GpuTables: " + dirtyPinned
          + " dirty buffer frame(s) pinned; the DB file is not current for row-range staging");
    return d;
  }

  public static synchronized long get(String columnarFile) throws Exception {
    Long t = tables.get(columnarFile);
    if (t == null) {
      long d = db();
      t = dirtyPinned == 0 ? Native.dbStage(GpuContext.ctx(), d, columnarFile) : stageDecoded(columnarFile);
      tables.put(columnarFile, t);
    }
    return t;
  }

  /**
   * A Columnarfile lifted through the buffer pool: every column heapfile
   * walked with heap.Scan (R/heap/Scan.java:84-113), each record placed at its
   * position (Heapfile.findPosition, R/heap/Heapfile.java:262-273) in a direct
   * ByteBuffer in host order -- int / float as their 4 big-endian bytes read
   * with Convert.getIntValue (R/global/Convert.java:18-37; a float keeps its
   * bits), char(n) as the record's writeUTF payload zero-padded to n bytes.
   * Positions some column lacks (holes) and cf.md's marks are deleted rows,
   * as TupleScan skips them (R/columnar/TupleScan.java:55-89).
   */
  static long stageDecoded(String name) throws Exception {
    Columnarfile f = new Columnarfile(name);
    final AttrType[] types = f.getAttributeTypes();
    final short[] sizes = f.getAttrSizes();
    final int nc = f.getFieldCount();
    final Heapfile[] hfs = f.getHeapfiles();
    int nrows = 0;
    for (int c = 0; c < nc; c++) {
      Scan s = hfs[c].openScan();
      RID rid = new RID();
      try {
        while (s.getNext(rid) != null) nrows = Math.max(nrows, hfs[c].findPosition(rid) + 1);
      } finally {
        s.closescan();
      }
    }
    int[] t = new int[nc];
    short[] w = new short[nc];
    ByteBuffer[] cols = new ByteBuffer[nc];
    BitSet present = new BitSet();
    present.set(0, nrows);
    for (int c = 0; c < nc; c++) {
      t[c] = types[c].attrType;
      w[c] = t[c] == AttrType.attrString ? sizes[c] : 4;
      ByteBuffer b = ByteBuffer.allocateDirect(Math.max(1, columnBytes(name, c, nrows, w[c])))
          .order(ByteOrder.nativeOrder());
      BitSet have = new BitSet(nrows);
      Scan s = hfs[c].openScan();
      RID rid = new RID();
      try {
        Tuple tu;
        while ((tu = s.getNext(rid)) != null) {
          int p = hfs[c].findPosition(rid);
          byte[] rec = tu.getTupleByteArray();
          if (t[c] == AttrType.attrString) {
            int len = ((rec[0] & 0xff) << 8) | (rec[1] & 0xff);
            // p * w[c] + k < nrows * w[c] <= Integer.MAX_VALUE (columnBytes)
            final int at = (int) ((long) p * w[c]);
            for (int k = 0; k < w[c]; k++) b.put(at + k, k < len ? rec[2 + k] : 0);
          } else {
            b.putInt((int) ((long) p * 4), Convert.getIntValue(0, rec));
          }
          have.set(p);
        }
      } finally {
        s.closescan();
      }
      present.and(have);
      cols[c] = b;
    }
    BitSet deleted = (BitSet) f.getMarkedDeleted().getBitSet().clone();
    BitSet holes = new BitSet();
    holes.set(0, nrows);
    holes.andNot(present);
    deleted.or(holes);
    return Native.tableStage(GpuContext.ctx(), t, w, nrows, cols, deleted.toLongArray(), 0);
  }

  /**
   * The bytes of one decoded column, computed in long: a direct ByteBuffer
   * holds at most Integer.MAX_VALUE bytes (e.g. a char(16) column past
   * 134,217,727 rows does not fit), so a larger column is refused with
   * FileScanException instead of an int product that wraps (to a negative
   * allocation or to offsets inside another row).  The DB-file path
   * (Native.dbStage) has no such limit.
   */
  static int columnBytes(String name, int col, long nrows, int width) throws iterator.FileScanException {
    final long bytes = nrows * (long) width;
    if (bytes > Integer.MAX_VALUE)
      throw new iterator.FileScanException(null, "GpuTables: column " + col + " of " + name + " needs " + bytes
          + " bytes; a decoded column (a dirty frame is pinned) holds at most " + Integer.MAX_VALUE
          + " -- unpin it so the DB file can be staged");
    return (int) bytes;
  }

  /**
   * Stage (if needed) a Columnarfile and add a column group over 2..4 of its
   * 4-byte columns (0-based): index / file scans projecting them gather one
   * 128-byte line per selected row (DESIGN.md section 2).  Lives with the
   * staged table (dropped by invalidate); an empty cols array drops the
   * table's groups (mbx_table_group with ncols = 0).
   */
  public static synchronized void group(String columnarFile, int[] cols) throws Exception {
    Native.tableGroup(GpuContext.ctx(), get(columnarFile), cols);
  }

  /** a BitMapFile's BitSet on the device (uploaded from the engine's own copy) */
  public static synchronized long bitmap(BitMapFile f, long nbits) throws Exception {
    Long b = bitmaps.get(f);
    if (b == null) {
      b = Native.bitmapUpload(GpuContext.ctx(), nbits, f.getBitSet().toLongArray());
      bitmaps.put(f, b);
    }
    return b;
  }

  /** call after insertTuple / markTupleDeleted / purgeAllDeletedTuples / createBitMapIndex */
  public static synchronized void invalidate(String columnarFile) {
    Long t = tables.remove(columnarFile);
    if (t != null) Native.tableFree(t);
    for (Long b : bitmaps.values()) Native.bitmapFree(b);
    bitmaps.clear();
  }

  public static synchronized void invalidateAll() {
    for (Long t : tables.values()) Native.tableFree(t);
    tables.clear();
    for (Long b : bitmaps.values()) Native.bitmapFree(b);
    bitmaps.clear();
  }
}
