package columnar;

import java.util.HashMap;
import java.util.IdentityHashMap;
import java.util.Map;

import bitmap.BitMapFile;
import global.GpuContext;
import global.Native;
import global.SystemDefs;

/**
 * HBM images of Columnarfiles and BitMapFiles, staged once per file and kept
 * until the file changes (tables are scanned many times, DESIGN.md section 2).
 * A Columnarfile is staged straight from the DB file (mbx_db_stage: pages ->
 * HBM -> GPU page decoder, the reference's positions kept, cf.md and holes
 * as deleted rows); the buffer pool is flushed first so the file on disk is
 * current.
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

  private static long db() throws Exception {
    if (dbPath == null) throw new IllegalStateException("GpuTables.open(dbPath) first");
    SystemDefs.JavabaseBM.flushAllPages();               // the pages the JVM still holds dirty
    if (db == 0) db = Native.dbOpen(dbPath);
    return db;
  }

  /** the DB file handle (buffer pool flushed first): sharded scans stage their row ranges from it */
  public static synchronized long dbHandle() throws Exception {
    return db();
  }

  public static synchronized long get(String columnarFile) throws Exception {
    Long t = tables.get(columnarFile);
    if (t == null) {
      t = Native.dbStage(GpuContext.ctx(), db(), columnarFile);
      tables.put(columnarFile, t);
    }
    return t;
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
