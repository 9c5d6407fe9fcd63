package global;

/**
 * The per-JVM GPU context(s), next to SystemDefs (R/global/SystemDefs.java:6-9):
 * one mbx_ctx per GPU, created on first use.  The engine is single threaded;
 * so is this class's contract.
 */
public final class GpuContext {
  private static long[] ctxs;
  private static long[] comms;   // one RCCL clique over the contexts of GPUs 0..n-1, shared

  private GpuContext() {}

  /** the context of GPU 0 (every single-GPU operator) */
  public static synchronized long ctx() throws Exception {
    return ctx(0);
  }

  public static synchronized long ctx(int device) throws Exception {
    if (ctxs == null) ctxs = new long[Math.max(1, Native.deviceCount())];
    if (device < 0 || device >= ctxs.length) throw new IllegalArgumentException("GPU " + device);
    if (ctxs[device] == 0) ctxs[device] = Native.init(device);
    return ctxs[device];
  }

  public static synchronized int devices() {
    return Math.max(1, Native.deviceCount());
  }

  /**
   * The communicators of one RCCL clique over every GPU (rank g = GPU g),
   * created once and shared by every sharded scan of the JVM: a context
   * carries at most one communicator (mbx_comm_init_all refuses a second).
   */
  public static synchronized long[] comms() throws Exception {
    if (comms == null) {
      long[] cs = new long[devices()];
      for (int g = 0; g < cs.length; g++) cs[g] = ctx(g);
      comms = Native.commInitAll(cs);
    }
    return comms;
  }

  /** releases the clique and every context (SystemDefs shutdown) */
  public static synchronized void shutdown() {
    if (comms != null) for (long m : comms) if (m != 0) Native.commFree(m);
    comms = null;
    if (ctxs == null) return;
    for (long c : ctxs) if (c != 0) Native.free(c);
    ctxs = null;
  }
}
