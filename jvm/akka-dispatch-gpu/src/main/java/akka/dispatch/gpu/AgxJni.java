/*
 * JNI binding of include/akka_gpu.h for the reference's own JDKs (8 and 11: .travis.yml:10 of the
 * reference), where java.lang.foreign (AgxNative.scala, JDK 22+) does not exist.  One native
 * method per C-ABI entry point; the glue is src/main/c/agx_jni.c (libakka_gpu_jni.so, linked
 * against libakka_gpu.so), each function a direct forward that turns a non-zero agx_status into
 * an exception carrying agx_last_error():
 *   AGX_EINVAL    -> akka.ConfigurationException
 *   AGX_ECAPACITY -> java.lang.IllegalStateException ("mailbox arena full ...")
 *   anything else -> java.lang.IllegalStateException ("akka-gpu status N: ...")
 * Arrays are copied (Get/Set<Type>ArrayRegion); bulk tells go through direct ByteBuffers
 * (GetDirectBufferAddress: no copy on the JVM side) or int[] arrays.
 */
package akka.dispatch.gpu;

import java.nio.ByteBuffer;

public final class AgxJni {
  static {
    System.loadLibrary(System.getProperty("akka.gpu.jni", "akka_gpu_jni"));
  }

  private AgxJni() {}

  public static native int abiVersion();

  public static native String lastError();

  /** agx_create; returns the engine handle (MessageDispatcherConfigurator.dispatcher()). */
  public static native long create(int device, long nActors, int throughput, int capacity, int nWords, int maxEmit,
                                   int nRanks, int rank, int numShards, int bucketActors, long msgCapacity);

  public static native void destroy(long engine);

  /** agx_register_range; initState: count x stateWords longs, actor-major, or null (zero state). */
  public static native void registerRange(long engine, long first, long count, int kind, long[] initState,
                                          int stateWords);

  /** agx_set_mailbox_class / agx_register_range_mailbox: a mailbox class (bounded capacity, 0 = unbounded)
   *  and a range of actors bound to it (Mailboxes.lookupConfigurator, per actor). */
  public static native void setMailboxClass(long engine, int mailboxClass, int capacity);

  public static native void setMailbox(long engine, long first, long count, int mailboxClass);

  public static native void setRing(long engine, int stride);

  public static native void setGossip(long engine, int fanout, long seed);

  public static native void setDeltaCrdt(long engine, int maxDeltaSize);

  /** agx_set_behaviors: the agx_case / agx_act tables as raw bytes (48 / 32 bytes per entry). */
  public static native void setBehaviors(long engine, byte[] cases, int nCases, byte[] acts, int nActs, int[] first,
                                         int nBehaviors);

  public static native void setFanout(long engine, int k, long seed, int[] cdf, int[] perm);

  public static native void setGraph(long engine, long[] rowPtr, int[] col);

  /** agx_stage_tells from direct ByteBuffers of n native-order ints each (src may be null = noSender). */
  public static native void stageTells(long engine, ByteBuffer dst, ByteBuffer src, ByteBuffer payload, int n);

  /** agx_stage_tells from int arrays. */
  public static native void stageTellsArrays(long engine, int[] dst, int[] src, int[] payload, int n);

  /** agx_run; stats (8 longs: delivered, dead letters, unhandled, emitted, staged, supersteps, in flight,
   *  algorithmic bytes) or null (no read-back; the error word is still checked). */
  /** agx_tell: lock-free, any thread; true iff the caller must submit the pump (idle -> scheduled). */
  public static native boolean tell(long engine, int dst, int src, int payload);

  /** agx_pump_idle: the pump's last call; true iff tells arrived meanwhile (submit the pump again). */
  public static native boolean pumpIdle(long engine);

  /** agx_pump_cancel: the executor rejected the pump; back to idle without the re-check. */
  public static native void pumpCancel(long engine);

  public static native void run(long engine, int maxSupersteps, long[] stats);

  public static native void getStats(long engine, long[] stats);

  /** agx_read_state: words (count x nWords) and alive (count) may each be null. */
  public static native void readState(long engine, long first, long count, long[] words, byte[] alive);

  /** agx_set_outbound: ids [firstHostId, firstHostId + nHost) are JVM actors; GPU tells to them
   *  are kept in an outbox of `capacity` envelopes instead of being dead letters. */
  public static native void setOutbound(long engine, int firstHostId, int nHost, long capacity);

  /** agx_take_outbound: up to cap outbound envelopes (dst host id, src GPU id, payload) in
   *  per-sender order; returns how many were written. */
  public static native int takeOutbound(long engine, int[] dst, int[] src, int[] payload, int cap);

  public static native int shardId(int id, int numShards);

  public static native int owner(int id, int numShards, int nRanks);
}
