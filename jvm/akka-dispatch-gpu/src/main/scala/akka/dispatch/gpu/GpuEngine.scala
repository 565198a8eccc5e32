/*
 * One engine (one agx_engine handle = one GPU rank) per GpuDispatcher instance: actor ids,
 * the MPSC staging buffer that ActorRef.! appends to, and the pump that runs supersteps.
 */
package akka.dispatch.gpu

import java.lang.foreign._
import java.lang.foreign.ValueLayout._
import java.util.concurrent.ConcurrentHashMap
import java.util.concurrent.atomic.{ AtomicBoolean, AtomicInteger }

import com.typesafe.config.Config

import akka.actor.ActorRef

final class GpuEngine(val dispatcherId: String, config: Config, throughput: Int) {
  import AgxNative._

  private val arena = Arena.ofShared()
  val maxActors: Long = config.getLong("gpu.actors")
  private val capacity: Int = if (config.hasPath("gpu.mailbox-capacity")) config.getInt("gpu.mailbox-capacity") else 0

  /** agx_create from the dispatcher's HOCON block (throughput: reference.conf:541, <= 0 behaves as 1) */
  val handle: MemorySegment = {
    val cfg = arena.allocate(Cfg)
    cfg.set(JAVA_INT, 0, AbiVersion)
    cfg.set(JAVA_INT, 4, if (config.hasPath("gpu.device")) config.getInt("gpu.device") else 0)
    cfg.set(JAVA_LONG, 8, maxActors)
    cfg.set(JAVA_INT, 16, math.max(throughput, 0))
    cfg.set(JAVA_INT, 20, capacity)
    cfg.set(JAVA_INT, 24, config.getInt("gpu.state-words"))
    cfg.set(JAVA_INT, 28, config.getInt("gpu.max-emit"))
    cfg.set(JAVA_INT, 32, 1)
    cfg.set(JAVA_INT, 36, 0)
    cfg.set(JAVA_INT, 40, 1000) // akka.cluster.sharding number-of-shards (typed reference.conf:10)
    cfg.set(JAVA_INT, 44, if (config.hasPath("gpu.bucket-actors")) config.getInt("gpu.bucket-actors") else 0)
    cfg.set(JAVA_LONG, 48, 0L)
    val out = arena.allocate(ADDRESS)
    check(create.invokeExact(cfg, out).asInstanceOf[Int])
    out.get(ADDRESS, 0)
  }

  // ---------------------------------------------------------------- actor ids
  private val nextId = new AtomicInteger(0)
  private val ids = new ConcurrentHashMap[ActorRef, Integer]()

  /** actorOf: one fixed-layout actor (GpuMailboxType.create) */
  def register(ref: ActorRef, kind: Int, init: Array[Long]): Int = {
    val id = nextId.getAndIncrement()
    if (id >= maxActors) throw new IllegalStateException(s"GPU dispatcher [$dispatcherId] is full ($maxActors actors)")
    val st = if (init == null) MemorySegment.NULL else arena.allocateFrom(JAVA_LONG, init: _*)
    synchronized { check(registerRange.invokeExact(handle, id.toLong, 1L, kind, st, init.length.toLong * 8).asInstanceOf[Int]) }
    ids.put(ref, id)
    id
  }

  /** a contiguous range of fixed-layout actors with no JVM ActorCell each (GpuDispatcher.spawnRange) */
  def registerRange(count: Int, kind: Int): Int = {
    val first = nextId.getAndAdd(count)
    if (first.toLong + count > maxActors) throw new IllegalStateException(s"GPU dispatcher [$dispatcherId] is full")
    synchronized {
      check(AgxNative.registerRange.invokeExact(handle, first.toLong, count.toLong, kind, MemorySegment.NULL, 0L).asInstanceOf[Int])
    }
    first
  }

  def idOf(ref: ActorRef): Int = {
    val i = ids.get(ref)
    if (i == null) NoSender else i.intValue
  }

  // ---------------------------------------------------------------- staging (MPSC)
  // Senders append under a lock (dispatch is called concurrently from any thread, AbstractDispatcher
  // contract); the pump swaps the buffer out and hands it to agx_stage_tells in one call.
  private var dst = new Array[Int](1024)
  private var src = new Array[Int](1024)
  private var pay = new Array[Int](1024)
  private var n = 0

  def stage(dstId: Int, srcId: Int, payload: Int): Unit = synchronized {
    if (n == dst.length) {
      dst = java.util.Arrays.copyOf(dst, 2 * n)
      src = java.util.Arrays.copyOf(src, 2 * n)
      pay = java.util.Arrays.copyOf(pay, 2 * n)
    }
    dst(n) = dstId
    src(n) = srcId
    pay(n) = payload
    n += 1
  }

  private val pumping = new AtomicBoolean(false)

  /** Run supersteps until the engine is quiescent.  One host thread drives the handle at a time
   *  (include/akka_gpu.h threading rule); returns false if another pump is running. */
  def pump(maxSupersteps: Int): Boolean = {
    if (!pumping.compareAndSet(false, true)) return false
    try {
      var more = true
      while (more) {
        val (d, s, p, k) = synchronized {
          val r = (dst, src, pay, n)
          dst = new Array[Int](math.max(1024, n)); src = new Array[Int](dst.length); pay = new Array[Int](dst.length)
          n = 0
          r
        }
        if (k > 0) {
          val a = Arena.ofConfined()
          try {
            check(stageTells.invokeExact(handle, a.allocateFrom(JAVA_INT, d.take(k): _*),
              a.allocateFrom(JAVA_INT, s.take(k): _*), a.allocateFrom(JAVA_INT, p.take(k): _*), k.toLong).asInstanceOf[Int])
          } finally a.close()
        }
        check(run.invokeExact(handle, maxSupersteps, MemorySegment.NULL).asInstanceOf[Int])
        more = synchronized(n > 0)
      }
      true
    } finally pumping.set(false)
  }

  def hasStaged: Boolean = synchronized(n > 0)

  /** delivered, dead letters, unhandled, emitted, staged, supersteps, in flight, bytes */
  def stats(): Array[Long] = {
    val a = Arena.ofConfined()
    try {
      val st = a.allocate(Stats)
      check(getStats.invokeExact(handle, st).asInstanceOf[Int])
      st.toArray(JAVA_LONG)
    } finally a.close()
  }

  def state(id: Int, words: Int): (Array[Long], Boolean) = {
    val a = Arena.ofConfined()
    try {
      val w = a.allocate(JAVA_LONG, words.toLong)
      val alive = a.allocate(JAVA_BYTE, 1)
      check(readState.invokeExact(handle, id.toLong, 1L, w, alive).asInstanceOf[Int])
      (w.toArray(JAVA_LONG), alive.get(JAVA_BYTE, 0) != 0)
    } finally a.close()
  }

  def close(): Unit = {
    check(destroy.invokeExact(handle).asInstanceOf[Int])
    arena.close()
  }
}

object GpuEngine {
  /** dispatcher id -> engine; GpuMailboxType finds its dispatcher's engine here */
  private val engines = new ConcurrentHashMap[String, GpuEngine]()
  def register(e: GpuEngine): Unit = engines.put(e.dispatcherId, e)
  def unregister(e: GpuEngine): Unit = engines.remove(e.dispatcherId, e)
  def forDispatcher(id: String): GpuEngine = {
    val e = engines.get(id)
    if (e == null) throw new akka.ConfigurationException(s"GPU dispatcher [$id] not created yet (mailbox before dispatcher)")
    e
  }
}
