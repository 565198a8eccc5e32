/*
 * One engine (one agx_engine handle = one GPU rank) per GpuDispatcher instance: actor ids, the
 * lock-free tell path that ActorRef.! appends to (agx_tell), the pump that runs supersteps, and the
 * reply path back to JVM actors.  All native calls go through an AgxBackend (JNI on JDK 8/11, Panama on
 * JDK 22+, AgxBackend.scala).
 *
 * Ids: GPU actors are [0, gpu.actors); a JVM actor that tells a GPU actor gets a host id in
 * [gpu.actors, gpu.actors + gpu.host-actors) (agx_set_outbound), so the GPU actor's sender() is a
 * real id: `sender() ! reply` (ActorCell.scala:583-587) lands in the engine's outbox, and the pump
 * delivers it to the JVM ActorRef with the replying GPU actor as sender.
 */
package akka.dispatch.gpu

import java.util.concurrent.ConcurrentHashMap
import java.util.concurrent.atomic.{ AtomicInteger, LongAdder }

import com.typesafe.config.Config

import akka.actor.ActorRef

final class GpuEngine(val dispatcherId: String, config: Config, throughput: Int) {
  private val native: AgxBackend = AgxBackend.load()
  if (native.abiVersion != Agx.AbiVersion)
    throw new akka.ConfigurationException(s"akka-gpu: native ABI ${native.abiVersion}, shim ABI ${Agx.AbiVersion}")

  private def opt(path: String, default: Int): Int = if (config.hasPath(path)) config.getInt(path) else default
  val maxActors: Long = config.getLong("gpu.actors")
  private val defaultCapacity: Int = opt("gpu.mailbox-capacity", 0)
  val stateWords: Int = config.getInt("gpu.state-words")
  private val nHost: Int = opt("gpu.host-actors", 65536)

  /** agx_create from the dispatcher's HOCON block (throughput: reference.conf:541, <= 0 behaves as 1) */
  val handle: Long = native.create(
    opt("gpu.device", 0),
    maxActors,
    math.max(throughput, 0),
    defaultCapacity,
    stateWords,
    config.getInt("gpu.max-emit"),
    1,
    0,
    1000, // akka.cluster.sharding number-of-shards (typed reference.conf:10)
    opt("gpu.bucket-actors", 0),
    0L)
  native.setOutbound(handle, maxActors.toInt, nHost, opt("gpu.outbox-capacity", 1 << 20).toLong)

  // ---------------------------------------------------------------- mailbox types (per actor)
  // Mailboxes.lookupConfigurator resolves a mailbox per actor (Mailboxes.scala:204-260): each distinct
  // capacity among this dispatcher's GPU mailbox types becomes one engine mailbox class (class 0 =
  // gpu.mailbox-capacity; at most Agx.MaxMailboxClasses - 1 further ones).
  private val classes = new ConcurrentHashMap[Integer, Integer]()
  classes.put(defaultCapacity, 0)
  def mailboxClass(capacity: Int): Int = synchronized {
    val c = classes.get(capacity)
    if (c != null) c.intValue
    else {
      val cls = classes.size
      if (cls >= Agx.MaxMailboxClasses)
        throw new akka.ConfigurationException(
          s"GPU dispatcher [$dispatcherId]: more than ${Agx.MaxMailboxClasses} distinct mailbox capacities")
      native.setMailboxClass(handle, cls, capacity)
      classes.put(capacity, cls)
      cls
    }
  }
  // capacities declared up front (gpu.mailbox-capacities = [64, 1000, 0]): their classes exist before
  // the first run -- with the ring apply on, the engine fixes its classes at that run, and a class added
  // later by an actorOf would be refused (INTEGRATION.md, "Ring apply and late mailbox types")
  if (config.hasPath("gpu.mailbox-capacities")) {
    val it = config.getIntList("gpu.mailbox-capacities").iterator()
    while (it.hasNext) mailboxClass(it.next().intValue)
  }

  // ---------------------------------------------------------------- actor ids
  private val nextId = new AtomicInteger(0)
  private val ids = new ConcurrentHashMap[ActorRef, Integer]()
  private val refs = new ConcurrentHashMap[Integer, ActorRef]() // GPU id -> its ActorRef (individually created)
  private val nextHost = new AtomicInteger(0)
  private val hostIds = new ConcurrentHashMap[ActorRef, Integer]()
  private val hostRefs = new ConcurrentHashMap[Integer, ActorRef]()

  /** actorOf: one fixed-layout actor (GpuMailboxType.create) with its mailbox class */
  def register(ref: ActorRef, kind: Int, init: Array[Long], mailboxCapacity: Int): Int = {
    val id = nextId.getAndIncrement()
    if (id >= maxActors) throw new IllegalStateException(s"GPU dispatcher [$dispatcherId] is full ($maxActors actors)")
    val cls = mailboxClass(mailboxCapacity)
    synchronized {
      native.registerRange(handle, id.toLong, 1L, kind, init, stateWords)
      if (cls != 0) native.setMailbox(handle, id.toLong, 1L, cls)
    }
    ids.put(ref, id)
    refs.put(id, ref)
    id
  }

  /** a contiguous range of fixed-layout actors with no JVM ActorCell each (GpuDispatcher.spawnRange) */
  def registerRange(count: Int, kind: Int, mailboxCapacity: Int): Int = {
    val first = nextId.getAndAdd(count)
    if (first.toLong + count > maxActors) throw new IllegalStateException(s"GPU dispatcher [$dispatcherId] is full")
    val cls = mailboxClass(mailboxCapacity)
    synchronized {
      native.registerRange(handle, first.toLong, count.toLong, kind, null, stateWords)
      if (cls != 0) native.setMailbox(handle, first.toLong, count.toLong, cls)
    }
    first
  }

  def setBehaviors(t: GpuBehaviors.Tables): Unit = synchronized(native.setBehaviors(handle, t))

  /** sender id of a tell: a GPU actor's own id, a host id for a JVM actor (the reply path), or
   *  noSender (deadLetters) when the host-id range is exhausted */
  def idOf(ref: ActorRef): Int = {
    if (ref == null || ref == ActorRef.noSender) return Agx.NoSender
    val i = ids.get(ref)
    if (i != null) return i.intValue
    val h = hostIds.get(ref)
    if (h != null) return h.intValue
    synchronized {
      val again = hostIds.get(ref)
      if (again != null) again.intValue
      else {
        val k = nextHost.getAndIncrement()
        if (k >= nHost) Agx.NoSender
        else {
          val id = maxActors.toInt + k
          hostIds.put(ref, id)
          hostRefs.put(id, ref)
          id
        }
      }
    }
  }

  // ---------------------------------------------------------------- the tell path (lock-free)
  // ActorRef.! from any thread appends through agx_tell to a native queue of the calling thread's
  // own (include/akka_gpu.h "lock-free tell path"; AbstractNodeQueue.java:79-82 enqueues with one
  // getAndSet): no monitor per tell.  agx_tell answers true exactly when the engine went from idle to
  // scheduled -- the caller then submits ONE pump task (Mailbox.setAsScheduled, Mailbox.scala:185-194).

  // the dispatcher's pump submission (GpuDispatcher sets it once it has an executor)
  @volatile private var submitPump: () => Unit = () => ()
  private[gpu] def setPumpSubmitter(f: () => Unit): Unit = submitPump = f

  // ---------------------------------------------------------------- close guard
  // Every native call that may race close() (tells from any thread, the pump) runs between enter()
  // and exit(); close() sets `closed`, then waits until every call that entered has exited before
  // agx_destroy frees the engine.  Two monotonic striped counters, so the tell path keeps no shared
  // contended word: entered >= exited always, and once closed is set a reading of exited followed by
  // an equal reading of entered means no call is inside (a call entering later sees closed).
  @volatile private var closed = false
  private val entered = new LongAdder
  private val exited = new LongAdder
  private[gpu] val lateTells = new LongAdder // tells after close: dead letters (the engine is gone)
  @inline private def enter(): Boolean = {
    entered.increment()
    if (closed) { exited.increment(); false }
    else true
  }
  @inline private def exit(): Unit = exited.increment()

  /** ActorRef.! : the tell enters the engine; the pump is submitted only on idle -> scheduled.
   *  After close() a tell is a dead letter (the dispatcher shut down, AbstractDispatcher.scala:325). */
  def tell(dstId: Int, srcId: Int, payload: Int): Unit =
    if (!enter()) lateTells.increment()
    else {
      val submit =
        try native.tell(handle, dstId, srcId, payload)
        finally exit()
      if (submit) submitPump()
    }

  private val outD = new Array[Int](4096)
  private val outS = new Array[Int](4096)
  private val outP = new Array[Int](4096)

  /** One pump task: take every tell published so far, run supersteps until the engine is
   *  quiescent, deliver the outbound replies to JVM actors, then the idle protocol (Mailbox.run's
   *  finally: setAsIdle + registerForExecution) -- returns true iff tells arrived meanwhile and
   *  the caller must submit the pump again.  At most one pump is scheduled at a time (the CAS in
   *  agx_tell / agx_pump_idle), so one host thread drives the handle (include/akka_gpu.h rule). */
  def pump(maxSupersteps: Int): Boolean =
    if (!enter()) false
    else
      try {
        native.run(handle, maxSupersteps, null)
        deliverOutbound()
        // also true while mail is still in flight after a run that hit gpu.supersteps-per-pump, or
        // while tells wait in the queue for capacity (agx_pump_idle; Mailbox.run's hasMessages re-check)
        native.pumpIdle(handle)
      } finally exit()

  /** a failed pump still ends with the idle protocol (else the engine would stay "scheduled") */
  private[gpu] def pumpIdleAfterFailure(): Boolean =
    if (!enter()) false
    else
      try native.pumpIdle(handle)
      catch { case _: Throwable => false }
      finally exit()

  /** the executor rejected the pump: back to idle, so the next tell submits it again */
  private[gpu] def pumpCancel(): Unit =
    if (enter())
      try native.pumpCancel(handle)
      finally exit()
  /** outbox -> JVM actors: `jvmRef ! GpuTell(payload)` with the replying GPU actor as sender
   *  (each GPU sender's replies in emission order, the only order Akka guarantees) */
  private def deliverOutbound(): Unit = {
    var k = native.takeOutbound(handle, outD, outS, outP, outD.length)
    while (k > 0) {
      var i = 0
      while (i < k) {
        val to = hostRefs.get(outD(i))
        if (to != null) to.tell(GpuTell(outP(i)), refs.getOrDefault(outS(i), ActorRef.noSender))
        i += 1
      }
      k = native.takeOutbound(handle, outD, outS, outP, outD.length)
    }
  }

  /** delivered, dead letters, unhandled, emitted, staged, supersteps, in flight, bytes */
  def stats(): Array[Long] = guarded {
    val st = new Array[Long](8)
    native.getStats(handle, st)
    st
  }

  def state(id: Int): (Array[Long], Boolean) = guarded {
    val w = new Array[Long](stateWords)
    val alive = new Array[Byte](1)
    native.readState(handle, id.toLong, 1L, w, alive)
    (w, alive(0) != 0)
  }

  private def guarded[T](f: => T): T =
    if (!enter()) throw new IllegalStateException(s"GPU dispatcher [$dispatcherId] is shut down")
    else
      try f
      finally exit()

  /** agx_destroy, once no tell or pump is inside the engine (idempotent) */
  def close(): Unit = synchronized {
    if (!closed) {
      closed = true
      while (exited.sum() != entered.sum()) Thread.`yield`() // (exited first: see the guard above)
      native.destroy(handle)
    }
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
