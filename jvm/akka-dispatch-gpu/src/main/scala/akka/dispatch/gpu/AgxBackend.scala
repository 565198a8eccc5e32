/*
 * The C ABI of include/akka_gpu.h as seen from the JVM, with plain JVM arrays and a `long` engine
 * handle, so GpuEngine does not care how the native library is reached:
 *   - JniBackend (this file): the JNI glue libakka_gpu_jni.so (src/main/c/agx_jni.c, AgxJni.java),
 *     for the reference's own JDKs 8 and 11 (.travis.yml:10 of the reference);
 *   - PanamaBackend (src/main/scala-jdk-22): java.lang.foreign downcalls, no native glue, JDK 22+.
 *     (Version-specific source directories follow the reference's own scala-jdk-9 layout,
 *     akka-remote/src/main/scala-jdk-9.)
 * Errors: every non-zero agx_status is an exception (akka.ConfigurationException for AGX_EINVAL,
 * IllegalStateException otherwise) carrying agx_last_error().
 */
package akka.dispatch.gpu

trait AgxBackend {
  def abiVersion: Int
  def create(device: Int, nActors: Long, throughput: Int, capacity: Int, nWords: Int, maxEmit: Int, nRanks: Int,
             rank: Int, numShards: Int, bucketActors: Int, msgCapacity: Long): Long
  def destroy(engine: Long): Unit
  def registerRange(engine: Long, first: Long, count: Long, kind: Int, init: Array[Long], stateWords: Int): Unit
  def setMailboxClass(engine: Long, mailboxClass: Int, capacity: Int): Unit
  def setMailbox(engine: Long, first: Long, count: Long, mailboxClass: Int): Unit
  def setBehaviors(engine: Long, t: GpuBehaviors.Tables): Unit
  def setOutbound(engine: Long, firstHostId: Int, nHost: Int, capacity: Long): Unit
  def takeOutbound(engine: Long, dst: Array[Int], src: Array[Int], payload: Array[Int], cap: Int): Int
  def stageTells(engine: Long, dst: Array[Int], src: Array[Int], payload: Array[Int], n: Int): Unit
  /** agx_tell (lock-free, any thread): true iff the caller must submit the pump */
  def tell(engine: Long, dst: Int, src: Int, payload: Int): Boolean
  /** agx_pump_idle (the pump's last call): true iff tells arrived meanwhile */
  def pumpIdle(engine: Long): Boolean
  /** agx_pump_cancel (the executor rejected the pump): back to idle, no re-check */
  def pumpCancel(engine: Long): Unit
  /** stats: 8 longs (delivered, dead letters, unhandled, emitted, staged, supersteps, in flight,
   *  algorithmic bytes), or null for no read-back */
  def run(engine: Long, maxSupersteps: Int, stats: Array[Long]): Unit
  def getStats(engine: Long, stats: Array[Long]): Unit
  def readState(engine: Long, first: Long, count: Long, words: Array[Long], alive: Array[Byte]): Unit
  def shardId(id: Int, numShards: Int): Int
}

object AgxBackend {
  /** `akka.dispatch.gpu.binding` system property: "jni", "panama" or "auto" (default): Panama when
   *  the JDK has java.lang.foreign (22+) and the module was built with scala-jdk-22, else JNI. */
  def load(): AgxBackend = System.getProperty("akka.dispatch.gpu.binding", "auto") match {
    case "jni"    => JniBackend
    case "panama" => panama().getOrElse(throw new akka.ConfigurationException("Panama binding needs JDK 22+"))
    case _        => panama().getOrElse(JniBackend)
  }

  private def panama(): Option[AgxBackend] =
    try {
      Class.forName("java.lang.foreign.Linker")
      Some(Class.forName("akka.dispatch.gpu.PanamaBackend$").getField("MODULE$").get(null).asInstanceOf[AgxBackend])
    } catch { case _: ClassNotFoundException | _: NoSuchFieldException => None }
}

/** JDK 8 / 11: every call is one AgxJni native method (src/main/c/agx_jni.c forwards it). */
object JniBackend extends AgxBackend {
  def abiVersion: Int = AgxJni.abiVersion()
  def create(device: Int, nActors: Long, throughput: Int, capacity: Int, nWords: Int, maxEmit: Int, nRanks: Int,
             rank: Int, numShards: Int, bucketActors: Int, msgCapacity: Long): Long =
    AgxJni.create(device, nActors, throughput, capacity, nWords, maxEmit, nRanks, rank, numShards, bucketActors,
      msgCapacity)
  def destroy(engine: Long): Unit = AgxJni.destroy(engine)
  def registerRange(engine: Long, first: Long, count: Long, kind: Int, init: Array[Long], stateWords: Int): Unit =
    AgxJni.registerRange(engine, first, count, kind, init, stateWords)
  def setMailboxClass(engine: Long, mailboxClass: Int, capacity: Int): Unit =
    AgxJni.setMailboxClass(engine, mailboxClass, capacity)
  def setMailbox(engine: Long, first: Long, count: Long, mailboxClass: Int): Unit =
    AgxJni.setMailbox(engine, first, count, mailboxClass)
  def setBehaviors(engine: Long, t: GpuBehaviors.Tables): Unit =
    AgxJni.setBehaviors(engine, t.cases, t.nCases, t.acts, t.nActs, t.first, t.behaviors.size)
  def setOutbound(engine: Long, firstHostId: Int, nHost: Int, capacity: Long): Unit =
    AgxJni.setOutbound(engine, firstHostId, nHost, capacity)
  def takeOutbound(engine: Long, dst: Array[Int], src: Array[Int], payload: Array[Int], cap: Int): Int =
    AgxJni.takeOutbound(engine, dst, src, payload, cap)
  def stageTells(engine: Long, dst: Array[Int], src: Array[Int], payload: Array[Int], n: Int): Unit =
    AgxJni.stageTellsArrays(engine, dst, src, payload, n)
  def tell(engine: Long, dst: Int, src: Int, payload: Int): Boolean = AgxJni.tell(engine, dst, src, payload)
  def pumpIdle(engine: Long): Boolean = AgxJni.pumpIdle(engine)
  def pumpCancel(engine: Long): Unit = AgxJni.pumpCancel(engine)
  def run(engine: Long, maxSupersteps: Int, stats: Array[Long]): Unit = AgxJni.run(engine, maxSupersteps, stats)
  def getStats(engine: Long, stats: Array[Long]): Unit = AgxJni.getStats(engine, stats)
  def readState(engine: Long, first: Long, count: Long, words: Array[Long], alive: Array[Byte]): Unit =
    AgxJni.readState(engine, first, count, words, alive)
  def shardId(id: Int, numShards: Int): Int = AgxJni.shardId(id, numShards)
}

/** Constants of include/akka_gpu.h shared by both bindings. */
object Agx {
  final val AbiVersion = 1
  final val NoSender = 0xFFFFFFFF // AGX_NO_SENDER (deadLetters as sender)
  final val KindNone = 0
  final val KindCounter = 1
  final val KindRing = 2
  final val KindFanout = 3
  final val KindForwardRR = 4
  final val KindStopAfter = 5
  final val KindPingPong = 6
  final val KindEven = 7
  final val KindGCounter = 8
  final val KindPNCounter = 9
  final val KindORSet = 10
  final val KindCompiled = 16 // + behaviour index (agx_set_behaviors)
  final val MaxMailboxClasses = 8
}
