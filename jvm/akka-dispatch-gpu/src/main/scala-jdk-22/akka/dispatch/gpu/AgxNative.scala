/*
 * Panama (java.lang.foreign, JDK 22+: Arena.allocateFrom) downcalls into include/akka_gpu.h -- the
 * AgxBackend for JVMs that have it.  No native glue: every handle binds one `extern "C"` symbol of
 * libakka_gpu.so with the C signature from the header.  JDK 8 / 11 use JniBackend instead
 * (src/main/scala/.../AgxBackend.scala).  Not compiled in the build image (no JVM, SURVEY.md
 * §8(c)); tests/c/abi_sequence.c and tests/c/jni_harness.c drive the same calls from C on the GPU.
 */
package akka.dispatch.gpu

import java.lang.foreign._
import java.lang.foreign.ValueLayout._
import java.lang.invoke.MethodHandle

import akka.ConfigurationException

object AgxNative {
  private val linker = Linker.nativeLinker()
  private val lib: SymbolLookup =
    SymbolLookup.libraryLookup(System.getProperty("akka.gpu.lib", "libakka_gpu.so"), Arena.global())
  private def h(name: String, fd: FunctionDescriptor): MethodHandle =
    linker.downcallHandle(lib.find(name).orElseThrow(() => new ConfigurationException(s"$name not found")), fd)

  /** struct agx_cfg: offsets 0 abi, 4 device, 8 n_actors, 16 throughput, 20 capacity, 24 n_words,
   *  28 max_emit, 32 n_ranks, 36 rank, 40 num_shards, 44 bucket_actors, 48 msg_capacity (56 bytes) */
  val Cfg: StructLayout = MemoryLayout.structLayout(
    JAVA_INT.withName("abi_version"),
    JAVA_INT.withName("device"),
    JAVA_LONG.withName("n_actors"),
    JAVA_INT.withName("throughput"),
    JAVA_INT.withName("capacity"),
    JAVA_INT.withName("n_words"),
    JAVA_INT.withName("max_emit"),
    JAVA_INT.withName("n_ranks"),
    JAVA_INT.withName("rank"),
    JAVA_INT.withName("num_shards"),
    JAVA_INT.withName("bucket_actors"),
    JAVA_LONG.withName("msg_capacity"))

  /** struct agx_stats: 8 x u64 */
  val Stats: SequenceLayout = MemoryLayout.sequenceLayout(8, JAVA_LONG)

  val abiVersion: MethodHandle = h("agx_abi_version", FunctionDescriptor.of(JAVA_INT))
  val create: MethodHandle = h("agx_create", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS))
  val destroy: MethodHandle = h("agx_destroy", FunctionDescriptor.of(JAVA_INT, ADDRESS))
  val lastError: MethodHandle = h("agx_last_error", FunctionDescriptor.of(ADDRESS))
  val registerRange: MethodHandle =
    h("agx_register_range", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, JAVA_LONG, JAVA_INT, ADDRESS, JAVA_LONG))
  val setMailboxClass: MethodHandle = h("agx_set_mailbox_class", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT))
  val setMailbox: MethodHandle =
    h("agx_set_mailbox", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, JAVA_LONG, JAVA_INT))
  val setBehaviors: MethodHandle = h(
    "agx_set_behaviors",
    FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT))
  val setOutbound: MethodHandle =
    h("agx_set_outbound", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_LONG))
  val takeOutbound: MethodHandle =
    h("agx_take_outbound", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS))
  val stageTells: MethodHandle =
    h("agx_stage_tells", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG))
  val tell: MethodHandle = h("agx_tell", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS))
  val pumpIdle: MethodHandle = h("agx_pump_idle", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS))
  val pumpCancel: MethodHandle = h("agx_pump_cancel", FunctionDescriptor.of(JAVA_INT, ADDRESS))
  val run: MethodHandle = h("agx_run", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS))
  val getStats: MethodHandle = h("agx_get_stats", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS))
  val readState: MethodHandle =
    h("agx_read_state", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, JAVA_LONG, ADDRESS, ADDRESS))
  val getShape: MethodHandle = h("agx_get_shape", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS))
  val shardId: MethodHandle = h("agx_shard_id", FunctionDescriptor.of(JAVA_INT, JAVA_INT, JAVA_INT))

  /** status -> exception (errors never cross the C ABI as exceptions; the message is agx_last_error) */
  def check(status: Int): Unit =
    if (status != 0) {
      val msg = lastError.invokeExact().asInstanceOf[MemorySegment].reinterpret(4096).getString(0)
      status match {
        case 1 => throw new ConfigurationException(s"akka-gpu: $msg")
        case 5 => throw new IllegalStateException(s"akka-gpu: mailbox arena full: $msg")
        case s => throw new IllegalStateException(s"akka-gpu status $s: $msg")
      }
    }
}

/** AgxBackend over java.lang.foreign: the engine handle is the native address as a long. */
object PanamaBackend extends AgxBackend {
  import AgxNative._
  private def seg(engine: Long): MemorySegment = MemorySegment.ofAddress(engine)
  private def ints(a: Arena, x: Array[Int], n: Int): MemorySegment =
    if (x == null) MemorySegment.NULL else a.allocateFrom(JAVA_INT, java.util.Arrays.copyOf(x, n): _*)

  def abiVersion: Int = AgxNative.abiVersion.invokeExact().asInstanceOf[Int]

  def create(device: Int, nActors: Long, throughput: Int, capacity: Int, nWords: Int, maxEmit: Int, nRanks: Int,
             rank: Int, numShards: Int, bucketActors: Int, msgCapacity: Long): Long = {
    val a = Arena.ofConfined()
    try {
      val cfg = a.allocate(Cfg)
      cfg.set(JAVA_INT, 0, Agx.AbiVersion)
      cfg.set(JAVA_INT, 4, device)
      cfg.set(JAVA_LONG, 8, nActors)
      cfg.set(JAVA_INT, 16, math.max(throughput, 0)) // <= 0 behaves as 1 (Mailbox.scala:261)
      cfg.set(JAVA_INT, 20, capacity)
      cfg.set(JAVA_INT, 24, nWords)
      cfg.set(JAVA_INT, 28, maxEmit)
      cfg.set(JAVA_INT, 32, nRanks)
      cfg.set(JAVA_INT, 36, rank)
      cfg.set(JAVA_INT, 40, numShards)
      cfg.set(JAVA_INT, 44, bucketActors)
      cfg.set(JAVA_LONG, 48, msgCapacity)
      val out = a.allocate(ADDRESS)
      check(AgxNative.create.invokeExact(cfg, out).asInstanceOf[Int])
      out.get(ADDRESS, 0).address()
    } finally a.close()
  }
  def destroy(engine: Long): Unit = check(AgxNative.destroy.invokeExact(seg(engine)).asInstanceOf[Int])
  def registerRange(engine: Long, first: Long, count: Long, kind: Int, init: Array[Long], stateWords: Int): Unit = {
    val a = Arena.ofConfined()
    try {
      val st = if (init == null) MemorySegment.NULL else a.allocateFrom(JAVA_LONG, init: _*)
      val stride = if (init == null) 0L else stateWords.toLong * 8
      check(AgxNative.registerRange.invokeExact(seg(engine), first, count, kind, st, stride).asInstanceOf[Int])
    } finally a.close()
  }
  def setMailboxClass(engine: Long, mailboxClass: Int, capacity: Int): Unit =
    check(AgxNative.setMailboxClass.invokeExact(seg(engine), mailboxClass, capacity).asInstanceOf[Int])
  def setMailbox(engine: Long, first: Long, count: Long, mailboxClass: Int): Unit =
    check(AgxNative.setMailbox.invokeExact(seg(engine), first, count, mailboxClass).asInstanceOf[Int])
  def setBehaviors(engine: Long, t: GpuBehaviors.Tables): Unit = {
    val a = Arena.ofConfined()
    try {
      val cs = a.allocateFrom(JAVA_BYTE, t.cases: _*)
      val as = a.allocateFrom(JAVA_BYTE, t.acts: _*)
      val fs = a.allocateFrom(JAVA_INT, t.first: _*)
      check(AgxNative.setBehaviors.invokeExact(seg(engine), cs, t.nCases, as, t.nActs, fs, t.behaviors.size)
        .asInstanceOf[Int])
    } finally a.close()
  }
  def setOutbound(engine: Long, firstHostId: Int, nHost: Int, capacity: Long): Unit =
    check(AgxNative.setOutbound.invokeExact(seg(engine), firstHostId, nHost, capacity).asInstanceOf[Int])
  def takeOutbound(engine: Long, dst: Array[Int], src: Array[Int], payload: Array[Int], cap: Int): Int = {
    val a = Arena.ofConfined()
    try {
      val d = a.allocate(JAVA_INT, math.max(cap, 1).toLong)
      val s = a.allocate(JAVA_INT, math.max(cap, 1).toLong)
      val p = a.allocate(JAVA_INT, math.max(cap, 1).toLong)
      val n = a.allocate(JAVA_LONG)
      check(AgxNative.takeOutbound.invokeExact(seg(engine), d, s, p, cap.toLong, n).asInstanceOf[Int])
      val k = n.get(JAVA_LONG, 0).toInt
      MemorySegment.copy(d, JAVA_INT, 0, dst, 0, k)
      MemorySegment.copy(s, JAVA_INT, 0, src, 0, k)
      MemorySegment.copy(p, JAVA_INT, 0, payload, 0, k)
      k
    } finally a.close()
  }
  def stageTells(engine: Long, dst: Array[Int], src: Array[Int], payload: Array[Int], n: Int): Unit = {
    val a = Arena.ofConfined()
    try check(AgxNative.stageTells.invokeExact(seg(engine), ints(a, dst, n), ints(a, src, n), ints(a, payload, n),
      n.toLong).asInstanceOf[Int])
    finally a.close()
  }
  // (one 4-byte out-parameter per call: a thread's own reusable slot, no Arena per tell)
  private val flag = ThreadLocal.withInitial[MemorySegment](() => Arena.global().allocate(JAVA_INT))
  def tell(engine: Long, dst: Int, src: Int, payload: Int): Boolean = {
    val f = flag.get()
    check(AgxNative.tell.invokeExact(seg(engine), dst, src, payload, f).asInstanceOf[Int])
    f.get(JAVA_INT, 0) != 0
  }
  def pumpIdle(engine: Long): Boolean = {
    val f = flag.get()
    check(AgxNative.pumpIdle.invokeExact(seg(engine), f).asInstanceOf[Int])
    f.get(JAVA_INT, 0) != 0
  }
  def pumpCancel(engine: Long): Unit = check(AgxNative.pumpCancel.invokeExact(seg(engine)).asInstanceOf[Int])
  def run(engine: Long, maxSupersteps: Int, stats: Array[Long]): Unit = {
    val a = Arena.ofConfined()
    try {
      val st = if (stats == null) MemorySegment.NULL else a.allocate(Stats)
      check(AgxNative.run.invokeExact(seg(engine), maxSupersteps, st).asInstanceOf[Int])
      if (stats != null) MemorySegment.copy(st, JAVA_LONG, 0, stats, 0, math.min(8, stats.length))
    } finally a.close()
  }
  def getStats(engine: Long, stats: Array[Long]): Unit = {
    val a = Arena.ofConfined()
    try {
      val st = a.allocate(Stats)
      check(AgxNative.getStats.invokeExact(seg(engine), st).asInstanceOf[Int])
      MemorySegment.copy(st, JAVA_LONG, 0, stats, 0, math.min(8, stats.length))
    } finally a.close()
  }
  def readState(engine: Long, first: Long, count: Long, words: Array[Long], alive: Array[Byte]): Unit = {
    val a = Arena.ofConfined()
    try {
      // agx_read_state writes count x n_words u64 and count bytes: the arrays must hold exactly that
      val shape = a.allocate(JAVA_INT)
      check(AgxNative.getShape.invokeExact(seg(engine), MemorySegment.NULL, shape).asInstanceOf[Int])
      val nWords = shape.get(JAVA_INT, 0).toLong
      if (count < 0 || (words != null && words.length.toLong != count * nWords) ||
          (alive != null && alive.length.toLong < count))
        throw new ConfigurationException(
          s"akka-gpu: readState needs words.length == count * $nWords and alive.length >= count")
      val w = if (words == null) MemorySegment.NULL else a.allocate(JAVA_LONG, math.max(words.length, 1).toLong)
      val al = if (alive == null) MemorySegment.NULL else a.allocate(JAVA_BYTE, math.max(alive.length, 1).toLong)
      check(AgxNative.readState.invokeExact(seg(engine), first, count, w, al).asInstanceOf[Int])
      if (words != null) MemorySegment.copy(w, JAVA_LONG, 0, words, 0, words.length)
      if (alive != null) MemorySegment.copy(al, JAVA_BYTE, 0, alive, 0, alive.length)
    } finally a.close()
  }
  def shardId(id: Int, numShards: Int): Int = AgxNative.shardId.invokeExact(id, numShards).asInstanceOf[Int]
}
