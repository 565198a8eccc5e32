/*
 * Panama (java.lang.foreign, JDK 22+) downcalls into include/akka_gpu.h.  No native glue:
 * every handle binds one `extern "C"` symbol of libakka_gpu.so with the C signature from the
 * header.  Not compiled in the build image (no JVM, SURVEY.md §8(c)); tests/c/abi_sequence.c
 * drives the same calls in the same order from C and runs on the GPU box.
 */
package akka.dispatch.gpu

import java.lang.foreign._
import java.lang.foreign.ValueLayout._
import java.lang.invoke.MethodHandle

import akka.ConfigurationException

object AgxNative {
  final val AbiVersion = 1
  final val NoSender = 0xFFFFFFFF // AGX_NO_SENDER (deadLetters as sender)

  // enum agx_behavior_kind
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

  // agx_status
  final val Ok = 0
  final val EInval = 1
  final val ECapacity = 5

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

  /** struct agx_stats: 8 x u64 (delivered, dead_letters, unhandled, emitted, staged, supersteps,
   *  in_flight, bytes_alg) */
  val Stats: SequenceLayout = MemoryLayout.sequenceLayout(8, JAVA_LONG)

  val create: MethodHandle = h("agx_create", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS))
  val destroy: MethodHandle = h("agx_destroy", FunctionDescriptor.of(JAVA_INT, ADDRESS))
  val lastError: MethodHandle = h("agx_last_error", FunctionDescriptor.of(ADDRESS))
  val registerRange: MethodHandle =
    h("agx_register_range", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, JAVA_LONG, JAVA_INT, ADDRESS, JAVA_LONG))
  val setRing: MethodHandle = h("agx_set_ring", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT))
  val setGossip: MethodHandle = h("agx_set_gossip", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_LONG))
  val setDeltaCrdt: MethodHandle = h("agx_set_delta_crdt", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT))
  val setBehaviors: MethodHandle = h(
    "agx_set_behaviors",
    FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT))

  /** struct agx_case (48 B): 12 x u8 (src1, word1, cmp1, src2, word2, src3, word3, cmp2, src4, word4,
   *  result, next), u16 act_first, u16 act_count, 4 x i64 (k1..k4) */
  val Case: StructLayout = MemoryLayout.structLayout(
    MemoryLayout.sequenceLayout(12, JAVA_BYTE).withName("bytes"),
    JAVA_SHORT.withName("act_first"),
    JAVA_SHORT.withName("act_count"),
    MemoryLayout.sequenceLayout(4, JAVA_LONG).withName("k"))

  /** struct agx_act (32 B): u8 op, word, src, sword, dsrc, dword, pad, pad; u32 or_mask; i64 k, dk */
  val Act: StructLayout = MemoryLayout.structLayout(
    MemoryLayout.sequenceLayout(8, JAVA_BYTE).withName("bytes"),
    JAVA_INT.withName("or_mask"),
    MemoryLayout.paddingLayout(4),
    JAVA_LONG.withName("k"),
    JAVA_LONG.withName("dk"))
  val stageTells: MethodHandle =
    h("agx_stage_tells", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG))
  val run: MethodHandle = h("agx_run", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS))
  val getStats: MethodHandle = h("agx_get_stats", FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS))
  val readState: MethodHandle =
    h("agx_read_state", FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, JAVA_LONG, ADDRESS, ADDRESS))
  val shardId: MethodHandle = h("agx_shard_id", FunctionDescriptor.of(JAVA_INT, JAVA_INT, JAVA_INT))

  /** status -> exception (errors never cross the C ABI as exceptions; the message is agx_last_error) */
  def check(status: Int): Unit =
    if (status != Ok) {
      val msg = lastError.invokeExact().asInstanceOf[MemorySegment].reinterpret(4096).getString(0)
      status match {
        case EInval    => throw new ConfigurationException(s"akka-gpu: $msg")
        case ECapacity => throw new IllegalStateException(s"akka-gpu: mailbox arena full: $msg")
        case other     => throw new IllegalStateException(s"akka-gpu status $other: $msg")
      }
    }
}
