/*
 * The Scala face of the behaviour-table compiler (the reference implementation of the lowering,
 * with its tests, is akka_amd/typed.py; both emit include/akka_gpu.h agx_case / agx_act tables).
 *
 * A typed Behaviors.receiveMessage / javadsl ReceiveBuilder subset
 * (akka-actor-typed/src/main/scala/akka/actor/typed/scaladsl/Behaviors.scala:101-121,
 *  akka-actor-typed/src/main/scala/akka/actor/typed/javadsl/ReceiveBuilder.scala:48-98,209-218)
 * written against symbolic messages and two u64 state fields:
 *
 *   val st = GpuBehaviors.State("count", "sum")
 *   val counter = GpuBehaviors.receiveBuilder(st)
 *     .onAnyMessage((m, s) => Seq(s("count").inc(), s("sum").add(m.payload)), GpuBehaviors.Same)
 *     .build("counter")
 *   val tables = GpuBehaviors.compile(Seq(counter))         // -> agx_set_behaviors
 *   engine.registerRange(0, n, tables.kindOf(counter))
 *
 * Not compiled in the build image (no JVM, SURVEY.md §8(c)); JDK 8+ (no java.lang.foreign).
 */
package akka.dispatch.gpu

import java.nio.{ ByteBuffer, ByteOrder }

import scala.collection.mutable

object GpuBehaviors {
  // operand sources / comparisons / actions / results (include/akka_gpu.h)
  final val VConst = 0; final val VPayload = 1; final val VTag = 2; final val VArg = 3
  final val VWord = 4; final val VSender = 5; final val VSelf = 6
  final val CmpAny = 0; final val CmpEq = 1; final val CmpNe = 2; final val CmpLt = 3
  final val CmpLe = 4; final val CmpGt = 5; final val CmpGe = 6
  final val ASet = 1; final val AAdd = 2; final val AMax = 3; final val AMin = 4; final val ATell = 5

  final case class Operand(src: Int, word: Int = 0, k: Long = 0) {
    def +(c: Long): Operand = copy(k = k + c)
    def -(c: Long): Operand = copy(k = k - c)
    def ===(o: Operand): Test = Test(CmpEq, this, o)
    def =!=(o: Operand): Test = Test(CmpNe, this, o)
    def <(o: Operand): Test = Test(CmpLt, this, o)
    def <=(o: Operand): Test = Test(CmpLe, this, o)
    def >(o: Operand): Test = Test(CmpGt, this, o)
    def >=(o: Operand): Test = Test(CmpGe, this, o)
  }
  implicit def const(v: Long): Operand = Operand(VConst, 0, v)

  final case class Test(cmp: Int, lhs: Operand, rhs: Operand)
  val Always: Test = Test(CmpAny, Operand(VConst), Operand(VConst))

  final case class Action(op: Int, word: Int, v: Operand, dst: Operand = Operand(VConst), orMask: Int = 0)

  final class Field(val word: Int) {
    def value: Operand = Operand(VWord, word)
    def set(v: Operand): Action = Action(ASet, word, v)
    def add(v: Operand): Action = Action(AAdd, word, v)
    def inc(n: Long = 1): Action = add(n)
    def max(v: Operand): Action = Action(AMax, word, v)
    def min(v: Operand): Action = Action(AMin, word, v)
  }
  final case class Ref(dst: Operand) {
    /** ActorRef.! (akka-actor/src/main/scala/akka/actor/ActorRef.scala:412-413) */
    def !(payload: Operand): Action = Action(ATell, 0, payload, dst)
    def tell(m: MessageType, arg: Operand): Action = Action(ATell, 0, arg, dst, m.tag << 24)
  }
  def selfRef(offset: Long = 0): Ref = Ref(Operand(VSelf, 0, offset))
  def actorRef(id: Long): Ref = Ref(Operand(VConst, 0, id))

  final case class MessageType(name: String, tag: Int) { require(tag >= 0 && tag <= 0xFF) }

  object Msg {
    val payload: Operand = Operand(VPayload)
    val tag: Operand = Operand(VTag)
    val arg: Operand = Operand(VArg)
    val sender: Ref = Ref(Operand(VSender))
  }

  final class State(names: String*) {
    require(names.size <= 2, "compiled behaviours hold at most two u64 state fields")
    private val fields = names.zipWithIndex.map { case (n, i) => n -> new Field(i) }.toMap
    def apply(name: String): Field = fields(name)
  }
  object State { def apply(names: String*): State = new State(names: _*) }

  sealed trait Next
  case object Same extends Next
  case object Stopped extends Next
  case object Unhandled extends Next
  final class Behavior(val name: String, val state: State) extends Next {
    private[gpu] var cases: Vector[Case] = Vector.empty
  }
  final case class Case(tests: Seq[Test], actions: Seq[Action], next: Next)

  /** javadsl ReceiveBuilder: handlers tried in the order added; none matching = Behaviors.unhandled */
  final class Builder(state: State) {
    private val cases = mutable.ArrayBuffer.empty[Case]
    private def add(tests: Seq[Test], actions: Seq[Action], next: Next): Builder = {
      require(tests.size <= 2, "a handler has at most two tests (message type / predicate / state guard)")
      cases += Case(tests, actions, next); this
    }
    def onMessage(t: MessageType, handler: (Msg.type, State) => Seq[Action], next: Next,
                  test: Option[Test] = None, when: Option[Test] = None): Builder =
      add(Seq(Msg.tag === t.tag.toLong) ++ test ++ when, handler(Msg, state), next)
    def onMessageEquals(payload: Long, handler: (Msg.type, State) => Seq[Action], next: Next): Builder =
      add(Seq(Msg.payload === payload), handler(Msg, state), next)
    def onAnyMessage(handler: (Msg.type, State) => Seq[Action], next: Next, test: Option[Test] = None,
                     when: Option[Test] = None): Builder =
      add(test.toSeq ++ when, handler(Msg, state), next)
    def build(name: String): Behavior = buildInto(new Behavior(name, state))
    def buildInto(b: Behavior): Behavior = { b.cases = cases.toVector; b }
  }
  def receiveBuilder(state: State): Builder = new Builder(state)

  /** The lowered tables (agx_set_behaviors arguments): agx_case (48 B) and agx_act (32 B) entries
   *  as little-endian bytes, and first[] -- handed to either binding (AgxBackend.setBehaviors). */
  final class Tables(val behaviors: Vector[Behavior], val cases: Array[Byte], val nCases: Int,
                     val acts: Array[Byte], val nActs: Int, val first: Array[Int]) {
    def kindOf(b: Behavior): Int = Agx.KindCompiled + behaviors.indexWhere(_ eq b)
    /** the most tells one message can emit: the dispatcher's gpu.max-emit must be at least this */
    def maxTells: Int = {
      var m = 0
      var c = 0
      while (c < nCases) {
        val first = (cases(48 * c + 12) & 0xFF) | ((cases(48 * c + 13) & 0xFF) << 8)
        val cnt = (cases(48 * c + 14) & 0xFF) | ((cases(48 * c + 15) & 0xFF) << 8)
        m = math.max(m, (first until first + cnt).count(i => acts(32 * i) == ATell))
        c += 1
      }
      m
    }
  }

  def compile(roots: Seq[Behavior]): Tables = {
    val order = mutable.ArrayBuffer.empty[Behavior]
    val todo = mutable.Queue(roots: _*)
    while (todo.nonEmpty) {
      val b = todo.dequeue()
      if (!order.exists(_ eq b)) {
        order += b
        b.cases.foreach { c => c.next match { case nb: Behavior => todo.enqueue(nb); case _ => } }
      }
    }
    val index = order.zipWithIndex.map { case (b, i) => (b: AnyRef) -> i }.toMap
    val allCases = order.flatMap(_.cases)
    val nActs = allCases.map(_.actions.size).sum
    val cs = ByteBuffer.allocate(48 * math.max(allCases.size, 1)).order(ByteOrder.LITTLE_ENDIAN)
    val as = ByteBuffer.allocate(32 * math.max(nActs, 1)).order(ByteOrder.LITTLE_ENDIAN)
    val first = new Array[Int](order.size + 1)
    var ci = 0; var ai = 0
    order.zipWithIndex.foreach { case (b, bi) =>
      b.cases.foreach { c =>
        val t = c.tests ++ Seq.fill(2 - c.tests.size)(Always)
        val base = ci * 48
        val bytes = Array(t(0).lhs.src, t(0).lhs.word, t(0).cmp, t(0).rhs.src, t(0).rhs.word, t(1).lhs.src,
                          t(1).lhs.word, t(1).cmp, t(1).rhs.src, t(1).rhs.word,
                          c.next match { case Same => 0; case Stopped => 1; case Unhandled => 2; case _ => 3 },
                          c.next match { case nb: Behavior => index(nb); case _ => 0 })
        bytes.zipWithIndex.foreach { case (v, i) => cs.put(base + i, v.toByte) }
        cs.putShort(base + 12, ai.toShort)
        cs.putShort(base + 14, c.actions.size.toShort)
        Seq(t(0).lhs.k, t(0).rhs.k, t(1).lhs.k, t(1).rhs.k).zipWithIndex.foreach { case (k, i) =>
          cs.putLong(base + 16 + 8 * i, k)
        }
        c.actions.foreach { a =>
          val ab = ai * 32
          Array(a.op, a.word, a.v.src, a.v.word, a.dst.src, a.dst.word, 0, 0).zipWithIndex.foreach { case (v, i) =>
            as.put(ab + i, v.toByte)
          }
          as.putInt(ab + 8, a.orMask)
          as.putLong(ab + 16, a.v.k)
          as.putLong(ab + 24, a.dst.k)
          ai += 1
        }
        ci += 1
      }
      first(bi + 1) = ci
    }
    new Tables(order.toVector, cs.array(), ci, as.array(), ai, first)
  }
}
