/*
 * mailbox-type = "akka.dispatch.gpu.GpuMailboxType": Mailboxes.lookupConfigurator instantiates
 * it reflectively with the (ActorSystem.Settings, Config) constructor (akka-actor/src/main/
 * scala/akka/dispatch/Mailboxes.scala:222-236); MailboxType.create (Mailbox.scala:638-640)
 * registers the owner as one fixed-layout actor of the dispatcher's engine, bound to the engine
 * mailbox class of this mailbox type's capacity -- so bounded and unbounded GPU mailboxes coexist
 * on one dispatcher, each actor with its own (Mailboxes.scala:204-260, ActorMailboxSpec.scala:245-450).
 *
 * Two mailbox types, like the reference's UnboundedMailbox / BoundedMailbox (Mailbox.scala:647-720):
 * GpuMailboxType (ProducesMessageQueue[GpuMessageQueue], UnboundedMessageQueueSemantics) and
 * GpuBoundedMailboxType (ProducesMessageQueue[GpuBoundedMessageQueue], BoundedMessageQueueSemantics,
 * mailbox-capacity > 0) -- Mailboxes.getMailboxType checks an actor's RequiresMessageQueue against
 * the type's marker (Mailboxes.scala:122-135,164-175), so an actor that requires bounded semantics
 * must be given the bounded type.  A GpuMailboxType with mailbox-capacity > 0 still tail-drops at
 * that capacity and its queues are GpuBoundedMessageQueue at run time.
 */
package akka.dispatch.gpu

import java.util.concurrent.atomic.AtomicInteger


import com.typesafe.config.Config

import scala.concurrent.duration.Duration

import akka.actor.{ ActorRef, ActorSystem, DeadLetter }
import akka.dispatch._

/** The fixed-layout message of a GPU actor: one u32 payload word (the sender travels in the Envelope). */
final case class GpuTell(payload: Int)

abstract class GpuMailboxTypeBase(settings: ActorSystem.Settings, config: Config) extends MailboxType {

  private val dispatcherId = config.getString("gpu.dispatcher")
  private val kind: Int = config.getString("gpu.behavior") match {
    case "counter"    => Agx.KindCounter
    case "ring"       => Agx.KindRing
    case "fanout"     => Agx.KindFanout
    case "forward-rr" => Agx.KindForwardRR
    case "stop-after" => Agx.KindStopAfter
    case "ping-pong"  => Agx.KindPingPong
    case "even"       => Agx.KindEven
    case "gcounter"   => Agx.KindGCounter
    case "pncounter"  => Agx.KindPNCounter
    case "orset"      => Agx.KindORSet
    case other        => throw new akka.ConfigurationException(s"Unknown GPU behavior [$other] in mailbox config")
  }

  /** BoundedMailbox's keys (Mailbox.scala:699-720): mailbox-capacity, mailbox-push-timeout-time.
   *  The GPU mailbox tail-drops at capacity (pushTimeOut 0, AbstractBoundedNodeQueue.java:92-113);
   *  a positive push timeout would block the sender, which a superstep cannot do. */
  protected val capacity: Int = if (config.hasPath("mailbox-capacity")) config.getInt("mailbox-capacity") else 0
  if (capacity < 0) throw new IllegalArgumentException("The capacity for GpuMailboxType can not be negative")
  if (capacity > 0 && config.hasPath("mailbox-push-timeout-time") &&
      config.getDuration("mailbox-push-timeout-time").toNanos != 0L)
    throw new akka.ConfigurationException(
      "GpuMailboxType is a non-blocking bounded mailbox: mailbox-push-timeout-time must be 0")

  override def create(owner: Option[ActorRef], system: Option[ActorSystem]): MessageQueue = {
    val engine = GpuEngine.forDispatcher(dispatcherId)
    val id = owner match {
      case Some(ref) => engine.register(ref, kind, Array.fill(engine.stateWords)(0L), capacity)
      case None      => Agx.NoSender // the dummy queue of a top-level actor under construction
    }
    val q: GpuQueue =
      if (capacity > 0) new GpuBoundedMessageQueue(id, engine, system, capacity)
      else new GpuMessageQueue(id, engine, system)
    q
  }
}

/** mailbox-type = "akka.dispatch.gpu.GpuMailboxType": unbounded semantics (UnboundedMailbox). */
class GpuMailboxType(settings: ActorSystem.Settings, config: Config)
    extends GpuMailboxTypeBase(settings, config)
    with ProducesMessageQueue[GpuMessageQueue]

/** mailbox-type = "akka.dispatch.gpu.GpuBoundedMailboxType": BoundedMailbox(mailbox-capacity, 0)
 *  semantics (Mailbox.scala:699-720), tail-drop to dead letters at the capacity. */
class GpuBoundedMailboxType(settings: ActorSystem.Settings, config: Config)
    extends GpuMailboxTypeBase(settings, config)
    with ProducesMessageQueue[GpuBoundedMessageQueue] {
  if (capacity <= 0)
    throw new IllegalArgumentException("The capacity for GpuBoundedMailboxType must be positive (mailbox-capacity)")
}

/** The device-side mailbox of one actor.  enqueue hands the tell to the engine through the
 *  lock-free tell path (GpuEngine.tell -> agx_tell: the calling thread's own queue, no lock;
 *  AbstractNodeQueue.java:79-82) and submits the dispatcher's pump only when the engine went from
 *  idle to scheduled (Mailbox.setAsScheduled, Mailbox.scala:185-194).  Nothing is ever dequeued on
 *  the JVM (MessageQueue contract, Mailbox.scala:359-390): the messages live in the engine, in its
 *  in-flight count (GpuEngine.stats()(6)), so numberOfMessages is 0 on the JVM side. */
sealed abstract class GpuQueue(val id: Int, engine: GpuEngine, system: Option[ActorSystem]) extends MessageQueue {

  def enqueue(receiver: ActorRef, handle: Envelope): Unit = {
    val payload = handle.message match {
      case GpuTell(p) => p
      case i: Int     => i
      case other =>
        // not in the fixed-layout protocol: deadLetters, like a tell the actor cannot accept
        system.foreach(_.deadLetters ! DeadLetter(other, handle.sender, receiver))
        return
    }
    engine.tell(id, engine.idOf(handle.sender), payload)
  }

  def dequeue(): Envelope = null
  def numberOfMessages: Int = 0
  def hasMessages: Boolean = false
  def cleanUp(owner: ActorRef, deadLetters: MessageQueue): Unit = () // the engine dead-letters them
}

/** A GPU actor's unbounded mailbox. */
final class GpuMessageQueue(id: Int, engine: GpuEngine, system: Option[ActorSystem])
    extends GpuQueue(id, engine, system)
    with UnboundedMessageQueueSemantics

/** A GPU actor's bounded mailbox: admission `p < capacity` on the device, the rest dead letters;
 *  never blocks a sender (pushTimeOut 0, AbstractBoundedNodeQueue.java:92-113). */
final class GpuBoundedMessageQueue(id: Int, engine: GpuEngine, system: Option[ActorSystem], val capacity: Int)
    extends GpuQueue(id, engine, system)
    with BoundedMessageQueueSemantics {
  def pushTimeOut: Duration = Duration.Zero
}
