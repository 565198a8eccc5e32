/*
 * mailbox-type = "akka.dispatch.gpu.GpuMailboxType": Mailboxes.lookupConfigurator instantiates
 * it reflectively with the (ActorSystem.Settings, Config) constructor (akka-actor/src/main/
 * scala/akka/dispatch/Mailboxes.scala:222-236); MailboxType.create (Mailbox.scala:638-640)
 * registers the owner as one fixed-layout actor of the dispatcher's engine.
 */
package akka.dispatch.gpu

import com.typesafe.config.Config

import akka.actor.{ ActorRef, ActorSystem, DeadLetter }
import akka.dispatch._

/** The fixed-layout message of a GPU actor: one u32 payload word (the sender travels in the Envelope). */
final case class GpuTell(payload: Int)

class GpuMailboxType(settings: ActorSystem.Settings, config: Config)
    extends MailboxType
    with ProducesMessageQueue[GpuMessageQueue] {

  private val dispatcherId = config.getString("gpu.dispatcher")
  private val kind: Int = config.getString("gpu.behavior") match {
    case "counter"    => AgxNative.KindCounter
    case "ring"       => AgxNative.KindRing
    case "fanout"     => AgxNative.KindFanout
    case "forward-rr" => AgxNative.KindForwardRR
    case "stop-after" => AgxNative.KindStopAfter
    case "ping-pong"  => AgxNative.KindPingPong
    case "even"       => AgxNative.KindEven
    case "gcounter"   => AgxNative.KindGCounter
    case "pncounter"  => AgxNative.KindPNCounter
    case "orset"      => AgxNative.KindORSet
    case other        => throw new akka.ConfigurationException(s"Unknown GPU behavior [$other] in mailbox config")
  }

  override def create(owner: Option[ActorRef], system: Option[ActorSystem]): MessageQueue = {
    val engine = GpuEngine.forDispatcher(dispatcherId)
    val id = owner match {
      case Some(ref) => engine.register(ref, kind, Array.fill(config.getInt("gpu.state-words"))(0L))
      case None      => AgxNative.NoSender // the dummy queue of a top-level actor under construction
    }
    new GpuMessageQueue(id, engine, system)
  }
}

/** The device-side mailbox of one actor.  enqueue stages the tell for the engine; nothing is
 *  ever dequeued on the JVM (MessageQueue contract, Mailbox.scala:359-390). */
final class GpuMessageQueue(val id: Int, engine: GpuEngine, system: Option[ActorSystem])
    extends MessageQueue
    with UnboundedMessageQueueSemantics {

  def enqueue(receiver: ActorRef, handle: Envelope): Unit = {
    val payload = handle.message match {
      case GpuTell(p) => p
      case i: Int     => i
      case other =>
        // not in the fixed-layout protocol: deadLetters, like a tell the actor cannot accept
        system.foreach(_.deadLetters ! DeadLetter(other, handle.sender, receiver))
        return
    }
    engine.stage(id, engine.idOf(handle.sender), payload)
  }

  def dequeue(): Envelope = null
  def numberOfMessages: Int = 0 // messages live on the device (agx_get_stats in_flight)
  def hasMessages: Boolean = false
  def cleanUp(owner: ActorRef, deadLetters: MessageQueue): Unit = () // the engine dead-letters them
}
