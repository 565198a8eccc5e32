/*
 * The drop-in: a MessageDispatcher whose actors' mailboxes live on the GPU.
 *
 *   gpu-dispatcher { type = "akka.dispatch.gpu.GpuDispatcherConfigurator", ... }
 *
 * Dispatchers.configuratorFrom instantiates GpuDispatcherConfigurator reflectively with the
 * (Config, DispatcherPrerequisites) constructor (akka-actor/src/main/scala/akka/dispatch/
 * Dispatchers.scala:235-262).  The dispatcher extends the reference's Dispatcher (constructor
 * Dispatcher.scala:32-38) so JVM actors bound to it still run on its executor; for actors whose
 * mailbox was created by GpuMailboxType:
 *   - dispatch (Dispatcher.scala:61-65): ActorRef.! -> ActorCell.sendMessage -> dispatch appends
 *     (dst id, sender id, payload) to the engine's staging buffer instead of a JVM queue, and
 *     schedules the pump instead of the mailbox;
 *   - registerForExecution (Dispatcher.scala:120-143): the pump task (agx_run) is what gets
 *     executed on the executor service; a GPU mailbox itself is only scheduled for system
 *     messages (Create / Terminate stay on the JVM ActorCell);
 *   - createMailbox (Dispatcher.scala:97-99) is inherited: mailboxType.create gives the
 *     GpuMessageQueue;
 *   - shutdown (AbstractDispatcher.scala:325) destroys the engine.
 */
package akka.dispatch.gpu

import java.util.concurrent.RejectedExecutionException

import scala.concurrent.duration.{ Duration, FiniteDuration }

import com.typesafe.config.Config

import akka.actor.ActorCell
import akka.dispatch._
import akka.event.Logging.Error
import akka.util.Helpers.ConfigOps

class GpuDispatcherConfigurator(config: Config, prerequisites: DispatcherPrerequisites)
    extends MessageDispatcherConfigurator(config, prerequisites) {

  private val instance = new GpuDispatcher(
    this,
    config.getString("id"),
    config.getInt("throughput"),
    config.getNanosDuration("throughput-deadline-time"),
    configureExecutor(),
    config.getMillisDuration("shutdown-timeout"),
    config)

  /** Returns the same dispatcher instance for each invocation (as DispatcherConfigurator) */
  override def dispatcher(): MessageDispatcher = instance
}

// (constructor parameters are prefixed: Dispatcher already declares `val id`, `val throughput`, ...)
class GpuDispatcher(
    _configurator: MessageDispatcherConfigurator,
    _id: String,
    _throughput: Int,
    _throughputDeadlineTime: Duration,
    _executorServiceFactoryProvider: ExecutorServiceFactoryProvider,
    _shutdownTimeout: FiniteDuration,
    config: Config)
    extends Dispatcher(
      _configurator,
      _id,
      _throughput,
      _throughputDeadlineTime,
      _executorServiceFactoryProvider,
      _shutdownTimeout) {

  val engine = new GpuEngine(id, config, throughput)
  GpuEngine.register(engine)

  private val maxSupersteps: Int =
    if (config.hasPath("gpu.supersteps-per-pump")) config.getInt("gpu.supersteps-per-pump") else Int.MaxValue

  // One pump task at a time: agx_tell answers "submit" only on idle -> scheduled, and the pump's
  // last call (agx_pump_idle) answers "submit again" only for tells that arrived while it ran --
  // Mailbox.run's finally { setAsIdle(); registerForExecution } (Mailbox.scala:227-240).
  private val pumpTask: Runnable = new Runnable {
    def run(): Unit = {
      val again =
        try engine.pump(maxSupersteps)
        catch {
          case e: Throwable =>
            eventStream.publish(Error(e, getClass.getName, getClass, "GPU pump failed"))
            engine.pumpIdleAfterFailure()
        }
      if (again) schedulePump()
    }
  }
  engine.setPumpSubmitter(() => schedulePump())

  private def schedulePump(): Unit =
    try executorService.execute(pumpTask)
    catch {
      case _: RejectedExecutionException =>
        try executorService.execute(pumpTask) // retry once, as registerForExecution does
        catch {
          case e: RejectedExecutionException =>
            // back to idle before rethrowing (Dispatcher.registerForExecution: mbox.setAsIdle(); throw,
            // Dispatcher.scala:130-138): agx_tell CASed idle -> scheduled for this submission, and a
            // status left at "scheduled" would make every later tell answer "do not submit" -- the GPU
            // actors would stall for good.  The next tell schedules the pump again.
            engine.pumpCancel()
            eventStream.publish(Error(e, getClass.getName, getClass, "GPU pump was rejected twice!"))
            throw e
        }
    }

  /** ActorRef.! for every actor bound to this dispatcher (Dispatcher.scala:61-65). */
  override protected[akka] def dispatch(receiver: ActorCell, invocation: Envelope): Unit =
    receiver.mailbox.messageQueue match {
      case q: GpuQueue =>
        q.enqueue(receiver.self, invocation) // -> agx_tell; submits the pump on idle -> scheduled
      case _ =>
        super.dispatch(receiver, invocation) // a JVM actor on this dispatcher
    }

  /** A GPU mailbox holds no JVM messages: it is scheduled only for system messages. */
  override protected[akka] def registerForExecution(
      mbox: Mailbox,
      hasMessageHint: Boolean,
      hasSystemMessageHint: Boolean): Boolean =
    mbox.messageQueue match {
      case _: GpuQueue if !hasSystemMessageHint && !mbox.hasSystemMessages => false
      case _                                                                       => super.registerForExecution(mbox, hasMessageHint, hasSystemMessageHint)
    }

  /** Large populations: `count` fixed-layout actors without a JVM ActorCell each; returns the
   *  first id (tell to them with tellRange / GpuRef). */
  def spawnRange(kind: Int, count: Int, mailboxCapacity: Int = defaultCapacity): Int =
    engine.registerRange(count, kind, mailboxCapacity)

  private def defaultCapacity: Int = if (config.hasPath("gpu.mailbox-capacity")) config.getInt("gpu.mailbox-capacity") else 0

  def tellRange(first: Int, count: Int, payload: Int): Unit = {
    var i = 0
    while (i < count) { engine.tell(first + i, Agx.NoSender, payload); i += 1 } // (one submission per burst)
  }

  override protected[akka] def shutdown(): Unit = {
    GpuEngine.unregister(engine)
    engine.close() // waits for tells and a pump inside the engine; later tells become dead letters
    super.shutdown()
  }
}
