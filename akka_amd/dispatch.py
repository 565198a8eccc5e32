"""The reference's dispatcher / mailbox plugin surface, backed by the GPU engine.

Akka resolves a dispatcher id to a MessageDispatcherConfigurator by HOCON
`type` (built-in name or FQCN constructed with (Config, DispatcherPrerequisites))
and a mailbox id to a MailboxType by `mailbox-type` FQCN or `bounded-capacity:N`:

  Dispatchers.lookup / lookupConfigurator / configuratorFrom
      akka-actor/src/main/scala/akka/dispatch/Dispatchers.scala:121-262
  MessageDispatcherConfigurator.dispatcher()
      akka-actor/src/main/scala/akka/dispatch/AbstractDispatcher.scala:338-382
  Mailboxes.lookup / lookupConfigurator
      akka-actor/src/main/scala/akka/dispatch/Mailboxes.scala:140-260
  typed DispatcherSelector.fromConfig / MailboxSelector.bounded
      akka-actor-typed/src/main/scala/akka/actor/typed/Props.scala:175,206

This module mirrors those names, argument meanings and error behaviour
(ConfigurationException) so that a config such as

    gpu-dispatcher {
      type = "akka_amd.dispatch.GpuDispatcherConfigurator"
      throughput = 5
      mailbox-type = "akka.dispatch.BoundedMailbox"
      mailbox-capacity = 64
      mailbox-push-timeout-time = 0s
      actors = 1000000
    }

selects the MI355X engine.  GPU actors are fixed-layout typed behaviours
(`Behaviors` below), addressed by integer ActorRef ids.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .config import Config, ConfigurationException
from .engine import EngineConfig, GpuEngine, Kind, NO_SENDER, Stats

MAX_DISPATCHER_ALIAS_DEPTH = 20          # Dispatchers.MaxDispatcherAliasDepth
BOUNDED_CAPACITY_PREFIX = "bounded-capacity:"  # Mailboxes.BoundedCapacityPrefix
GPU_CONFIGURATOR_FQCNS = ("akka_amd.dispatch.GpuDispatcherConfigurator",
                          "akka.dispatch.gpu.GpuDispatcherConfigurator")

# akka-actor/src/main/resources/reference.conf:364-555 (subset used here)
REFERENCE_CONF = Config.parse_string("""
akka.actor.default-dispatcher {
  type = "Dispatcher"
  executor = "default-executor"
  throughput = 5
  throughput-deadline-time = 0ms
  mailbox-requirement = ""
}
akka.actor.default-mailbox {
  mailbox-type = "akka.dispatch.UnboundedMailbox"
  mailbox-capacity = 1000
  mailbox-push-timeout-time = 10s
}
akka.actor.typed.default-mailbox {
  mailbox-type = "akka.dispatch.SingleConsumerOnlyUnboundedMailbox"
}
""")


# ------------------------------------------------------------------ mailboxes
class MailboxType:
    """MailboxType.create(owner, system): MessageQueue (Mailbox.scala:638-640).
    On the GPU a mailbox type is a queue *semantics*: capacity 0 = unbounded."""
    capacity = 0


@dataclass(frozen=True)
class UnboundedMailbox(MailboxType):
    capacity: int = 0


@dataclass(frozen=True)
class SingleConsumerOnlyUnboundedMailbox(MailboxType):
    capacity: int = 0


@dataclass(frozen=True)
class BoundedMailbox(MailboxType):
    """BoundedMailbox(capacity, pushTimeOut) (Mailbox.scala:699-720).  The GPU
    queue is non-blocking: overflow is a DeadLetter, i.e. pushTimeOut must be 0
    (Mailbox.scala:551-565 with offer timeout 0)."""
    capacity: int
    push_timeout_s: float = 0.0

    def __post_init__(self):
        if self.capacity < 0:
            raise ValueError("The capacity for BoundedMailbox can not be negative")
        if self.push_timeout_s > 0:
            raise ConfigurationException(
                "GPU mailboxes never block the sender: set mailbox-push-timeout-time = 0 "
                "(BoundedMailbox with pushTimeOut > 0 would block; Mailboxes.scala:238-249)")


@dataclass(frozen=True)
class NonBlockingBoundedMailbox(MailboxType):
    capacity: int


_MAILBOX_FQCN = {
    "akka.dispatch.UnboundedMailbox": lambda c: UnboundedMailbox(),
    "akka.dispatch.SingleConsumerOnlyUnboundedMailbox": lambda c: SingleConsumerOnlyUnboundedMailbox(),
    "akka.dispatch.BoundedMailbox": lambda c: BoundedMailbox(c.get_int("mailbox-capacity"),
                                                             c.get_duration_s("mailbox-push-timeout-time")),
    "akka.dispatch.NonBlockingBoundedMailbox": lambda c: NonBlockingBoundedMailbox(c.get_int("mailbox-capacity")),
}


class Mailboxes:
    """Mailboxes.lookup (Mailboxes.scala:140-260)."""

    def __init__(self, config: Config):
        self.config = config.with_fallback(REFERENCE_CONF)
        self._cache: dict = {}

    def lookup(self, mailbox_id: str) -> MailboxType:
        if mailbox_id in self._cache:
            return self._cache[mailbox_id]
        if mailbox_id == "unbounded":
            mt = UnboundedMailbox()
        elif mailbox_id == "bounded":
            # Mailboxes.scala:211 builds a BoundedMailbox from default-mailbox; the GPU mailbox
            # tail-drops (push timeout 0), so the lookup id keeps the capacity and drops the timeout
            dm = self.config.get_config("akka.actor.default-mailbox")
            mt = BoundedMailbox(dm.get_int("mailbox-capacity"), 0.0)
        elif mailbox_id.startswith(BOUNDED_CAPACITY_PREFIX):
            mt = BoundedMailbox(int(mailbox_id.split(":")[1]), 0.0)  # Mailboxes.scala:212-216
        else:
            if not self.config.has_path(mailbox_id):
                raise ConfigurationException(f"Mailbox Type [{mailbox_id}] not configured")
            conf = self.config.get_config(mailbox_id).with_fallback(
                self.config.get_config("akka.actor.default-mailbox"))
            mt = self.from_config(conf, conf.get_string("mailbox-type"), mailbox_id)
        self._cache[mailbox_id] = mt
        return mt

    @staticmethod
    def from_config(conf: Config, fqcn: str, where: str = "") -> MailboxType:
        if fqcn == "":
            raise ConfigurationException(f"The setting mailbox-type, defined in [{where}] is empty")
        ctor = _MAILBOX_FQCN.get(fqcn)
        if ctor is None:
            raise ConfigurationException(
                f"Cannot instantiate MailboxType [{fqcn}], defined in [{where}]: not supported by the GPU dispatcher "
                f"(supported: {sorted(_MAILBOX_FQCN)})")
        return ctor(conf.with_fallback(REFERENCE_CONF.get_config("akka.actor.default-mailbox")))


# ------------------------------------------------------------------ typed behaviours
@dataclass(frozen=True)
class Behavior:
    """A fixed-layout typed behaviour: kind + initial state words."""
    kind: int
    init: tuple = ()
    params: tuple = ()
    min_words: int = 1


class Behaviors:
    """The fixed-layout subset of typed Behaviors.receive
    (akka-actor-typed/src/main/scala/akka/actor/typed/scaladsl/Behaviors.scala:101-121).
    Each returns same / stopped / unhandled per message, like ActorAdapter.next."""

    @staticmethod
    def counter() -> Behavior:
        return Behavior(Kind.COUNTER, (0, 0), min_words=1)

    @staticmethod
    def ring(stride: int = 1) -> Behavior:
        return Behavior(Kind.RING, (0,), ("ring", stride))

    @staticmethod
    def fanout(k: int, cdf, perm, seed: int) -> Behavior:
        return Behavior(Kind.FANOUT, (0, 0), ("fanout", k, seed, cdf, perm))

    @staticmethod
    def forward_round_robin(row_ptr, col) -> Behavior:
        return Behavior(Kind.FORWARD_RR, (0, 0), ("graph", row_ptr, col), min_words=2)

    @staticmethod
    def stop_after(n: int) -> Behavior:
        return Behavior(Kind.STOP_AFTER, (0, n), min_words=2)

    @staticmethod
    def ping_pong(messages_per_pair: int) -> Behavior:
        return Behavior(Kind.PINGPONG, (messages_per_pair // 2, 0))

    @staticmethod
    def even_only() -> Behavior:
        return Behavior(Kind.EVEN, (0,))


class MailboxSelector:
    """typed MailboxSelector (Props.scala:196-216)."""

    @staticmethod
    def bounded(capacity: int) -> str:
        return f"{BOUNDED_CAPACITY_PREFIX}{capacity}"

    @staticmethod
    def default() -> str:
        return "akka.actor.typed.default-mailbox"

    @staticmethod
    def from_config(path: str) -> str:
        return path


class DispatcherSelector:
    """typed DispatcherSelector (Props.scala:150-176)."""

    @staticmethod
    def from_config(path: str) -> str:
        return path


# ------------------------------------------------------------------ dispatchers
@dataclass
class DispatcherPrerequisites:
    """DispatcherPrerequisites (Dispatchers.scala:24-32): here the GPU placement."""
    device: int = 0
    n_ranks: int = 1
    rank: int = 0
    mailboxes: Mailboxes | None = None


@dataclass
class ActorRange:
    first: int
    count: int
    behavior: Behavior

    def ref(self, i: int = 0) -> int:
        if not 0 <= i < self.count:
            raise IndexError(i)
        return self.first + i


class MessageDispatcherConfigurator:
    """Base of dispatcher configurators (AbstractDispatcher.scala:338-347)."""

    def __init__(self, config: Config, prerequisites: DispatcherPrerequisites):
        self.config = config
        self.prerequisites = prerequisites

    def dispatcher(self):
        raise NotImplementedError


class GpuDispatcher:
    """MessageDispatcher backed by one GpuEngine (one rank of a population).

    dispatch(receiver, message, sender)  <- Dispatcher.dispatch (Dispatcher.scala:61-65)
    run(max_supersteps)                  <- registerForExecution + Mailbox.run (Dispatcher.scala:120-143,
                                            Mailbox.scala:227-277) as BSP supersteps
    shutdown()                           <- MessageDispatcher.shutdown (AbstractDispatcher.scala:325)
    """

    def __init__(self, id: str, throughput: int, mailbox: MailboxType, actors: int, state_words: int,
                 max_emit: int, prerequisites: DispatcherPrerequisites, msg_capacity: int = 0,
                 num_shards: int = 1000):
        self.id = id
        self.throughput = throughput
        self.mailbox_type = mailbox
        self.shutdown_timeout_s = 1.0
        self._cfg = EngineConfig(n_actors=actors, throughput=throughput, capacity=mailbox.capacity,
                                 n_words=state_words, max_emit=max_emit, n_ranks=prerequisites.n_ranks,
                                 rank=prerequisites.rank, device=prerequisites.device, msg_capacity=msg_capacity,
                                 num_shards=num_shards)
        self._engine: GpuEngine | None = None
        self._next_id = 0
        self._ranges: list[ActorRange] = []
        self._shut = False

    @property
    def engine(self) -> GpuEngine:
        if self._shut:
            raise RuntimeError(f"dispatcher [{self.id}] is shut down")
        if self._engine is None:
            self._engine = GpuEngine(self._cfg)  # created lazily, like the executor service
        return self._engine

    def is_throughput_deadline_time_defined(self) -> bool:
        return False

    def spawn(self, behavior: Behavior, count: int = 1, mailbox: str | None = None,
              mailboxes: Mailboxes | None = None, init_state=None) -> ActorRange:
        """actorOf for `count` actors with one behaviour: a contiguous ActorRef id range."""
        if mailbox is not None:
            mb = (mailboxes or self._cfg_mailboxes()).lookup(mailbox)
            if mb.capacity != self.mailbox_type.capacity:
                raise ConfigurationException(
                    f"dispatcher [{self.id}] runs one mailbox semantics (capacity {self.mailbox_type.capacity}); "
                    f"props asked for {mb}")
        if behavior.min_words > self._cfg.n_words:
            raise ConfigurationException(f"behaviour needs state-words >= {behavior.min_words}")
        if self._next_id + count > self._cfg.n_actors:
            raise ConfigurationException(f"dispatcher [{self.id}] is configured for {self._cfg.n_actors} actors")
        first = self._next_id
        eng = self.engine
        if init_state is None:
            init = np.zeros((count, self._cfg.n_words), np.uint64)
            for i, v in enumerate(behavior.init[: self._cfg.n_words]):
                init[:, i] = v
        else:
            init = init_state
        eng.register_range(first, count, behavior.kind, init)
        p = behavior.params
        if p and p[0] == "ring":
            eng.set_ring(p[1])
        elif p and p[0] == "fanout":
            eng.set_fanout(p[1], p[2], p[3], p[4])
        elif p and p[0] == "graph":
            eng.set_graph(p[1], p[2])
        self._next_id += count
        r = ActorRange(first, count, behavior)
        self._ranges.append(r)
        return r

    def _cfg_mailboxes(self):
        return self._mailboxes if hasattr(self, "_mailboxes") else Mailboxes(Config())

    def dispatch(self, receiver, message, sender=NO_SENDER) -> None:
        """tell(s): receiver/message/sender may be scalars or arrays."""
        r = np.atleast_1d(np.asarray(receiver, dtype=np.uint32))
        m = np.broadcast_to(np.asarray(message, dtype=np.uint32), r.shape)
        s = np.broadcast_to(np.asarray(sender, dtype=np.uint32), r.shape)
        self.engine.tell(r, m, s)

    tell = dispatch

    def run(self, max_supersteps: int = 1 << 30) -> Stats:
        return self.engine.run(max_supersteps)

    def state(self, rng: ActorRange | None = None):
        if rng is None:
            return self.engine.read_state()
        return self.engine.read_state(rng.first, rng.count)

    def shutdown(self) -> None:
        if self._engine is not None:
            self._engine.close()
            self._engine = None
        self._shut = True


class GpuDispatcherConfigurator(MessageDispatcherConfigurator):
    """`type = "akka_amd.dispatch.GpuDispatcherConfigurator"`.

    Keys (besides the reference's `throughput`, `throughput-deadline-time`,
    `mailbox-type`, `mailbox-capacity`, `mailbox-push-timeout-time`):
      actors, state-words, max-emit, msg-capacity, number-of-shards."""

    def __init__(self, config: Config, prerequisites: DispatcherPrerequisites):
        super().__init__(config, prerequisites)
        c = config.with_fallback(REFERENCE_CONF.get_config("akka.actor.default-dispatcher"))
        if c.get_duration_s("throughput-deadline-time") > 0:
            raise ConfigurationException(
                "throughput-deadline-time is not supported by the GPU dispatcher (a superstep drains "
                "exactly max(throughput,1) messages per mailbox, Mailbox.scala:260-277)")
        mbs = prerequisites.mailboxes or Mailboxes(Config())
        if c.has_path("mailbox-type") and c.get_string("mailbox-type"):
            mb = Mailboxes.from_config(c, c.get_string("mailbox-type"), c.get_string("id") if c.has_path("id") else "")
        else:
            mb = mbs.lookup("akka.actor.typed.default-mailbox")
        self._dispatcher = GpuDispatcher(
            id=c.get_string("id") if c.has_path("id") else "gpu-dispatcher",
            throughput=c.get_int("throughput"),
            mailbox=mb,
            actors=c.get_int("actors") if c.has_path("actors") else 1 << 20,
            state_words=c.get_int("state-words") if c.has_path("state-words") else 2,
            max_emit=c.get_int("max-emit") if c.has_path("max-emit") else 4,
            prerequisites=prerequisites,
            msg_capacity=c.get_int("msg-capacity") if c.has_path("msg-capacity") else 0,
            num_shards=c.get_int("number-of-shards") if c.has_path("number-of-shards") else 1000,
        )
        self._dispatcher._mailboxes = mbs

    def dispatcher(self) -> GpuDispatcher:
        return self._dispatcher


class Dispatchers:
    """Dispatchers.lookup (Dispatchers.scala:121-262): id -> configurator, aliases
    followed up to MaxDispatcherAliasDepth, configurator built from `type`."""

    def __init__(self, config: Config, prerequisites: DispatcherPrerequisites | None = None):
        self.config = config.with_fallback(REFERENCE_CONF)
        self.prerequisites = prerequisites or DispatcherPrerequisites()
        if self.prerequisites.mailboxes is None:
            self.prerequisites.mailboxes = Mailboxes(self.config)
        self._configurators: dict = {}

    def has_dispatcher(self, id: str) -> bool:
        return id in self._configurators or self.config.has_path(id)

    def register_configurator(self, id: str, configurator: MessageDispatcherConfigurator) -> bool:
        if id in self._configurators:
            return False
        self._configurators[id] = configurator
        return True

    def lookup(self, id: str):
        return self._lookup_configurator(id, 0).dispatcher()

    def _lookup_configurator(self, id: str, depth: int) -> MessageDispatcherConfigurator:
        if depth > MAX_DISPATCHER_ALIAS_DEPTH:
            raise ConfigurationException(
                f"Didn't find a concrete dispatcher config after following {MAX_DISPATCHER_ALIAS_DEPTH}, "
                f"is there a loop in your config? last looked for id was {id}")
        if id in self._configurators:
            return self._configurators[id]
        if not self.config.has_path(id):
            raise ConfigurationException(f"Dispatcher [{id}] not configured")
        v = self.config.get_value(id)
        if isinstance(v, str):  # alias
            conf = self._lookup_configurator(v, depth + 1)
        elif isinstance(v, dict):
            c = Config(dict(v))
            c.root.setdefault("id", id)
            conf = self._configurator_from(c)
        else:
            raise ConfigurationException(f"Expected either a dispatcher config or an alias at [{id}] but found [{v!r}]")
        self._configurators.setdefault(id, conf)
        return self._configurators[id]

    def _configurator_from(self, cfg: Config) -> MessageDispatcherConfigurator:
        if not cfg.has_path("id"):
            raise ConfigurationException("Missing dispatcher 'id' property in config")
        t = cfg.get_string("type") if cfg.has_path("type") else "Dispatcher"
        if t in GPU_CONFIGURATOR_FQCNS:
            return GpuDispatcherConfigurator(cfg, self.prerequisites)
        if t in ("Dispatcher", "PinnedDispatcher", "BalancingDispatcher"):
            raise ConfigurationException(
                f"dispatcher [{cfg.get_string('id')}] has type [{t}]: the JVM ForkJoinPool dispatcher is not part "
                f"of this engine; use type = \"{GPU_CONFIGURATOR_FQCNS[0]}\"")
        raise ConfigurationException(
            f"Cannot instantiate MessageDispatcherConfigurator type [{t}], defined in [{cfg.get_string('id')}], "
            "make sure it has constructor with [com.typesafe.config.Config] and "
            "[akka.dispatch.DispatcherPrerequisites] parameters")
