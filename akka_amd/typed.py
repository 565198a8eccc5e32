"""Typed behaviours lowered to compiled behaviour tables.

A subset of the typed actor DSL -- ``Behaviors.receiveMessage`` / ``Behaviors.same`` /
``Behaviors.stopped`` / ``Behaviors.unhandled`` (akka-actor-typed/src/main/scala/akka/actor/typed/
scaladsl/Behaviors.scala:101-121) and the javadsl ``ReceiveBuilder`` (onMessage / onMessageEquals /
onAnyMessage, akka-actor-typed/src/main/scala/akka/actor/typed/javadsl/ReceiveBuilder.scala:48-98)
-- is written here against symbolic messages and state, and lowered to the engine's case/action
tables (include/akka_gpu.h "compiled behaviours", ``agx_set_behaviors``).  The engine (and the
oracle) then run every actor registered with ``kind_of(behavior)`` through those tables:
ReceiveBuilder.receive's first-matching-handler rule (:209-218), ``Behaviors.unhandled`` when no
handler matches, and ``become`` when a handler returns another behaviour (TY/Behavior.scala:150,
ActorAdapter.next TY/internal/adapter/ActorAdapter.scala:152-168).

What lowers:
  * messages are u32 payloads; a ``MessageType`` owns a tag (payload >> 24) and carries a 24-bit
    argument, ``m.payload`` / ``m.tag`` / ``m.arg`` / ``m.sender`` are the message's fields;
  * state is at most two u64 fields (the actor's state words 0 and 1);
  * a handler returns a list of effects -- ``field.set/add/inc/max/min(v)``, ``ref.tell(v)`` --
    followed by the next behaviour; ``test=`` (a message predicate, like ReceiveBuilder's
    ``JPredicate``) and ``when=`` (a state guard: the lowering of an ``if`` inside a handler into
    two handlers) give each handler at most two tests beside its message type.

    counter = (ReceiveBuilder.create(State("count", "sum"))
               .on_any_message(lambda m, s: [s.count.inc(), s.sum.add(m.payload), Behaviors.same])
               .build("counter"))
    tables = compile_behaviors([counter])     # -> engine.set_behaviors(tables)
    engine.register_range(0, n, tables.kind_of(counter))
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

KIND_COMPILED = 16
MAX_BEHAVIORS, MAX_CASES, MAX_ACTS = 64, 1024, 4096

V_CONST, V_PAYLOAD, V_TAG, V_ARG, V_WORD, V_SENDER, V_SELF = range(7)
CMP_ANY, CMP_EQ, CMP_NE, CMP_LT, CMP_LE, CMP_GT, CMP_GE = range(7)
A_SET, A_ADD, A_MAX, A_MIN, A_TELL = 1, 2, 3, 4, 5
RES_SAME, RES_STOPPED, RES_UNHANDLED, RES_BECOME = 0, 1, 2, 3


class AgxCase(ctypes.Structure):
    """include/akka_gpu.h agx_case (48 B)."""
    _fields_ = [("src1", ctypes.c_uint8), ("word1", ctypes.c_uint8), ("cmp1", ctypes.c_uint8), ("src2", ctypes.c_uint8),
                ("word2", ctypes.c_uint8), ("src3", ctypes.c_uint8), ("word3", ctypes.c_uint8), ("cmp2", ctypes.c_uint8),
                ("src4", ctypes.c_uint8), ("word4", ctypes.c_uint8), ("result", ctypes.c_uint8), ("next", ctypes.c_uint8),
                ("act_first", ctypes.c_uint16), ("act_count", ctypes.c_uint16),
                ("k1", ctypes.c_int64), ("k2", ctypes.c_int64), ("k3", ctypes.c_int64), ("k4", ctypes.c_int64)]


class AgxAct(ctypes.Structure):
    """include/akka_gpu.h agx_act (32 B)."""
    _fields_ = [("op", ctypes.c_uint8), ("word", ctypes.c_uint8), ("src", ctypes.c_uint8), ("sword", ctypes.c_uint8),
                ("dsrc", ctypes.c_uint8), ("dword", ctypes.c_uint8), ("pad0", ctypes.c_uint8), ("pad1", ctypes.c_uint8),
                ("or_mask", ctypes.c_uint32), ("k", ctypes.c_int64), ("dk", ctypes.c_int64)]


assert ctypes.sizeof(AgxCase) == 48 and ctypes.sizeof(AgxAct) == 32


class CompileError(ValueError):
    """The behaviour uses something the tables cannot express."""


# ------------------------------------------------------------------ symbolic values
@dataclass(frozen=True)
class Operand:
    """value = base(src, word) + k (u64 wrapping)."""
    src: int
    word: int = 0
    k: int = 0

    def __add__(self, c):
        if not isinstance(c, int):
            raise CompileError("only a constant can be added to an operand")
        return Operand(self.src, self.word, self.k + c)

    def __sub__(self, c):
        return self + (-c)

    def _test(self, cmp, other):
        return Test(cmp, self, lift(other))

    def __eq__(self, o):  # noqa: D105 -- builds a Test, like the Scala `==` inside a guard
        return self._test(CMP_EQ, o)

    def __ne__(self, o):
        return self._test(CMP_NE, o)

    def __lt__(self, o):
        return self._test(CMP_LT, o)

    def __le__(self, o):
        return self._test(CMP_LE, o)

    def __gt__(self, o):
        return self._test(CMP_GT, o)

    def __ge__(self, o):
        return self._test(CMP_GE, o)

    __hash__ = object.__hash__


def lift(x) -> Operand:
    if isinstance(x, Operand):
        return x
    if isinstance(x, (int, np.integer)):
        return Operand(V_CONST, 0, int(x))
    raise CompileError(f"not an operand: {x!r}")


@dataclass(frozen=True)
class Test:
    cmp: int
    lhs: Operand
    rhs: Operand


ALWAYS = Test(CMP_ANY, Operand(V_CONST), Operand(V_CONST))


@dataclass(frozen=True)
class Action:
    op: int
    word: int = 0
    val: Operand = Operand(V_CONST)
    dst: Operand | None = None
    or_mask: int = 0


class Field(Operand):
    """A state field (state word 0 or 1)."""

    def set(self, v):
        return Action(A_SET, self.word, lift(v))

    def add(self, v):
        return Action(A_ADD, self.word, lift(v))

    def inc(self, n: int = 1):
        return self.add(n)

    def max(self, v):
        return Action(A_MAX, self.word, lift(v))

    def min(self, v):
        return Action(A_MIN, self.word, lift(v))

    @property
    def ref(self) -> "Ref":
        """The field's value as an ActorRef (an actor id)."""
        return Ref(Operand(V_WORD, self.word))


@dataclass(frozen=True)
class Ref:
    """An ActorRef: `dst` operand; based on the actor's own id it wraps mod n (ring neighbours)."""
    dst: Operand

    def tell(self, msg, tag: int | None = None):
        """ActorRef.! (AA/ActorRef.scala:412-413).  `msg`: an operand (the payload) or a
        MessageType application; `tag` ORs a message tag into the payload."""
        if isinstance(msg, Message):
            val, mask = msg.arg, msg.or_mask
        else:
            val, mask = lift(msg), 0
        if tag is not None:
            mask |= (tag & 0xFF) << 24
        return Action(A_TELL, 0, val, self.dst, mask)

    __call__ = tell


def self_ref(offset: int = 0) -> Ref:
    """context.self, or the actor `offset` ids further on (mod the population)."""
    return Ref(Operand(V_SELF, 0, offset))


def actor_ref(actor_id: int) -> Ref:
    return Ref(Operand(V_CONST, 0, actor_id))


@dataclass(frozen=True)
class Message:
    """An outgoing message of a MessageType: payload = (tag << 24) | arg."""
    arg: Operand
    or_mask: int


@dataclass(frozen=True)
class MessageType:
    """A message class: its instances are the payloads carrying `tag` in bits 24..31."""
    name: str
    tag: int

    def __post_init__(self):
        if not 0 <= self.tag <= 0xFF:
            raise CompileError("message tags are 8 bits")

    def __call__(self, arg=0) -> Message:
        return Message(lift(arg), self.tag << 24)

    def payload(self, arg: int = 0) -> int:
        """The u32 payload of an instance (for host tells)."""
        return (self.tag << 24) | (arg & 0xFFFFFF)


class Incoming:
    """The message being handled (symbolic)."""
    payload = Operand(V_PAYLOAD)
    tag = Operand(V_TAG)
    arg = Operand(V_ARG)
    sender = Ref(Operand(V_SENDER))


class State:
    """Named state fields -> words 0, 1."""

    def __init__(self, *names: str):
        if len(names) > 2:
            raise CompileError("compiled behaviours hold at most two u64 state fields")
        self.names = names
        for i, n in enumerate(names):
            setattr(self, n, Field(V_WORD, i))


# ------------------------------------------------------------------ behaviours
@dataclass(frozen=True)
class _Result:
    code: int
    name: str


class Behaviors:
    """Behaviors.same / stopped / unhandled (TY/scaladsl/Behaviors.scala) and receiveMessage."""
    same = _Result(RES_SAME, "same")
    stopped = _Result(RES_STOPPED, "stopped")
    unhandled = _Result(RES_UNHANDLED, "unhandled")

    @staticmethod
    def receive_message(state: State, *handlers, name: str = "behavior") -> "Behavior":
        """Behaviors.receiveMessage with a partial function: `handlers` are
        (type or None, handler[, test[, when]]) tuples tried in order."""
        b = ReceiveBuilder.create(state)
        for h in handlers:
            b.on_message(*h)
        return b.build(name)


@dataclass
class _Case:
    tests: list
    effects: list
    result: object  # _Result or Behavior


@dataclass(eq=False)
class Behavior:
    name: str
    state: State
    cases: list = field(default_factory=list)


class ReceiveBuilder:
    """javadsl ReceiveBuilder (TY/javadsl/ReceiveBuilder.scala): handlers in the order added."""

    def __init__(self, state: State):
        self.state = state
        self.cases: list[_Case] = []

    @staticmethod
    def create(state: State | None = None) -> "ReceiveBuilder":
        return ReceiveBuilder(state or State())

    def _add(self, tests, handler, when):
        m, s = Incoming, self.state
        if when is not None:
            tests.append(when(m, s))
        out = handler(m, s)
        if not isinstance(out, (list, tuple)):
            out = [out]
        effects, result = list(out[:-1]), out[-1]
        if not isinstance(result, (_Result, Behavior)):
            raise CompileError("a handler's last element must be Behaviors.same/stopped/unhandled or a Behavior")
        for e in effects:
            if not isinstance(e, Action):
                raise CompileError(f"not an effect: {e!r}")
        for t in tests:
            if not isinstance(t, Test):
                raise CompileError(f"not a test: {t!r}")
        if len(tests) > 2:
            raise CompileError("a handler has at most two tests (message type / predicate / state guard)")
        self.cases.append(_Case(tests, effects, result))
        return self

    def on_message(self, mtype: MessageType | None, handler, test=None, when=None) -> "ReceiveBuilder":
        """onMessage(type, [test,] handler) (:48-60); `when` guards on the actor's state."""
        tests = [] if mtype is None else [Incoming.tag == mtype.tag]
        if test is not None:
            tests.append(test(Incoming))
        return self._add(tests, handler, when)

    def on_message_equals(self, payload: int, handler, when=None) -> "ReceiveBuilder":
        """onMessageEquals(msg, handler) (:83-90)."""
        return self._add([Incoming.payload == payload], lambda m, s: handler(m, s), when)

    def on_any_message(self, handler, test=None, when=None) -> "ReceiveBuilder":
        """onAnyMessage(handler) (:98)."""
        return self.on_message(None, handler, test, when)

    def build(self, name: str = "behavior", into: Behavior | None = None) -> Behavior:
        """The built behaviour; `into` fills a Behavior created beforehand (mutually recursive
        behaviours that become each other)."""
        if into is not None:
            into.cases = list(self.cases)
            return into
        return Behavior(name, self.state, list(self.cases))


# ------------------------------------------------------------------ lowering
@dataclass
class Tables:
    """The lowered tables of a set of behaviours (agx_set_behaviors arguments)."""
    behaviors: list
    cases: ctypes.Array
    acts: ctypes.Array
    first: np.ndarray

    @property
    def n_behaviors(self) -> int:
        return len(self.behaviors)

    @property
    def max_tells(self) -> int:
        """The most tells one message can emit (the largest tell count of any case): the engine's
        max_emit must be at least this (agx_set_behaviors rejects the tables otherwise)."""
        return max((sum(1 for i in range(c.act_first, c.act_first + c.act_count) if self.acts[i].op == A_TELL)
                    for c in self.cases[:int(self.first[-1])]), default=0)

    def kind_of(self, b: Behavior) -> int:
        """The actor kind that starts in behaviour `b`."""
        for i, x in enumerate(self.behaviors):
            if x is b:
                return KIND_COMPILED + i
        raise KeyError(b.name)


def _reachable(roots) -> list:
    seen, order = set(), []
    todo = list(roots)
    while todo:
        b = todo.pop(0)
        if id(b) in seen:
            continue
        seen.add(id(b))
        order.append(b)
        todo.extend(c.result for c in b.cases if isinstance(c.result, Behavior))
    return order


def compile_behaviors(roots, max_emit: int | None = None) -> Tables:
    """Lower `roots` and every behaviour they become into the engine's tables.  With `max_emit`
    (the engine's agx_cfg.max_emit), a case that tells more often than that is a CompileError:
    the apply kernels reserve max_emit tell slots per message."""
    behs = _reachable(roots)
    if len(behs) > MAX_BEHAVIORS:
        raise CompileError(f"more than {MAX_BEHAVIORS} behaviours")
    index = {id(b): i for i, b in enumerate(behs)}
    cases, acts, first = [], [], [0]
    for b in behs:
        for c in b.cases:
            t = c.tests + [ALWAYS] * (2 - len(c.tests))
            res = c.result
            code, nxt = (RES_BECOME, index[id(res)]) if isinstance(res, Behavior) else (res.code, 0)
            if len(acts) + len(c.effects) > 0xFFFF:
                raise CompileError("too many actions")
            cases.append(AgxCase(src1=t[0].lhs.src, word1=t[0].lhs.word, k1=t[0].lhs.k, cmp1=t[0].cmp,
                                 src2=t[0].rhs.src, word2=t[0].rhs.word, k2=t[0].rhs.k,
                                 src3=t[1].lhs.src, word3=t[1].lhs.word, k3=t[1].lhs.k, cmp2=t[1].cmp,
                                 src4=t[1].rhs.src, word4=t[1].rhs.word, k4=t[1].rhs.k,
                                 result=code, next=nxt, act_first=len(acts), act_count=len(c.effects)))
            for e in c.effects:
                d = e.dst or Operand(V_CONST)
                acts.append(AgxAct(op=e.op, word=e.word, src=e.val.src, sword=e.val.word, k=e.val.k,
                                   dsrc=d.src, dword=d.word, dk=d.k, or_mask=e.or_mask))
        first.append(len(cases))
    if len(cases) > MAX_CASES or len(acts) > MAX_ACTS:
        raise CompileError("tables too large")
    t = Tables(behs, (AgxCase * max(len(cases), 1))(*cases), (AgxAct * max(len(acts), 1))(*acts),
               np.asarray(first, dtype=np.uint32))
    if max_emit is not None and t.max_tells > max(1, max_emit):
        raise CompileError(f"a case tells {t.max_tells} times per message but max_emit is {max_emit}")
    return t


# ------------------------------------------------------------------ the built-in kinds, as typed behaviours
def library(ring_stride: int = 1) -> dict:
    """The engine's fixed behaviour kinds written in the DSL (used to cross-check the lowering
    against the hand-written kinds, include/akka_gpu.h agx_behavior_kind)."""
    st2 = State("count", "sum")
    counter = (ReceiveBuilder.create(st2)
               .on_any_message(lambda m, s: [s.count.inc(), s.sum.add(m.payload), Behaviors.same])
               .build("counter"))
    ring_state = State("count")
    ring = (ReceiveBuilder.create(ring_state)
            .on_any_message(lambda m, s: [s.count.inc(), self_ref(ring_stride).tell(m.payload - 1), Behaviors.same],
                            test=lambda m: m.payload > 0)
            .on_any_message(lambda m, s: [s.count.inc(), Behaviors.same])
            .build("ring"))
    sa = State("count", "limit")
    stop_after = (ReceiveBuilder.create(sa)
                  .on_any_message(lambda m, s: [s.count.inc(), Behaviors.stopped], when=lambda m, s: s.count + 1 >= s.limit)
                  .on_any_message(lambda m, s: [s.count.inc(), Behaviors.same])
                  .build("stop_after"))
    pp = State("left", "count")
    # BenchmarkActors.PingPong (akka-bench-jmh/src/main/scala/akka/actor/BenchmarkActors.scala:20-32)
    reply = lambda m, s: [s.count.inc(), m.sender.tell(m.payload), s.left.add(-1)]
    ping_pong = (ReceiveBuilder.create(pp)
                 .on_any_message(lambda m, s: reply(m, s) + [Behaviors.stopped], when=lambda m, s: s.left == 0)
                 .on_any_message(lambda m, s: reply(m, s) + [Behaviors.same])
                 .build("ping_pong"))
    return {"counter": counter, "ring": ring, "stop_after": stop_after, "ping_pong": ping_pong}


SWITCH_ON, SWITCH_OFF, PING = MessageType("SwitchOn", 1), MessageType("SwitchOff", 2), MessageType("Ping", 3)


def switch() -> Behavior:
    """Two behaviours that become each other (TY/Behavior.scala:150): `off` counts a SwitchOn and
    becomes `on`, leaves Ping unhandled; `on` sums Ping arguments, answers Ping(n) with Ping(n - 1)
    while n > 0, and becomes `off` on SwitchOff."""
    st = State("flips", "sum")
    on, off = Behavior("on", st), Behavior("off", st)
    (ReceiveBuilder.create(st)
     .on_message(SWITCH_ON, lambda m, s: [s.flips.inc(), on])
     .on_message(SWITCH_OFF, lambda m, s: [Behaviors.same])
     .build(into=off))
    (ReceiveBuilder.create(st)
     .on_message(SWITCH_OFF, lambda m, s: [s.flips.inc(), off])
     .on_message(PING, lambda m, s: [s.sum.add(m.arg), m.sender.tell(PING(m.arg - 1)), Behaviors.same],
                 test=lambda m: m.arg > 0)
     .on_message(PING, lambda m, s: [Behaviors.same])
     .build(into=on))
    return off
