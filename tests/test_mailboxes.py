"""Per-actor mailbox types and the reply path on the CPU oracle (bsp_ref.c), pinned by the
reference's mailbox specs.  The GPU parity of the same workloads is in tests/test_gpu_mailboxes.py.

- Mailboxes.lookupConfigurator resolves a mailbox per actor (akka-actor/src/main/scala/akka/
  dispatch/Mailboxes.scala:204-260; selection precedence: akka-actor-tests/.../ActorMailboxSpec.
  scala:245-450): a bounded-capacity:N actor beside unbounded ones drops exactly its arrivals
  beyond N (MailboxConfigSpec.scala:47-66), FIFO survivors; its neighbours drop nothing.
- sender() ! reply (akka-actor/src/main/scala/akka/actor/ActorCell.scala:583-587): a PingPong
  actor answering a host-side sender leaves its replies in the outbox, not in dead letters.
"""
import numpy as np
import pytest

from akka_amd import workloads as wl
from akka_amd.engine import Kind, NO_SENDER
from oracle import BspOracle


def test_bounded_beside_unbounded_kat():
    o = BspOracle(n_actors=8, throughput=1000, capacity=0, n_words=2)
    o.register_range(0, 8, Kind.COUNTER)
    o.set_mailbox_class(1, 10)   # bounded-capacity:10
    o.set_mailbox(2, 1, 1)
    pay = np.arange(1, 21, dtype=np.uint32)
    for a in (1, 2, 3):
        o.tell(np.full(20, a, np.uint32), pay)
    st = o.run()
    w, _ = o.read_state()
    assert st["delivered"] == 20 + 10 + 20 and st["dead_letters"] == 10
    assert (w[2] == [10, 55]).all() and (w[1] == [20, 210]).all() and (w[3] == [20, 210]).all()


def test_bounded_class_clamps_throughput():
    """A bounded queue never holds more than C: a class of capacity 3 drains <= 3 per run even
    with throughput 5 (the default class drains 5)."""
    o = BspOracle(n_actors=4, throughput=5, capacity=0, n_words=2)
    o.register_range(0, 4, Kind.COUNTER)
    o.set_mailbox_class(1, 3)
    o.set_mailbox(0, 1, 1)
    o.tell(np.zeros(3, np.uint32), [1, 2, 3])
    o.tell(np.ones(5, np.uint32), [1, 2, 3, 4, 5])
    st = o.run()
    assert st["delivered"] == 8 and st["supersteps"] == 1


def test_outbox_ping_pong():
    """Host probe 100 pings PingPong actor 5 (left 2): three replies reach the probe through the
    outbox (left 2 -> 0, then stopped); nothing is a dead letter; the 4th ping is."""
    o = BspOracle(n_actors=16, throughput=5, capacity=0, n_words=2)
    init = np.zeros((1, 2), np.uint64)
    init[0, 0] = 2
    o.register_range(0, 16, Kind.COUNTER)
    o.register_range(5, 1, Kind.PINGPONG, init)
    o.set_outbound(100, 4)
    replies = []
    for k in range(4):
        o.tell([5], [10 + k], [100])
        o.run()
        d, s, p = o.take_outbound()
        replies += list(zip(d.tolist(), s.tolist(), p.tolist()))
    assert replies == [(100, 5, 10), (100, 5, 11), (100, 5, 12)]
    st = o.run()
    assert st["dead_letters"] == 1 and st["emitted"] == 0


def test_mailbox_mix_conservation():
    """staged + emitted = delivered + dead letters + in flight, with outbound tells outside the engine."""
    w = wl.mailbox_mix(4096, seed=3, throughput=2)
    o = BspOracle(**w.engine_kwargs())
    w.apply_to(o)
    st = o.run()
    d, s, p = o.take_outbound()
    assert d.size > 0 and (d >= w.n_actors).all()
    assert st["staged"] + st["emitted"] == st["delivered"] + st["dead_letters"] + st["in_flight"]


def test_outbox_overflow_oracle_matches_engine_rule():
    """The oracle's outbox overflow follows the engine (agx_take_outbound): the run goes
    on, the next take reports the drop once (OutboxOverflow = AGX_ECAPACITY), the kept tells (the
    capacity's worth) come out of the take after it, and the counters are unaffected."""
    from oracle.oracle import OutboxOverflow
    w = wl.mailbox_mix(4096, seed=1, throughput=5)
    big = BspOracle(**w.engine_kwargs())
    w.apply_to(big)
    big.set_outbound(w.n_actors, 32, capacity=1 << 20)
    sb = big.run(3)
    total = big.take_outbound()[0].size
    assert total > 4
    o = BspOracle(**w.engine_kwargs())
    w.apply_to(o)
    o.set_outbound(w.n_actors, 32, capacity=4)
    st = o.run(3)
    assert st == sb  # (outbound tells leave the engine: no counter depends on the outbox)
    with pytest.raises(OutboxOverflow):
        o.take_outbound()
    d, s, p = o.take_outbound()
    assert d.size == 4 and (d >= w.n_actors).all()
    o.take_outbound()  # nothing lost since: no report
    st2, sb2 = o.run(), big.run()
    assert st2 == sb2
