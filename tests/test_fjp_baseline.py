"""The multi-threaded ForkJoin restatement (oracle/fjp_ref.cpp, the CPU baseline) on the
benchmark's workload shapes, at small sizes: it must agree bit-exactly with the BSP oracle
wherever the workload is confluent (schedule independent), for any worker count, and its
counters must be conserved.  tools/sanitize.sh runs this file under TSan and ASan/UBSan."""
import numpy as np
import pytest

from akka_amd import workloads as wl
from akka_amd.engine import Kind
from oracle import BspOracle, FjpOracle

CASES = {
    "ring": lambda: wl.token_ring(20_000, 12),
    "pingpong": lambda: wl.ping_pong(200, 400, 50),
    "zipf": lambda: wl.zipf_fanout(20_000, k=4, ttl=3, root_every=16, throughput=5),
}
CRDT = {
    "gcounter": lambda: wl.crdt_gossip(2_000, Kind.GCOUNTER, rounds=8),
    "orset": lambda: wl.crdt_gossip(1_000, Kind.ORSET, rounds=6),
    "pncounter": lambda: wl.crdt_gossip(2_000, Kind.PNCOUNTER, rounds=8),
}


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("case", sorted(CASES))
def test_fjp_matches_bsp_on_confluent_workloads(case, threads):
    w = CASES[case]()
    b = BspOracle(**w.engine_kwargs())
    w.apply_to(b)
    sb = b.run()
    f = FjpOracle(**w.engine_kwargs())
    w.apply_to(f)
    sf = f.run(threads)
    for k in ("delivered", "dead_letters", "unhandled", "emitted", "staged", "in_flight"):
        assert sb[k] == sf[k], (case, k, sb[k], sf[k])
    assert np.array_equal(b.read_state()[0], f.read_state()[0]), case


@pytest.mark.parametrize("threads", [2, 8])
def test_fjp_bounded_conservation(threads):
    """Bounded mailboxes are schedule-sensitive (MailboxSelectorSpec.scala:73-75): only the
    conservation law and the per-mailbox bound are checked."""
    w = wl.power_law_forward(20_000, ttl=6, capacity=4, throughput=5)
    f = FjpOracle(**w.engine_kwargs())
    w.apply_to(f)
    st = f.run(threads)
    assert st["in_flight"] == 0
    assert st["staged"] + st["emitted"] == st["delivered"] + st["dead_letters"]


@pytest.mark.parametrize("threads", [1, 4, 8])
@pytest.mark.parametrize("case", sorted(CRDT))
def test_fjp_crdt_gossip(case, threads):
    """Replicator-style gossip: the message counts are schedule independent, the replica
    states are not (a gossip carries the sender's state at send time) -- every final state
    must lie below the join of the writers' updates, and merging it in changes nothing."""
    from oracle.oracle import orset
    w = CRDT[case]()
    b = BspOracle(**w.engine_kwargs())
    w.apply_to(b)
    sb = b.run()
    f = FjpOracle(**w.engine_kwargs())
    w.apply_to(f)
    sf = f.run(threads)
    for k in ("delivered", "dead_letters", "unhandled", "emitted", "staged", "in_flight"):
        assert sb[k] == sf[k], (case, k, sb[k], sf[k])
    ws = f.read_state()[0]
    ops = wl.crdt_ops(8, w.ranges[0][2], 16)
    if case == "orset":
        join = orset.empty()
        for k in range(8):
            r = orset.empty()
            for p in ops[k]:
                op, arg = int(p) >> 24, int(p) & 0xFFFFFF
                r = orset.add(r, k, arg) if op == 3 else orset.remove(r, arg)
            join = orset.merge(join, r)
        assert all(np.array_equal(orset.merge(x, join), join) for x in ws)
    else:
        join = np.zeros(w.n_words, np.uint64)
        for k in range(8):
            for p in ops[k]:
                op, arg = int(p) >> 24, int(p) & 0xFFFFFF
                join[k if op == 1 else 8 + k] += arg
        assert (ws <= join[None, :]).all()
