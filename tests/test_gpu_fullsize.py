"""GPU parity at the FULL sizes bench.py reports (BASELINE.json configs C1, C3, C4, C5), through the
C ABI, against the BSP oracle -- the same workload constructors, throughputs, capacities, message
capacities and superstep windows as `bench.py other_configs()`, so every number the bench prints
comes from a configuration whose results are checked bit-exactly here:

* C3 10M Zipf, steady state and fan-out tree: the bench window, then on to quiescence (the hot
  actors' BoundedMailbox(1000) backlogs drain at 5 per superstep: ~1600 supersteps);
* C4 1M GCounter / ORSet full-state gossip and GCounter / ORSet delta-CRDT: the bench window
  (warmup + timed supersteps);
* C5 100M power-law R-MAT, BoundedMailbox(64): the bench window (2 + 10 supersteps) at 10^8 actors
  -- the structure that only exists at that size (first-pass units of G = 24 buckets, 48 828
  buckets, tens of thousands of skewed parts) -- plus conservation; and a 10M run to quiescence;
* C1 ping-pong, 1000 pairs as benched, over the bench's 16 + 400 supersteps.

Reference semantics pinned: Mailbox.processMailbox / BoundedMailbox admission
(akka-actor/src/main/scala/akka/dispatch/Mailbox.scala:260-277,551-565;
akka-actor/src/main/java/akka/dispatch/AbstractBoundedNodeQueue.java:92-113), ORSet / GCounter merge
(akka-distributed-data/src/main/scala/akka/cluster/ddata/ORSet.scala:427-501, GCounter.scala:113-125),
delta propagation (Replicator.scala:1953-2027).  The oracle runs its apply on host threads
(oracle/bsp_ref.c: identical output for any thread count, tests/test_oracle_golden.py).
"""
import numpy as np
import pytest

from akka_amd import workloads as wl
from akka_amd.engine import EngineConfig, GpuEngine, Kind

pytestmark = [pytest.mark.gpu, pytest.mark.fullsize]

COUNT_KEYS = ("delivered", "dead_letters", "unhandled", "emitted", "staged", "supersteps", "in_flight")


def _gpu(w, windows, msg_capacity=0):
    """Run the HIP engine through `windows` (cumulative superstep budgets); stats + state after each."""
    eng = GpuEngine(EngineConfig(msg_capacity=msg_capacity, **w.gpu_kwargs()))
    w.apply_to(eng)
    out, done = [], 0
    for k in windows:
        st = eng.run(k - done)
        done = k
        out.append((st, eng.read_state()))
    eng.close()
    return out


def _oracle(w, windows):
    from oracle import BspOracle
    ref = BspOracle(**w.engine_kwargs())
    w.apply_to(ref)
    out, done = [], 0
    for k in windows:
        st = ref.run(k - done)
        done = k
        out.append((st, ref.read_state()))
    ref.close()
    return out


def _check(w, windows, name, msg_capacity=0):
    g = _gpu(w, windows, msg_capacity)
    o = _oracle(w, windows)
    for k, (sg, (wg, ag)), (so, (wo, ao)) in zip(windows, g, o):
        tag = f"{name} after {k if k < 1 << 29 else 'quiescence'}"
        for key in COUNT_KEYS:
            assert getattr(sg, key) == so[key], f"{tag}: {key} gpu={getattr(sg, key)} oracle={so[key]}"
        # conservation: staged + emitted = delivered + dead letters + in flight (outbound: none here)
        assert sg.staged + sg.emitted == sg.delivered + sg.dead_letters + sg.in_flight, tag
        assert np.array_equal(ag, ao), f"{tag}: alive differs"
        diff = np.nonzero((wg != wo).any(axis=1))[0]
        assert diff.size == 0, f"{tag}: state differs at {diff[:10]}"
    return g


QUIET = 1 << 30


# ------------------------------------------------------------------ C3 10M (bench: 2 + 10 / 0 + 8)
@pytest.mark.timeout(600)
def test_c3_steady_10m_as_benched(built):
    w = wl.zipf_fanout(10_000_000, k=1, ttl=15, root_every=1, capacity=1000)
    g = _check(w, [12, QUIET], "C3 steady 10M")
    assert g[0][0].dead_letters > 0 and g[0][0].in_flight > 0 and g[1][0].in_flight == 0


@pytest.mark.timeout(600)
def test_c3_tree_10m_as_benched(built):
    w = wl.zipf_fanout(10_000_000, k=4, ttl=3, root_every=64, capacity=1000)
    g = _check(w, [8, QUIET], "C3 tree 10M")
    assert g[0][0].dead_letters > 0 and g[1][0].in_flight == 0


# ------------------------------------------------------------------ C4 1M (bench windows)
@pytest.mark.timeout(600)
def test_c4_gcounter_1m_as_benched(built):
    _check(wl.crdt_gossip(1_000_000, Kind.GCOUNTER, rounds=40), [4, 28], "C4 GCounter 1M")


@pytest.mark.timeout(600)
def test_c4_orset_1m_as_benched(built):
    g = _check(wl.crdt_gossip(1_000_000, Kind.ORSET, rounds=20), [2, 14], "C4 ORSet 1M")
    assert g[-1][0].unhandled == 0


@pytest.mark.timeout(900)
def test_c4_orset_delta_1m_as_benched(built):
    w = wl.crdt_delta(1_000_000, Kind.ORSET, rounds=40, write=True)
    _check(w, [4, 28], "C4 ORSet delta 1M", msg_capacity=8_000_000)


@pytest.mark.timeout(600)
def test_c4_gcounter_delta_1m_as_benched(built):
    w = wl.crdt_delta(1_000_000, Kind.GCOUNTER, rounds=40, write=True)
    _check(w, [4, 28], "C4 GCounter delta 1M", msg_capacity=8_000_000)


# ------------------------------------------------------------------ C5 (bench: 100M, 2 + 10)
@pytest.mark.timeout(900)
def test_c5_100m_as_benched(built):
    """10^8 actors, the device R-MAT graph (~3.6e8 edges), BoundedMailbox(64), throughput 5: the
    bench's warmup and timed window, bit-exact counts and every actor's state and alive flag."""
    w = wl.power_law_forward(100_000_000, ttl=15, capacity=64, throughput=5, device_graph=True)
    g = _check(w, [2, 12], "C5 100M")
    st = g[-1][0]
    assert st.dead_letters > 0 and st.in_flight > 0
    # every delivered message was admitted: at most T = 5 per actor per superstep
    assert st.delivered <= 5 * 100_000_000 * 12


@pytest.mark.timeout(600)
def test_c5_10m_to_quiescence(built):
    w = wl.power_law_forward(10_000_000, ttl=15, capacity=64, throughput=5, device_graph=True)
    g = _check(w, [12, QUIET], "C5 10M")
    assert g[-1][0].in_flight == 0


# ------------------------------------------------------------------ C1 (bench: 16 + 400)
@pytest.mark.timeout(600)
def test_c1_ping_pong_as_benched(built):
    w = wl.ping_pong(1000, messages_per_pair=2_000_000, throughput=50)
    _check(w, [16, 416], "C1 ping-pong", msg_capacity=1 << 20)


# ------------------------------------------------------------------ the 100M ring (bench's second line)
@pytest.mark.timeout(600)
def test_ring_100m_properties(built):
    """10^8 actors, one token each (the bench's 100M ring): size-independent properties to
    quiescence -- every actor counted exactly hops + 1 deliveries, hops + 1 supersteps, nothing dead
    or in flight -- and identity grouping on (agx_identity_supersteps: every superstep after the first
    grouped its mail without a radix pass), with the dense-bucket launch (its
    default for rings) taking the buckets."""
    n, hops = 100_000_000, 6
    w = wl.token_ring(n, hops)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    st = eng.run()
    assert st.delivered == n * (hops + 1) and st.emitted == n * hops and st.staged == n
    assert st.dead_letters == 0 and st.unhandled == 0 and st.in_flight == 0
    assert st.supersteps == hops + 1
    assert eng.identity_supersteps() >= hops - 1
    words, alive = eng.read_state()
    assert (words[:, 0] == hops + 1).all() and alive.all()
    eng.close()
