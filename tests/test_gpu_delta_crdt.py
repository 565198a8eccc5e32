"""GPU parity of delta-CRDT replication (agx_set_delta_crdt): DeltaPropagationSelector,
causal receiveDeltaPropagation, ORSet.mergeDelta / mergeRemoveDelta and counter deltas
(DD/DeltaPropagationSelector.scala, DD/Replicator.scala:1646-1695,1953-2027,
DD/ORSet.scala:43-120,455-501) -- the HIP engine through the C ABI vs the BSP oracle, bit-exact
on every counter and every state word (data, deltaVersions, selector state and delta log)."""
import numpy as np
import pytest

from akka_amd import workloads as wl
from akka_amd.engine import EngineConfig, GpuEngine, Kind, Op
from tests.test_gpu_parity import assert_same, run_both

pytestmark = pytest.mark.gpu

KINDS = [Kind.GCOUNTER, Kind.PNCOUNTER, Kind.ORSET]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("T,C", [(5, 0), (1, 0), (2, 6)])
def test_delta_writer_ticks(built, kind, T, C):
    """Writer clients + DeltaPropagationTicks + full-state gossip, with throughput caps (queued
    DeltaPropagations keep their rows) and bounded mailboxes (dropped ones leave seqNr gaps that
    the causal check skips)."""
    w = wl.crdt_delta(8 * 300 + 5, kind, rounds=10, write=True, ops_per_replica=3, gossip_rounds=6, throughput=T,
                      capacity=C)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"delta kind={kind} T={T} C={C}")


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("max_delta", [1, 2, 50])
def test_delta_groups_and_placeholders(built, kind, max_delta):
    """Groups over several seqNrs (host updates before the ticks), coalesced AddDeltaOps, groups at
    max-delta-size (NoDeltaPlaceholder) and counter updates by 0 (placeholder entries)."""
    n = 8 * 200
    w = wl.crdt_delta(n, kind, rounds=6, write=False, ops_per_replica=9, max_delta_size=max_delta)
    ids = np.arange(n, dtype=np.uint32)
    zero = Op.make(Op.INCREMENT, 0) if kind != Kind.ORSET else Op.make(Op.CLEAR, 0)
    dst, src, pay = w.tells
    w.tells = (np.concatenate([ids[::3], dst]), np.concatenate([src[:ids[::3].size], src]),
               np.concatenate([np.full(ids[::3].size, zero, np.uint32), pay]))
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"delta groups kind={kind} M={max_delta}")


@pytest.mark.parametrize("ba", [32, 512, 2048])
def test_delta_orset_bucket_widths(built, ba):
    w = wl.crdt_delta(8 * 500, Kind.ORSET, rounds=8, write=True, gossip_rounds=3)
    sg, so, a, b = run_both(w, bucket_actors=ba)
    assert_same(sg, so, a, b, f"delta orset ba={ba}")


def test_delta_orset_skew_path(built):
    """One 2048-actor bucket with ~4 messages per replica: over one LDS tile, the skew launch."""
    w = wl.crdt_delta(8 * 1000, Kind.ORSET, rounds=6, write=True, bucket_actors=2048)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "delta orset skew")


def test_delta_multipass(built, monkeypatch):
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    w = wl.crdt_delta(8 * 1000 + 3, Kind.ORSET, rounds=6, write=True, gossip_rounds=2)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "delta multipass")


@pytest.mark.parametrize("ranks", [2, 3])
def test_delta_loopback_sharded(built, ranks):
    """Hash-sharded replicas: DeltaPropagation rows travel with the tells between ranks."""
    from oracle import BspOracle
    from akka_amd.engine import owner
    w = wl.crdt_delta(8 * 250, Kind.ORSET, rounds=6, write=True, gossip_rounds=2, throughput=3)
    engs = [GpuEngine(EngineConfig(n_ranks=ranks, rank=r, **w.gpu_kwargs())) for r in range(ranks)]
    for e in engs:
        w.apply_to(e)
    sg = GpuEngine.group_run(engs)
    ref = BspOracle(n_ranks=ranks, **w.engine_kwargs())
    w.apply_to(ref)
    so = ref.run()
    for k in ("delivered", "dead_letters", "unhandled", "emitted", "staged", "in_flight"):
        assert getattr(sg, k) == so[k], (k, getattr(sg, k), so[k])
    wo, _ = ref.read_state()
    wg = np.zeros_like(wo)
    own_of = np.array([owner(i, 1000, ranks) for i in range(w.n_actors)])
    for e in engs:
        a, _ = e.read_state()
        own = own_of == e.cfg.rank
        wg[own] = a[own]
        e.close()
    diff = np.nonzero((wg != wo).any(axis=1))[0]
    assert diff.size == 0, diff[:10]


@pytest.mark.parametrize("kind", [Kind.GCOUNTER, Kind.PNCOUNTER])
def test_delta_counters_unbounded_log(built, kind):
    """Counter groups over 150 unsent seqNrs, some with a no-delta update (a placeholder) among
    them, then writer ticks: the counters keep each slot's last delta, so no log bound applies
    (the reference's deltaEntries map is unbounded)."""
    n = 8 * 100 + 3
    w = wl.crdt_delta(n, kind, rounds=6, write=True, ops_per_replica=150, gossip_rounds=2)
    ids = np.arange(n, dtype=np.uint32)
    dst, src, pay = w.tells
    w.tells = (np.concatenate([ids[::5], dst]), np.concatenate([src[:ids[::5].size], src]),
               np.concatenate([np.full(ids[::5].size, Op.make(Op.INCREMENT, 0), np.uint32), pay]))
    from oracle import BspOracle
    eng = GpuEngine(EngineConfig(msg_capacity=1 << 18, **w.gpu_kwargs()))
    w.apply_to(eng)
    sg = eng.run()
    ref = BspOracle(**w.engine_kwargs())
    w.apply_to(ref)
    so = ref.run()
    a, b = eng.read_state(), ref.read_state()
    eng.close()
    assert sg.in_flight == 0
    assert_same(sg, so, a, b, f"delta counters unbounded kind={kind}")


def test_delta_log_overflow_is_loud(built):
    """More than AGX_DELTA_LOG unsent ORSet seqNrs: AGX_ECAPACITY, as the oracle."""
    w = wl.crdt_delta(64, Kind.ORSET, rounds=0, write=False, ops_per_replica=70)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    with pytest.raises(Exception):
        eng.run()
    eng.close()


def test_delta_orset_converges_100k(built):
    """Size-independent property at 100k replicas: deltas plus full-state gossip converge every
    key's 8 replicas to one value, with every replica's deltaVersions at each writer's last seqNr."""
    n = 100_000
    w = wl.crdt_delta(n, Kind.ORSET, rounds=12, write=False, ops_per_replica=4, gossip_rounds=40)
    eng = GpuEngine(EngineConfig(msg_capacity=8 * n, **w.gpu_kwargs()))
    w.apply_to(eng)
    st = eng.run()
    assert st.in_flight == 0 and st.unhandled == 0 and st.dead_letters == 0
    ws, _ = eng.read_state()
    eng.close()
    data = ws[:, :260].reshape(-1, 8, 260)
    assert (data == data[:, :1]).all()
    env = ws[:, 260:272].view(np.uint32)
    assert (env[:, 8] == 4).all()


@pytest.mark.parametrize("kind", [Kind.GCOUNTER, Kind.PNCOUNTER])
def test_counter_slot_wrap_is_loud(built, kind):
    """A counter slot past 2^64 - 1: the reference's BigInt (DD/GCounter.scala:53) never wraps, the
    u64 slot would -- the engine reports AGX_ERANGE instead of a silently wrapped counter."""
    n, W = 16, 8 if kind == Kind.GCOUNTER else 16
    eng = GpuEngine(EngineConfig(n_actors=n, n_words=W, max_emit=1))
    init = np.zeros((n, W), np.uint64)
    init[3, 3] = np.uint64(0xFFFFFFFFFFFFFFF0)  # actor 3 = node 3: its own increment slot
    eng.register_range(0, n, kind, init)
    eng.tell([3], [Op.make(Op.INCREMENT, 32)])
    with pytest.raises(Exception, match="AGX_ERANGE"):
        eng.run()
    eng.close()
