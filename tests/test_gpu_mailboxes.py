"""GPU parity of per-actor mailbox types and of the reply path (the HIP engine through the C ABI vs
the BSP oracle, bit-exact): a population with bounded-capacity:2 / unbounded / bounded-capacity:16 /
default mailboxes in one dispatcher (Mailboxes.lookupConfigurator per actor, akka-actor/src/main/
scala/akka/dispatch/Mailboxes.scala:204-260), host-side senders answered through the outbox
(ActorCell.scala:583-587), on the fused, multi-pass, tiny-wave, skew and sharded paths."""
import numpy as np
import pytest

from akka_amd import workloads as wl
from akka_amd.engine import EngineConfig, GpuEngine, owner
from tests.test_gpu_parity import COUNT_KEYS

pytestmark = pytest.mark.gpu


def _per_sender(d, s, p):
    """outbox -> canonical per-sender sequences (a stable sort by sender keeps each sender's order)"""
    o = np.argsort(s, kind="stable")
    return np.stack([s[o], d[o], p[o]])


def _run(w, ranks=1, max_steps=1 << 30, probe=None, **cfg):
    from oracle import BspOracle
    ba = cfg.pop("bucket_actors", w.bucket_actors)
    kw = dict(w.engine_kwargs(), **cfg)
    engs = [GpuEngine(EngineConfig(n_ranks=ranks, rank=r, bucket_actors=ba, **kw)) for r in range(ranks)]
    for e in engs:
        w.apply_to(e)
    sg = engs[0].run(max_steps) if ranks == 1 else GpuEngine.group_run(engs, max_steps)
    outs = [e.take_outbound() for e in engs]
    if probe is not None:
        probe(engs[0])
    ref = BspOracle(n_ranks=ranks, **kw)
    w.apply_to(ref)
    so = ref.run(max_steps)
    od = ref.take_outbound()
    wo, ao = ref.read_state()
    ref.close()
    own_of = np.array([owner(i, 1000, ranks) for i in range(w.n_actors)]) if ranks > 1 else np.zeros(w.n_actors, int)
    wg, ag = np.zeros_like(wo), np.zeros_like(ao)
    for e in engs:
        x, y = e.read_state()
        own = own_of == e.cfg.rank
        wg[own], ag[own] = x[own], y[own]
        e.close()
    keys = COUNT_KEYS if ranks == 1 else tuple(k for k in COUNT_KEYS if k != "supersteps")
    for k in keys:
        assert getattr(sg, k) == so[k], f"{k}: gpu={getattr(sg, k)} oracle={so[k]}"
    assert np.array_equal(ag, ao), "alive differs"
    diff = np.nonzero((wg != wo).any(axis=1))[0]
    assert diff.size == 0, f"state differs at {diff[:10]}"
    d = np.concatenate([o[0] for o in outs])
    s = np.concatenate([o[1] for o in outs])
    p = np.concatenate([o[2] for o in outs])
    assert d.size == od[0].size and d.size > 0, (d.size, od[0].size)
    assert np.array_equal(_per_sender(d, s, p), _per_sender(*od)), "outbox differs"
    return sg


@pytest.mark.parametrize("T,C", [(1, 0), (3, 0), (5, 4), (50, 1)])
def test_mailbox_classes_fused(built, T, C):
    _run(wl.mailbox_mix(6000, seed=T + C, throughput=T, capacity=C))


@pytest.mark.parametrize("tiny", ["0", "128"])
def test_mailbox_classes_multipass(built, monkeypatch, tiny):
    """multi-pass grouping (narrow radix digits), wave path on / off, skewed buckets (32-actor buckets)"""
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    monkeypatch.setenv("AGX_TINY", tiny)
    _run(wl.mailbox_mix(30_000, seed=5, throughput=2, capacity=6))
    _run(wl.mailbox_mix(30_000, seed=6, throughput=3, capacity=0), bucket_actors=32)


@pytest.mark.parametrize("slots", ["8192", "3"])
def test_bounded_rings_multipass(built, monkeypatch, slots):
    """Every mailbox class bounded: buckets that reach the skew path keep their actors' queued
    messages in per-actor rings (a 3-slot pool: ring and backlog buckets side by side), with stops,
    replies to host senders and capacity classes 2 / 5 / 16 / 40 in one population."""
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    monkeypatch.setenv("AGX_RING_SLOTS", slots)
    rings = []
    w = wl.mailbox_mix(30_000, seed=9, throughput=3, capacity=5, classes={1: 2, 2: 40, 3: 16})
    # a hot spot: 6000 more tells to the 64 actors from 7500 (class 2) -- two buckets over one LDS tile
    rng = np.random.default_rng(9)
    dst, src, pay = w.tells
    hd = rng.integers(7500, 7564, 6000).astype(np.uint32)
    w.tells = (np.concatenate([dst, hd]), np.concatenate([src, rng.integers(0, 30_000, 6000).astype(np.uint32)]),
               np.concatenate([pay, rng.integers(0, 12, 6000).astype(np.uint32)]))
    _run(w, bucket_actors=32, probe=lambda e: rings.append(e.ring_buckets()))
    assert 0 < rings[0] <= int(slots), rings
    _run(w, bucket_actors=32, max_steps=3)  # stopped with messages in the rings


def test_rings_fix_mailbox_classes(built, monkeypatch):
    """Once the rings are allocated (first run), a class they cannot hold is refused loudly."""
    from akka_amd._lib import AgxError
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    monkeypatch.setenv("AGX_RING_SLOTS", "8192")
    w = wl.mailbox_mix(30_000, seed=3, throughput=3, capacity=5, classes={1: 2, 2: 40, 3: 16})
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    eng.run(2)
    eng.set_mailbox_class(1, 30)  # within the ring capacity (40)
    with pytest.raises(AgxError):
        eng.set_mailbox_class(2, 0)
    with pytest.raises(AgxError):
        eng.set_mailbox_class(3, 41)
    eng.close()


@pytest.mark.parametrize("ranks", [2, 5])
def test_mailbox_classes_sharded(built, ranks):
    _run(wl.mailbox_mix(5000, seed=ranks, throughput=2, capacity=3), ranks=ranks)


def test_outbox_capacity_is_loud(built):
    """More outbound tells than the outbox holds between two takes: agx_take_outbound reports
    AGX_ECAPACITY once (not a silent drop) and the engine stays usable -- agx_run itself does not
    fail, the kept tells are handed out by the next take, and later runs and takes work."""
    from akka_amd._lib import AgxError
    w = wl.mailbox_mix(4096, seed=1, throughput=5)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    eng.set_outbound(w.n_actors, 32, capacity=4)
    st = eng.run(3)  # the run itself succeeds: the overflow belongs to the outbox, not the engine
    with pytest.raises(AgxError, match="outbound tells dropped"):
        eng.take_outbound()
    d, s, p = eng.take_outbound()  # reported once: the 4 kept tells come out now
    assert d.size == 4 and (d >= w.n_actors).all()
    st2 = eng.run()
    assert st2.delivered >= st.delivered
    try:
        eng.take_outbound()
    except AgxError:
        pass  # another overflow during the second run is reported the same way
    eng.take_outbound()
    eng.close()


def test_outbox_overflow_parity(built):
    """Outbox overflow, engine against the oracle (the oracle used to halt its run): both
    keep running, both report the drop at the same take, the counters and final states agree, and
    the take after the report hands out the capacity's worth of kept tells on both.  (Which tells are
    kept differs: the device keeps the first appends to land, the oracle the first in canonical order.)"""
    from akka_amd._lib import AgxError
    from oracle import BspOracle
    from oracle.oracle import OutboxOverflow
    w = wl.mailbox_mix(4096, seed=1, throughput=5)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    ref = BspOracle(**w.engine_kwargs())
    for t in (eng, ref):
        w.apply_to(t)
        t.set_outbound(w.n_actors, 32, capacity=4)
    sg, so = eng.run(3), ref.run(3)
    for k in COUNT_KEYS:
        assert getattr(sg, k) == so[k], (k, getattr(sg, k), so[k])
    with pytest.raises(AgxError, match="outbound tells dropped"):
        eng.take_outbound()
    with pytest.raises(OutboxOverflow):
        ref.take_outbound()
    assert eng.take_outbound()[0].size == ref.take_outbound()[0].size == 4
    sg, so = eng.run(), ref.run()
    for k in COUNT_KEYS:
        assert getattr(sg, k) == so[k], (k, getattr(sg, k), so[k])
    assert np.array_equal(eng.read_state()[0], ref.read_state()[0])
    eng.close()


def test_outbox_capacity_change_keeps_pending(built):
    """agx_set_outbound with a new capacity while tells wait in the device outbox: they move to the
    host queue first and come out of the next take, in order (they were lost)."""
    w = wl.mailbox_mix(4096, seed=1, throughput=5)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    eng.set_outbound(w.n_actors, 32, capacity=1 << 16)
    eng.run(1)
    ref = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(ref)
    ref.set_outbound(w.n_actors, 32, capacity=1 << 16)
    ref.run(1)
    want = ref.take_outbound()
    ref.close()
    eng.set_outbound(w.n_actors, 32, capacity=1 << 17)
    got = eng.take_outbound()
    eng.close()
    assert want[0].size > 0
    # (different senders interleave arbitrarily in the outbox: compare as sets of envelopes)
    assert np.array_equal(_per_sender(*got), _per_sender(*want))


def test_set_mailbox_rejects_unconfigured_class(built):
    from akka_amd._lib import AgxError
    eng = GpuEngine(EngineConfig(n_actors=64))
    with pytest.raises(AgxError):
        eng.set_mailbox(0, 8, 3)
    with pytest.raises(AgxError):
        eng.set_mailbox_class(0, 5)  # class 0 is agx_cfg.capacity
    with pytest.raises(AgxError):
        eng.set_outbound(10, 4)      # host ids inside the population
    eng.close()
