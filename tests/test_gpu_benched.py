"""GPU parity at the parameters the benchmark reports (bench.py `configs`), and the
reference's golden known-answer tests run through the HIP engine itself.

Each benched configuration is run here at its own throughput / capacity / behaviour /
graph generator, at a population large enough to take the same kernel path as the
bench (multi-pass grouping above 2^20 actors, the skew launch, R = 8 sharding), and
compared bit-exactly with the BSP oracle.  Golden fixtures: tests/golden/*.json
(transcribed from the reference's specs by tests/golden/make_golden.py).
"""
import json
import pathlib

import numpy as np
import pytest

from akka_amd import workloads as wl
from akka_amd.engine import EngineConfig, GpuEngine, Kind, owner

pytestmark = pytest.mark.gpu

GOLD = pathlib.Path(__file__).resolve().parent / "golden"
COUNT_KEYS = ("delivered", "dead_letters", "unhandled", "emitted", "staged", "supersteps", "in_flight")


def _load(name):
    return json.loads((GOLD / name).read_text())


def _run_both(w, max_steps=1 << 30, bucket_actors=None, probe=None, **cfg):
    from oracle import BspOracle
    kw = w.engine_kwargs()
    kw.update(cfg)
    mcap = kw.pop("msg_capacity", 0)
    ba = w.bucket_actors if bucket_actors is None else bucket_actors
    eng = GpuEngine(EngineConfig(msg_capacity=mcap, bucket_actors=ba, **kw))
    w.apply_to(eng)
    sg = eng.run(max_steps)
    wg, ag = eng.read_state()
    if probe is not None:
        probe(eng)
    eng.close()
    ref = BspOracle(**kw)
    w.apply_to(ref)
    so = ref.run(max_steps)
    wo, ao = ref.read_state()
    ref.close()
    return sg, so, (wg, ag), (wo, ao)


def _assert_same(sg, so, a, b, name):
    for k in COUNT_KEYS:
        assert getattr(sg, k) == so[k], f"{name}: {k} gpu={getattr(sg, k)} oracle={so[k]}"
    assert np.array_equal(a[1], b[1]), f"{name}: alive differs"
    diff = np.nonzero((a[0] != b[0]).any(axis=1))[0]
    assert diff.size == 0, f"{name}: state differs at {diff[:10]}"


# ------------------------------------------------------------------ golden KATs through the engine
def test_mailbox_kats_on_gpu(built):
    """MailboxConfigSpec (akka-actor-tests/.../dispatch/MailboxConfigSpec.scala:47-66,84-116):
    capacity C => exactly the (C+1)th.. enqueues are dead letters, FIFO survivors."""
    for case in _load("mailbox_kat.json")["cases"]:
        eng = GpuEngine(EngineConfig(n_actors=1, throughput=case["throughput"], capacity=case["capacity"], n_words=2))
        eng.register_range(0, 1, Kind.COUNTER)
        eng.tell(np.zeros(len(case["payloads"]), np.uint32), case["payloads"])
        st = eng.run()
        w, _ = eng.read_state()
        eng.close()
        assert st.delivered == case["delivered"], case["name"]
        assert st.dead_letters == case["dead_letters"], case["name"]
        assert int(w[0, 1]) == case["sum"], case["name"]
        if "supersteps" in case:
            assert st.supersteps == case["supersteps"], case["name"]


def test_pingpong_kats_on_gpu(built):
    """BenchmarkActors.PingPong invocation counts (pingpong_kat.json)."""
    for c in _load("pingpong_kat.json")["cases"]:
        w = wl.ping_pong(c["pairs"], c["messages_per_pair"], c["throughput"], c["in_flight"])
        eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
        w.apply_to(eng)
        st = eng.run()
        eng.close()
        assert st.delivered == c["delivered"] and st.dead_letters == c["dead_letters"], c


def test_ring_kats_on_gpu(built):
    for c in _load("ring_kat.json")["cases"]:
        w = wl.token_ring(c["n"], c["hops"])
        eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
        w.apply_to(eng)
        st = eng.run()
        words, alive = eng.read_state()
        eng.close()
        assert st.delivered == c["delivered"] and st.supersteps == c["supersteps"], c
        assert (words[:, 0] == c["count"]).all() and alive.all(), c


@pytest.mark.parametrize("C", [0, 3])
def test_throughput_zero_behaves_as_one(built, C):
    """throughput = 0 drains one message per mailbox run: the code clamps to max(throughput, 1)
    (akka-actor/src/main/scala/akka/dispatch/Mailbox.scala:261), not "drain until empty"."""
    w = wl.mixed(3000, seed=17 + C, throughput=0, capacity=C)
    sg, so, a, b = _run_both(w)
    _assert_same(sg, so, a, b, f"T=0 C={C}")
    w1 = wl.mixed(3000, seed=17 + C, throughput=1, capacity=C)
    s1, _, a1, _ = _run_both(w1)
    assert (sg.delivered, sg.dead_letters, sg.supersteps) == (s1.delivered, s1.dead_letters, s1.supersteps)
    assert np.array_equal(a[0], a1[0])


# ------------------------------------------------------------------ C5 as benched
@pytest.mark.parametrize("ring_slots", [None, "8192", "5"])
def test_c5_power_law_bounded_as_benched(built, monkeypatch, ring_slots):
    """bench C5: FORWARD_RR over the device-generated R-MAT power-law graph, BoundedMailbox(64),
    throughput 5, one message per actor with ttl 15 -- at 2.2M actors (> 2^20: the multi-pass
    grouping + in-place backlog path of the 100M bench) and the bench's 2 + 10 superstep window,
    then to quiescence.  ring_slots: as benched (None: no ring pool, the backlog arena), the
    bounded-mailbox ring pool (8192 slots), or 5 slots (ring and backlog buckets side by side)."""
    if ring_slots is not None:
        monkeypatch.setenv("AGX_RING_SLOTS", ring_slots)
    w = wl.power_law_forward(2_200_000, ttl=15, capacity=64, throughput=5, device_graph=True)
    rings = []
    sg, so, a, b = _run_both(w, max_steps=12, probe=lambda e: rings.append(e.ring_buckets()))
    _assert_same(sg, so, a, b, "C5 12 supersteps")
    assert sg.dead_letters > 0 and sg.in_flight > 0
    if ring_slots is None:
        assert rings[0] == 0, rings
    elif ring_slots == "8192":
        assert rings[0] > 5, rings
    else:
        assert 0 < rings[0] <= int(ring_slots), rings
    sg, so, a, b = _run_both(w)
    _assert_same(sg, so, a, b, "C5 to quiescence")


def test_c5_power_law_cap1000_as_benched(built):
    """bench C5's second mailbox setting: the reference's default capacity 1000 --
    at 2.2M actors, the bench window then to quiescence (the ring apply is not used at this shape: its
    rings of 1000 slots per actor would not fit; the backlog arena and the skew pre-pass take the hubs)."""
    w = wl.power_law_forward(2_200_000, ttl=15, capacity=1000, throughput=5, device_graph=True)
    sg, so, a, b = _run_both(w, max_steps=12)
    _assert_same(sg, so, a, b, "C5 cap 1000, 12 supersteps")
    assert sg.in_flight > 0
    sg, so, a, b = _run_both(w)
    _assert_same(sg, so, a, b, "C5 cap 1000 to quiescence")


@pytest.mark.parametrize("ranks", [8])
def test_c5_power_law_sharded_loopback(built, ranks):
    """C5 hash-sharded over 8 ranks (ShardRegion extractShardId ownership, loopback exchange)."""
    from oracle import BspOracle
    w = wl.power_law_forward(300_000, ttl=10, capacity=64, throughput=5, device_graph=True)
    engs = [GpuEngine(EngineConfig(n_ranks=ranks, rank=r, **w.gpu_kwargs())) for r in range(ranks)]
    for e in engs:
        w.apply_to(e)
    sg = GpuEngine.group_run(engs)
    ref = BspOracle(n_ranks=ranks, **w.engine_kwargs())
    w.apply_to(ref)
    so = ref.run()
    for k in ("delivered", "dead_letters", "unhandled", "emitted", "staged", "in_flight"):
        assert getattr(sg, k) == so[k], (k, getattr(sg, k), so[k])
    wo, ao = ref.read_state()
    own_of = np.array([owner(i, 1000, ranks) for i in range(w.n_actors)])
    wg = np.zeros_like(wo)
    ag = np.zeros_like(ao)
    for e in engs:
        x, y = e.read_state()
        own = own_of == e.cfg.rank
        wg[own] = x[own]
        ag[own] = y[own]
        e.close()
    assert np.array_equal(wg, wo) and np.array_equal(ag, ao)
    assert sg.dead_letters > 0


# ------------------------------------------------------------------ C4 ORSet on the skew path
@pytest.mark.parametrize("ba", [512, 2048])
def test_c4_orset_100k(built, ba):
    """bench C4 ORSet at 100k replicas: 3 messages per replica per superstep (tick + 2 gossips).
    With the workload's 512-replica buckets they fit the fast path's 2048-message tile; with
    2048-replica buckets every bucket takes the skew launch."""
    w = wl.crdt_gossip(100_000, Kind.ORSET, rounds=5)
    sg, so, a, b = _run_both(w, bucket_actors=ba)
    _assert_same(sg, so, a, b, f"C4 ORSet 100k bucket {ba}")
    assert sg.in_flight == 0 and sg.unhandled == 0


def test_c4_gcounter_as_benched_window(built):
    """bench C4 GCounter shape (fanout 2, throughput 5) at 200k replicas, partial window."""
    w = wl.crdt_gossip(200_000, Kind.GCOUNTER, rounds=40)
    sg, so, a, b = _run_both(w, max_steps=28)
    _assert_same(sg, so, a, b, "C4 GCounter 28 supersteps")


# ------------------------------------------------------------------ C3
@pytest.mark.parametrize("variant", ["tree", "steady"])
def test_c3_zipf_unbounded_shapes(built, variant):
    """SURVEY.md §8(d)'s C3 shapes with an UNBOUNDED mailbox (the bench's own parameters are in
    test_c3_zipf_as_benched): Zipf(1.1) FANOUT, 1/64 roots, throughput 5; 'tree' = k 4, ttl 3;
    'steady' = k 1, ttl 64 -- 2M actors, 24 supersteps."""
    if variant == "tree":
        w = wl.zipf_fanout(2_000_000, k=4, ttl=3, root_every=64, throughput=5)
    else:
        w = wl.zipf_fanout(2_000_000, k=1, ttl=64, root_every=64, throughput=5)
    sg, so, a, b = _run_both(w, max_steps=24)
    _assert_same(sg, so, a, b, f"C3 unbounded {variant}")


@pytest.mark.parametrize("variant", ["steady", "tree"])
def test_c3_zipf_as_benched(built, variant):
    """bench.py's two C3 lines at their own parameters, at 2.2M actors (> 2^20: the multi-pass
    grouping, in-place backlog, tiny-wave and skewed-bucket paths of the 10M bench):
    'steady' = zipf_fanout(k=1, ttl=15, root_every=1, BoundedMailbox(1000)), throughput 5, timed
    from superstep 2 for 10 supersteps; 'tree' = zipf_fanout(k=4, ttl=3, root_every=64,
    BoundedMailbox(1000)), timed from superstep 0 for 8.  Checked after the bench's window and
    again to quiescence (the hot actors' bounded backlogs drain at 5 per superstep)."""
    if variant == "steady":
        w, window = wl.zipf_fanout(2_200_000, k=1, ttl=15, root_every=1, capacity=1000), 12
    else:
        w, window = wl.zipf_fanout(2_200_000, k=4, ttl=3, root_every=64, capacity=1000), 8
    assert w.throughput == 5 and w.capacity == 1000
    sg, so, a, b = _run_both(w, max_steps=window)
    _assert_same(sg, so, a, b, f"C3 {variant} bench window")
    assert sg.dead_letters > 0 and sg.in_flight > 0  # hot actors tail-drop at 1000 and keep backlogs
    sg, so, a, b = _run_both(w)
    _assert_same(sg, so, a, b, f"C3 {variant} to quiescence")
    assert sg.in_flight == 0


# ------------------------------------------------------------------ 8-way sharding (loopback)
def _run_sharded(w, ranks):
    from oracle import BspOracle
    engs = [GpuEngine(EngineConfig(n_ranks=ranks, rank=r, **w.gpu_kwargs())) for r in range(ranks)]
    for e in engs:
        w.apply_to(e)
    sg = GpuEngine.group_run(engs)
    ref = BspOracle(n_ranks=ranks, **w.engine_kwargs())
    w.apply_to(ref)
    so = ref.run()
    wo, ao = ref.read_state()
    ref.close()
    own_of = np.array([owner(i, 1000, ranks) for i in range(w.n_actors)])
    wg = np.zeros_like(wo)
    ag = np.zeros_like(ao)
    for e in engs:
        x, y = e.read_state()
        own = own_of == e.cfg.rank
        wg[own] = x[own]
        ag[own] = y[own]
        e.close()
    return sg, so, (wg, ag), (wo, ao)


@pytest.mark.parametrize("case", ["zipf", "zipf_bounded", "orset", "orset_delta", "gcounter_delta"])
def test_sharded_8_ranks(built, case):
    """C3 Zipf fan-out and C4 ORSet (full-state and delta-CRDT) hash-sharded over 8 ranks
    (ShardRegion extractShardId ownership, SH/ShardRegion.scala:154-158; loopback exchange of the
    RCCL path's kernels), bit-exact against the oracle in the sharded canonical order."""
    w = {
        "zipf": lambda: wl.zipf_fanout(60_000, k=4, ttl=3, root_every=16, throughput=3),
        "zipf_bounded": lambda: wl.zipf_fanout(60_000, k=1, ttl=8, root_every=1, capacity=64),
        "orset": lambda: wl.crdt_gossip(4_000, Kind.ORSET, rounds=8, throughput=2),
        "orset_delta": lambda: wl.crdt_delta(8 * 400, Kind.ORSET, rounds=8, write=True, gossip_rounds=2,
                                             throughput=3),
        "gcounter_delta": lambda: wl.crdt_delta(8 * 400, Kind.GCOUNTER, rounds=8, write=True, throughput=3),
    }[case]()
    sg, so, a, b = _run_sharded(w, 8)
    for k in ("delivered", "dead_letters", "unhandled", "emitted", "staged", "in_flight"):
        assert getattr(sg, k) == so[k], f"{case}: {k} gpu={getattr(sg, k)} oracle={so[k]}"
    assert np.array_equal(a[1], b[1]), f"{case}: alive differs"
    diff = np.nonzero((a[0] != b[0]).any(axis=1))[0]
    assert diff.size == 0, f"{case}: state differs at {diff[:10]}"
    assert sg.delivered > 0


# ------------------------------------------------------------------ skewed-bucket partitions
def test_skew_parts_many_saturated_buckets(built):
    """Many skewed buckets just over one LDS tile, each with a backlog, on a multi-pass population
    with a small message capacity: k_skew_plan rounds every bucket's backlog parts and new-mail
    parts up separately, so the parts reach budget + 2 x (skewed buckets) -- the pc table must
    hold them (k_skew_scan wrote past it).  800 of 1075 buckets hold 2048 + 60 tokens
    that RING-forward to themselves (stride 0) at throughput 1: every superstep each of them has
    a 60-message backlog and 2048 new messages."""
    n, hot, extra, hops = 2_200_000, 800, 60, 5
    base = np.arange(hot * 2048, dtype=np.uint32)
    dup = (np.arange(hot, dtype=np.uint32)[:, None] * 2048 + np.arange(extra, dtype=np.uint32)[None, :] * 31).reshape(-1)
    dst = np.concatenate([base, dup])
    pay = np.full(dst.size, hops, np.uint32)
    src = np.full(dst.size, 0xFFFFFFFF, np.uint32)
    w = wl.Workload("skew_parts", n, 1, 1, 1, 0, [(0, n, Kind.RING, None)], ring_stride=0, tells=(dst, src, pay))
    sg, so, a, b = _run_both(w, msg_capacity=3_200_000)
    _assert_same(sg, so, a, b, "skew parts")
    assert sg.delivered == dst.size * (hops + 1)


def test_c1_ping_pong_as_benched(built):
    """bench C1 shape: 1000 pairs, 100 in flight per pair, throughput 50, short messages-per-pair
    so the oracle finishes in seconds; run to completion -- with the workload's 32-actor buckets
    (fast path) and with one 2048-actor bucket (the skew path)."""
    w = wl.ping_pong(1000, messages_per_pair=2_000, throughput=50)
    sg, so, a, b = _run_both(w, msg_capacity=1 << 20)
    _assert_same(sg, so, a, b, "C1")
    sg, so, a, b = _run_both(w, msg_capacity=1 << 20, bucket_actors=2048)
    _assert_same(sg, so, a, b, "C1")
