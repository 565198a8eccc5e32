"""GPU parity: the HIP engine (through the C ABI) vs the BSP oracle, bit-exact.

Every case runs the same seeded workload through GpuEngine and BspOracle and
compares delivered / dead-letter / unhandled / emitted / staged / superstep
counts and the final state of every actor.
"""
import numpy as np
import pytest

from akka_amd import workloads as wl
from akka_amd.engine import EngineConfig, GpuEngine, Kind, NO_SENDER

pytestmark = pytest.mark.gpu

COUNT_KEYS = ("delivered", "dead_letters", "unhandled", "emitted", "staged", "supersteps", "in_flight")


def run_both(w, max_steps=1 << 30, bucket_actors=None, **cfg):
    from oracle import BspOracle
    kw = w.engine_kwargs()
    kw.update(cfg)
    ba = w.bucket_actors if bucket_actors is None else bucket_actors
    eng = GpuEngine(EngineConfig(bucket_actors=ba, **kw))
    w.apply_to(eng)
    sg = eng.run(max_steps)
    ref = BspOracle(**kw)
    w.apply_to(ref)
    so = ref.run(max_steps)
    wg, ag = eng.read_state()
    wo, ao = ref.read_state()
    eng.close()
    return sg, so, (wg, ag), (wo, ao)


def assert_same(sg, so, stg, sto, name=""):
    for k in COUNT_KEYS:
        assert getattr(sg, k) == so[k], f"{name}: {k} gpu={getattr(sg, k)} oracle={so[k]}"
    assert np.array_equal(stg[1], sto[1]), f"{name}: alive differs"
    diff = np.nonzero((stg[0] != sto[0]).any(axis=1))[0]
    assert diff.size == 0, f"{name}: state differs at {diff[:10]} gpu={stg[0][diff[:3]]} oracle={sto[0][diff[:3]]}"


@pytest.mark.parametrize("n,hops", [(1, 5), (7, 3), (4096, 8), (100_000, 12)])
def test_ring(built, n, hops):
    w = wl.token_ring(n, hops)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "ring")
    assert sg.delivered == n * (hops + 1)


@pytest.mark.parametrize("T", [1, 2, 5, 50])
@pytest.mark.parametrize("C", [0, 1, 3, 16])
def test_mixed_throughput_capacity(built, T, C):
    w = wl.mixed(3000, seed=T * 31 + C, throughput=T, capacity=C)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"mixed T={T} C={C}")
    assert sg.staged + sg.emitted == sg.delivered + sg.dead_letters + sg.in_flight


def test_partial_run_and_resume(built):
    """agx_run with a superstep budget, then resume: same as one long run."""
    from oracle import BspOracle
    w = wl.mixed(2000, seed=9, throughput=2, capacity=5)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    ref = BspOracle(**w.engine_kwargs())
    w.apply_to(ref)
    for budget in (1, 2, 3, 5, 1000):
        sg = eng.run(budget)
        so = ref.run(budget)
        for k in COUNT_KEYS:
            assert getattr(sg, k) == so[k], (budget, k)
        assert np.array_equal(eng.read_state()[0], ref.read_state()[0])
    # stage more tells between runs (appended after the pending mail)
    dst = np.arange(0, 2000, 3, dtype=np.uint32)
    pay = (dst % 5).astype(np.uint32)
    eng.tell(dst, pay, dst[::-1].copy())
    ref.tell(dst, pay, dst[::-1].copy())
    sg, so = eng.run(), ref.run()
    for k in COUNT_KEYS:
        assert getattr(sg, k) == so[k], k
    assert np.array_equal(eng.read_state()[0], ref.read_state()[0])
    eng.close()


@pytest.mark.parametrize("budgets", [(1000,), (3, 4, 1000)])
@pytest.mark.parametrize("strict", [True, False])
def test_strict_replay_recovery(built, monkeypatch, strict, budgets):
    """Fused graphs without skew launches ("strict" replays): Zipf fan-out (k = 4) multiplies the
    mail each hop until a hot bucket's inbox passes one LDS tile a few supersteps in -- in the
    middle of an 8-superstep replay (one long run) or while single-superstep replays are in flight
    (short budgets).  The rest of that replay is void, the deferred skew launch runs, the run goes
    on with the full graphs; every budget must match the oracle (and the full-graph mode)."""
    from oracle import BspOracle
    if not strict:
        monkeypatch.setenv("AGX_NO_STRICT", "1")
    w = wl.zipf_fanout(20_000, k=4, ttl=6, root_every=256, throughput=1000)
    eng = GpuEngine(EngineConfig(msg_capacity=1 << 20, **w.gpu_kwargs()))  # (234 K in flight at the peak)
    w.apply_to(eng)
    ref = BspOracle(**w.engine_kwargs())
    w.apply_to(ref)
    for budget in budgets:
        sg = eng.run(budget)
        so = ref.run(budget)
        for k in COUNT_KEYS:
            assert getattr(sg, k) == so[k], (budget, k, getattr(sg, k), so[k])
        assert np.array_equal(eng.read_state()[0], ref.read_state()[0]), budget
    assert sg.in_flight == 0
    eng.close()


@pytest.mark.parametrize("mpp,T,inflight", [(300, 50, None), (333, 50, None), (101, 7, 9), (64, 50, 1)])
def test_ping_pong(built, mpp, T, inflight):
    """PingPong pairs to their stop (the message-parallel drain: the stopping message at the start,
    in the middle and past the end of a run; throughput caps below and above the run lengths)."""
    w = wl.ping_pong(pairs=200, messages_per_pair=mpp, throughput=T, in_flight=inflight)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"ping_pong mpp={mpp} T={T} inflight={inflight}")


def test_zipf_fanout(built):
    w = wl.zipf_fanout(20_000, k=4, ttl=3, root_every=16, throughput=1000)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "zipf_fanout")


def test_power_law_bounded(built):
    w = wl.power_law_forward(20_000, ttl=6, capacity=8, throughput=5)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "power_law")
    assert sg.dead_letters > 0


def test_empty_and_unknown(built):
    w = wl.token_ring(64, 0)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "hop0")
    eng = GpuEngine(EngineConfig(n_actors=16, n_words=1))
    eng.register_range(0, 16, Kind.COUNTER)
    assert eng.run().delivered == 0  # nothing staged: quiescent immediately
    eng.tell([3, 99, 0xFFFFFFFF], [1, 2, 3])
    st = eng.run()
    assert st.delivered == 1 and st.dead_letters == 2
    eng.close()


@pytest.mark.parametrize("ranks", [2, 3, 8])
def test_loopback_sharded(built, ranks):
    """Hash-sharded over `ranks` virtual GPUs (one device, loopback exchange):
    bit-exact vs the oracle in the sharded canonical order."""
    from oracle import BspOracle
    w = wl.mixed(3000, seed=ranks, throughput=2, capacity=6)
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
    wg = np.zeros_like(wo)
    ag = np.zeros_like(ao)
    for e in engs:
        a, b = e.read_state()  # only owned ids are written
        from akka_amd.engine import owner
        own = np.array([owner(i, 1000, ranks) == e.cfg.rank for i in range(w.n_actors)])
        wg[own] = a[own]
        ag[own] = b[own]
    assert np.array_equal(wg, wo) and np.array_equal(ag, ao)
    for e in engs:
        e.close()


def test_ring_1m_properties(built):
    """Full C2 size (1M actors): size-independent properties."""
    n, hops = 1_000_000, 16
    w = wl.token_ring(n, hops)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    st = eng.run()
    words, alive = eng.read_state()
    assert st.delivered == n * (hops + 1) and st.dead_letters == 0 and st.supersteps == hops + 1
    assert (words[:, 0] == hops + 1).all() and alive.all()
    eng.close()


# ------------------------------------------------------------------ CRDT replicas (C4; rows a9, a10)
@pytest.mark.parametrize("kind", [Kind.GCOUNTER, Kind.PNCOUNTER, Kind.ORSET])
@pytest.mark.parametrize("T,C", [(5, 0), (1, 0), (2, 3)])
def test_crdt_gossip(built, kind, T, C):
    """Full-state gossip rounds: merges, snapshot rows, rows forwarded for queued
    gossips (T=1), tail-dropped gossips (C=3) — bit-exact vs the oracle."""
    w = wl.crdt_gossip(3000, kind, rounds=12, throughput=T, capacity=C)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"crdt kind={kind} T={T} C={C}")


@pytest.mark.parametrize("T,C", [(3, 0), (1, 4)])
def test_crdt_mixed_protocols(built, T, C):
    """CRDT replicas beside classic kinds: gossips to a non-CRDT actor and ops of the
    wrong data type are Behaviors.unhandled."""
    w = wl.crdt_mixed(5000, rounds=5, throughput=T, capacity=C)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"crdt_mixed T={T} C={C}")
    assert sg.unhandled > 0


def test_crdt_gcounter_1m_converges(built):
    """C4 size (1M replicas): every replica converges to the join of the 8 writers."""
    n, rounds = 1_000_000, 40
    w = wl.crdt_gossip(n, Kind.GCOUNTER, rounds=rounds)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    st = eng.run()
    words, _ = eng.read_state()
    eng.close()
    ops = wl.crdt_ops(8, Kind.GCOUNTER, 16)
    exp = (ops & 0xFFFFFF).astype(np.uint64).sum(axis=1)
    assert st.in_flight == 0 and st.unhandled == 0 and st.delivered == 8 * 16 + 3 * n * rounds
    assert (words == exp[None, :]).all()


@pytest.mark.parametrize("ranks", [2, 5])
@pytest.mark.parametrize("workload", ["orset", "mixed"])
def test_crdt_loopback_sharded(built, ranks, workload):
    """C4 hash-sharded: snapshot rows travel with the gossips between ranks."""
    from oracle import BspOracle
    from akka_amd.engine import owner
    if workload == "orset":
        w = wl.crdt_gossip(2000, Kind.ORSET, rounds=8, throughput=2, capacity=0)
    else:
        w = wl.crdt_mixed(3000, rounds=4, throughput=2, capacity=5)
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
    wg = np.zeros_like(wo)
    own_of = np.array([owner(i, 1000, ranks) for i in range(w.n_actors)])
    for e in engs:
        a, _ = e.read_state()
        own = own_of == e.cfg.rank
        wg[own] = a[own]
        e.close()
    diff = np.nonzero((wg != wo).any(axis=1))[0]
    assert diff.size == 0, diff[:10]


# ------------------------------------------------------------------ multi-pass bucket grouping
# Populations above 2^20 actors per rank group mail by bucket with more than one radix
# pass (and find bucket starts with k_bucket_bounds).  AGX_RADIX_BITS narrows the digits
# so that the same code path runs at oracle-friendly sizes.
MULTIPASS_CASES = {
    "ring": lambda: wl.token_ring(100_000, 9),
    "mixed": lambda: wl.mixed(30_000, seed=4, throughput=2, capacity=5),
    "zipf": lambda: wl.zipf_fanout(40_000, k=4, ttl=3, root_every=32, throughput=1000),
    "power_law": lambda: wl.power_law_forward(50_000, ttl=5, capacity=8, throughput=5),
    "crdt": lambda: wl.crdt_mixed(20_000, rounds=4, throughput=2, capacity=5),
    # (ORSet-only full state: the wave path, orset_protocol + k_orset_merge, with sparse snapshot rows)
    "orset": lambda: wl.crdt_gossip(20_000, Kind.ORSET, rounds=6),
}


@pytest.mark.parametrize("ring", ["1", "0"])
@pytest.mark.parametrize("bits,G", [(2, 1), (3, 5), (9, 3)])
@pytest.mark.parametrize("case", sorted(MULTIPASS_CASES))
def test_multipass_grouping(built, monkeypatch, bits, G, case, ring):
    """AGX_UNIT_G groups G buckets per first-pass histogram column (as at 100M actors); bounded
    cases with ring apply (AGX_RING_APPLY=1) and with the backlog arena (AGX_RING_APPLY=0; the
    default below a bounded capacity of 256)."""
    monkeypatch.setenv("AGX_RADIX_BITS", str(bits))
    monkeypatch.setenv("AGX_UNIT_G", str(G))
    monkeypatch.setenv("AGX_RING_APPLY", ring)
    w = MULTIPASS_CASES[case]()
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"multipass {case} bits={bits}")


@pytest.mark.parametrize("bits,G", [(2, 1), (3, 5), (9, 3)])
@pytest.mark.parametrize("case", ["crdt", "orset", "mixed", "power_law"])
def test_multipass_emitted_conservation(built, monkeypatch, bits, G, case):
    """The apply's emitted counter against the mail it actually wrote, superstep by superstep (engine
    alone, no oracle): with no host actors, staged + emitted == delivered + dead_letters + in_flight,
    where in_flight is the size of the next superstep's grouped inbox, counted independently of the
    per-block counters.  (Round 4's sparse ORSet rows in crdt_apply broke exactly this: the summed
    per-block emitted counter came out wrong while every state row matched -- DESIGN.md §7.)"""
    monkeypatch.setenv("AGX_RADIX_BITS", str(bits))
    monkeypatch.setenv("AGX_UNIT_G", str(G))
    w = MULTIPASS_CASES[case]()
    eng = GpuEngine(EngineConfig(bucket_actors=w.bucket_actors, **w.engine_kwargs()))
    w.apply_to(eng)
    try:
        for step in range(60):
            s = eng.run(1)
            assert s.staged + s.emitted == s.delivered + s.dead_letters + s.in_flight, (case, step, s)
            if s.in_flight == 0:
                break
        assert s.emitted > 0
    finally:
        eng.close()


def test_multipass_loopback_sharded(built, monkeypatch):
    from oracle import BspOracle
    from akka_amd.engine import owner
    monkeypatch.setenv("AGX_RADIX_BITS", "2")
    ranks = 3
    w = wl.mixed(30_000, seed=11, throughput=2, capacity=6)
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
    assert np.array_equal(wg, wo)


def test_ring_2m_multipass_native(built):
    """2.1M actors: the real (9-bit digit) multi-pass path, bit-exact vs the oracle."""
    w = wl.token_ring(2_100_000, 6)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "ring 2.1M")


@pytest.mark.parametrize("case", sorted(MULTIPASS_CASES))
def test_unfused_single_pass(built, monkeypatch, case):
    """AGX_NO_FUSED: the chunk-pass + apply pipeline at one radix pass (the fused
    gather-apply superstep is the default there)."""
    monkeypatch.setenv("AGX_NO_FUSED", "1")
    w = MULTIPASS_CASES[case]()
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"unfused {case}")


def test_power_law_device_graph(built):
    """agx_set_graph_rmat: device-generated R-MAT destinations equal the host generator's
    (the oracle gets the host ones), so the whole run is bit-exact."""
    w = wl.power_law_forward(40_000, ttl=6, capacity=8, throughput=5, device_graph=True)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "power_law device graph")
    assert sg.dead_letters > 0


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("case", sorted(MULTIPASS_CASES))
def test_grid_stride_apply(built, monkeypatch, fused, case):
    """AGX_APPLY_GRID: few apply blocks, each looping over many buckets (as above 8M actors),
    with skewed buckets deferred to the skew launch in between."""
    monkeypatch.setenv("AGX_APPLY_GRID", "3")
    if not fused:
        monkeypatch.setenv("AGX_NO_FUSED", "1")
    w = MULTIPASS_CASES[case]()
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"grid-stride {case} fused={fused}")


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("shape", ["steps", "dup_edges", "tiny"])
def test_zipf_index_ranges(built, shape, k):
    """The device's indexed CDF search (top 20 bits of the draw pick an index entry: the
    destination itself when the whole range has one answer, else a search range) returns the
    plain binary search's answer: thresholds on range boundaries, long runs of equal thresholds,
    0 and 0xFFFFFFFF entries, tables shorter than the index.  k = 1 takes the kernels' lockstep
    lookups (block, wave and ring launches), k = 3 the per-message one in apply_msg."""
    import dataclasses
    n = 50_000
    w = wl.zipf_fanout(n, k=k, ttl=3, root_every=7, throughput=3)
    k, seed, _, perm = w.fanout
    rng = np.random.default_rng(5)
    if shape == "steps":  # every threshold on a multiple of 2^12 (a range boundary)
        cdf = np.sort(rng.integers(0, 1 << 20, n, dtype=np.uint64) << np.uint64(12)).astype(np.uint32)
    elif shape == "dup_edges":  # few distinct values, both extremes
        cdf = np.sort(rng.choice(np.array([0, 1, 4095, 4096, 1 << 31, 0xFFFFFFFE, 0xFFFFFFFF], np.uint32), n))
    else:  # 5 targets
        cdf, perm = np.array([1 << 30, 1 << 31, 3 << 30, 0xF0000000, 0xFFFFFFFF], np.uint32), perm[:5]
    w = dataclasses.replace(w, fanout=(k, seed, cdf, perm))
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"zipf index {shape}")


# ------------------------------------------------------------------ bucket width (agx_cfg.bucket_actors)
BUCKET_CASES = {
    "mixed": lambda: wl.mixed(6000, seed=21, throughput=3, capacity=5),
    "ping_pong": lambda: wl.ping_pong(300, messages_per_pair=600, throughput=50),
    "zipf": lambda: wl.zipf_fanout(30_000, k=4, ttl=3, root_every=16, throughput=7),
    "power_law": lambda: wl.power_law_forward(30_000, ttl=6, capacity=8, throughput=5),
    "orset": lambda: wl.crdt_gossip(6000, Kind.ORSET, rounds=5),
    "crdt_mixed": lambda: wl.crdt_mixed(6000, rounds=4, throughput=2, capacity=5),
}


@pytest.mark.parametrize("ba", [32, 128, 512, 2048])
@pytest.mark.parametrize("case", sorted(BUCKET_CASES))
def test_bucket_width(built, case, ba):
    """Any bucket width gives the oracle's result (buckets only group actors for the apply)."""
    w = BUCKET_CASES[case]()
    sg, so, a, b = run_both(w, bucket_actors=ba)
    assert_same(sg, so, a, b, f"bucket {ba} {case}")


@pytest.mark.parametrize("ba", [32, 512])
@pytest.mark.parametrize("case", ["mixed", "zipf", "orset"])
def test_bucket_width_multipass(built, monkeypatch, case, ba):
    """Small buckets on the multi-pass grouping path (narrow radix digits)."""
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    w = BUCKET_CASES[case]()
    sg, so, a, b = run_both(w, bucket_actors=ba)
    assert_same(sg, so, a, b, f"multipass bucket {ba} {case}")


def test_bucket_width_rejects_bad_values(built):
    from akka_amd._lib import AgxError
    for ba in (3, 16, 48, 4096):
        with pytest.raises(AgxError):
            GpuEngine(EngineConfig(n_actors=100, bucket_actors=ba))


@pytest.mark.parametrize("launch", ["1", "0"])
@pytest.mark.parametrize("tiny", [0, 16, 128])
@pytest.mark.parametrize("ba", [32, 2048])
@pytest.mark.parametrize("case", sorted(set(MULTIPASS_CASES) - {"crdt", "orset"}))
def test_tiny_wave_path(built, monkeypatch, launch, tiny, ba, case):
    """Multi-pass supersteps: inboxes of <= AGX_TINY messages are drained by one wave (no block
    barrier), the others by the block path -- both bit-exact against the oracle (0 = block only).
    launch 1: the wave path is its own launch (k_tiny_apply) that marks the other buckets for the
    block launch; 0: no wave path, the block launch takes every bucket (AGX_TINY_LAUNCH=0)."""
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    monkeypatch.setenv("AGX_TINY", str(tiny))
    monkeypatch.setenv("AGX_TINY_LAUNCH", launch)
    monkeypatch.setenv("AGX_RING_APPLY", "0")  # (bounded cases: the backlog arena's wave / block paths)
    w = MULTIPASS_CASES[case]()
    sg, so, a, b = run_both(w, bucket_actors=ba)
    assert_same(sg, so, a, b, f"tiny={tiny} ba={ba} {case}")


@pytest.mark.parametrize("launch", ["1", "0"])
@pytest.mark.parametrize("tiny", [0, 128])
def test_tiny_wave_path_compiled(built, monkeypatch, launch, tiny):
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    monkeypatch.setenv("AGX_TINY", str(tiny))
    monkeypatch.setenv("AGX_TINY_LAUNCH", launch)
    monkeypatch.setenv("AGX_RING_APPLY", "0")
    w = wl.compiled(20_000, seed=5, throughput=2, capacity=4, builtin=True)
    sg, so, a, b = run_both(w, bucket_actors=64)
    assert_same(sg, so, a, b, f"compiled tiny={tiny}")


# ------------------------------------------------------------------ identity grouping (multi-pass, no sort)
def _ring_and_forwarders(n=120_000, seed=3):
    """a ring over [0, 100000) whose tokens never leave it (tokens on [0, 90000), 30 hops) beside
    FORWARD_RR actors on [100000, n) forwarding among themselves for 4 hops: the first supersteps'
    mail is not in destination order (radix passes), the later ones are (identity grouping)"""
    rng = np.random.default_rng(seed)
    f0 = 100_000
    deg = np.zeros(n, np.uint64)
    deg[f0:] = rng.integers(1, 6, n - f0)
    row = np.zeros(n + 1, np.uint64)
    np.cumsum(deg, out=row[1:])
    col = rng.integers(f0, n, int(row[-1])).astype(np.uint32)
    ring_dst = np.arange(0, 90_000, dtype=np.uint32)
    fw_dst = np.arange(f0, n, 3, dtype=np.uint32)
    dst = np.concatenate([ring_dst, fw_dst])
    pay = np.concatenate([np.full(ring_dst.size, 30, np.uint32), np.full(fw_dst.size, 4, np.uint32)])
    src = np.full(dst.size, NO_SENDER, np.uint32)
    return wl.Workload("ring_and_forwarders", n, 2, 1, 5, 0,
                       [(0, f0, Kind.RING, None), (f0, n - f0, Kind.FORWARD_RR, None)], ring_stride=1,
                       graph=(row, col), tells=(dst, src, pay))


@pytest.mark.parametrize("bits,ba", [(3, 0), (9, 0), (3, 32)])
def test_identity_grouping(built, monkeypatch, bits, ba):
    """Multi-pass supersteps whose tells are already in destination order skip the radix passes
    (identity grouping; a ring's wrap-around is a rotation) -- bit-exact against the oracle and
    against the same engine with identity grouping off, through transitions in both directions
    (forwarders at first; host tells staged mid-run).  ba = 32: 32-actor buckets, so the chunk
    summaries span several slices of 2048 chunks (the 10^8-actor shape)."""
    monkeypatch.setenv("AGX_RADIX_BITS", str(bits))
    if ba:
        monkeypatch.setenv("AGX_TINY", "0")  # (a wave-path bucket is never summarised: no identity)
    from oracle import BspOracle
    # (9-bit digits: the production plan, multi-pass only above 2^20 actors)
    big = bits >= 9
    for w in (wl.token_ring(1_200_000 if big else 100_000, 12), _ring_and_forwarders(1_300_000 if big else 120_000)):
        res = {}
        for ident in (True, False):
            if ident:
                monkeypatch.delenv("AGX_NO_IDENT", raising=False)
            else:
                monkeypatch.setenv("AGX_NO_IDENT", "1")
            eng = GpuEngine(EngineConfig(**dict(w.gpu_kwargs(), bucket_actors=ba or w.bucket_actors)))
            w.apply_to(eng)
            s1 = eng.run(9)
            eng.tell(np.arange(0, w.n_actors, 97, dtype=np.uint32), 2)  # a staged burst: sort path once
            s2 = eng.run()
            res[ident] = (s1, s2, eng.read_state(), eng.identity_supersteps())
            eng.close()
        ref = BspOracle(**w.engine_kwargs())
        w.apply_to(ref)
        o1 = ref.run(9)
        ref.tell(np.arange(0, w.n_actors, 97, dtype=np.uint32), 2)
        o2 = ref.run()
        st_o = ref.read_state()
        ref.close()
        for ident, (s1, s2, st, nid) in res.items():
            for k in COUNT_KEYS:
                assert getattr(s1, k) == o1[k], f"{w.name} ident={ident}: {k} after 9 supersteps"
            for k in COUNT_KEYS:
                assert getattr(s2, k) == o2[k], f"{w.name} ident={ident}: {k}"
            assert_same(s2, o2, st, st_o, f"{w.name} ident={ident}")
        assert res[False][3] == 0
        assert res[True][3] > 0, f"{w.name}: identity grouping never engaged"


# ------------------------------------------------------------------ ring apply (bounded mailboxes, agx_ring.h)
def _compiled_classes_host(n=40_000, seed=9):  # (> 8 buckets: 3-bit digits take two passes, not fused)
    """typed + built-in behaviours (one tell per message) under three bounded mailbox classes and
    the dispatcher default, with host-side senders that PINGPONG actors answer through the outbox"""
    w = wl.compiled(n, seed=seed, throughput=3, capacity=6, builtin=True)
    q = n // 4
    w.name = "compiled_classes_host"
    w.mailbox_classes = {1: 2, 2: 9, 3: 17}
    w.mailboxes = [(0, q, 1), (q, q, 2), (2 * q, q, 3)]
    w.outbound = (n, 32)
    rng = np.random.default_rng(seed + 101)
    m = n // 4
    dst, src, pay = w.tells
    w.tells = (np.concatenate([dst, rng.integers(0, n, m).astype(np.uint32)]),
               np.concatenate([src, rng.integers(n, n + 32, m).astype(np.uint32)]),
               np.concatenate([pay, rng.integers(0, 12, m).astype(np.uint32)]))
    return w


def _bounded_ring(n=50_000, hops=7, tokens=3, C=2, T=2):
    w = wl.token_ring(n, hops, throughput=T, tokens_per_actor=tokens)
    w.name, w.capacity = "bounded_ring", C
    return w


RING_APPLY_CASES = {
    "power_law_c8": lambda: wl.power_law_forward(50_000, ttl=5, capacity=8, throughput=5),
    # (C5's shape: hub buckets take more than one tile of arrivals and drain more than kBucket)
    "power_law_c64": lambda: wl.power_law_forward(60_000, ttl=14, capacity=64, throughput=5),
    "power_law_t1": lambda: wl.power_law_forward(30_000, ttl=8, capacity=3, throughput=1),
    "compiled": lambda: wl.compiled(20_000, seed=5, throughput=2, capacity=4, builtin=True),
    "classes_host": _compiled_classes_host,
    "bounded_ring": _bounded_ring,
}


def _run_profiled(w, ba, max_steps=1 << 30):
    eng = GpuEngine(EngineConfig(**dict(w.gpu_kwargs(), bucket_actors=ba or w.bucket_actors)))
    w.apply_to(eng)
    eng.profile(True)
    sg = eng.run(max_steps)
    prof = eng.profile_read()
    launches = prof.get("ring_apply", {"launches": 0})["launches"]
    st = eng.read_state()
    eng.tiny_launches = prof.get("bucket_apply_tiny", {"launches": 0})["launches"]
    return eng, sg, st, launches


@pytest.mark.parametrize("mode", ["bits3", "single_pass"])
@pytest.mark.parametrize("ba", [0, 64])
@pytest.mark.parametrize("case", sorted(RING_APPLY_CASES))
def test_ring_apply(built, monkeypatch, mode, ba, case):
    """Bounded mailboxes whose queued messages stay in per-actor rings (one k_ring_apply per
    superstep): bit-exact against the oracle and against the backlog arena (AGX_RING_APPLY=0), at
    multi-pass grouping (3-bit digits) and at one unfused pass; 64-actor buckets put several
    tiles of arrivals and drains larger than kBucket into one bucket."""
    from oracle import BspOracle
    if mode == "bits3":
        monkeypatch.setenv("AGX_RADIX_BITS", "3")
    else:
        monkeypatch.setenv("AGX_NO_FUSED", "1")
    w = RING_APPLY_CASES[case]()
    ref = BspOracle(**w.engine_kwargs())
    w.apply_to(ref)
    so = ref.run()
    sto = ref.read_state()
    ref.close()
    for ring in ("1", "0"):
        monkeypatch.setenv("AGX_RING_APPLY", ring)
        eng, sg, st, launches = _run_profiled(w, ba)
        eng.close()
        assert (launches > 0) == (ring == "1"), f"{case}: ring_apply launches {launches} with AGX_RING_APPLY={ring}"
        assert_same(sg, so, st, sto, f"{case} ring={ring}")


@pytest.mark.parametrize("capacity,rings,n", [(64, False, 60_000), (255, False, 60_000), (256, True, 60_000),
                                              (1000, True, 60_000), (1000, True, 60_001), (300, True, 30_003)])
def test_ring_apply_default(built, monkeypatch, capacity, rings, n):
    """Without AGX_RING_APPLY the ring apply is on exactly when the largest bounded capacity is
    >= 256 (deep queues: C3's BoundedMailbox(1000)), and either way bit-exact against the oracle
    (C3's FANOUT shape at 3-bit digits, hot actors' queues filling up).  Populations that are not a
    multiple of 4 (or of the bucket width) put actors past n_local into the last bucket's threads:
    their ring-head loads must stay inside the n_local rings."""
    from oracle import BspOracle
    monkeypatch.delenv("AGX_RING_APPLY", raising=False)
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    w = wl.zipf_fanout(n, k=1, ttl=12, root_every=1, capacity=capacity)
    ref = BspOracle(**w.engine_kwargs())
    w.apply_to(ref)
    so = ref.run()
    sto = ref.read_state()
    ref.close()
    eng, sg, st, launches = _run_profiled(w, 0)
    eng.close()
    assert (launches > 0) == rings, f"capacity {capacity}: ring_apply launches {launches}"
    assert_same(sg, so, st, sto, f"zipf capacity={capacity}")


@pytest.mark.parametrize("case", ["power_law_c64", "compiled", "classes_host", "bounded_ring"])
def test_ring_apply_wave_and_block(built, monkeypatch, case):
    """The wave-per-bucket ring launch (k_ring_tiny: sparse buckets a wave each, the rest marked for
    k_ring_apply) and the block kernel alone (AGX_TINY_LAUNCH=0), both bit-exact against the oracle."""
    from oracle import BspOracle
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    monkeypatch.setenv("AGX_RING_APPLY", "1")
    w = RING_APPLY_CASES[case]()
    ref = BspOracle(**w.engine_kwargs())
    w.apply_to(ref)
    so = ref.run()
    sto = ref.read_state()
    ref.close()
    for tl in ("1", "0"):
        monkeypatch.setenv("AGX_TINY_LAUNCH", tl)
        eng, sg, st, launches = _run_profiled(w, 0)
        tiny = eng.tiny_launches
        eng.close()
        assert launches > 0 and (tiny > 0) == (tl == "1"), f"{case}: ring {launches} / wave {tiny} launches, TINY_LAUNCH={tl}"
        assert_same(sg, so, st, sto, f"{case} tiny_launch={tl}")


@pytest.mark.parametrize("case", ["power_law_c64", "classes_host"])
def test_ring_apply_resume_and_shrink(built, monkeypatch, case):
    """Runs split into budgets (the rings persist across agx_run calls), a host burst staged
    mid-run, then a mailbox class shrunk below what its rings hold (keep = min(len, C): the
    excess queued messages become dead letters) -- counts after every leg and the final state
    bit-exact against the oracle."""
    from oracle import BspOracle
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    monkeypatch.setenv("AGX_RING_APPLY", "1")
    w = RING_APPLY_CASES[case]()
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    ref = BspOracle(**w.engine_kwargs())
    for t in (eng, ref):
        w.apply_to(t)
    eng.profile(True)
    burst = np.arange(0, w.n_actors, 5, dtype=np.uint32)
    for leg, steps in enumerate((2, 3, 1, 4, 1 << 30)):
        if leg == 2:
            eng.tell(burst, 3)
            ref.tell(burst, 3)
        if leg == 3:
            for t in (eng, ref):
                if w.mailbox_classes:
                    t.set_mailbox_class(3, 5)  # (17 -> 5)
                else:
                    t.set_mailbox_class(1, 4)  # (the default 64 -> 4 for half the population)
                    t.set_mailbox(0, w.n_actors // 2, 1)
        sg, so = eng.run(steps), ref.run(steps)
        for k in COUNT_KEYS:
            assert getattr(sg, k) == so[k], f"{case} leg {leg}: {k} gpu={getattr(sg, k)} oracle={so[k]}"
    assert eng.profile_read()["ring_apply"]["launches"] > 0
    assert_same(sg, so, eng.read_state(), ref.read_state(), case)
    eng.close()
    ref.close()


@pytest.mark.parametrize("mode", ["fused", "bits3"])
@pytest.mark.parametrize("case", ["mixed", "zipf_tree", "ring"])
def test_run_zero_captures_graphs(built, monkeypatch, mode, case):
    """agx_run(0) captures the replay graphs (bench.py times C3 tree from its first superstep): with
    host-staged tells pending -- the multi-pass staged chunk is set aside for the capture and consumed
    by the next run's first superstep -- the results match the oracle, budgets before and after."""
    from oracle import BspOracle
    if mode == "bits3":
        monkeypatch.setenv("AGX_RADIX_BITS", "3")
    w = {"mixed": lambda: wl.mixed(20_000, seed=2, throughput=2, capacity=5),
         "zipf_tree": lambda: wl.zipf_fanout(40_000, k=4, ttl=3, root_every=64, capacity=100),
         "ring": lambda: wl.token_ring(30_000, 20)}[case]()
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    ref = BspOracle(**w.engine_kwargs())
    w.apply_to(ref)
    for budget in (0, 0, 9, 0, 1 << 30):
        sg, so = eng.run(budget), ref.run(budget)
        for k in COUNT_KEYS:
            assert getattr(sg, k) == so[k], (case, mode, budget, k, getattr(sg, k), so[k])
        assert np.array_equal(eng.read_state()[0], ref.read_state()[0]), (case, mode, budget)
    eng.close()


@pytest.mark.parametrize("strict", ["1", "0"])
def test_fused_capacity_error_reported(built, monkeypatch, strict):
    """A kernel-raised capacity error in a fused run (a hot bucket's inbox past the message arena)
    reaches agx_run: through the last replay's ring row (full graphs, the skew launch inside the
    replay) or through the copy after a strict replay's recovery."""
    from akka_amd._lib import AgxError
    if strict == "0":
        monkeypatch.setenv("AGX_NO_STRICT", "1")
    w = wl.zipf_fanout(20_000, k=4, ttl=6, root_every=256, throughput=1000)
    eng = GpuEngine(EngineConfig(msg_capacity=20_000, **w.gpu_kwargs()))
    w.apply_to(eng)
    with pytest.raises(AgxError):
        eng.run()
    eng.close()
