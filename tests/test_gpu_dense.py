"""Dense buckets (agx_kernels.h dense_finish): a bucket whose inbox keys are strictly increasing holds
at most one message per actor, so each message is applied by the thread that holds it and its tell
goes to its rank among the bucket's tells -- the same admission / drain / emission order as
bucket_finish (AD/Mailbox.scala:261,551-565).  Every case is bit-exact against the BSP oracle:
one staged tell per actor (a permutation) over every behaviour kind, so dense buckets run beside
buckets whose forwards collide, with stops, dead letters to stopped actors, unknown refs and replies
to host-side actors; in the fused superstep, the multi-pass bypass (3-bit digits) and the unfused
single pass, and over a loopback-sharded group (owner grouping, R = 3)."""
import numpy as np
import pytest

from akka_amd import workloads as wl
from akka_amd.engine import EngineConfig, GpuEngine, owner
from tests.test_gpu_parity import COUNT_KEYS, assert_same, run_both

pytestmark = pytest.mark.gpu

MODES = {"fused": {}, "bits3": {"AGX_RADIX_BITS": "3"}, "unfused": {"AGX_NO_FUSED": "1"}}


@pytest.mark.parametrize("launch", ["1", "0"])
@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("compiled,capacity", [(False, 0), (False, 1), (True, 0), (True, 3)])
def test_dense_one_per_actor(built, monkeypatch, mode, compiled, capacity, launch):
    """(launch: the lean dense-bucket launch -- k_dense_apply in the multi-pass modes, k_dense_fused in
    the fused superstep -- forced on / off; the block launch (and the multi-pass wave-per-bucket
    launch) then takes only the buckets it left)"""
    monkeypatch.setenv("AGX_DENSE_LAUNCH", launch)
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    w = wl.one_per_actor(20_000, seed=5 + capacity, compiled_kinds=compiled, capacity=capacity)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"one_per_actor compiled={compiled} C={capacity} {mode}")


@pytest.mark.parametrize("n,hops", [(2047, 9), (2049, 9), (20_001, 7)])
@pytest.mark.parametrize("mode", sorted(MODES))
def test_dense_ring_partial_buckets(built, monkeypatch, n, hops, mode):
    """Token rings whose last bucket is partial (and a ring of one bucket +- 1 actor): every bucket
    dense, the wrap-around tell crossing into bucket 0 (the ring's multi-pass supersteps take the
    dense launch by default)."""
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    sg, so, a, b = run_both(wl.token_ring(n, hops))
    assert_same(sg, so, a, b, f"ring n={n} {mode}")


@pytest.mark.parametrize("launch,persist", [("1", "1"), ("1", "0"), ("0", "1")])
@pytest.mark.parametrize("n,tokens,hops", [(1_000_000, 1, 6), (1_000_000, 1, 37), (300_001, 2, 4), (65_536, 1, 9),
                                           (4_099, 1, 5)])
def test_dense_fused_ring(built, monkeypatch, n, tokens, hops, launch, persist):
    """The fused superstep's dense launch (k_dense_fused, default for rings): every bucket of a
    one-token ring is dense -- bucket 0 included, whose wrap-around tell arrives after its own
    (distinct actors, not increasing keys) -- and none of a two-token ring, which the block launch
    then takes whole.  persist: a replay of dense-alone strict supersteps as ONE persistent launch
    (grid barrier between supersteps) or one launch per superstep; 37 hops cross
    several replays of 8 and 16."""
    monkeypatch.setenv("AGX_DENSE_FUSED", launch)
    monkeypatch.setenv("AGX_PERSIST", persist)
    sg, so, a, b = run_both(wl.token_ring(n, hops, tokens_per_actor=tokens))
    assert_same(sg, so, a, b, f"fused ring n={n} x{tokens}")


@pytest.mark.parametrize("persist", ["1", "0"])
@pytest.mark.parametrize("budgets", [(1000,), (5, 3, 1000), (17, 9, 1000)])
def test_dense_fused_recovery(built, monkeypatch, budgets, persist):
    """Dense-alone strict replays (k_dense_fused the whole superstep) meeting a bucket it cannot take:
    a one-token ring with one actor holding a second token -- that pair travels together, so one
    bucket per superstep has two messages for one actor.  The first replay voids from that
    superstep on, run_single runs its block + skew launches, and the engine continues on graphs
    with the block launch beside the dense launch; and the same pair staged between runs of a
    clean ring (its superstep runs eagerly, then the replays recover).  Every budget matches the
    oracle -- with the replays as persistent launches (the void mark crosses the grid barrier) and as
    one launch per superstep."""
    from oracle import BspOracle
    monkeypatch.setenv("AGX_PERSIST", persist)
    n, hops = 200_003, 40
    w = wl.token_ring(n, hops)
    dst, src, pay = w.tells
    for staged_later in (False, True):
        extra = (np.array([77], np.uint32), np.array([hops // 2], np.uint32))
        if not staged_later:
            w.tells = (np.concatenate([dst, extra[0]]), np.concatenate([src, [src[0]]]).astype(np.uint32),
                       np.concatenate([pay, extra[1]]))
        else:
            w.tells = (dst, src, pay)
        eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
        ref = BspOracle(**w.engine_kwargs())
        w.apply_to(eng)
        w.apply_to(ref)
        for i, budget in enumerate(budgets + ((7, 1000) if staged_later else ())):
            if staged_later and i == len(budgets):
                eng.tell(extra[0], extra[1])
                ref.tell(extra[0], extra[1])
            sg, so = eng.run(budget), ref.run(budget)
            for k in COUNT_KEYS:
                assert getattr(sg, k) == so[k], (staged_later, budget, k, getattr(sg, k), so[k])
            assert np.array_equal(eng.read_state()[0], ref.read_state()[0]), (staged_later, budget)
        eng.close()


@pytest.mark.parametrize("tokens", [1, 2])
def test_dense_launch_ring_2m(built, tokens):
    """2.1M actors (native 9-bit multi-pass, identity grouping): one token per actor -- every bucket
    dense -- and two -- none dense, every bucket left to the block launch."""
    sg, so, a, b = run_both(wl.token_ring(2_100_000, 5, tokens_per_actor=tokens))
    assert_same(sg, so, a, b, f"ring 2.1M x{tokens}")


@pytest.mark.parametrize("launch", ["1", "0"])
@pytest.mark.parametrize("ranks,case", [(3, "one_per_actor"), (2, "ring"), (8, "ring"), (3, "ring2")])
def test_dense_sharded_loopback(built, monkeypatch, ranks, case, launch):
    """Owner grouping (multi-rank superstep) with the dense launch (k_dense_fused<kOwner>: the sorted
    inbox of each bucket, the tells grouped by owner rank) forced on / off: one message per actor over
    every kind, a hash-sharded token ring (every bucket dense), a two-token ring (none dense)."""
    from oracle import BspOracle
    monkeypatch.setenv("AGX_DENSE_LAUNCH", launch)
    monkeypatch.setenv("AGX_DENSE_OWNER", launch)
    w = {"one_per_actor": lambda: wl.one_per_actor(30_000, seed=9, capacity=2),
         "ring": lambda: wl.token_ring(40_000, 9),
         "ring2": lambda: wl.token_ring(30_001, 5, tokens_per_actor=2)}[case]()
    engs = [GpuEngine(EngineConfig(n_ranks=ranks, rank=r, **w.gpu_kwargs())) for r in range(ranks)]
    for e in engs:
        w.apply_to(e)
    sg = GpuEngine.group_run(engs)
    ref = BspOracle(n_ranks=ranks, **w.engine_kwargs())
    w.apply_to(ref)
    so = ref.run()
    for k in COUNT_KEYS:
        if k != "supersteps":
            assert getattr(sg, k) == so[k], (k, getattr(sg, k), so[k])
    wo, _ = ref.read_state()
    wg = np.zeros_like(wo)
    own_of = np.array([owner(i, 1000, ranks) for i in range(w.n_actors)])
    for e in engs:
        st, _ = e.read_state()
        own = own_of == e.cfg.rank
        wg[own] = st[own]
        e.close()
    assert np.array_equal(wg, wo)


@pytest.mark.parametrize("tokens", [1, 2])
def test_profile_counts_dense_launches_that_took_every_bucket(built, monkeypatch, tokens):
    """agx_profile_read's items for bucket_apply_dense: the profiled dense launches after which the
    device's dense_left flags were both clear (the wave / block launches returned at entry; bench.py
    marks them returned_at_entry from this count, not from a rate).  A one-token ring (multi-pass,
    3-bit digits) leaves no bucket; a two-token ring leaves every bucket to the block launch."""
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    w = wl.token_ring(40_000, 12, tokens_per_actor=tokens)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    eng.run(2)
    eng.profile(True)
    eng.profile_reset()
    eng.run(4)
    p = eng.profile_read()
    eng.profile(False)
    eng.close()
    d = p["bucket_apply_dense"]
    assert d["launches"] == 4
    assert d["items"] == (4 if tokens == 1 else 0)
    assert all(v["items"] == 0 for k, v in p.items() if k != "bucket_apply_dense")
