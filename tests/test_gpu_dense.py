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
    """(launch: the multi-pass modes' lean dense-bucket launch, k_dense_apply, forced on / off -- beside
    the wave-per-bucket launch, which then takes only the buckets the dense launch left)"""
    if launch == "1" and mode == "fused":
        pytest.skip("the dense launch is a multi-pass launch")
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


@pytest.mark.parametrize("tokens", [1, 2])
def test_dense_launch_ring_2m(built, tokens):
    """2.1M actors (native 9-bit multi-pass, identity grouping): one token per actor -- every bucket
    dense -- and two -- none dense, every bucket left to the block launch."""
    sg, so, a, b = run_both(wl.token_ring(2_100_000, 5, tokens_per_actor=tokens))
    assert_same(sg, so, a, b, f"ring 2.1M x{tokens}")


def test_dense_sharded_loopback(built):
    from oracle import BspOracle
    ranks = 3
    w = wl.one_per_actor(30_000, seed=9, capacity=2)
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
