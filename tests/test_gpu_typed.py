"""GPU parity of compiled behaviours (typed DSL tables, akka_amd/typed.py -> agx_set_behaviors):
the HIP engine through the C ABI vs the BSP oracle, bit-exact; and the DSL ring equals the
hand-written RING kind on the GPU."""
import numpy as np
import pytest

from akka_amd import typed
from akka_amd import workloads as wl
from akka_amd.engine import EngineConfig, GpuEngine
from tests.test_gpu_parity import assert_same, run_both

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,C", [(3, 0), (1, 2), (50, 0), (2, 5)])
@pytest.mark.parametrize("builtin", [False, True])
def test_compiled_behaviors(built, T, C, builtin):
    w = wl.compiled(6000, seed=T * 7 + C, throughput=T, capacity=C, builtin=builtin)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, f"compiled T={T} C={C} builtin={builtin}")


@pytest.mark.parametrize("ba", [32, 2048])
def test_compiled_behaviors_bucket_widths(built, ba):
    w = wl.compiled(20_000, seed=3, throughput=3, capacity=0)
    sg, so, a, b = run_both(w, bucket_actors=ba)
    assert_same(sg, so, a, b, f"compiled ba={ba}")


def test_compiled_multipass(built, monkeypatch):
    monkeypatch.setenv("AGX_RADIX_BITS", "3")
    w = wl.compiled(20_000, seed=11, throughput=2, capacity=4, builtin=True)
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "compiled multipass")


def test_compiled_ring_equals_builtin_ring(built):
    n, hops = 100_000, 12
    out = []
    for w in (wl.token_ring(n, hops), wl.compiled_ring(n, hops)):
        eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
        w.apply_to(eng)
        st = eng.run()
        ws, _ = eng.read_state()
        eng.close()
        out.append((st, ws[:, 0]))
    (s0, w0), (s1, w1) = out
    assert s0.delivered == s1.delivered == n * (hops + 1)
    assert s0.supersteps == s1.supersteps and np.array_equal(w0, w1)


def test_compiled_rejects_crdt_mix(built):
    from akka_amd.engine import Kind
    t = typed.compile_behaviors([typed.library()["counter"]])
    eng = GpuEngine(EngineConfig(n_actors=64, n_words=8, max_emit=3))
    eng.set_behaviors(t)
    eng.register_range(0, 32, Kind.GCOUNTER)
    with pytest.raises(Exception):
        eng.register_range(32, 32, t.kind_of(t.behaviors[0]))
    eng.close()
