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


def test_compiled_tells_beyond_max_emit_rejected(built):
    """A case that tells twice per message needs max_emit >= 2 (the apply reserves max_emit tell
    slots per message): agx_set_behaviors rejects it with AGX_EINVAL at max_emit 1, and accepts it,
    bit-exact against the oracle, at max_emit 2."""
    from akka_amd import typed
    from akka_amd._lib import AgxError
    st = typed.State("count")
    two = (typed.ReceiveBuilder.create(st)
           .on_any_message(lambda m, s: [s.count.inc(), typed.self_ref(1).tell(m.payload - 1),
                                         typed.self_ref(2).tell(m.payload - 1), typed.Behaviors.same],
                           test=lambda m: m.payload > 0)
           .on_any_message(lambda m, s: [s.count.inc(), typed.Behaviors.same])
           .build("two_tells"))
    tables = typed.compile_behaviors([two])
    assert tables.max_tells == 2
    eng = GpuEngine(EngineConfig(n_actors=64, n_words=2, max_emit=1))
    with pytest.raises(AgxError):
        eng.set_behaviors(tables)
    eng.close()
    n = 4096
    w = wl.Workload("two_tells", n, 2, 2, 3, 0, [(0, n, tables.kind_of(two), None)], behaviors=tables,
                    tells=(np.arange(0, n, 97, dtype=np.uint32), np.full(43, 0xFFFFFFFF, np.uint32),
                           np.full(43, 6, np.uint32)))
    sg, so, a, b = run_both(w)
    assert_same(sg, so, a, b, "two tells")
