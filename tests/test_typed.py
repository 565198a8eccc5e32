"""Typed behaviours lowered to compiled behaviour tables (akka_amd/typed.py) -- CPU tests:
the lowering, and the oracle running the tables (ReceiveBuilder.receive's first-match rule,
TY/javadsl/ReceiveBuilder.scala:209-218; become, TY/Behavior.scala:150)."""
import numpy as np
import pytest

from akka_amd import typed
from akka_amd import workloads as wl
from akka_amd.engine import Kind, NO_SENDER
from oracle import BspOracle


def test_lowering_shapes():
    lib = typed.library(ring_stride=3)
    t = typed.compile_behaviors([lib["ring"], lib["ping_pong"]])
    assert t.n_behaviors == 2 and list(t.first) == [0, 2, 4]
    ring0 = t.cases[0]  # test: payload > 0; actions: count += 1, tell(self + 3, payload - 1)
    assert (ring0.src1, ring0.cmp1, ring0.src2, ring0.k2) == (typed.V_PAYLOAD, typed.CMP_GT, typed.V_CONST, 0)
    a = t.acts[ring0.act_first + 1]
    assert (a.op, a.dsrc, a.dk, a.src, a.k) == (typed.A_TELL, typed.V_SELF, 3, typed.V_PAYLOAD, -1)
    pp0 = t.cases[2]  # state guard left == 0 -> stopped
    assert (pp0.src1, pp0.word1, pp0.cmp1, pp0.result) == (typed.V_WORD, 0, typed.CMP_EQ, typed.RES_STOPPED)
    sw = typed.switch()
    t2 = typed.compile_behaviors([sw])
    assert t2.n_behaviors == 2  # off and the `on` it becomes
    assert any(c.result == typed.RES_BECOME for c in t2.cases)


def test_lowering_rejects():
    with pytest.raises(typed.CompileError):
        typed.State("a", "b", "c")
    st = typed.State("a")
    with pytest.raises(typed.CompileError):  # type + predicate + guard = three tests
        typed.ReceiveBuilder.create(st).on_message(typed.PING, lambda m, s: [typed.Behaviors.same],
                                                   test=lambda m: m.arg > 1, when=lambda m, s: s.a == 0)
    with pytest.raises(typed.CompileError):
        typed.ReceiveBuilder.create(st).on_any_message(lambda m, s: [s.a.inc()])  # no next behaviour


def _kinds_workload(kinds, inits, seed=5, n=4000, T=3, C=0, tables=None):
    rng = np.random.default_rng(seed)
    per = n // len(kinds)
    ranges = [(i * per, per if i < len(kinds) - 1 else n - i * per, k, inits[i]) for i, k in enumerate(kinds)]
    m = 3 * n
    dst = rng.integers(0, n + 8, m).astype(np.uint32)
    src = rng.integers(0, n, m).astype(np.uint32)
    src[rng.random(m) < 0.1] = NO_SENDER
    pay = rng.integers(0, 12, m).astype(np.uint32)
    return wl.Workload("kinds", n, 2, 1, T, C, ranges, ring_stride=7, tells=(dst, src, pay), behaviors=tables)


@pytest.mark.parametrize("T,C", [(3, 0), (1, 2), (50, 0)])
def test_compiled_library_equals_builtin_kinds(T, C):
    """The DSL versions of COUNTER / RING / STOP_AFTER / PINGPONG give the same counts and states
    as the hand-written kinds on the same tells."""
    rng = np.random.default_rng(9)
    n, per = 4000, 1000
    sa = np.zeros((per, 2), np.uint64)
    sa[:, 1] = rng.integers(1, 6, per)
    pp = np.zeros((per, 2), np.uint64)
    pp[:, 0] = rng.integers(0, 5, per)
    inits = [None, None, sa, pp]
    lib = typed.library(ring_stride=7)
    t = typed.compile_behaviors([lib[k] for k in ("counter", "ring", "stop_after", "ping_pong")])
    wb = _kinds_workload([Kind.COUNTER, Kind.RING, Kind.STOP_AFTER, Kind.PINGPONG], inits, T=T, C=C)
    wc = _kinds_workload([t.kind_of(lib[k]) for k in ("counter", "ring", "stop_after", "ping_pong")], inits, T=T, C=C,
                         tables=t)
    out = []
    for w in (wb, wc):
        o = BspOracle(**w.engine_kwargs())
        w.apply_to(o)
        out.append((o.run(), o.read_state()))
    (sb, (wsb, ab)), (sc, (wsc, ac)) = out
    assert sb == sc
    assert np.array_equal(ab, ac)
    # the built-in RING kind keeps one word; compare the words the behaviours define
    assert np.array_equal(wsb, wsc)


def test_switch_become_semantics():
    """off: Ping unhandled, SwitchOn -> flips + 1, become on; on: Ping(n) sums n and answers
    Ping(n - 1) while n > 0, SwitchOff -> become off."""
    sw = typed.switch()
    lib = typed.library()
    t = typed.compile_behaviors([sw, lib["counter"]])
    w = wl.Workload("switch", 2, 2, 1, 100, 0, [(0, 1, t.kind_of(sw), None), (1, 1, t.kind_of(lib["counter"]), None)],
                    behaviors=t)
    o = BspOracle(**w.engine_kwargs())
    w.apply_to(o)
    P, ON, OFF = typed.PING.payload, typed.SWITCH_ON.payload(), typed.SWITCH_OFF.payload()
    o.tell([0, 0, 0, 0, 0], [P(3), ON, P(2), OFF, P(5)], src=np.array([1, NO_SENDER, 1, NO_SENDER, 1], np.uint32))
    st = o.run()
    ws, _ = o.read_state()
    assert st["delivered"] == 6 and st["unhandled"] == 2 and st["emitted"] == 1
    assert list(ws[0]) == [2, 2]                 # flips, sum
    assert list(ws[1]) == [1, P(1)]              # the reply Ping(1)


def test_compile_rejects_tells_beyond_max_emit():
    """compile_behaviors(max_emit=k) refuses a case that tells more than k times per message
    (the engine reserves max_emit tell slots per message, agx_set_behaviors checks the same)."""
    st = typed.State("count")
    two = (typed.ReceiveBuilder.create(st)
           .on_any_message(lambda m, s: [typed.self_ref(1).tell(m.payload), m.sender.tell(m.payload),
                                         typed.Behaviors.same])
           .build("two"))
    assert typed.compile_behaviors([two]).max_tells == 2
    assert typed.compile_behaviors([two], max_emit=2).max_tells == 2
    with pytest.raises(typed.CompileError):
        typed.compile_behaviors([two], max_emit=1)
    assert typed.compile_behaviors([typed.library()["ring"]], max_emit=1).max_tells == 1
