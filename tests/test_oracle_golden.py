"""The CPU oracle (test infrastructure) pinned against the reference's own
known-answer tests, transcribed into tests/golden/*.json (see make_golden.py)."""
import json
import pathlib

import numpy as np
import pytest

from akka_amd import workloads as wl
from akka_amd.engine import Kind, Op
from oracle import BspOracle, FjpOracle, crdt, java_hash, shard_id

GOLD = pathlib.Path(__file__).resolve().parent / "golden"


def load(name):
    return json.loads((GOLD / name).read_text())


def test_shard_ids_oracle_and_host_mirror():
    from akka_amd import sharding
    for v in load("shard_ids.json")["vectors"]:
        assert sharding.java_string_hash(v["entity_id"]) == v["hash"]
        assert int(sharding.shard_id(v["entity_id"], v["num_shards"])) == v["shard"]
        if v["entity_id"].isdigit() and int(v["entity_id"]) < 2**32:
            assert java_hash(int(v["entity_id"])) == v["hash"]
            assert shard_id(int(v["entity_id"]), v["num_shards"]) == v["shard"]


def test_vectorised_owner_matches_scalar():
    from akka_amd import sharding
    n = 20000
    own = sharding.owners(n, 1000, 8)
    ref = np.array([sharding.rank_of_shard(sharding.shard_of_actor(i, 1000), 8) for i in range(n)])
    assert np.array_equal(own, ref)


def _apply_ops(ops, slots):
    c = np.zeros(slots, np.uint64)
    for op, slot, n in ops:
        assert op == "inc"
        c = crdt.gcounter_increment(c, slot, n)
    return c


def test_gcounter_kats():
    g = load("gcounter_kat.json")
    for case in g["cases"]:
        c = _apply_ops(case["ops"], g["slots"])
        assert c.tolist() == case["state"], case["name"]
        if "value" in case:
            assert crdt.gcounter_value(c) == case["value"]
    for m in g["merges"]:
        a = _apply_ops(m["a_ops"], g["slots"])
        b = _apply_ops(m["b_ops"], g["slots"])
        assert a.tolist() == m["a_state"] and crdt.gcounter_value(a) == m["a_value"], m["name"]
        assert b.tolist() == m["b_state"] and crdt.gcounter_value(b) == m["b_value"], m["name"]
        for x, y in ((a, b), (b, a)):  # merge both ways
            mg = crdt.gcounter_merge(x, y)
            assert mg.tolist() == m["merged_state"] and crdt.gcounter_value(mg) == m["merged_value"], m["name"]
        # join laws: idempotent, commutative
        assert np.array_equal(crdt.gcounter_merge(a, a), a)


@pytest.mark.parametrize("Oracle", [BspOracle, FjpOracle])
def test_mailbox_kats(Oracle):
    for case in load("mailbox_kat.json")["cases"]:
        o = Oracle(1, throughput=case["throughput"], capacity=case["capacity"], n_words=2)
        o.register_range(0, 1, Kind.COUNTER)
        o.tell(np.zeros(len(case["payloads"]), np.uint32), case["payloads"])
        st = o.run() if Oracle is BspOracle else o.run(2)
        w, _ = o.read_state()
        assert st["delivered"] == case["delivered"], case["name"]
        assert st["dead_letters"] == case["dead_letters"], case["name"]
        assert int(w[0, 1]) == case["sum"], case["name"]
        if Oracle is BspOracle and "supersteps" in case:
            assert st["supersteps"] == case["supersteps"], case["name"]


@pytest.mark.parametrize("Oracle", [BspOracle, FjpOracle])
def test_pingpong_kats(Oracle):
    for c in load("pingpong_kat.json")["cases"]:
        w = wl.ping_pong(c["pairs"], c["messages_per_pair"], c["throughput"], c["in_flight"])
        o = Oracle(**w.engine_kwargs())
        w.apply_to(o)
        st = o.run() if Oracle is BspOracle else o.run(4)
        assert st["delivered"] == c["delivered"] and st["dead_letters"] == c["dead_letters"], c


def test_ring_kats():
    for c in load("ring_kat.json")["cases"]:
        w = wl.token_ring(c["n"], c["hops"])
        o = BspOracle(**w.engine_kwargs())
        w.apply_to(o)
        st = o.run()
        words, alive = o.read_state()
        assert st["delivered"] == c["delivered"] and st["supersteps"] == c["supersteps"]
        assert (words[:, 0] == c["count"]).all() and alive.all()


@pytest.mark.parametrize("make", [lambda: wl.token_ring(3000, 17, throughput=2),
                                  lambda: wl.zipf_fanout(4000, k=3, ttl=3, root_every=8, throughput=7),
                                  lambda: wl.ping_pong(50, 60, 5)])
def test_fjp_restatement_agrees_with_bsp_on_confluent_workloads(make):
    """For confluent workloads the final state is schedule independent: the
    multi-threaded ForkJoin restatement and the BSP oracle agree bit for bit."""
    w = make()
    b = BspOracle(**w.engine_kwargs())
    w.apply_to(b)
    sb = b.run()
    f = FjpOracle(**w.engine_kwargs())
    w.apply_to(f)
    sf = f.run(4)
    for k in ("delivered", "dead_letters", "unhandled", "emitted", "staged"):
        assert sb[k] == sf[k], k
    assert np.array_equal(b.read_state()[0], f.read_state()[0])


@pytest.mark.parametrize("T,C", [(1, 0), (3, 4), (5, 1), (50, 16)])
def test_conservation(T, C):
    """delivered + dead letters + in flight = staged + emitted (MailboxConfigSpec:132-182)."""
    w = wl.mixed(2000, seed=T + 7 * C, throughput=T, capacity=C)
    for budget in (1, 4, 1 << 20):
        o = BspOracle(**w.engine_kwargs())
        w.apply_to(o)
        st = o.run(budget)
        assert st["delivered"] + st["dead_letters"] + st["in_flight"] == st["staged"] + st["emitted"]


def test_sharded_order_is_rank_major():
    """With n_ranks > 1 arrivals are ordered by (owner(src), src): a bounded
    mailbox then admits a different subset, but totals are conserved."""
    w = wl.mixed(1500, seed=3, throughput=2, capacity=3)
    res = []
    for R in (1, 2, 4):
        o = BspOracle(n_ranks=R, **w.engine_kwargs())
        w.apply_to(o)
        st = o.run()
        res.append(st)
        assert st["delivered"] + st["dead_letters"] + st["in_flight"] == st["staged"] + st["emitted"]
    ring = wl.token_ring(500, 9)
    outs = []
    for R in (1, 2, 8):
        o = BspOracle(n_ranks=R, **ring.engine_kwargs())
        ring.apply_to(o)
        o.run()
        outs.append(o.read_state()[0])
    assert all(np.array_equal(outs[0], x) for x in outs[1:])  # confluent: same for any R


# ------------------------------------------------------------------ CRDT KATs (a9, a10)
def _pn_apply(ops, slots):
    inc = np.zeros(slots, np.uint64)
    dec = np.zeros(slots, np.uint64)
    for op, slot, n in ops:
        if op == "inc":
            inc = crdt.gcounter_increment(inc, slot, n)
        else:
            dec = crdt.gcounter_increment(dec, slot, n)
    return inc, dec


def test_pncounter_kats():
    g = load("pncounter_kat.json")
    for case in g["cases"]:
        inc, dec = _pn_apply(case["ops"], g["slots"])
        if "increments" in case:
            assert inc.tolist() == case["increments"] and dec.tolist() == case["decrements"], case["name"]
        if "value" in case:
            assert crdt.gcounter_value(inc) == case["increments_value"], case["name"]
            assert crdt.gcounter_value(dec) == case["decrements_value"], case["name"]
            assert crdt.gcounter_value(inc) - crdt.gcounter_value(dec) == case["value"], case["name"]
    for m in g["merges"]:
        a = _pn_apply(m["a_ops"], g["slots"])
        b = _pn_apply(m["b_ops"], g["slots"])
        assert crdt.gcounter_value(b[0]) == m["b_increments_value"]
        assert crdt.gcounter_value(b[1]) == m["b_decrements_value"]
        for x, y in ((a, b), (b, a)):  # PNCounter.merge = GCounter.merge of each half (PNCounter.scala:178)
            mi, md = crdt.gcounter_merge(x[0], y[0]), crdt.gcounter_merge(x[1], y[1])
            assert crdt.gcounter_value(mi) == m["merged_increments_value"], m["name"]
            assert crdt.gcounter_value(md) == m["merged_decrements_value"], m["name"]
            assert crdt.gcounter_value(mi) - crdt.gcounter_value(md) == m["merged_value"], m["name"]


def _ikeys(d):
    return {int(k): v for k, v in d.items()}


def test_orset_subtract_dots_kat():
    from oracle.oracle import orset
    for c in load("orset_kat.json")["subtract_dots"]:
        assert orset.subtract_dots(_ikeys(c["dot"]), _ikeys(c["vvector"])) == _ikeys(c["expected"]), c["name"]


def test_orset_merge_kats():
    from oracle.oracle import orset
    for c in load("orset_kat.json")["merges"]:
        names = sorted(set(c["this"]["elements"]) | set(c["that"]["elements"]) | set(c["expected_elements"]))
        idx = {k: i for i, k in enumerate(names)}
        a = orset.from_dict({k: _ikeys(v) for k, v in c["this"]["elements"].items()}, _ikeys(c["this"]["vvector"]), idx)
        b = orset.from_dict({k: _ikeys(v) for k, v in c["that"]["elements"].items()}, _ikeys(c["that"]["vvector"]), idx)
        m = orset.merge(a, b)
        got = {k: orset.dots(m, idx[k]) for k in names if orset.dots(m, idx[k])}
        assert got == {k: _ikeys(v) for k, v in c["expected_elements"].items()}, c["name"]
        # vvector = VersionVector.merge (pointwise max)
        vv = {**_ikeys(c["this"]["vvector"])}
        for n, v in _ikeys(c["that"]["vvector"]).items():
            vv[n] = max(vv.get(n, 0), v)
        assert orset.vvector(m) == vv


def test_orset_replica_scripts():
    """ORSetSpec 'verify disjoint merge' / 'removed after merge' (1, 2): add/remove/merge
    sequences on named replicas, checked on the element sets."""
    from oracle.oracle import orset
    for c in load("orset_kat.json")["scripts"]:
        reps, idx = {}, {}
        for op in c["ops"]:
            if op[0] == "new":
                reps[op[1]] = orset.empty()
            elif op[0] == "add":
                reps[op[1]] = orset.add(reps[op[1]], op[2], idx.setdefault(op[3], len(idx)))
            elif op[0] == "remove":
                reps[op[1]] = orset.remove(reps[op[1]], idx.setdefault(op[2], len(idx)))
            elif op[0] == "copy":
                reps[op[1]] = reps[op[2]].copy()
            elif op[0] == "merge":
                reps[op[1]] = orset.merge(reps[op[2]], reps[op[3]])
        inv = {v: k for k, v in idx.items()}
        for chk in c["checks"]:
            assert {inv[e] for e in orset.elements(reps[chk[1]])} == set(chk[2]), (c["name"], chk)


@pytest.mark.parametrize("kind", [Kind.GCOUNTER, Kind.PNCOUNTER, Kind.ORSET])
def test_crdt_gossip_converges_to_writers_merge(kind):
    """C4 on the oracle: after enough GossipTicks every replica holds the join of the
    8 writers' values (computed here from the ops with the KAT-pinned functions)."""
    from oracle.oracle import orset
    n, rounds, opw = 384, 24, 16
    w = wl.crdt_gossip(n, kind, rounds=rounds, ops_per_writer=opw)
    o = BspOracle(**w.engine_kwargs())
    w.apply_to(o)
    st = o.run()
    assert st["in_flight"] == 0 and st["unhandled"] == 0
    assert st["delivered"] == 8 * opw + n * rounds * 3  # ops + ticks + 2 gossips per tick
    ws, _ = o.read_state()
    ops = wl.crdt_ops(8, kind, opw)
    if kind == Kind.ORSET:
        exp = orset.empty()
        for k in range(8):
            r = orset.empty()
            for p in ops[k]:
                op, arg = int(p) >> 24, int(p) & 0xFFFFFF
                r = orset.add(r, k, arg) if op == 3 else orset.remove(r, arg)
            exp = orset.merge(exp, r)
    else:
        exp = np.zeros(w.n_words, np.uint64)
        for k in range(8):
            for p in ops[k]:
                op, arg = int(p) >> 24, int(p) & 0xFFFFFF
                exp[k if op == 1 else 8 + k] += arg
    assert all(np.array_equal(r, exp) for r in ws)


def test_versionvector_kats():
    """VersionVectorSpec (merge / compare / increment) on the fixed 8-node layout; versions come
    from one global counter like Timestamp.counter (VersionVector.scala:277-281)."""
    from oracle.oracle import vv_compare
    for c in load("versionvector_kat.json")["cases"]:
        vs, clock = {}, [0]
        for op in c["ops"]:
            if op[0] == "new":
                vs[op[1]] = np.zeros(8, np.uint32)
            elif op[0] == "copy":
                vs[op[1]] = vs[op[2]].copy()
            elif op[0] == "inc":
                clock[0] += 1
                v = vs[op[2]].copy()
                v[op[3]] = clock[0]
                vs[op[1]] = v
            elif op[0] == "merge":
                vs[op[1]] = np.maximum(vs[op[2]], vs[op[3]])
        for chk in c["checks"]:
            k = chk[0]
            if k == "size":
                assert int(np.count_nonzero(vs[chk[1]])) == chk[2], (c["name"], chk)
            elif k == "contains":
                assert bool(vs[chk[1]][chk[2]]) == chk[3], (c["name"], chk)
            elif k == "cmp":
                assert (vv_compare(vs[chk[1]], vs[chk[2]]) == chk[3]) == chk[4], (c["name"], chk)
            elif k == "gt_at":
                assert vs[chk[1]][chk[3]] > vs[chk[2]][chk[3]], (c["name"], chk)
            elif k == "eq_at":
                assert vs[chk[1]][chk[3]] == vs[chk[2]][chk[3]], (c["name"], chk)


def test_orset_delta_kats():
    """ORSetSpec "ORSet deltas" (AddDeltaOp / RemoveDeltaOp / FullStateDeltaOp / DeltaGroup,
    mergeDelta, mergeRemoveDelta) through the oracle's restatement (crdt_ref.h)."""
    from oracle.oracle import OrsetDelta, orset, orset_delta
    for c in load("orset_delta_kat.json")["cases"]:
        vals, deltas, idx, clock = {}, {}, {}, [0]
        el = lambda name: idx.setdefault(name, len(idx))
        for op in c["ops"]:
            k = op[0]
            if k == "empty":
                vals[op[1]] = orset_delta.empty()
            elif k == "add":
                clock[0] += 1
                vals[op[1]] = orset_delta.add(vals[op[2]], op[3], el(op[4]), clock[0])
            elif k == "remove":
                vals[op[1]] = orset_delta.remove(vals[op[2]], op[3], el(op[4]))
            elif k == "clear":
                vals[op[1]] = orset_delta.clear(vals[op[2]])
            elif k == "reset":
                vals[op[1]] = orset_delta.reset(vals[op[2]])
            elif k == "merge":
                vals[op[1]] = orset_delta.merge(vals[op[2]], vals[op[3]])
            elif k == "merge_delta":
                vals[op[1]] = orset_delta.merge_delta(vals[op[2]], deltas[op[3]])
            elif k == "delta":
                d = vals[op[2]][1]
                assert d.nops > 0, (c["name"], op, "delta.get on None")
                deltas[op[1]] = d
            elif k == "dmerge":
                deltas[op[1]] = orset_delta.delta_merge(deltas[op[2]], deltas[op[3]])
            else:
                raise AssertionError(op)
        inv = lambda: {v: k for k, v in idx.items()}
        for chk in c["checks"]:
            k = chk[0]
            if k == "elements":
                assert {inv()[e] for e in orset.elements(vals[chk[1]][0])} == set(chk[2]), (c["name"], chk)
            elif k == "absent":
                assert el(chk[2]) not in orset.elements(vals[chk[1]][0]), (c["name"], chk)
            elif k == "equal":  # ORSet.equals: elementsMap and vvector, not the delta
                assert np.array_equal(vals[chk[1]][0], vals[chk[2]][0]), (c["name"], chk)
            elif k == "vv_has":
                assert bool(orset.vvector(vals[chk[1]][0]).get(chk[2], 0)) == chk[3], (c["name"], chk)
            elif k in ("add_op", "last_add"):
                d = deltas[chk[1]]
                op = d.ops[d.nops - 1]
                assert (k == "last_add") == bool(d.group) and OrsetDelta.TYPES[op.type] == "add", (c["name"], chk)
                assert {inv()[op.elem[i]] for i in range(op.n)} == set(chk[2]), (c["name"], chk)
            elif k == "group":
                d = deltas[chk[1]]
                assert d.group and d.nops == chk[2], (c["name"], chk)
                assert OrsetDelta.TYPES[d.ops[d.nops - 1].type] == chk[3], (c["name"], chk)


@pytest.mark.parametrize("kind,opr", [(Kind.GCOUNTER, 6), (Kind.PNCOUNTER, 6), (Kind.ORSET, 6),
                                      (Kind.GCOUNTER, 150), (Kind.PNCOUNTER, 150)])
def test_delta_crdt_converges(kind, opr):
    """Delta-CRDT replication on the oracle (DeltaPropagationSelector + receiveDeltaPropagation):
    counters converge from deltas alone to the slot-wise sums of each node's updates; ORSet
    replicas converge once full-state gossip runs beside the deltas (a RemoveDeltaOp only removes
    an element whose dots it covers, DD/ORSet.scala:471-501, so deltas alone can leave dots that
    the full-state merge drops -- as in the reference).  opr = 150: every replica's first group
    covers 150 unsent seqNrs (the reference's deltaEntries map is unbounded; counters are too)."""
    n = 8 * 40
    gossip = 40 if kind == Kind.ORSET else 0
    w = wl.crdt_delta(n, kind, rounds=24, write=False, ops_per_replica=opr, gossip_rounds=gossip)
    o = BspOracle(**w.engine_kwargs())
    w.apply_to(o)
    st = o.run()
    assert st["in_flight"] == 0 and st["unhandled"] == 0 and st["dead_letters"] == 0
    ws, _ = o.read_state()
    D = wl.CRDT_WORDS[kind]
    data = ws[:, :D].reshape(-1, 8, D)
    assert all(np.array_equal(g[0], g[i]) for g in data for i in range(8))
    env = ws[:, D:D + 12].view(np.uint32)
    assert (env[:, 8] == opr).all()  # deltaCounter: one seqNr per update
    if kind != Kind.ORSET:
        ops = wl.crdt_ops(n, kind, opr)
        exp = np.zeros((n, D), np.uint64)
        for a in range(n):
            for p in ops[a]:
                op, arg = int(p) >> 24, int(p) & 0xFFFFFF
                exp[a & ~7, (8 if op == Op.DECREMENT else 0) + a % 8] += arg
        assert np.array_equal(data[:, 0], exp[::8])
    else:  # causal delivery: every replica applied every other node's deltas in order
        for a in range(n):
            dv = env[a, :8].copy()
            dv[a % 8] = opr
            assert (dv == opr).all()


def test_delta_crdt_placeholders_and_log_capacity():
    """max-delta-size: a group of >= M ops is a NoDeltaPlaceholder (never applied; deltaSentToNode
    still advances, DD/DeltaPropagationSelector.scala:112-131), so without full-state gossip the
    receivers keep nothing; a counter update by 0 records a NoDeltaPlaceholder
    (DD/Replicator.scala:1648-1652).  More than AGX_DELTA_LOG unsent seqNrs overflow the ORSet log
    (counters keep each slot's last delta: no bound)."""
    n = 16
    w = wl.crdt_delta(n, Kind.ORSET, rounds=4, write=False, ops_per_replica=6, max_delta_size=2)
    o = BspOracle(**w.engine_kwargs())
    w.apply_to(o)
    o.run()
    ws, _ = o.read_state()
    env = ws[:, 260:272].view(np.uint32)
    adds_only = (wl.crdt_ops(n, Kind.ORSET, 6) >> 24 == Op.ADD).all(axis=1)  # one AddDeltaOp: deltaSize 1
    assert adds_only.any() and not adds_only.all()
    for a in range(n):
        for b in range(8):
            if b != a % 8:
                assert env[a, b] == (6 if adds_only[(a & ~7) + b] else 0), (a, b)
    assert (env[:, 8] == 6).all()
    # a zero increment in the range turns the whole counter group into a placeholder
    w = wl.crdt_delta(n, Kind.GCOUNTER, rounds=4, write=False)
    o = BspOracle(**w.engine_kwargs())
    w.apply_to(o, stage_tells=False)
    ids = np.arange(n, dtype=np.uint32)
    o.tell(np.concatenate([ids, ids, ids]),
           np.concatenate([np.full(n, Op.make(Op.INCREMENT, 5), np.uint32), np.full(n, Op.make(Op.INCREMENT, 0), np.uint32),
                           np.full(n, Op.make(Op.DELTA_TICK, 3), np.uint32)]))
    o.run()
    ws, _ = o.read_state()
    assert all(ws[a, b] == (5 if b == a % 8 else 0) for a in range(n) for b in range(8))
    # ... also when it lies among 100 unsent seqNrs; a group after it carries the slot's last value
    w = wl.crdt_delta(n, Kind.GCOUNTER, rounds=4, write=False)
    o = BspOracle(**w.engine_kwargs())
    w.apply_to(o, stage_tells=False)
    pays = [Op.make(Op.INCREMENT, 5)] * 60 + [Op.make(Op.INCREMENT, 0)] + [Op.make(Op.INCREMENT, 5)] * 39
    o.tell(np.repeat(ids, len(pays)), np.tile(np.array(pays, np.uint32), n))
    o.tell(ids, np.full(n, Op.make(Op.DELTA_TICK, 3), np.uint32))
    o.run()
    o.tell(np.repeat(ids, 2), np.tile(np.array([Op.make(Op.INCREMENT, 7), Op.make(Op.DELTA_TICK, 3)], np.uint32), n))
    o.run()
    ws, _ = o.read_state()
    assert (ws[:, :8] == 495 + 7).all()  # (the first groups were placeholders: nothing of them applied)
    # ORSet log overflow: 70 updates with no propagation
    w = wl.crdt_delta(n, Kind.ORSET, rounds=0, write=False, ops_per_replica=70)
    o = BspOracle(**w.engine_kwargs())
    w.apply_to(o)
    with pytest.raises(OverflowError):
        o.run()


# ------------------------------------------------------------------ the oracle's own execution
@pytest.mark.parametrize("case", ["mixed", "zipf", "plaw", "orset", "orset_delta", "mbox", "sharded"])
def test_oracle_threads_identical(monkeypatch, case):
    """bsp_ref.c applies the actors with mail on host threads, in contiguous runs of the canonical
    order whose outputs are concatenated in order: every count, state word, alive flag and outbox
    envelope is the same for 1 thread and for 7 (and the dense / sparse inbox sorts agree)."""
    w = {
        "mixed": lambda: wl.mixed(20000, seed=3, throughput=2, capacity=3),
        "zipf": lambda: wl.zipf_fanout(100_000, k=4, ttl=3, root_every=16, capacity=50),
        "plaw": lambda: wl.power_law_forward(100_000, ttl=8, capacity=64, device_graph=True),
        "orset": lambda: wl.crdt_gossip(3_000, Kind.ORSET, rounds=4),
        "orset_delta": lambda: wl.crdt_delta(8 * 300, Kind.ORSET, rounds=6, write=True, gossip_rounds=2),
        "mbox": lambda: wl.mailbox_mix(8192, seed=2, throughput=3, capacity=4),
        "sharded": lambda: wl.zipf_fanout(50_000, k=2, ttl=3, root_every=8, capacity=20),
    }[case]
    ranks = 5 if case == "sharded" else 1
    res = []
    for threads in ("1", "7"):
        monkeypatch.setenv("BSP_THREADS", threads)
        x = w()
        o = BspOracle(n_ranks=ranks, **x.engine_kwargs())
        x.apply_to(o)
        sts = [o.run(2), o.run(3), o.run()]
        ws, al = o.read_state()
        ob = o.take_outbound() if x.outbound else ()
        o.close()
        res.append((sts, ws, al, ob))
    (s1, w1, a1, o1), (s7, w7, a7, o7) = res
    assert s1 == s7 and np.array_equal(w1, w7) and np.array_equal(a1, a7)
    assert all(np.array_equal(p, q) for p, q in zip(o1, o7))
    assert s1[-1]["delivered"] > 0


def test_oracle_rmat_generator_matches_workloads():
    """bsp_set_graph_rmat (the device generator's formula, restated in C and threaded) gives the
    same graph as workloads.rmat_cols: the power-law run is identical either way."""
    runs = []
    for dev in (True, False):
        x = wl.power_law_forward(60_000, ttl=6, capacity=16, device_graph=dev)
        o = BspOracle(**x.engine_kwargs())
        x.apply_to(o)
        st = o.run()
        runs.append((st, o.read_state()[0]))
        o.close()
    assert runs[0][0] == runs[1][0] and np.array_equal(runs[0][1], runs[1][1])
