"""Deterministic synthetic workloads (BASELINE.json configs C1..C5).

Everything is integer and seeded (SplitMix64 counter RNG),
so the same inputs feed the GPU engine, the CPU oracles and the benchmark.
A workload is a plain description: actor ranges + behaviour params + initial
tells; `apply_to(target)` installs it into anything with the engine's
register_range / set_* / tell interface.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .engine import CRDT_DELTA_WORDS, CRDT_NODES, CRDT_WORDS, DELTA_WRITE, Kind, NO_SENDER, Op

SEED = 0x5EED
M64 = (1 << 64) - 1


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    """Vectorised SplitMix64 finaliser (uint64 wrapping arithmetic)."""
    z = (np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15))
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


@dataclass
class Workload:
    name: str
    n_actors: int
    n_words: int
    max_emit: int
    throughput: int
    capacity: int
    ranges: list = field(default_factory=list)  # (first, count, kind, init_state or None)
    ring_stride: int | None = None
    gossip: tuple | None = None  # (fanout, seed)
    delta_crdt: int = 0          # Replicator max-delta-size (0 = full-state gossip only)
    behaviors: object = None     # compiled behaviour tables (akka_amd.typed.Tables)
    fanout: tuple | None = None  # (k, seed, cdf, perm)
    graph: tuple | None = None   # (row_ptr, col)
    tells: tuple | None = None   # (dst, src, payload)
    bucket_actors: int = 0       # GPU engine hint (agx_cfg.bucket_actors): deep mailboxes want small buckets
    mailbox_classes: dict = field(default_factory=dict)  # class -> capacity (agx_set_mailbox_class)
    mailboxes: list = field(default_factory=list)         # (first, count, class) (agx_set_mailbox)
    outbound: tuple | None = None                         # (first_host_id, n_host) (agx_set_outbound)

    def engine_kwargs(self) -> dict:
        """Semantic parameters (shared by the GPU engine and the CPU oracles)."""
        return dict(n_actors=self.n_actors, throughput=self.throughput, capacity=self.capacity,
                    n_words=self.n_words, max_emit=self.max_emit)

    def gpu_kwargs(self) -> dict:
        """engine_kwargs + the GPU engine's layout hints (EngineConfig)."""
        return dict(self.engine_kwargs(), bucket_actors=self.bucket_actors)

    def apply_to(self, target, stage_tells: bool = True) -> None:
        for first, count, kind, init in self.ranges:
            target.register_range(first, count, kind, init)
        for cls, cap in self.mailbox_classes.items():
            target.set_mailbox_class(cls, cap)
        for first, count, cls in self.mailboxes:
            target.set_mailbox(first, count, cls)
        if self.outbound is not None:
            target.set_outbound(*self.outbound)
        if self.ring_stride is not None:
            target.set_ring(self.ring_stride)
        if self.gossip is not None:
            target.set_gossip(*self.gossip)
        if self.delta_crdt:
            target.set_delta_crdt(self.delta_crdt)
        if self.behaviors is not None:
            target.set_behaviors(self.behaviors)
        if self.fanout is not None:
            target.set_fanout(*self.fanout)
        if self.graph is not None:
            if len(self.graph) == 3 and isinstance(self.graph[0], str):  # ("rmat", row_ptr, params)
                _, row, prm = self.graph
                if hasattr(target, "set_graph_rmat"):
                    target.set_graph_rmat(row, *prm)
                else:
                    target.set_graph(row, rmat_cols(int(row[-1]), self.n_actors, *prm))
            else:
                target.set_graph(*self.graph)
        if stage_tells and self.tells is not None:
            dst, src, pay = self.tells
            target.tell(dst, pay, src)

    @property
    def n_tells(self) -> int:
        return 0 if self.tells is None else int(len(self.tells[0]))


# ------------------------------------------------------------------ C2
def token_ring(n: int = 1_000_000, hops: int = 256, throughput: int = 5, tokens_per_actor: int = 1) -> Workload:
    """C2: every actor starts with `tokens_per_actor` tokens with hop budget H;
    RING behaviour: count++, forward payload-1 to (self+1) mod N while > 0.
    Delivered = tokens * N * (H + 1)."""
    dst = np.tile(np.arange(n, dtype=np.uint32), tokens_per_actor)
    pay = np.full(dst.size, hops, np.uint32)
    src = np.full(dst.size, NO_SENDER, np.uint32)
    return Workload("token_ring", n, 1, 1, throughput, 0, [(0, n, Kind.RING, None)], ring_stride=1,
                    tells=(dst, src, pay))


# ------------------------------------------------------------------ C3
def zipf_tables(n: int, s: float = 1.1, seed: int = SEED):
    """Zipf(s) over a seeded permutation of the actors, as u32 CDF thresholds:
    sample i = smallest i with u32(r >> 32) <= cdf[i]; actor = perm[i]."""
    ranks = np.arange(1, n + 1, dtype=np.float64)
    w = ranks ** (-s)
    cum = np.cumsum(w)
    cum /= cum[-1]
    cdf = np.floor(cum * 4294967296.0) - 1.0
    cdf = np.clip(cdf, 0, 4294967295.0).astype(np.uint64)
    cdf = np.maximum.accumulate(cdf)
    cdf[-1] = 0xFFFFFFFF
    key = splitmix64_np(np.arange(n, dtype=np.uint64) ^ np.uint64(seed))
    perm = np.argsort(key, kind="stable").astype(np.uint32)
    return cdf.astype(np.uint32), perm


def zipf_fanout(n: int = 10_000_000, k: int = 4, ttl: int = 3, root_every: int = 64, s: float = 1.1,
                throughput: int = 5, seed: int = SEED, capacity: int = 0) -> Workload:
    """C3: 1/root_every actors are roots holding one message with ttl; FANOUT
    behaviour: count++, sum += payload, if ttl > 0 emit k tells to Zipf targets."""
    cdf, perm = zipf_tables(n, s, seed)
    roots = np.arange(0, n, root_every, dtype=np.uint32)
    h = (splitmix64_np(roots.astype(np.uint64) ^ np.uint64(seed * 3)) & np.uint64(0x00FFFFFF)).astype(np.uint32)
    pay = (np.uint32(ttl) << np.uint32(24)) | h
    src = np.full(roots.size, NO_SENDER, np.uint32)
    return Workload("zipf_fanout", n, 2, k, throughput, capacity, [(0, n, Kind.FANOUT, None)],
                    fanout=(k, seed, cdf, perm), tells=(roots, src, pay.astype(np.uint32)))


# ------------------------------------------------------------------ C4
def crdt_ops(n: int, kind: int, ops_per_actor: int, seed: int = SEED):
    """Round-0 local updates, one row per actor: INCREMENT (GCounter), INCREMENT/DECREMENT
    (PNCounter), ADD/REMOVE of one of the 64 elements, 3:1 (ORSet)."""
    a = np.arange(n, dtype=np.uint64)
    out = np.zeros((n, ops_per_actor), np.uint32)
    for j in range(ops_per_actor):
        r = splitmix64_np((a << np.uint64(8)) ^ np.uint64(j) ^ np.uint64(seed * 11))
        lo = (r & np.uint64(0xFFFF)).astype(np.uint32)
        hi = ((r >> np.uint64(32)) & np.uint64(0xFF)).astype(np.uint32)
        if kind == Kind.GCOUNTER:
            op, arg = np.full(n, Op.INCREMENT, np.uint32), lo % 100 + 1
        elif kind == Kind.PNCOUNTER:
            op = np.where(hi % 3 == 0, Op.DECREMENT, Op.INCREMENT).astype(np.uint32)
            arg = lo % 100 + 1
        else:
            op = np.where(hi % 4 == 0, Op.REMOVE, Op.ADD).astype(np.uint32)
            arg = lo % 64
        out[:, j] = (op << np.uint32(24)) | arg
    return out


def crdt_gossip(n: int = 1_000_000, kind: int = Kind.GCOUNTER, rounds: int = 32, fanout: int = 2,
                ops_per_writer: int = 16, throughput: int = 5, seed: int = SEED, capacity: int = 0) -> Workload:
    """C4: Replicator-style replicas.  Actors 0..7 are the writers of node slots 0..7
    (one writer per UniqueAddress, as the CRDTs require) and first apply `ops_per_writer`
    local updates (host tells); then every actor runs `rounds` GossipTicks: each tick sends
    its full state to `fanout` random peers, which merge it
    (DD/Replicator.scala:2029-2064,2118-2133).  The population converges to the merge
    of the 8 writers' values."""
    nw = min(n, CRDT_NODES)
    ops = crdt_ops(nw, kind, ops_per_writer, seed).reshape(-1)
    odst = np.repeat(np.arange(nw, dtype=np.uint32), ops_per_writer)
    tdst = np.arange(n, dtype=np.uint32)
    tick = np.full(n, Op.make(Op.GOSSIP, rounds - 1), np.uint32)
    dst = np.concatenate([odst, tdst])
    pay = np.concatenate([ops, tick])
    src = np.full(dst.size, NO_SENDER, np.uint32)
    # a replica receives its tick + `fanout` gossips per superstep: buckets of 512 replicas keep
    # the ~3 x 512 messages in one 2048-message apply tile (the fast path)
    return Workload(f"crdt_gossip_{kind}", n, CRDT_WORDS[kind], fanout + 1, throughput, capacity,
                    [(0, n, kind, None)], gossip=(fanout, seed), tells=(dst, src, pay), bucket_actors=512)


def crdt_delta(n: int = 1_000_000, kind: int = Kind.ORSET, rounds: int = 32, write: bool = True,
               ops_per_replica: int = 0, gossip_rounds: int = 0, fanout: int = 1, max_delta_size: int = 50,
               throughput: int = 5, seed: int = SEED, capacity: int = 0, bucket_actors: int = 0) -> Workload:
    """C4 with delta-CRDT replication (Replicator delta-crdt.enabled, DD/Replicator.scala:1646-1695,
    1953-2027; DD/DeltaPropagationSelector.scala): keys of 8 replicas (id = 8 * key + node).  Each
    replica first applies `ops_per_replica` host updates, then runs `rounds` DeltaPropagationTicks
    (`write`: each tick also tells the replica one seeded Update, a writer client) and, if
    `gossip_rounds`, that many full-state GossipTicks to `fanout` random replicas of its key.
    bucket_actors 0: 2048 replicas per bucket (every bucket in the skew launch), measured after
    round 6's phase-B schedule against 512 / 1024: ORSet +8 %, GCounter +10 %."""
    if not bucket_actors:
        bucket_actors = 2048
    ids = np.arange(n, dtype=np.uint32)
    dsts, pays = [], []
    if ops_per_replica:
        dsts.append(np.repeat(ids, ops_per_replica))
        pays.append(crdt_ops(n, kind, ops_per_replica, seed).reshape(-1))
    if rounds:
        dsts.append(ids)
        pays.append(np.full(n, Op.make(Op.DELTA_TICK, (rounds - 1) | (DELTA_WRITE if write else 0)), np.uint32))
    if gossip_rounds:
        dsts.append(ids)
        pays.append(np.full(n, Op.make(Op.GOSSIP, gossip_rounds - 1), np.uint32))
    dst = np.concatenate(dsts)
    pay = np.concatenate(pays)
    src = np.full(dst.size, NO_SENDER, np.uint32)
    return Workload(f"crdt_delta_{kind}", n, CRDT_DELTA_WORDS[kind], max(4, fanout + 1), throughput, capacity,
                    [(0, n, kind, None)], gossip=(fanout, seed), delta_crdt=max_delta_size, tells=(dst, src, pay),
                    bucket_actors=bucket_actors)


def crdt_mixed(n: int = 4096, rounds: int = 4, seed: int = 3, throughput: int = 3, capacity: int = 0) -> Workload:
    """GCounter / PNCounter / ORSet replicas beside COUNTER and EVEN actors: gossips that
    land on a non-CRDT actor (or an ORSet op on a counter) are Behaviors.unhandled."""
    kinds = [Kind.GCOUNTER, Kind.PNCOUNTER, Kind.ORSET, Kind.COUNTER, Kind.EVEN]
    per = n // len(kinds)
    ranges, dsts, pays = [], [], []
    rng = np.random.default_rng(seed)
    for i, kd in enumerate(kinds):
        first = i * per
        count = per if i < len(kinds) - 1 else n - first
        ranges.append((first, count, kd, None))
        ids = np.arange(first, first + count, dtype=np.uint32)
        if kd in CRDT_WORDS:
            ops = crdt_ops(count, kd, 3, seed + i)
            tick = np.full((count, 1), Op.make(Op.GOSSIP, rounds - 1), np.uint32)
            dsts.append(np.repeat(ids, 4))
            pays.append(np.concatenate([ops, tick], axis=1).reshape(-1))
    m = n
    dsts.append(rng.integers(0, n, m).astype(np.uint32))  # random control ops everywhere
    pays.append(((rng.integers(1, 8, m).astype(np.uint32) << 24) | rng.integers(0, 70, m).astype(np.uint32)))
    dst = np.concatenate(dsts)
    pay = np.concatenate(pays)
    src = np.full(dst.size, NO_SENDER, np.uint32)
    return Workload("crdt_mixed", n, CRDT_WORDS[Kind.ORSET], 3, throughput, capacity, ranges, gossip=(2, seed),
                    tells=(dst, src, pay))


# ------------------------------------------------------------------ C5
RMAT_ABC = (0.57, 0.19, 0.19)


def power_law_degrees(n: int, alpha: float = 2.1, dmax: int = 1024, seed: int = SEED) -> np.ndarray:
    """CSR row pointer (u64, n+1) of out-degrees ~ d^-alpha on [1, dmax], one integer
    draw per actor against host-built u32-scaled thresholds."""
    d = np.arange(1, dmax + 1, dtype=np.float64)
    p = d ** (-alpha)
    cdf = np.cumsum(p) / p.sum()
    thr = np.floor(cdf * 4294967296.0).astype(np.uint64)
    thr[-1] = 1 << 32
    row = np.zeros(n + 1, np.uint64)
    for lo in range(0, n, 1 << 24):  # chunked: bounded temporaries at 10^8 actors
        hi = min(n, lo + (1 << 24))
        r = splitmix64_np(np.arange(lo, hi, dtype=np.uint64) ^ np.uint64(seed * 7)) >> np.uint64(32)
        deg = np.minimum(np.searchsorted(thr, r, side="right") + 1, dmax).astype(np.uint64)
        row[lo + 1:hi + 1] = deg
    np.cumsum(row, out=row)
    return row


def rmat_params(n: int, a: float = RMAT_ABC[0], b: float = RMAT_ABC[1], c: float = RMAT_ABC[2],
                seed: int = SEED) -> tuple:
    """(bits, ta, tb, tc, seed) of the R-MAT destination draw (agx_set_graph_rmat)."""
    bits = max(1, int(np.ceil(np.log2(max(n, 2)))))
    return bits, int(a * 65536), int((a + b) * 65536), int((a + b + c) * 65536), seed


def rmat_cols(m: int, n: int, bits: int, ta: int, tb: int, tc: int, seed: int) -> np.ndarray:
    """Destination of every edge id in [0, m): `bits` quadrant draws q = splitmix64(e*64 + bit +
    seed) & 0xFFFF, destination bit = (ta <= q < tb) | (q >= tc), reduced mod n."""
    col = np.zeros(m, np.uint64)
    eid = np.arange(m, dtype=np.uint64)
    for bit in range(bits):
        rr = splitmix64_np(eid * np.uint64(64) + np.uint64(bit) + np.uint64(seed)) & np.uint64(0xFFFF)
        dst_bit = ((rr >= np.uint64(ta)) & (rr < np.uint64(tb))) | (rr >= np.uint64(tc))
        col |= dst_bit.astype(np.uint64) << np.uint64(bits - 1 - bit)
    col %= np.uint64(n)
    return col.astype(np.uint32)


def power_law_graph(n: int, alpha: float = 2.1, dmax: int = 1024, a: float = RMAT_ABC[0], b: float = RMAT_ABC[1],
                    c: float = RMAT_ABC[2], seed: int = SEED):
    """Out-degrees ~ d^-alpha on [1, dmax]; endpoints by R-MAT bit sampling.
    Integer RNG throughout (float only to build the host-side degree table)."""
    row = power_law_degrees(n, alpha, dmax, seed)
    return row, rmat_cols(int(row[-1]), n, *rmat_params(n, a, b, c, seed))


def power_law_forward(n: int = 100_000_000, ttl: int = 16, capacity: int = 64, throughput: int = 5,
                      msgs_per_actor_den: int = 1, seed: int = SEED, device_graph: bool = False) -> Workload:
    """C5: FORWARD_RR over a power-law graph with BoundedMailbox(capacity).
    device_graph: the R-MAT destinations are generated by the engine (agx_set_graph_rmat);
    targets without that entry point (the CPU oracle) get them from rmat_cols."""
    row = power_law_degrees(n, seed=seed)
    graph = ("rmat", row, rmat_params(n, seed=seed)) if device_graph else (row, rmat_cols(
        int(row[-1]), n, *rmat_params(n, seed=seed)))
    dst = np.arange(0, n, msgs_per_actor_den, dtype=np.uint32)
    pay = np.full(dst.size, ttl, np.uint32)
    src = np.full(dst.size, NO_SENDER, np.uint32)
    return Workload("power_law_forward", n, 2, 1, throughput, capacity, [(0, n, Kind.FORWARD_RR, None)],
                    graph=graph, tells=(dst, src, pay))


# ------------------------------------------------------------------ C1
def ping_pong(pairs: int = 1000, messages_per_pair: int = 2_000_000, throughput: int = 50,
              in_flight: int | None = None) -> Workload:
    """C1: BenchmarkActors.PingPong pairs (akka-bench-jmh/.../BenchmarkActors.scala:20-32,96-117):
    left = messagesPerPair/2 per actor, inFlight = 2*throughput initial tells
    `ping.tell(Message, pong)` per pair."""
    if in_flight is None:
        in_flight = 2 * throughput
    n = 2 * pairs
    init = np.zeros((n, 2), np.uint64)
    init[:, 0] = messages_per_pair // 2
    ping = np.arange(0, n, 2, dtype=np.uint32)
    dst = np.repeat(ping, in_flight)
    src = dst + np.uint32(1)
    pay = np.zeros(dst.size, np.uint32)
    # in_flight tells per pair: ~in_flight/2 queued per actor -> buckets of 2048/in_flight actors fit one tile
    ba = max(32, min(2048, 1 << max(0, (2048 // max(in_flight, 1)).bit_length() - 1)))
    return Workload("ping_pong", n, 2, 1, throughput, 0, [(0, n, Kind.PINGPONG, init)], tells=(dst, src, pay),
                    bucket_actors=ba)


# ------------------------------------------------------------------ small mixed workload for parity tests
def mixed(n: int = 4096, seed: int = 1, throughput: int = 3, capacity: int = 0, tells_per_actor: int = 3) -> Workload:
    """Every behaviour kind side by side (ranges), random tells between them."""
    rng = np.random.default_rng(seed)
    kinds = [Kind.COUNTER, Kind.RING, Kind.FANOUT, Kind.FORWARD_RR, Kind.STOP_AFTER, Kind.PINGPONG, Kind.EVEN,
             Kind.NONE]
    per = n // len(kinds)
    ranges = []
    for i, kd in enumerate(kinds):
        first = i * per
        count = per if i < len(kinds) - 1 else n - first
        init = None
        if kd == Kind.STOP_AFTER:
            init = np.zeros((count, 2), np.uint64)
            init[:, 1] = rng.integers(1, 6, count)
        elif kd == Kind.PINGPONG:
            init = np.zeros((count, 2), np.uint64)
            init[:, 0] = rng.integers(0, 5, count)
        ranges.append((first, count, kd, init))
    cdf, perm = zipf_tables(n, 1.1, seed)
    row, col = power_law_graph(n, seed=seed)
    m = n * tells_per_actor
    dst = rng.integers(0, n + 8, m).astype(np.uint32)  # a few unknown refs -> dead letters
    src = rng.integers(0, n, m).astype(np.uint32)
    src[rng.random(m) < 0.1] = NO_SENDER
    pay = rng.integers(0, 12, m).astype(np.uint32)
    # fan-out payloads carry ttl in the top 8 bits
    fan_first, fan_count = ranges[2][0], ranges[2][1]
    is_fan = (dst >= fan_first) & (dst < fan_first + fan_count)
    pay[is_fan] = (rng.integers(0, 3, int(is_fan.sum())).astype(np.uint32) << 24) | rng.integers(
        0, 1 << 24, int(is_fan.sum())).astype(np.uint32)
    return Workload("mixed", n, 2, 2, throughput, capacity, ranges, ring_stride=7, fanout=(2, seed, cdf, perm),
                    graph=(row, col), tells=(dst, src, pay))


def one_per_actor(n: int = 4096, seed: int = 1, throughput: int = 3, capacity: int = 0, compiled_kinds: bool = False,
                  n_host: int = 16) -> Workload:
    """mixed()'s behaviour kinds (or the compiled library with `compiled_kinds`) with exactly one
    staged tell per actor (a permutation of the population): buckets whose inbox holds at most one
    message per actor (the dense path, agx_kernels.h dense_finish) beside buckets where forwards
    collide; stops, dead letters to stopped actors, unknown refs and replies to host-side actors
    (PINGPONG -> outbox) included."""
    rng = np.random.default_rng(seed)
    w = compiled(n, seed=seed, throughput=throughput, capacity=capacity, builtin=True) if compiled_kinds else \
        mixed(n, seed=seed, throughput=throughput, capacity=capacity)
    dst = rng.permutation(n).astype(np.uint32)
    src = rng.integers(0, n, n).astype(np.uint32)
    src[rng.random(n) < 0.1] = NO_SENDER
    if n_host:
        hs = rng.random(n) < 0.05
        src[hs] = rng.integers(n, n + n_host, int(hs.sum())).astype(np.uint32)
        w.outbound = (n, n_host)
    pay = rng.integers(0, 12, n).astype(np.uint32)
    if not compiled_kinds:  # fan-out payloads carry ttl in the top 8 bits
        fan_first, fan_count = w.ranges[2][0], w.ranges[2][1]
        is_fan = (dst >= fan_first) & (dst < fan_first + fan_count)
        pay[is_fan] = (rng.integers(0, 3, int(is_fan.sum())).astype(np.uint32) << 24) | rng.integers(
            0, 1 << 24, int(is_fan.sum())).astype(np.uint32)
    w.name = "one_per_actor"
    w.tells = (dst, src, pay)
    return w


def compiled(n: int = 4096, seed: int = 1, throughput: int = 3, capacity: int = 0, tells_per_actor: int = 3,
             builtin: bool = False) -> Workload:
    """Typed behaviours lowered by akka_amd.typed (compiled behaviour tables): the DSL versions of
    counter / ring / stop-after / ping-pong and a pair of behaviours that become each other, side
    by side (and beside the built-in kinds with `builtin`), random tells between them."""
    from . import typed
    rng = np.random.default_rng(seed)
    lib = typed.library(ring_stride=7)
    sw = typed.switch()
    tables = typed.compile_behaviors([lib["counter"], lib["ring"], lib["stop_after"], lib["ping_pong"], sw])
    kinds = [tables.kind_of(lib[k]) for k in ("counter", "ring", "stop_after", "ping_pong")] + [tables.kind_of(sw)]
    if builtin:
        kinds += [Kind.COUNTER, Kind.RING, Kind.PINGPONG, Kind.STOP_AFTER]
    per = n // len(kinds)
    ranges = []
    for i, kd in enumerate(kinds):
        first = i * per
        count = per if i < len(kinds) - 1 else n - first
        init = None
        if kd in (tables.kind_of(lib["stop_after"]), Kind.STOP_AFTER):
            init = np.zeros((count, 2), np.uint64)
            init[:, 1] = rng.integers(1, 6, count)
        elif kd in (tables.kind_of(lib["ping_pong"]), Kind.PINGPONG):
            init = np.zeros((count, 2), np.uint64)
            init[:, 0] = rng.integers(0, 5, count)
        ranges.append((first, count, kd, init))
    m = n * tells_per_actor
    dst = rng.integers(0, n + 8, m).astype(np.uint32)  # a few unknown refs -> dead letters
    src = rng.integers(0, n, m).astype(np.uint32)
    src[rng.random(m) < 0.1] = NO_SENDER
    pay = rng.integers(0, 12, m).astype(np.uint32)
    sw_first, sw_count = ranges[4][0], ranges[4][1]
    is_sw = (dst >= sw_first) & (dst < sw_first + sw_count)
    k = int(is_sw.sum())
    pay[is_sw] = (rng.integers(1, 4, k).astype(np.uint32) << 24) | rng.integers(0, 6, k).astype(np.uint32)
    return Workload("compiled", n, 2, 1, throughput, capacity, ranges, ring_stride=7, tells=(dst, src, pay),
                    behaviors=tables)


def compiled_ring(n: int = 1_000_000, hops: int = 256, throughput: int = 5) -> Workload:
    """C2's token ring with the ring behaviour written in the typed DSL (akka_amd.typed.library)."""
    from . import typed
    ring = typed.library(ring_stride=1)["ring"]
    tables = typed.compile_behaviors([ring])
    w = token_ring(n, hops, throughput)
    w.name, w.ranges, w.behaviors = "compiled_ring", [(0, n, tables.kind_of(ring), None)], tables
    return w


# ------------------------------------------------------------------ per-actor mailboxes + the reply path
def mailbox_mix(n: int = 4096, seed: int = 7, throughput: int = 3, capacity: int = 0, n_host: int = 32,
                tells_per_actor: int = 3, classes: dict | None = None) -> Workload:
    """mixed() with several mailbox types in one dispatcher (Mailboxes.lookupConfigurator per actor,
    Mailboxes.scala:204-260): quarters of the population bound to bounded-capacity:2, an unbounded
    type, bounded-capacity:16 and the dispatcher default (`capacity`) -- or `classes` {class: capacity}
    for classes 1..3; plus `n_host` host-side actors
    (ids n..n+n_host-1, e.g. JVM TestProbes) that tell GPU actors -- PINGPONG actors answer them
    through the outbox (sender() ! reply, ActorCell.scala:583-587)."""
    w = mixed(n, seed=seed, throughput=throughput, capacity=capacity, tells_per_actor=tells_per_actor)
    q = n // 4
    w.name = "mailbox_mix"
    w.mailbox_classes = dict(classes) if classes else {1: 2, 2: 0, 3: 16}
    w.mailboxes = [(0, q, 1), (q, q, 2), (2 * q, q, 3)]
    if n_host:
        w.outbound = (n, n_host)
        rng = np.random.default_rng(seed + 101)
        m = max(1, n // 4)
        dst, src, pay = w.tells
        hs = rng.integers(n, n + n_host, m).astype(np.uint32)
        hd = rng.integers(0, n, m).astype(np.uint32)
        hp = rng.integers(0, 12, m).astype(np.uint32)
        # host senders to every kind; the PINGPONG range answers them
        w.tells = (np.concatenate([dst, hd]), np.concatenate([src, hs]), np.concatenate([pay, hp]))
    return w
