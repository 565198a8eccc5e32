"""GpuEngine: the Python host over the C ABI (include/akka_gpu.h).

One GpuEngine = one rank of the actor population on one GPU.  All arrays that
cross the boundary are plain numpy buffers (u32 ids/payloads, u64 state words).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import AgxCfg, AgxStats, check

NO_SENDER = 0xFFFFFFFF


class Kind:
    """Behaviour kinds (enum agx_behavior_kind)."""
    NONE = 0
    COUNTER = 1
    RING = 2
    FANOUT = 3
    FORWARD_RR = 4
    STOP_AFTER = 5
    PINGPONG = 6
    EVEN = 7
    GCOUNTER = 8      # Replicator-style replicas (akka-distributed-data), include/akka_gpu.h "CRDT behaviours"
    PNCOUNTER = 9
    ORSET = 10


CRDT_NODES = 8
ORSET_ELEMS = 64
CRDT_WORDS = {Kind.GCOUNTER: 8, Kind.PNCOUNTER: 16, Kind.ORSET: 260}
# delta-CRDT mode (agx_set_delta_crdt): data + envelope/selector area + delta log (include/akka_gpu.h)
DELTA_ENV_WORDS, DELTA_LOG = 12, 64
CRDT_DELTA_WORDS = {k: w + DELTA_ENV_WORDS + (DELTA_LOG * 6 if k == Kind.ORSET else 4) for k, w in CRDT_WORDS.items()}
DELTA_WRITE = 0x800000
WIDE_BIT = 0x80000000


class Op:
    """Control-tell opcodes of the CRDT kinds: payload = (op << 24) | arg."""
    INCREMENT = 1
    DECREMENT = 2
    ADD = 3
    REMOVE = 4
    CLEAR = 5
    GOSSIP = 6
    DELTA_TICK = 7

    @staticmethod
    def make(op: int, arg: int = 0) -> int:
        return ((op & 0xFF) << 24) | (arg & 0xFFFFFF)


@dataclass
class EngineConfig:
    n_actors: int
    throughput: int = 5          # akka.actor.default-dispatcher.throughput (reference.conf:541)
    capacity: int = 0            # bounded mailbox capacity, 0 = unbounded
    n_words: int = 2
    max_emit: int = 1
    n_ranks: int = 1
    rank: int = 0
    num_shards: int = 1000
    device: int = 0
    msg_capacity: int = 0
    bucket_actors: int = 0       # actors per apply bucket (0 = 2048; power of two in [32, 2048])

    def to_c(self) -> AgxCfg:
        c = AgxCfg()
        c.abi_version = _lib.ABI_VERSION
        c.device = self.device
        c.n_actors = self.n_actors
        # throughput <= 0 behaves as 1 (Mailbox.scala:261); keep the value, the engine clamps
        c.throughput = max(int(self.throughput), 0) & 0xFFFFFFFF
        c.capacity = int(self.capacity)
        c.n_words = int(self.n_words)
        c.max_emit = int(self.max_emit)
        c.n_ranks = int(self.n_ranks)
        c.rank = int(self.rank)
        c.num_shards = int(self.num_shards)
        c.msg_capacity = int(self.msg_capacity)
        c.bucket_actors = int(self.bucket_actors)
        return c


@dataclass
class Stats:
    delivered: int = 0
    dead_letters: int = 0
    unhandled: int = 0
    emitted: int = 0
    staged: int = 0
    supersteps: int = 0
    in_flight: int = 0
    bytes_alg: int = 0

    @classmethod
    def from_c(cls, s: AgxStats) -> "Stats":
        return cls(**s.as_dict())


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


def _ptr(a: np.ndarray, ty):
    return a.ctypes.data_as(ctypes.POINTER(ty))


class GpuEngine:
    """One rank of the batched dispatcher.  Mirrors agx_* one to one."""

    def __init__(self, cfg: EngineConfig):
        self.lib = _lib.load()
        self.cfg = cfg
        h = ctypes.c_void_p()
        c = cfg.to_c()
        check(self.lib.agx_create(ctypes.byref(c), ctypes.byref(h)))
        self._h = h

    # -- lifecycle
    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            check(self.lib.agx_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    # -- registration
    def register_range(self, first: int, count: int, kind: int, init_state=None) -> None:
        W = self.cfg.n_words
        if init_state is None:
            check(self.lib.agx_register_range(self._h, first, count, kind, None, 0))
            return
        st = np.ascontiguousarray(np.asarray(init_state, dtype=np.uint64).reshape(count, -1))
        if st.shape[1] < W:
            st = np.concatenate([st, np.zeros((count, W - st.shape[1]), np.uint64)], axis=1)
        st = np.ascontiguousarray(st[:, :W])
        check(self.lib.agx_register_range(self._h, first, count, kind, st.ctypes.data_as(ctypes.c_void_p), W * 8))

    def set_ring(self, stride: int = 1) -> None:
        check(self.lib.agx_set_ring(self._h, stride))

    def set_mailbox_class(self, cls: int, capacity: int) -> None:
        """A further mailbox type of this dispatcher (agx_set_mailbox_class): bounded-capacity:N -> N,
        an unbounded type -> 0 (Mailboxes.lookupConfigurator, Mailboxes.scala:204-260)."""
        check(self.lib.agx_set_mailbox_class(self._h, cls, capacity))

    def set_mailbox(self, first: int, count: int, cls: int) -> None:
        """Bind actors [first, first + count) to mailbox class `cls` (agx_set_mailbox)."""
        check(self.lib.agx_set_mailbox(self._h, first, count, cls))

    def set_outbound(self, first_host_id: int, n_host: int, capacity: int = 1 << 20) -> None:
        """Host-side actor ids [first_host_id, +n_host): GPU tells to them go to the outbox
        (agx_set_outbound; the reply path of sender() ! reply, ActorCell.scala:583-587)."""
        check(self.lib.agx_set_outbound(self._h, first_host_id, n_host, capacity))

    def take_outbound(self, cap: int = 1 << 24):
        """agx_take_outbound: (dst, src, payload) arrays, each sender's tells in emission order."""
        d, s, p = (np.zeros(cap, np.uint32) for _ in range(3))
        n = ctypes.c_uint64()
        check(self.lib.agx_take_outbound(self._h, _ptr(d, ctypes.c_uint32), _ptr(s, ctypes.c_uint32),
                                         _ptr(p, ctypes.c_uint32), cap, ctypes.byref(n)))
        k = int(n.value)
        return d[:k], s[:k], p[:k]

    def set_gossip(self, fanout: int, seed: int) -> None:
        check(self.lib.agx_set_gossip(self._h, fanout, seed))

    def set_behaviors(self, tables) -> None:
        """Compiled behaviours (akka_amd.typed.compile_behaviors -> agx_set_behaviors)."""
        check(self.lib.agx_set_behaviors(self._h, ctypes.addressof(tables.cases), len(tables.cases),
                                         ctypes.addressof(tables.acts), len(tables.acts),
                                         _ptr(tables.first, ctypes.c_uint32), tables.n_behaviors))

    def set_delta_crdt(self, max_delta_size: int) -> None:
        """Replicator delta-crdt.enabled / max-delta-size (0 = off)."""
        check(self.lib.agx_set_delta_crdt(self._h, max_delta_size))

    def set_fanout(self, k: int, seed: int, cdf, perm) -> None:
        cdf = _u32(cdf)
        perm = _u32(perm)
        check(self.lib.agx_set_fanout(self._h, k, seed, _ptr(cdf, ctypes.c_uint32), _ptr(perm, ctypes.c_uint32),
                                      cdf.size))

    def set_graph(self, row_ptr, col) -> None:
        rp = np.ascontiguousarray(np.asarray(row_ptr, dtype=np.uint64))
        cl = _u32(col) if len(col) else np.zeros(1, np.uint32)
        check(self.lib.agx_set_graph(self._h, _ptr(rp, ctypes.c_uint64), _ptr(cl, ctypes.c_uint32)))

    def set_graph_rmat(self, row_ptr, bits: int, ta: int, tb: int, tc: int, seed: int) -> None:
        """CSR rows from the host, R-MAT destinations generated on the device."""
        rp = np.ascontiguousarray(np.asarray(row_ptr, dtype=np.uint64))
        check(self.lib.agx_set_graph_rmat(self._h, _ptr(rp, ctypes.c_uint64), bits, ta, tb, tc, seed))

    # -- tell / run
    def tell(self, dst, payload, src=None) -> None:
        dst = _u32(dst)
        pay = _u32(np.broadcast_to(np.asarray(payload, dtype=np.uint32), dst.shape))  # (a scalar: every tell)
        srcp = None
        if src is not None:
            s = _u32(np.broadcast_to(np.asarray(src, dtype=np.uint32), dst.shape))
            srcp = _ptr(s, ctypes.c_uint32)
        check(self.lib.agx_stage_tells(self._h, _ptr(dst, ctypes.c_uint32), srcp, _ptr(pay, ctypes.c_uint32),
                                       dst.size))

    def tell_one(self, dst: int, payload: int, src: int = NO_SENDER) -> bool:
        """agx_tell (any thread, lock-free): True iff the caller must submit the pump (the engine
        went from idle to scheduled)."""
        sched = ctypes.c_int32(0)
        check(self.lib.agx_tell(self._h, dst, src, payload, ctypes.byref(sched)))
        return bool(sched.value)

    def pump_idle(self) -> bool:
        """agx_pump_idle (the pump's last call): True iff the pump must be submitted again -- tells
        arrived meanwhile or wait for capacity, or the last run left mail in flight."""
        again = ctypes.c_int32(0)
        check(self.lib.agx_pump_idle(self._h, ctypes.byref(again)))
        return bool(again.value)

    def pump_cancel(self) -> None:
        """agx_pump_cancel: the pump could not be submitted; back to idle without the re-check."""
        check(self.lib.agx_pump_cancel(self._h))

    def run(self, max_supersteps: int = 1 << 30, stats: bool = True) -> Stats | None:
        """agx_run.  stats=False skips the counter read-back (read them with stats())."""
        if not stats:
            check(self.lib.agx_run(self._h, min(int(max_supersteps), 0xFFFFFFFF), None))
            return None
        st = AgxStats()
        check(self.lib.agx_run(self._h, min(int(max_supersteps), 0xFFFFFFFF), ctypes.byref(st)))
        return Stats.from_c(st)

    def run_timed(self, max_supersteps: int) -> tuple:
        """agx_run_timed: (stats, device ms of the run: HIP events on the engine stream)."""
        st = AgxStats()
        ms = ctypes.c_float()
        check(self.lib.agx_run_timed(self._h, min(int(max_supersteps), 0xFFFFFFFF), ctypes.byref(st), ctypes.byref(ms)))
        return Stats.from_c(st), float(ms.value)

    def identity_supersteps(self) -> int:
        """Multi-pass supersteps grouped without a radix pass (agx_identity_supersteps)."""
        v = ctypes.c_uint64()
        check(self.lib.agx_identity_supersteps(self._h, ctypes.byref(v)))
        return int(v.value)

    def ring_buckets(self) -> int:
        """Buckets whose queued messages live in bounded-mailbox rings (agx_ring_buckets)."""
        v = ctypes.c_uint64()
        check(self.lib.agx_ring_buckets(self._h, ctypes.byref(v)))
        return v.value

    def exchange_info(self) -> dict:
        """This rank's multi-rank exchange accounting (agx_exchange_info)."""
        v = (ctypes.c_uint64 * 6)()
        check(self.lib.agx_exchange_info(self._h, v))
        return {"dev_steps": v[0], "host_steps": v[1], "env_bytes": v[2], "row_bytes": v[3],
                "rows_on_host": bool(v[4]), "slab": v[5]}

    def persist_info(self) -> dict:
        """Replays run as one persistent launch and their supersteps (agx_persist_info)."""
        v = (ctypes.c_uint64 * 2)()
        check(self.lib.agx_persist_info(self._h, v))
        return {"launches": v[0], "supersteps": v[1]}

    def stats(self) -> Stats:
        st = AgxStats()
        check(self.lib.agx_get_stats(self._h, ctypes.byref(st)))
        return Stats.from_c(st)

    def read_state(self, first: int = 0, count: int | None = None):
        if count is None:
            count = self.cfg.n_actors - first
        W = self.cfg.n_words
        words = np.zeros((count, W), np.uint64)
        alive = np.zeros(count, np.uint8)
        check(self.lib.agx_read_state(self._h, first, count, _ptr(words, ctypes.c_uint64),
                                      _ptr(alive, ctypes.c_uint8)))
        return words, alive

    # -- multi-GPU
    @staticmethod
    def comm_unique_id() -> bytes:
        lib = _lib.load()
        buf = (ctypes.c_uint8 * 128)()
        check(lib.agx_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid: bytes) -> None:
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(self.lib.agx_comm_init(self._h, buf))

    @staticmethod
    def group_run(engines: list["GpuEngine"], max_supersteps: int = 1 << 30) -> Stats:
        lib = _lib.load()
        arr = (ctypes.c_void_p * len(engines))(*[e._h.value for e in engines])
        st = AgxStats()
        check(lib.agx_group_run(arr, len(engines), min(int(max_supersteps), 0xFFFFFFFF), ctypes.byref(st)))
        return Stats.from_c(st)

    # -- measurement
    def profile(self, on: bool = True) -> None:
        check(self.lib.agx_profile_enable(self._h, 1 if on else 0))

    def profile_reset(self) -> None:
        check(self.lib.agx_profile_reset(self._h))

    def profile_read(self) -> dict:
        cap = 16
        names = (ctypes.c_char * 32 * cap)()
        ms = (ctypes.c_double * cap)()
        launches = (ctypes.c_uint64 * cap)()
        items = (ctypes.c_uint64 * cap)()
        n = ctypes.c_uint32()
        check(self.lib.agx_profile_read(self._h, names, ms, launches, items, cap, ctypes.byref(n)))
        out = {}
        for i in range(min(n.value, cap)):
            out[bytes(names[i]).split(b"\0")[0].decode()] = {"total_ms": ms[i], "launches": int(launches[i]),
                                                             "items": int(items[i])}
        return out


def shard_id(entity_id: int, num_shards: int = 1000) -> int:
    """HashCodeMessageExtractor.shardId for a numeric entity id (native helper)."""
    return int(_lib.load().agx_shard_id(entity_id, num_shards))


def owner(entity_id: int, num_shards: int, n_ranks: int) -> int:
    return int(_lib.load().agx_owner(entity_id, num_shards, n_ranks))


MR_GO, MR_OVER_SLAB, MR_QUIET, MR_OVER_CAPACITY = 0, 1, 2, 3


def mr_plan(mat, rank: int, slab: int, cap: int) -> dict:
    """agx_mr_plan: the device-resident replays' decision for one superstep (the same code as
    k_mr_pack): code (MR_*), this rank's send / receive offsets (R + 1 each) and backlog."""
    m = np.ascontiguousarray(np.asarray(mat, dtype=np.uint64))
    R = m.shape[0]
    so, ro = np.zeros(R + 1, np.uint64), np.zeros(R + 1, np.uint64)
    code, nbl = ctypes.c_uint32(), ctypes.c_uint64()
    check(_lib.load().agx_mr_plan(_ptr(m, ctypes.c_uint64), R, rank, slab, cap, ctypes.byref(code),
                                  _ptr(so, ctypes.c_uint64), _ptr(ro, ctypes.c_uint64), ctypes.byref(nbl)))
    return {"code": int(code.value), "send_off": so, "recv_off": ro, "n_backlog": int(nbl.value)}


def mr_initial_slab(n_global: int, max_emit: int, R: int) -> int:
    """The first slab size of the device-resident replays (agx_engine.hip mr_initial_slab)."""
    share = n_global * max_emit // (R * R)
    return min(share + share // 4 + 1024, 1 << 30)


def exchange_plan(mat, rank: int) -> dict:
    """agx_exchange_plan: this rank's send/recv counts and offsets (host only)."""
    m = np.ascontiguousarray(np.asarray(mat, dtype=np.uint64))
    R = m.shape[0]
    out = {k: np.zeros(R, np.uint64) for k in ("send_cnt", "send_off", "recv_cnt", "recv_off")}
    infl = ctypes.c_uint64()
    check(_lib.load().agx_exchange_plan(_ptr(m, ctypes.c_uint64), R, rank, *(_ptr(out[k], ctypes.c_uint64) for k in
                                                                          ("send_cnt", "send_off", "recv_cnt",
                                                                           "recv_off")), ctypes.byref(infl)))
    out["inflight"] = int(infl.value)
    return out
