"""TEST INFRASTRUCTURE ONLY.  ctypes wrappers of the C/C++ oracles in this
directory (bsp_ref.c, fjp_ref.cpp).  Never imported by akka_amd/.

The oracles are CPU restatements of the reference's Dispatcher/Mailbox drain
loop (see the header of bsp_ref.c for the file:line map).  Their interface
mirrors akka_amd.engine.GpuEngine so tests can drive both with one workload.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import subprocess
import threading

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
BUILD = HERE / "_build"
_lock = threading.Lock()
_bsp = None
_fjp = None

W_MAX = 656
NO_SENDER = 0xFFFFFFFF


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("delivered", "dead_letters", "unhandled", "emitted", "staged", "supersteps", "in_flight",
                 "bytes_alg")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


def build(force: bool = False) -> None:
    """Compile the oracles with the committed Makefile (gcc/g++)."""
    with _lock:
        if force or not (BUILD / "libbsp_ref.so").exists() or not (BUILD / "libfjp_ref.so").exists():
            subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


class OutboxOverflow(RuntimeError):
    """bsp_take_outbound's AGX_ECAPACITY: outbound tells were dropped at a full outbox."""


def _u32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _load_bsp():
    global _bsp
    if _bsp is None:
        build()
        lib = ctypes.CDLL(str(BUILD / os.environ.get("AGX_BSP_LIB", "libbsp_ref.so")))
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        P32, P64, P8 = ctypes.POINTER(u32), ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_uint8)
        sig = {
            "bsp_create": (vp, [u64, u32, u32, u32, u32, u32]),
            "bsp_destroy": (None, [vp]),
            "bsp_register_range": (ctypes.c_int, [vp, u64, u64, u32, P64, u64]),
            "bsp_set_ring": (None, [vp, u32]),
            "bsp_set_mailbox_class": (ctypes.c_int, [vp, u32, u32]),
            "bsp_set_mailbox": (ctypes.c_int, [vp, u64, u64, u32]),
            "bsp_set_outbound": (ctypes.c_int, [vp, u32, u32, u64]),
            "bsp_take_outbound": (ctypes.c_int, [vp, P32, P32, P32, u64, P64]),
            "bsp_set_gossip": (None, [vp, u32, u64]),
            "bsp_set_delta_crdt": (ctypes.c_int, [vp, u32]),
            "bsp_set_behaviors": (ctypes.c_int, [vp, vp, u32, vp, u32, P32, u32]),
            "bsp_orset_merge": (None, [P64, P64]),
            "bsp_orset_add": (None, [P64, u32, u32]),
            "bsp_orset_remove": (None, [P64, u32]),
            "bsp_orset_subtract_dots": (None, [P32, P32, P32]),
            "bsp_crdt_peer": (u32, [u64, u32, u32, u32, u64]),
            "bsp_orset_delta_bytes": (u32, []),
            "bsp_orset_add_d": (None, [P64, vp, u32, u32, u32]),
            "bsp_orset_remove_d": (None, [P64, vp, u32, u32]),
            "bsp_orset_clear_d": (None, [P64, vp]),
            "bsp_orset_delta_merge": (ctypes.c_int, [vp, vp]),
            "bsp_orset_merge_delta": (None, [P64, vp]),
            "bsp_vv_compare": (u32, [P32, P32]),
            "bsp_set_fanout": (ctypes.c_int, [vp, u32, u64, P32, P32, u64]),
            "bsp_set_graph": (ctypes.c_int, [vp, P64, P32]),
            "bsp_set_graph_rmat": (ctypes.c_int, [vp, P64, u32, u32, u32, u32, u64, u32]),
            "bsp_stage": (ctypes.c_int, [vp, P32, P32, P32, u64]),
            "bsp_run": (ctypes.c_int, [vp, u32, ctypes.POINTER(Stats)]),
            "bsp_read_state": (None, [vp, u64, u64, P64, P8]),
            "bsp_java_hash_decimal": (ctypes.c_int32, [u32]),
            "bsp_shard_id": (ctypes.c_int32, [u32, u32]),
            "bsp_owner": (u32, [u32, u32, u32]),
            "bsp_splitmix64": (u64, [u64]),
            "bsp_gcounter_merge": (None, [P64, P64, P64, u32]),
            "bsp_gcounter_value": (u64, [P64, u32]),
            "bsp_gcounter_increment": (None, [P64, u32, u64]),
        }
        for k, (r, a) in sig.items():
            f = getattr(lib, k)
            f.restype = r
            f.argtypes = a
        _bsp = lib
    return _bsp


def _load_fjp():
    global _fjp
    if _fjp is None:
        build()
        lib = ctypes.CDLL(str(BUILD / os.environ.get("AGX_FJP_LIB", "libfjp_ref.so")))
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        P32, P64, P8 = ctypes.POINTER(u32), ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_uint8)
        sig = {
            "fjp_create": (vp, [u64, u32, u32, u32]),
            "fjp_destroy": (None, [vp]),
            "fjp_register_range": (ctypes.c_int, [vp, u64, u64, u32, P64, u64]),
            "fjp_set_ring": (None, [vp, u32]),
            "fjp_set_gossip": (None, [vp, u32, u64]),
            "fjp_set_delta_crdt": (ctypes.c_int, [vp, u32]),
            "fjp_set_behaviors": (ctypes.c_int, [vp, vp, u32, vp, u32, P32, u32]),
            "fjp_set_fanout": (None, [vp, u32, u64, P32, P32, u64]),
            "fjp_set_graph": (None, [vp, P64, P32]),
            "fjp_stage": (None, [vp, P32, P32, P32, u64]),
            "fjp_run": (ctypes.c_double, [vp, u32, ctypes.POINTER(Stats)]),
            "fjp_read_state": (None, [vp, u64, u64, P64, P8]),
        }
        for k, (r, a) in sig.items():
            f = getattr(lib, k)
            f.restype = r
            f.argtypes = a
        _fjp = lib
    return _fjp


class _Base:
    def _init_arr(self, count, init):
        if init is None:
            return None, 0
        st = np.ascontiguousarray(np.asarray(init, dtype=np.uint64).reshape(count, -1))
        return st, st.shape[1]


class BspOracle(_Base):
    """Deterministic BSP restatement (bsp_ref.c).  n_ranks selects the
    canonical sharded order (owner rank of the sender first)."""

    def __init__(self, n_actors, throughput=5, capacity=0, n_words=2, max_emit=1, n_ranks=1, num_shards=1000):
        self.lib = _load_bsp()
        self.n, self.W = n_actors, n_words
        self.h = self.lib.bsp_create(n_actors, max(int(throughput), 0), capacity, n_words, n_ranks, num_shards)
        if not self.h:
            raise ValueError("bsp_create failed")
        self._keep = []

    def close(self):
        if self.h:
            self.lib.bsp_destroy(self.h)
            self.h = None

    __del__ = close

    def register_range(self, first, count, kind, init=None):
        st, stride = self._init_arr(count, init)
        p = _p(st, ctypes.c_uint64) if st is not None else None
        if self.lib.bsp_register_range(self.h, first, count, kind, p, stride):
            raise ValueError("bsp_register_range failed")

    def set_ring(self, stride):
        self.lib.bsp_set_ring(self.h, stride)

    def set_mailbox_class(self, cls, capacity):
        if self.lib.bsp_set_mailbox_class(self.h, cls, capacity):
            raise ValueError("bsp_set_mailbox_class failed")

    def set_mailbox(self, first, count, cls):
        if self.lib.bsp_set_mailbox(self.h, first, count, cls):
            raise ValueError("bsp_set_mailbox failed")

    def set_outbound(self, first_host_id, n_host, capacity=1 << 20):
        if self.lib.bsp_set_outbound(self.h, first_host_id, n_host, capacity):
            raise ValueError("bsp_set_outbound failed")

    def take_outbound(self, cap=1 << 24):
        """(dst, src, payload) arrays of the outbox, canonical emission order.  Raises OutboxOverflow
        once when more than the outbox capacity was appended since the last take (the engine's
        AGX_ECAPACITY from agx_take_outbound); the kept tells come out of the next take."""
        d, s, p = (np.zeros(cap, np.uint32) for _ in range(3))
        n = ctypes.c_uint64()
        rc = self.lib.bsp_take_outbound(self.h, _p(d, ctypes.c_uint32), _p(s, ctypes.c_uint32),
                                        _p(p, ctypes.c_uint32), cap, ctypes.byref(n))
        if rc:
            raise OutboxOverflow("outbound tells dropped: more than the outbox capacity between two takes")
        k = int(n.value)
        return d[:k], s[:k], p[:k]

    def set_gossip(self, fanout, seed):
        self.lib.bsp_set_gossip(self.h, fanout, seed)

    def set_behaviors(self, t):
        first = _u32(t.first)
        self._keep.append(t) if hasattr(self, "_keep") else None
        if self.lib.bsp_set_behaviors(self.h, ctypes.addressof(t.cases), len(t.cases), ctypes.addressof(t.acts),
                                       len(t.acts), _p(first, ctypes.c_uint32), t.n_behaviors):
            raise ValueError("bsp_set_behaviors failed")

    def set_delta_crdt(self, max_delta_size):
        if self.lib.bsp_set_delta_crdt(self.h, max_delta_size):
            raise ValueError("bsp_set_delta_crdt failed")

    def set_fanout(self, k, seed, cdf, perm):
        cdf, perm = _u32(cdf), _u32(perm)
        self.lib.bsp_set_fanout(self.h, k, seed, _p(cdf, ctypes.c_uint32), _p(perm, ctypes.c_uint32), cdf.size)

    def set_graph(self, row_ptr, col):
        rp = np.ascontiguousarray(np.asarray(row_ptr, dtype=np.uint64))
        cl = _u32(col) if len(col) else np.zeros(1, np.uint32)
        self.lib.bsp_set_graph(self.h, _p(rp, ctypes.c_uint64), _p(cl, ctypes.c_uint32))

    def set_graph_rmat(self, row_ptr, bits, ta, tb, tc, seed):
        """agx_set_graph_rmat's destinations generated on the host (bsp_ref.c bsp_set_graph_rmat; the
        same formula as workloads.rmat_cols, threaded for 10^8-actor graphs)."""
        rp = np.ascontiguousarray(np.asarray(row_ptr, dtype=np.uint64))
        threads = min(len(os.sched_getaffinity(0)), 16)
        if self.lib.bsp_set_graph_rmat(self.h, _p(rp, ctypes.c_uint64), bits, ta, tb, tc, seed, threads):
            raise MemoryError("bsp_set_graph_rmat: allocation failed")

    def tell(self, dst, payload, src=None):
        dst = _u32(dst)
        pay = _u32(np.broadcast_to(np.asarray(payload, dtype=np.uint32), dst.shape))  # (a scalar: every tell)
        s = _u32(np.broadcast_to(np.asarray(NO_SENDER if src is None else src, dtype=np.uint32), dst.shape))
        if self.lib.bsp_stage(self.h, _p(dst, ctypes.c_uint32), _p(s, ctypes.c_uint32), _p(pay, ctypes.c_uint32),
                              dst.size):
            raise ValueError("bsp_stage rejected the tells")

    def run(self, max_supersteps=1 << 30):
        st = Stats()
        rc = self.lib.bsp_run(self.h, min(int(max_supersteps), 0xFFFFFFFF), ctypes.byref(st))
        if rc:
            raise OverflowError(f"bsp_run: status {rc} (delta log overflow)")
        return st.as_dict()

    def read_state(self, first=0, count=None):
        count = self.n - first if count is None else count
        w = np.zeros((count, self.W), np.uint64)
        a = np.zeros(count, np.uint8)
        self.lib.bsp_read_state(self.h, first, count, _p(w, ctypes.c_uint64), _p(a, ctypes.c_uint8))
        return w, a


class FjpOracle(_Base):
    """Multi-threaded Dispatcher/Mailbox/ForkJoinPool restatement (fjp_ref.cpp)."""

    def __init__(self, n_actors, throughput=5, capacity=0, n_words=2, max_emit=1, **_):
        self.lib = _load_fjp()
        self.n, self.W = n_actors, n_words
        self.h = self.lib.fjp_create(n_actors, max(int(throughput), 0), capacity, n_words)
        if not self.h:
            raise ValueError("fjp_create failed")
        self.wall_s = 0.0

    def close(self):
        if self.h:
            self.lib.fjp_destroy(self.h)
            self.h = None

    __del__ = close

    def register_range(self, first, count, kind, init=None):
        st, stride = self._init_arr(count, init)
        p = _p(st, ctypes.c_uint64) if st is not None else None
        if self.lib.fjp_register_range(self.h, first, count, kind, p, stride):
            raise ValueError("fjp_register_range failed")

    def set_ring(self, stride):
        self.lib.fjp_set_ring(self.h, stride)

    def set_gossip(self, fanout, seed):
        self.lib.fjp_set_gossip(self.h, fanout, seed)

    def set_behaviors(self, t):
        first = _u32(t.first)
        self._keep.append(t) if hasattr(self, "_keep") else None
        if self.lib.fjp_set_behaviors(self.h, ctypes.addressof(t.cases), len(t.cases), ctypes.addressof(t.acts),
                                       len(t.acts), _p(first, ctypes.c_uint32), t.n_behaviors):
            raise ValueError("fjp_set_behaviors failed")

    def set_delta_crdt(self, max_delta_size):
        if self.lib.fjp_set_delta_crdt(self.h, max_delta_size):
            raise ValueError("fjp_set_delta_crdt failed")

    def set_fanout(self, k, seed, cdf, perm):
        cdf, perm = _u32(cdf), _u32(perm)
        self.lib.fjp_set_fanout(self.h, k, seed, _p(cdf, ctypes.c_uint32), _p(perm, ctypes.c_uint32), cdf.size)

    def set_graph(self, row_ptr, col):
        rp = np.ascontiguousarray(np.asarray(row_ptr, dtype=np.uint64))
        cl = _u32(col) if len(col) else np.zeros(1, np.uint32)
        self._g = (rp, cl)
        self.lib.fjp_set_graph(self.h, _p(rp, ctypes.c_uint64), _p(cl, ctypes.c_uint32))

    def tell(self, dst, payload, src=None):
        dst = _u32(dst)
        pay = _u32(np.broadcast_to(np.asarray(payload, dtype=np.uint32), dst.shape))  # (a scalar: every tell)
        s = _u32(np.broadcast_to(np.asarray(NO_SENDER if src is None else src, dtype=np.uint32), dst.shape))
        self.lib.fjp_stage(self.h, _p(dst, ctypes.c_uint32), _p(s, ctypes.c_uint32), _p(pay, ctypes.c_uint32),
                           dst.size)

    def run(self, threads=1):
        st = Stats()
        self.wall_s = self.lib.fjp_run(self.h, threads, ctypes.byref(st))
        return st.as_dict()

    def read_state(self, first=0, count=None):
        count = self.n - first if count is None else count
        w = np.zeros((count, self.W), np.uint64)
        a = np.zeros(count, np.uint8)
        self.lib.fjp_read_state(self.h, first, count, _p(w, ctypes.c_uint64), _p(a, ctypes.c_uint8))
        return w, a


# ------------------------------------------------------------------ pure functions
def java_hash(id_: int) -> int:
    return int(_load_bsp().bsp_java_hash_decimal(id_))


def shard_id(id_: int, num_shards: int = 1000) -> int:
    return int(_load_bsp().bsp_shard_id(id_, num_shards))


class crdt:
    """GCounter restatement (DD/GCounter.scala:62-64,97-125) over R node slots."""

    @staticmethod
    def gcounter_merge(a, b):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
        b = np.ascontiguousarray(np.asarray(b, dtype=np.uint64))
        out = np.zeros_like(a)
        _load_bsp().bsp_gcounter_merge(_p(out, ctypes.c_uint64), _p(a, ctypes.c_uint64), _p(b, ctypes.c_uint64),
                                       a.size)
        return out

    @staticmethod
    def gcounter_value(a):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
        return int(_load_bsp().bsp_gcounter_value(_p(a, ctypes.c_uint64), a.size))

    @staticmethod
    def gcounter_increment(a, slot, n=1):
        a = np.ascontiguousarray(np.asarray(a, dtype=np.uint64)).copy()
        _load_bsp().bsp_gcounter_increment(_p(a, ctypes.c_uint64), slot, n)
        return a


class orset:
    """ORSet restatement on the engine layout (crdt_ref.h; DD/ORSet.scala).  A value is a
    u64[260] array: u32 dots[64][8] then u32 vvector[8] (node index = UniqueAddress order)."""
    WORDS = 260
    ELEMS = 64
    NODES = 8

    @staticmethod
    def empty():
        return np.zeros(orset.WORDS, np.uint64)

    @staticmethod
    def from_dict(elements: dict, vvector: dict, index: dict):
        """elements {name: {node: version}}, vvector {node: version}; index maps name -> element slot."""
        w = orset.empty()
        u = w.view(np.uint32)
        for name, dot in elements.items():
            for n, v in dot.items():
                u[index[name] * orset.NODES + int(n)] = v
        for n, v in vvector.items():
            u[orset.ELEMS * orset.NODES + int(n)] = v
        return w

    @staticmethod
    def dots(w, e):
        u = np.asarray(w, np.uint64).view(np.uint32)
        d = u[e * orset.NODES:(e + 1) * orset.NODES]
        return {n: int(v) for n, v in enumerate(d) if v}

    @staticmethod
    def vvector(w):
        u = np.asarray(w, np.uint64).view(np.uint32)[orset.ELEMS * orset.NODES:]
        return {n: int(v) for n, v in enumerate(u) if v}

    @staticmethod
    def elements(w):
        u = np.asarray(w, np.uint64).view(np.uint32)[:orset.ELEMS * orset.NODES].reshape(orset.ELEMS, orset.NODES)
        return set(np.nonzero(u.any(axis=1))[0].tolist())

    @staticmethod
    def merge(a, b):
        out = np.ascontiguousarray(np.asarray(a, np.uint64)).copy()
        b = np.ascontiguousarray(np.asarray(b, np.uint64))
        _load_bsp().bsp_orset_merge(_p(out, ctypes.c_uint64), _p(b, ctypes.c_uint64))
        return out

    @staticmethod
    def add(a, node, e):
        out = np.ascontiguousarray(np.asarray(a, np.uint64)).copy()
        _load_bsp().bsp_orset_add(_p(out, ctypes.c_uint64), node, e)
        return out

    @staticmethod
    def remove(a, e):
        out = np.ascontiguousarray(np.asarray(a, np.uint64)).copy()
        _load_bsp().bsp_orset_remove(_p(out, ctypes.c_uint64), e)
        return out

    @staticmethod
    def subtract_dots(dot: dict, vv: dict) -> dict:
        d = np.zeros(orset.NODES, np.uint32)
        v = np.zeros(orset.NODES, np.uint32)
        for n, x in dot.items():
            d[int(n)] = x
        for n, x in vv.items():
            v[int(n)] = x
        out = np.zeros(orset.NODES, np.uint32)
        _load_bsp().bsp_orset_subtract_dots(_p(out, ctypes.c_uint32), _p(d, ctypes.c_uint32), _p(v, ctypes.c_uint32))
        return {n: int(x) for n, x in enumerate(out) if x}


def crdt_peer(seed: int, self_id: int, round_: int, j: int, n: int) -> int:
    return int(_load_bsp().bsp_crdt_peer(seed, self_id, round_, j, n))


class OrsetDop(ctypes.Structure):
    """crdt_ref.h orset_dop: one AtomicDeltaOp (DD/ORSet.scala:43-96)."""
    _fields_ = [("type", ctypes.c_uint32), ("n", ctypes.c_uint32), ("elem", ctypes.c_uint32 * 64),
                ("dot", (ctypes.c_uint32 * 8) * 64), ("vv", ctypes.c_uint32 * 8)]


class OrsetDelta(ctypes.Structure):
    """crdt_ref.h orset_delta: None (nops 0), an AtomicDeltaOp or a DeltaGroup (DD/ORSet.scala:99-120)."""
    _fields_ = [("group", ctypes.c_uint32), ("nops", ctypes.c_uint32), ("ops", OrsetDop * 64)]
    TYPES = {1: "add", 2: "remove", 3: "full"}


class orset_delta:
    """ORSet values with their delta (ORSet.add/remove/clear/mergeDelta/DeltaOp.merge restated in
    crdt_ref.h) -- for the ORSetSpec delta KATs.  A value is (state words, OrsetDelta)."""

    @staticmethod
    def _lib():
        lib = _load_bsp()
        assert lib.bsp_orset_delta_bytes() == ctypes.sizeof(OrsetDelta)
        return lib

    @staticmethod
    def empty():
        return orset.empty(), OrsetDelta()

    @staticmethod
    def _copy(v):
        w, d = v
        d2 = OrsetDelta()
        ctypes.memmove(ctypes.byref(d2), ctypes.byref(d), ctypes.sizeof(OrsetDelta))
        return np.array(w, copy=True), d2

    @staticmethod
    def add(v, node, e, ver):
        w, d = orset_delta._copy(v)
        orset_delta._lib().bsp_orset_add_d(_p(w, ctypes.c_uint64), ctypes.byref(d), node, e, ver)
        return w, d

    @staticmethod
    def remove(v, node, e):
        w, d = orset_delta._copy(v)
        orset_delta._lib().bsp_orset_remove_d(_p(w, ctypes.c_uint64), ctypes.byref(d), node, e)
        return w, d

    @staticmethod
    def clear(v):
        w, d = orset_delta._copy(v)
        orset_delta._lib().bsp_orset_clear_d(_p(w, ctypes.c_uint64), ctypes.byref(d))
        return w, d

    @staticmethod
    def reset(v):
        return np.array(v[0], copy=True), OrsetDelta()

    @staticmethod
    def merge(a, b):
        return orset.merge(a[0], b[0]), OrsetDelta()

    @staticmethod
    def merge_delta(v, d):
        w = np.array(v[0], copy=True)
        orset_delta._lib().bsp_orset_merge_delta(_p(w, ctypes.c_uint64), ctypes.byref(d))
        return w, OrsetDelta()

    @staticmethod
    def delta_merge(d1, d2):
        out = OrsetDelta()
        ctypes.memmove(ctypes.byref(out), ctypes.byref(d1), ctypes.sizeof(OrsetDelta))
        if orset_delta._lib().bsp_orset_delta_merge(ctypes.byref(out), ctypes.byref(d2)):
            raise OverflowError("delta group too long")
        return out


def vv_compare(a, b) -> str:
    """VersionVector.compareTo on the fixed layout: '==' | '<' | '>' | '<>'."""
    a, b = _u32(a), _u32(b)
    return ("==", "<", ">", "<>")[_load_bsp().bsp_vv_compare(_p(a, ctypes.c_uint32), _p(b, ctypes.c_uint32))]
