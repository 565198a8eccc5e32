"""ctypes binding of the C ABI in include/akka_gpu.h (libakka_gpu.so).

This is the product path: there is no CPU fallback.  If the HIP library is
missing, `load()` raises; build it with `__graft_entry__.build()` (or
`python -m akka_amd.build`).
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import threading

LIB_PATH = pathlib.Path(__file__).resolve().parent / "lib" / "libakka_gpu.so"
if os.environ.get("AKKA_AMD_LIB"):  # A/B diagnostics: an alternative in-tree build
    LIB_PATH = pathlib.Path(os.environ["AKKA_AMD_LIB"]).resolve()

_lib = None
_lock = threading.Lock()

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)


class AgxCfg(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_uint32),
        ("device", ctypes.c_uint32),
        ("n_actors", ctypes.c_uint64),
        ("throughput", ctypes.c_uint32),
        ("capacity", ctypes.c_uint32),
        ("n_words", ctypes.c_uint32),
        ("max_emit", ctypes.c_uint32),
        ("n_ranks", ctypes.c_uint32),
        ("rank", ctypes.c_uint32),
        ("num_shards", ctypes.c_uint32),
        ("bucket_actors", ctypes.c_uint32),
        ("msg_capacity", ctypes.c_uint64),
    ]


class AgxStats(ctypes.Structure):
    _fields_ = [
        ("delivered", ctypes.c_uint64),
        ("dead_letters", ctypes.c_uint64),
        ("unhandled", ctypes.c_uint64),
        ("emitted", ctypes.c_uint64),
        ("staged", ctypes.c_uint64),
        ("supersteps", ctypes.c_uint64),
        ("in_flight", ctypes.c_uint64),
        ("bytes_alg", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {name: int(getattr(self, name)) for name, _ in self._fields_}


ABI_VERSION = 1

# status codes (akka_gpu.h)
STATUS = {0: "AGX_OK", 1: "AGX_EINVAL", 2: "AGX_ENOMEM", 3: "AGX_EDEVICE", 4: "AGX_ECOMM",
          5: "AGX_ECAPACITY", 6: "AGX_ESTATE", 7: "AGX_ERANGE"}


class AgxError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS.get(status, status)}: {msg}")
        self.status = status


# name -> (restype, argtypes)
_E = ctypes.POINTER(ctypes.c_void_p)  # opaque agx_engine*
SIGNATURES = {
    "agx_create": (ctypes.c_int32, [ctypes.POINTER(AgxCfg), ctypes.POINTER(ctypes.c_void_p)]),
    "agx_destroy": (ctypes.c_int32, [ctypes.c_void_p]),
    "agx_last_error": (ctypes.c_char_p, []),
    "agx_abi_version": (ctypes.c_uint32, []),
    "agx_register_range": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_size_t]),
    "agx_set_ring": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32]),
    "agx_set_mailbox_class": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]),
    "agx_set_mailbox": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]),
    "agx_set_outbound": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    "agx_take_outbound": (ctypes.c_int32, [ctypes.c_void_p, c_u32p, c_u32p, c_u32p, ctypes.c_uint64, c_u64p]),
    "agx_set_gossip": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64]),
    "agx_set_delta_crdt": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32]),
    "agx_set_behaviors": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]),
    "agx_set_fanout": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, c_u32p, c_u32p,
                                        ctypes.c_uint64]),
    "agx_set_graph": (ctypes.c_int32, [ctypes.c_void_p, c_u64p, c_u32p]),
    "agx_set_graph_rmat": (ctypes.c_int32, [ctypes.c_void_p, c_u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint64]),
    "agx_stage_tells": (ctypes.c_int32, [ctypes.c_void_p, c_u32p, c_u32p, c_u32p, ctypes.c_size_t]),
    "agx_tell": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.POINTER(ctypes.c_int32)]),
    "agx_pump_idle": (ctypes.c_int32, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]),
    "agx_pump_cancel": (ctypes.c_int32, [ctypes.c_void_p]),
    "agx_build_hash": (ctypes.c_char_p, []),
    "agx_run": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(AgxStats)]),
    "agx_get_stats": (ctypes.c_int32, [ctypes.c_void_p, ctypes.POINTER(AgxStats)]),
    "agx_identity_supersteps": (ctypes.c_int32, [ctypes.c_void_p, c_u64p]),
    "agx_ring_buckets": (ctypes.c_int32, [ctypes.c_void_p, c_u64p]),
    "agx_exchange_info": (ctypes.c_int32, [ctypes.c_void_p, c_u64p]),
    "agx_persist_info": (ctypes.c_int32, [ctypes.c_void_p, c_u64p]),
    "agx_run_timed": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]),
    "agx_get_shape": (ctypes.c_int32, [ctypes.c_void_p, c_u64p, c_u32p]),
    "agx_read_state": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, c_u64p, c_u8p]),
    "agx_comm_unique_id": (ctypes.c_int32, [ctypes.c_void_p]),
    "agx_comm_init": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_void_p]),
    "agx_group_run": (ctypes.c_int32, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.POINTER(AgxStats)]),
    "agx_profile_enable": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int]),
    "agx_profile_read": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                          c_u64p, c_u64p, ctypes.c_uint32, c_u32p]),
    "agx_profile_reset": (ctypes.c_int32, [ctypes.c_void_p]),
    "agx_exchange_plan": (ctypes.c_int32, [c_u64p, ctypes.c_uint32, ctypes.c_uint32, c_u64p, c_u64p, c_u64p, c_u64p,
                                           c_u64p]),
    "agx_mr_plan": (ctypes.c_int32, [c_u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                     c_u32p, c_u64p, c_u64p, c_u64p]),
    "agx_shard_id": (ctypes.c_int32, [ctypes.c_uint32, ctypes.c_uint32]),
    "agx_owner": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
}


# entry points newer than some A/B diagnostic builds (tools/build_variant.sh of an older checkout)
OPTIONAL = {"agx_tell", "agx_pump_idle", "agx_pump_cancel", "agx_exchange_info", "agx_run_timed", "agx_build_hash",
            "agx_persist_info"}


def load():
    """Load libakka_gpu.so (fails loudly when it is missing)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            raise RuntimeError(
                f"akka_amd: native HIP library not found at {LIB_PATH}; "
                "build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        # torch ships its own libamdhip64 (same SONAME): load it first so both share one HIP runtime.
        if os.environ.get("AKKA_AMD_NO_TORCH") != "1":
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        lib = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            if name in OPTIONAL and not hasattr(lib, name):  # (an older A/B build: AKKA_AMD_LIB)
                continue
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.agx_abi_version() != ABI_VERSION:
            raise RuntimeError("akka_amd: ABI version mismatch")
        _lib = lib
        return lib


def check(status: int) -> None:
    if status != 0:
        msg = _lib.agx_last_error().decode(errors="replace") if _lib is not None else ""
        raise AgxError(status, msg)
