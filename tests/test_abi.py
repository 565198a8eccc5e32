"""The C-ABI library loads and exports every symbol include/akka_gpu.h declares.
Host-only helpers (no GPU) are exercised; compute entry points are not called."""
import ctypes
import pathlib
import re

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]


def declared_symbols():
    text = (ROOT / "include" / "akka_gpu.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(agx_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(built):
    from akka_amd import _lib
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the Python binding declares a signature for each
    assert set(syms) <= set(_lib.SIGNATURES), set(syms) - set(_lib.SIGNATURES)
    assert lib.agx_abi_version() == _lib.ABI_VERSION


def test_gfx950_code_object_present(built):
    from akka_amd import _lib
    data = _lib.LIB_PATH.read_bytes()
    assert b"gfx950" in data and b"k_bucket_apply" in data and b"k_chunk_downsweep" in data


def test_host_shard_helpers_match_golden(built):
    import json
    from akka_amd.engine import owner, shard_id
    gold = json.loads((ROOT / "tests" / "golden" / "shard_ids.json").read_text())
    for v in gold["vectors"]:
        if v["entity_id"].isdigit() and int(v["entity_id"]) < 2**32:
            assert shard_id(int(v["entity_id"]), v["num_shards"]) == v["shard"]
            assert owner(int(v["entity_id"]), v["num_shards"], 8) == v["shard"] % 8


def test_exchange_plan(built):
    from akka_amd.engine import exchange_plan
    R = 3
    S = R + 2
    mat = np.zeros((R, S), np.uint64)
    mat[0, :R] = [1, 2, 3]
    mat[1, :R] = [4, 5, 6]
    mat[2, :R] = [7, 8, 9]
    mat[:, R] = [10, 20, 30]  # backlog
    mat[:, R + 1] = [0, 1, 0]  # staged
    p = exchange_plan(mat, 1)
    assert p["send_cnt"].tolist() == [4, 5, 6] and p["send_off"].tolist() == [0, 4, 9]
    assert p["recv_cnt"].tolist() == [2, 5, 8]
    assert p["recv_off"].tolist() == [20, 22, 27]  # after this rank's backlog, sender-rank order
    assert p["inflight"] == int(mat.sum())


def test_errors_are_status_codes_not_crashes(built):
    from akka_amd import _lib
    from akka_amd._lib import AgxCfg
    lib = _lib.load()
    cfg = AgxCfg()
    cfg.abi_version = 999
    h = ctypes.c_void_p()
    assert lib.agx_create(ctypes.byref(cfg), ctypes.byref(h)) == 1  # AGX_EINVAL before touching a device
    assert b"abi_version" in lib.agx_last_error()
    assert lib.agx_create(None, ctypes.byref(h)) == 1
    assert lib.agx_destroy(None) == 0


def test_library_stamped_with_source_hash(built, tmp_path):
    """build_native rebuilds by source hash, not by file times: the built library carries the hash of
    the sources it was built from (found in its bytes), agx_build_hash returns it, and a library
    stamped with any other hash -- a stale build shipped beside newer sources -- reads as stale."""
    import __graft_entry__ as ge
    want = ge.source_hash()
    assert len(want) == 16
    assert ge.library_hash(ge.LIB) == want
    from akka_amd import _lib
    assert _lib.load().agx_build_hash().decode() == want
    stale = tmp_path / "libakka_gpu.so"
    data = ge.LIB.read_bytes()
    i = data.find(ge.STAMP) + len(ge.STAMP)
    stale.write_bytes(data[:i] + b"0123456789abcdef" + data[i + 16:])
    assert ge.library_hash(stale) == "0123456789abcdef" != want
    assert ge.library_hash(tmp_path / "missing.so") is None
