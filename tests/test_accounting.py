"""The roofline accounting the bench line and profiles/ rest on, on synthetic inputs (CPU):

* tools/pmc_window.py: dispatches attributed to supersteps by the kernel-sequence rules, the window
  [warmup, warmup + steps) of engine 1, HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB) with the raw
  FETCH_SIZE + WRITE_SIZE kept beside it, ratios against alg_bytes_per_msg x delivered;
* bench.py: kernel_rooflines' achieved = algorithmic bytes per message x messages per launch / the
  average launch time, and every dominant kernel class has an algorithmic byte count.
"""
import csv
import json
import pathlib
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _pass(d: pathlib.Path, seq, counter):
    d.mkdir(parents=True)
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (k, fetch, write) in enumerate(seq):
            w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": f"agx::{k}(agx::Args)", "Counter_Name": counter,
                        "Counter_Value": fetch if counter == "FETCH_SIZE" else write})


def test_pmc_window_counts_the_window_and_keeps_raw(tmp_path):
    # engine 1: staged superstep 0, then supersteps 1..4; engine 2 (the profiled replay) after it
    seq = [("k_chunk_hist", 1, 1), ("k_bucket_apply", 10, 5)]
    for s in range(1, 5):
        seq += [("k_chunk_rowscan", 1, 0), ("k_chunk_downsweep", 100 * s, 50 * s), ("k_bucket_apply", 10 * s, 4 * s)]
    seq += [("k_chunk_hist", 7, 7), ("k_bucket_apply", 999, 999)]
    _pass(tmp_path / "f", seq, "FETCH_SIZE")
    _pass(tmp_path / "w", seq, "WRITE_SIZE")
    log = tmp_path / "cfg.log"
    log.write_text("noise\n" + json.dumps({"CFG": {"alg_bytes_per_msg": 40.0, "delivered": 1000,
                                                   "supersteps_timed": 2}}) + "\n")
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_window.py"), "CFG", str(tmp_path / "f"),
                        str(tmp_path / "w"), str(log), "--warmup", "2"], capture_output=True, text=True, check=True)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    # window = supersteps 2 and 3 of engine 1 (superstep index s counts from 0: warm < s + 1 <= warm + 2)
    fetch = sum(f for k, f, _ in seq[2 + 3 * 1:2 + 3 * 3])
    write = sum(w for k, _, w in seq[2 + 3 * 1:2 + 3 * 3])
    assert out["window"] == {"warmup": 2, "supersteps": 2}
    assert out["counted_bytes_per_superstep"] == pytest.approx((2 * fetch + write) * 1024 / 2)
    assert out["counted_bytes_per_superstep_raw"] == pytest.approx((fetch + write) * 1024 / 2)
    assert out["raw_fetch_bytes_per_superstep"] == pytest.approx(fetch * 1024 / 2)
    assert out["write_bytes_per_superstep"] == pytest.approx(write * 1024 / 2)
    assert out["alg_bytes_per_superstep"] == pytest.approx(40.0 * 1000 / 2)
    assert out["ratio"] == pytest.approx(round((2 * fetch + write) * 1024 / 40000.0, 3))
    assert out["ratio_raw"] == pytest.approx(round((fetch + write) * 1024 / 40000.0, 3))


def test_bench_kernel_rooflines():
    sys.path.insert(0, str(ROOT))
    import bench
    per = bench.kernel_bytes_per_msg(1)
    # the C2 dominant classes (the fused dense launch; the block kernel) carry the §8(d) bytes
    assert per["bucket_apply_dense"] == per["bucket_apply"] == 12 + 12 + 16 + 2
    prof = {"bucket_apply_dense": {"total_ms": 0.254, "launches": 20}, "bucket_apply": {"total_ms": 0.0, "launches": 0}}
    rr = bench.kernel_rooflines(prof, per, 1_000_000)
    assert rr["dominant"] == "bucket_apply_dense" and rr["peak"] == bench.PEAK_HBM_GBS
    r = rr["kernels"]
    avg = 0.254 / 20
    assert r["bucket_apply_dense"]["avg_launch_ms"] == pytest.approx(round(avg, 4))
    assert r["bucket_apply_dense"]["achieved"] == pytest.approx(round(42 * 1_000_000 / (avg * 1e-3) / 1e9, 1))
    assert r["bucket_apply_dense"]["frac"] == pytest.approx(round(42e6 / (avg * 1e-3) / 1e9 / bench.PEAK_HBM_GBS, 4))
    assert "bucket_apply" not in r  # (no launches: no roofline)


def test_bench_rooflines_after_a_dense_launch():
    """At 100M the block launch follows the dense launch and returns at entry when it took every
    bucket -- as the device's dense_left flags say (agx_profile_read items: the profiled dense launches
    that took every bucket), not as a > peak rate suggests: the block class then gets no fraction, the
    dense class keeps its own.  When the flags say a dense launch left buckets, the block class keeps its
    number (a fraction > 1 stays visible instead of being relabelled)."""
    sys.path.insert(0, str(ROOT))
    import bench
    per = bench.kernel_bytes_per_msg(1)
    prof = {"bucket_apply_dense": {"total_ms": 16.8, "launches": 25, "items": 25},
            "bucket_apply": {"total_ms": 0.19, "launches": 25, "items": 0}}
    rr = bench.kernel_rooflines(prof, per, 100_000_000, identity=True)
    r = rr["kernels"]
    assert rr["dominant"] == "bucket_apply_dense"
    assert r["bucket_apply"] == {"returned_at_entry": True, "avg_launch_ms": 0.0076,
                                 "reason": "the dense launch before it took every bucket (device dense_left flags)"}
    assert 0 < r["bucket_apply_dense"]["frac"] < 1
    # one profiled dense launch left a bucket: the block launch did work in that superstep
    prof["bucket_apply_dense"]["items"] = 24
    r1 = bench.kernel_rooflines(prof, per, 100_000_000, identity=True)["kernels"]
    assert "returned_at_entry" not in r1["bucket_apply"] and r1["bucket_apply"]["frac"] > 1
    # without a dense launch in the profile the same numbers stay a (bad) fraction, not hidden
    r2 = bench.kernel_rooflines({"bucket_apply": prof["bucket_apply"]}, per, 100_000_000)["kernels"]
    assert r2["bucket_apply"]["frac"] > 1
