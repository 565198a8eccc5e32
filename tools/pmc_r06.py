#!/usr/bin/env python3
"""profiles/pmc_r06.json from the round-6 counter passes.

Ring operating points (tools/gpu_r04.sh TAG=r06 step pmcring, copied to profiles/r06/pmc/ring_p{1,2,3}):
per kernel instantiation the mean FETCH_SIZE / WRITE_SIZE per dispatch (KiB, raw), HBM bytes with
FETCH doubled (MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE reports half of a wide streaming
read; WRITE_SIZE exact) and the SQ wait/issue split.  `kernels.bucket_apply_dense` is the 1M fused dense launch
(bench.py's headline roofline.traffic).  The BASELINE configs come from the per-superstep windows
of tools/pmc_window.py (profiles/r06/pmc/window_*.json: counted vs algorithmic bytes per superstep
over the bench window).

    python tools/pmc_r06.py
"""
import collections
import csv
import glob
import json
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
P = ROOT / "profiles" / "r06" / "pmc"
FUSED = "agx::k_dense_fused<4u, false, false>"  # (round 6: owner and persistent flags in the name)
BYPASS = "agx::k_dense_apply<4u>"


def load(pat):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(str(P / pat / "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def traffic(d, alg):
    f, w = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0)
    out = {"fetch_kib_raw": round(f, 1), "write_kib_raw": round(w, 1),
           "hbm_bytes_per_launch": int((2 * f + w) * 1024), "hbm_bytes_raw": int((f + w) * 1024),
           "alg_bytes_per_launch": alg}
    out["ratio_corrected"] = round(out["hbm_bytes_per_launch"] / alg, 3)
    out["ratio_raw"] = round(out["hbm_bytes_raw"] / alg, 3)
    return out


def sq(d):
    wc = d["SQ_WAVE_CYCLES"]
    return {"wave_cycles_per_wave": round(wc / d["SQ_WAVES"], 1),
            "wait_any": round(d["SQ_WAIT_ANY"] / wc, 3), "wait_inst_any": round(d["SQ_WAIT_INST_ANY"] / wc, 3),
            "active_inst_any": round(d["SQ_ACTIVE_INST_ANY"] / wc, 3)}


def main():
    ring = load("ring_p*")
    out = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / SQ_* (separate runs, TAG=r06 tools/gpu_r04.sh pmcring / pmc)",
        "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes; raw sums kept beside",
        "note": "round 6: bench.py --steps 20 --warmup 4 --no-configs --no-cpu-baseline --large-steps 8 (1M fused "
                "ring: k_dense_fused; 100M multi-pass ring with identity grouping: k_dense_apply); configs: per-superstep windows over the bench "
                "window (tools/pmc_window.py)",
        "kernels": {"bucket_apply_dense": traffic(ring[FUSED], 42_000_000)},
        "ring_1M_fused_apply": dict(traffic(ring[FUSED], 42_000_000), sq=sq(ring[FUSED])),
        "ring_100M_apply": dict(traffic(ring[BYPASS], 4_200_000_000), sq=sq(ring[BYPASS])),
        "configs": {},
    }
    for f in sorted(P.glob("window_*.json")):
        d = json.loads(f.read_text())
        out["configs"][f.stem[len("window_"):]] = {k: d[k] for k in ("counted_bytes_per_superstep",
                                                                      "alg_bytes_per_superstep", "ratio",
                                                                      "counted_bytes_per_superstep_raw", "ratio_raw",
                                                                      "per_kernel_gb_per_superstep", "window") if k in d}
    (ROOT / "profiles" / "pmc_r06.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps({k: out[k] for k in ("ring_1M_fused_apply", "ring_100M_apply")}, indent=1))
    print({k: v["ratio"] for k, v in out["configs"].items()})


if __name__ == "__main__":
    main()
