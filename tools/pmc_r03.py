#!/usr/bin/env python3
"""profiles/pmc_r03.json from the round-3 counter passes (tools/gpu_pmc_r03.sh, copied to
profiles/r03/pmc/): per kernel instantiation, mean FETCH_SIZE / WRITE_SIZE per dispatch (KiB,
raw), HBM bytes with FETCH doubled (MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE reports
half of a wide streaming read; WRITE_SIZE exact), and the SQ wait/issue split of the ring's
applies.  `kernels.bucket_apply` is the 1M fused apply (bench.py's headline roofline.traffic)."""
import collections
import csv
import glob
import json
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
P = ROOT / "profiles" / "r03" / "pmc"


def load(pat):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(str(P / pat / "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def traffic(d, alg=None):
    f, w = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0)
    out = {"fetch_kib_raw": round(f, 1), "write_kib_raw": round(w, 1),
           "hbm_bytes_per_launch": int((2 * f + w) * 1024), "hbm_bytes_raw": int((f + w) * 1024)}
    if alg:
        out["alg_bytes_per_launch"] = alg
        out["ratio_corrected"] = round(out["hbm_bytes_per_launch"] / alg, 3)
        out["ratio_raw"] = round(out["hbm_bytes_raw"] / alg, 3)
    return out


def sq(d):
    wc = d["SQ_WAVE_CYCLES"]
    return {"wave_cycles_per_wave": round(wc / d["SQ_WAVES"], 1),
            "wait_any": round(d["SQ_WAIT_ANY"] / wc, 3), "wait_inst_any": round(d["SQ_WAIT_INST_ANY"] / wc, 3),
            "active_inst_any": round(d["SQ_ACTIVE_INST_ANY"] / wc, 3)}


ring = load("pmc3_ring_p*")
fused = "agx::k_bucket_apply<false, 4u, true, false, false>"
bypass = "agx::k_bucket_apply<false, 4u, false, false, false>"
c4 = load("pmc3_C4_orset_gossip_p*")
c5 = load("pmc3_C5_power_law_bounded_p*")
c4d = load("pmc3_C4_orset_delta_gossip_p*")
out = {
    "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / SQ_* (separate passes, tools/gpu_pmc_r03.sh)",
    "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes; raw sums kept beside",
    "note": "round 3: bench.py --steps 20 --warmup 4 --no-configs --no-cpu-baseline --large-steps 8 (1M fused ring "
            "+ 100M multi-pass ring with identity grouping); tools/cfg_one.py C4_orset_gossip / C4_orset_delta_gossip / C5_power_law_bounded",
    "kernels": {"bucket_apply": traffic(ring[fused], 42_000_000)},
    "ring_1M_fused_apply": dict(traffic(ring[fused], 42_000_000), sq=sq(ring[fused])),
    "ring_100M_apply": dict(traffic(ring[bypass], 4_200_000_000), sq=sq(ring[bypass])),
    "C4_orset_gossip": {k.replace("agx::", ""): traffic(v) for k, v in c4.items()
                        if v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0) > 1000},
    "C4_orset_delta_gossip": {k.replace("agx::", ""): traffic(v) for k, v in c4d.items()
                              if v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0) > 1000},
    "C5_power_law_bounded": {k.replace("agx::", ""): traffic(v) for k, v in c5.items()
                             if v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0) > 1000 and "gen_rmat" not in k
                             and "chunk_hist" not in k},
}
for cfg in ("C4_orset_gossip", "C4_orset_delta_gossip", "C5_power_law_bounded"):
    t = out[cfg]
    t["per_superstep_total"] = {"hbm_bytes": sum(v["hbm_bytes_per_launch"] for v in t.values()),
                                "hbm_bytes_raw": sum(v["hbm_bytes_raw"] for v in t.values())}
(ROOT / "profiles" / "pmc_r03.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps({k: out[k] for k in ("ring_1M_fused_apply", "ring_100M_apply")}, indent=1))
print(out["C4_orset_gossip"]["per_superstep_total"], out["C4_orset_delta_gossip"]["per_superstep_total"],
      out["C5_power_law_bounded"]["per_superstep_total"])
