#!/usr/bin/env python3
"""Counted HBM traffic per superstep over the bench window of one BASELINE config.

Input: two rocprofv3 counter passes of `tools/cfg_one.py CONFIG` (one FETCH_SIZE run, one WRITE_SIZE
run: rocprofv3 never splits counters over passes) and the config's JSON line (its stdout).  cfg_one
runs the config as bench.py does: engine 1 = warmup + the timed supersteps, engine 2 = the same window
again with per-kernel HIP events.  Every dispatch is attributed to a superstep of its engine:
  * an engine starts at its host-staged tells (k_chunk_hist), the first superstep's first kernel;
  * a later superstep starts at its first-pass rowscan (k_chunk_rowscan; with identity grouping the
    split launch's first part, the one followed by k_ident_combine);
  * engine setup (k_gen_rmat: the next engine's graph) closes the previous engine's last superstep.
The window is engine 1's supersteps [warmup, warmup + timed).  HBM bytes per dispatch = 2 x FETCH_SIZE
+ WRITE_SIZE (KiB; MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE counts half of a wide streaming
read, WRITE_SIZE is exact).  Algorithmic bytes = the config's alg_bytes_per_msg x delivered (SURVEY.md
§8(d) formula, accumulated by the engine), per superstep of the same window.

    python tools/pmc_window.py CONFIG FETCH_DIR WRITE_DIR CFG_JSON_LOG [--warmup W --steps K]
"""
import argparse
import collections
import csv
import json
import pathlib

def dispatches(d):
    rows = []
    for f in sorted(pathlib.Path(d).rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("void ", "").replace("agx::", ""),
                         float(r["Counter_Value"])))
    rows.sort()
    return rows


SETUP_KERNELS = ("k_gen_rmat",)  # engine setup (the device R-MAT graph): not part of any superstep


def supersteps(rows):
    """[(engine, superstep) per dispatch] by the kernel-sequence rules above; dispatches from an
    engine-setup kernel up to the next engine's first superstep get superstep -1 (outside every window)."""
    out, eng, step, started = [], -1, -1, False
    for i, (_, k, _) in enumerate(rows):
        if k in SETUP_KERNELS:
            started = False
            step = -1
        if k == "k_chunk_hist":
            if not (out and out[-1][1] == step and rows[i - 1][1] == "k_chunk_hist"):
                eng += 1
                step = 0
                started = True
        elif k == "k_chunk_rowscan" and started:
            prev = rows[i - 1][1] if i else ""
            first_of_step = prev not in ("k_chunk_hist", "k_chunk_rowscan", "k_ident_combine")
            if first_of_step:
                step += 1
        out.append((eng, step))
    # the memsets / copies right before an engine's first superstep are that engine's setup
    for i, (_, k, _) in enumerate(rows):
        if (k in SETUP_KERNELS or k == "k_chunk_hist") and i and rows[i - 1][1] != "k_chunk_hist":
            j = i - 1
            while j >= 0 and rows[j][1].startswith("__amd_rocclr"):
                out[j] = (out[j][0], -1)
                j -= 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("cfg_log")
    ap.add_argument("--warmup", type=int, required=True, help="the config's warmup supersteps (bench.py other_configs)")
    ap.add_argument("--steps", type=int, default=None)
    a = ap.parse_args()
    line = [ln for ln in open(a.cfg_log).read().splitlines() if ln.startswith("{")][-1]
    cfg = json.loads(line)[a.config]
    warm = a.warmup
    steps = a.steps if a.steps is not None else cfg["supersteps_timed"]
    fr, wr = dispatches(a.fetch_dir), dispatches(a.write_dir)
    if [k for _, k, _ in fr] != [k for _, k, _ in wr]:
        raise SystemExit("the FETCH and WRITE passes dispatched different kernel sequences")
    tags = supersteps(fr)
    per_k = collections.defaultdict(float)
    per_k_raw = collections.defaultdict(float)
    tot = tot_raw = fetch_raw = write_raw = 0.0
    for (_, k, f), (_, _, w), (e, s) in zip(fr, wr, tags):
        if e == 0 and warm < s + 1 <= warm + steps:  # superstep index s counts from 0 (the staged one)
            b = (2 * f + w) * 1024
            r = (f + w) * 1024  # raw: FETCH_SIZE as counted, no gfx950 correction
            per_k[k] += b
            per_k_raw[k] += r
            tot += b
            tot_raw += r
            fetch_raw += f * 1024
            write_raw += w * 1024
    alg = cfg["alg_bytes_per_msg"] * cfg["delivered"]
    out = {"config": a.config, "window": {"warmup": warm, "supersteps": steps},
           "counted_bytes_per_superstep": tot / steps, "alg_bytes_per_superstep": alg / steps,
           "ratio": round(tot / alg, 3) if alg else None,
           # the x2 FETCH correction is calibrated for 16-B-per-lane streaming reads only
           # (MI355X_MICROARCH.md HBM section); the raw counts bound the scattered kernels from below
           "raw_fetch_bytes_per_superstep": fetch_raw / steps, "write_bytes_per_superstep": write_raw / steps,
           "counted_bytes_per_superstep_raw": tot_raw / steps,
           "ratio_raw": round(tot_raw / alg, 3) if alg else None,
           "per_kernel_gb_per_superstep": {k: round(v / steps / 1e9, 4) for k, v in
                                           sorted(per_k.items(), key=lambda kv: -kv[1]) if v / steps > 1e6},
           "per_kernel_gb_per_superstep_raw": {k: round(v / steps / 1e9, 4) for k, v in
                                               sorted(per_k_raw.items(), key=lambda kv: -kv[1]) if v / steps > 1e6},
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs) of tools/cfg_one.py; "
                     "HBM = 2 x FETCH + WRITE (gfx950 correction); *_raw: FETCH + WRITE as counted"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
