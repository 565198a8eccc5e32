#!/usr/bin/env python3
"""A/B timing helper: median of several timed regions in ONE process (the
bench's single region is noisy across boxes).  Usage:
  python tools/perf.py [--n 1000000] [--steps 100] [--reps 7] [--workload ring|powerlaw|fanout]"""
import argparse
import json
import pathlib
import statistics
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--workload", default="ring")
    ap.add_argument("--prof", action="store_true")
    a = ap.parse_args()
    import torch
    import __graft_entry__ as g
    g.build_native()
    from akka_amd import workloads as wl
    from akka_amd.engine import EngineConfig, GpuEngine
    hops = 16 + a.steps * (a.reps + 1) + 8
    if a.workload == "ring":
        w = wl.token_ring(a.n, hops)
    elif a.workload == "powerlaw":
        w = wl.power_law_forward(a.n, ttl=hops, capacity=64, throughput=5)
    else:
        raise SystemExit("unknown workload")
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    t0 = time.perf_counter()
    w.apply_to(eng)
    eng.run(16)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    res = []
    for _ in range(a.reps):
        s0 = eng.stats()
        t0 = time.perf_counter()
        s1 = eng.run(a.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res.append((dt / a.steps * 1e6, (s1.delivered - s0.delivered) / dt))
    out = {"workload": a.workload, "n": a.n, "setup_s": round(setup, 2),
           "us_per_step_median": statistics.median(r[0] for r in res),
           "us_per_step_min": min(r[0] for r in res),
           "msg_per_s_median": statistics.median(r[1] for r in res)}
    if a.prof:
        eng.profile(True)
        eng.run(a.steps)
        p = eng.profile_read()
        out["kernel_us_per_step"] = {k: round(v["total_ms"] * 1e3 / a.steps, 2) for k, v in p.items() if v["launches"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
