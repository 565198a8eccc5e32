#!/usr/bin/env python3
"""Multi-rank superstep cost without RCCL: R engines on one device (agx_group_run loopback
exchange), token ring with `n` actors per rank.  Prints wall µs per superstep and the per-kernel
µs per superstep of rank 0 (eager launches, HIP events).

    python tools/perf_group.py [--ranks 2] [--n 1000000] [--steps 20]"""
import argparse
import json
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from akka_amd import workloads as wl
    from akka_amd.engine import EngineConfig, GpuEngine
    R = a.ranks
    w = wl.token_ring(a.n * R, 4 * a.steps + 8)
    engs = [GpuEngine(EngineConfig(n_ranks=R, rank=r, msg_capacity=int(2.5 * a.n), **w.engine_kwargs()))
            for r in range(R)]
    for e in engs:
        w.apply_to(e)
    GpuEngine.group_run(engs, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s0 = engs[0].stats()
    s1 = GpuEngine.group_run(engs, a.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    engs[0].profile(True)
    engs[0].profile_reset()
    GpuEngine.group_run(engs, a.steps)
    prof = engs[0].profile_read()
    out = {"ranks": R, "n_per_rank": a.n, "us_per_step_wall_all_ranks": dt / a.steps * 1e6,
           "delivered_per_step": (s1.delivered) / max(1, a.steps + 2),
           "rank0_kernel_us_per_step": {k: round(v["total_ms"] * 1e3 / a.steps, 2) for k, v in prof.items()
                                        if v["launches"]}}
    print(json.dumps(out))
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
