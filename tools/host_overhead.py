#!/usr/bin/env python3
"""Host overhead of agx_run on the 1M ring: wall time of run(k) (host call + sync, as bench.py
times it) against the device time of the same supersteps (agx_run_timed), per budget k."""
import statistics
import sys
import time

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), ".."))


def main():
    import torch
    from akka_amd import workloads as wl
    from akka_amd.engine import EngineConfig, GpuEngine
    w = wl.token_ring(1_000_000, 4000)
    eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
    w.apply_to(eng)
    eng.run(16)
    torch.cuda.synchronize()
    for k in (1, 4, 16, 20, 32, 64):
        walls, devs = [], []
        for _ in range(5):
            t0 = time.perf_counter()
            eng.run(k, stats=False)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
            _, ms = eng.run_timed(k)
            devs.append(ms * 1e3)
        wm, dm = statistics.median(walls), statistics.median(devs)
        print(f"k={k:3d} wall {wm:8.1f} us  device {dm:8.1f} us  host overhead {wm - dm:6.1f} us "
              f"({(wm - dm) / k:5.2f} us/step)", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
