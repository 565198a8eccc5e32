#!/usr/bin/env python3
"""Where the first timed agx_run(20) after the warmup loses ~20 us: fresh 1M-ring engines, the warmup
run(5) followed by MODE, then the wall time of run(20) (host call + sync) three times."""
import sys
import time

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), ".."))


def main():
    import torch
    from akka_amd import workloads as wl
    from akka_amd.engine import EngineConfig, GpuEngine
    for mode in ("none", "run5", "run1x4", "run20", "none"):
        w = wl.token_ring(1_000_000, 400)
        eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
        w.apply_to(eng)
        eng.run(5)
        if mode == "run5":
            eng.run(5)
        elif mode == "run1x4":
            for _ in range(4):
                eng.run(1)
        elif mode == "run20":
            eng.run(20)
        torch.cuda.synchronize()
        walls = []
        for _ in range(3):
            t0 = time.perf_counter()
            eng.run(20, stats=False)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
        print(f"{mode:7s} run(20) wall us: {walls[0]:.1f} {walls[1]:.1f} {walls[2]:.1f}", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
