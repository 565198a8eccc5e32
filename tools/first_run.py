#!/usr/bin/env python3
"""The bench's timed region in isolation: a fresh 1M-ring engine, run(warmup) with graph capture,
then the wall time of run(steps) (host call + sync, as bench.py times it) -- the first run after the
warmup -- against a second and third run(steps) and the device time (agx_run_timed)."""
import sys
import time

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), ".."))


def main():
    import torch
    from akka_amd import workloads as wl
    from akka_amd.engine import EngineConfig, GpuEngine
    for trial in range(3):
        w = wl.token_ring(1_000_000, 400)
        eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
        w.apply_to(eng)
        if "--capture-first" in sys.argv:
            eng.run(0)  # capture every replay graph before the warmup (setup)
        eng.run(5)
        torch.cuda.synchronize()
        walls = []
        for _ in range(3):
            t0 = time.perf_counter()
            eng.run(20, stats=False)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
        _, ms = eng.run_timed(20)
        # a replay size the warmup already launched (4) against one it only captured (8)
        t0 = time.perf_counter(); eng.run(4, stats=False); torch.cuda.synchronize(); w4 = (time.perf_counter() - t0) * 1e6
        t0 = time.perf_counter(); eng.run(4, stats=False); torch.cuda.synchronize(); w4b = (time.perf_counter() - t0) * 1e6
        t0 = time.perf_counter(); eng.run(8, stats=False); torch.cuda.synchronize(); w8 = (time.perf_counter() - t0) * 1e6
        t0 = time.perf_counter(); eng.run(8, stats=False); torch.cuda.synchronize(); w8b = (time.perf_counter() - t0) * 1e6
        print(f"trial {trial}: run(4) {w4:.1f} {w4b:.1f}; run(8) first {w8:.1f} then {w8b:.1f}", flush=True)
        print(f"trial {trial}: run(20) wall us: first {walls[0]:.1f}, then {walls[1]:.1f} {walls[2]:.1f}; "
              f"device {ms * 1e3:.1f} us", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
