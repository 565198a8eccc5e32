"""Diagnostic: wall time per superstep of the C2 ring for several agx_run budgets (stats=False),
to see launch/poll overheads of the graph replays (AGX_MAX_REPLAY caps the replay length)."""
import sys, time, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import torch
from akka_amd import workloads as wl
from akka_amd.engine import EngineConfig, GpuEngine
w = wl.token_ring(1_000_000, 2000)
eng = GpuEngine(EngineConfig(**w.engine_kwargs()))
w.apply_to(eng)
eng.run(17)
torch.cuda.synchronize()
for K in (16, 20, 32, 64, 128, 200, 400):
    t0 = time.perf_counter()
    eng.run(K, stats=False)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"K={K} total {el*1e3:.3f} ms  per step {el/K*1e6:.2f} us", flush=True)
eng.close()
