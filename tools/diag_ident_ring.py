#!/usr/bin/env python3
"""Diagnostic: identity grouping on the token ring at scale, one superstep per run call
(AGX_IDENT_DEBUG=1 prints each run's slice summaries).  python tools/diag_ident_ring.py N [steps]"""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
from akka_amd import workloads as wl  # noqa: E402
from akka_amd.engine import EngineConfig, GpuEngine  # noqa: E402

n = int(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
w = wl.token_ring(n, 256)
eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
w.apply_to(eng)
del w
for s in range(steps):
    g = eng.run(1)
    print(f"n={n} step {s}: delivered={g.delivered} in_flight={g.in_flight} ident={eng.identity_supersteps()}",
          flush=True)
eng.close()
