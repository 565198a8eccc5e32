#!/usr/bin/env python3
"""Diagnostic: identity grouping superstep by superstep (tests/test_gpu_parity.py::test_identity_grouping
scenario), engine vs oracle counters after every superstep.

    AGX_RADIX_BITS=3 python tools/diag_ident.py [--n 100000] [--hops 12] [--steps 40]"""
import argparse
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

from akka_amd import workloads as wl  # noqa: E402
from akka_amd.engine import EngineConfig, GpuEngine  # noqa: E402
from oracle import BspOracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000)
ap.add_argument("--hops", type=int, default=12)
ap.add_argument("--steps", type=int, default=40)
a = ap.parse_args()
w = wl.token_ring(a.n, a.hops)
eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
w.apply_to(eng)
ref = BspOracle(**w.engine_kwargs())
w.apply_to(ref)
for s in range(a.steps):
    if s == 9:
        eng.tell(np.arange(0, w.n_actors, 97, dtype=np.uint32), 2)
        ref.tell(np.arange(0, w.n_actors, 97, dtype=np.uint32), 2)
    g = eng.run(1)
    o = ref.run(1)
    print(f"step {s}: gpu delivered={g.delivered} in_flight={g.in_flight} steps={g.supersteps} "
          f"ident={eng.identity_supersteps()} | oracle delivered={o['delivered']} in_flight={o['in_flight']} "
          f"steps={o['supersteps']}", flush=True)
    if o["in_flight"] == 0 and g.in_flight == 0:
        break
wg, _ = eng.read_state()
wo, _ = ref.read_state()
print("state equal:", bool(np.array_equal(wg, wo)), flush=True)
# the test's shape: replays of up to 16 supersteps, bounded
eng.close()
eng = GpuEngine(EngineConfig(**w.gpu_kwargs()))
w.apply_to(eng)
g1 = eng.run(9)
eng.tell(np.arange(0, w.n_actors, 97, dtype=np.uint32), 2)
g2 = eng.run(300)
print(f"replays: after 9 delivered={g1.delivered} in_flight={g1.in_flight}; after 300 more delivered={g2.delivered} "
      f"in_flight={g2.in_flight} steps={g2.supersteps} ident={eng.identity_supersteps()}", flush=True)
ref2 = BspOracle(**w.engine_kwargs())
w.apply_to(ref2)
ref2.run(9)
ref2.tell(np.arange(0, w.n_actors, 97, dtype=np.uint32), 2)
o2 = ref2.run()
print(f"oracle to quiescence: delivered={o2['delivered']} steps={o2['supersteps']}", flush=True)
