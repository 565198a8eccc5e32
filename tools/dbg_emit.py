#!/usr/bin/env python3
"""Diagnostic: run a multi-pass parity case one superstep at a time on the GPU engine and the BSP
oracle and print the first superstep whose counters differ (emitted / delivered / dead / ...).

  AGX_RADIX_BITS=2 AGX_UNIT_G=1 AKKA_AMD_LIB=akka_amd/lib/var/x.so python tools/dbg_emit.py --case crdt
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402

from akka_amd import workloads as wl  # noqa: E402
from akka_amd.engine import EngineConfig, GpuEngine, Kind  # noqa: E402
from oracle import BspOracle  # noqa: E402

CASES = {
    "crdt": lambda: wl.crdt_mixed(20_000, rounds=4, throughput=2, capacity=5),
    "orset": lambda: wl.crdt_gossip(20_000, Kind.ORSET, rounds=6),
}
KEYS = ("delivered", "dead_letters", "unhandled", "emitted", "staged", "supersteps", "in_flight")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="crdt")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--budget", type=int, default=1, help="supersteps per agx_run call (graph replays when > 1)")
    args = ap.parse_args()
    w = CASES[args.case]()
    kw = w.engine_kwargs()
    eng = GpuEngine(EngineConfig(bucket_actors=w.bucket_actors, **kw))
    w.apply_to(eng)
    ref = BspOracle(**kw)
    w.apply_to(ref)
    for s in range(args.steps):
        sg = eng.run(args.budget)
        so = ref.run(args.budget)
        bad = [k for k in KEYS if getattr(sg, k) != so[k]]
        print(f"step {s}: " + " ".join(f"{k}={getattr(sg, k)}/{so[k]}" for k in KEYS), flush=True)
        if bad:
            wg, ag = eng.read_state()
            wo, ao = ref.read_state()
            diff = np.nonzero((wg != wo).any(axis=1))[0]
            print(f"DIVERGED at step {s}: {bad}; state rows differing: {diff.size}, alive differs: "
                  f"{int((ag != ao).sum())}", flush=True)
            break
        if so["in_flight"] == 0:
            print("quiescent, no divergence", flush=True)
            break
    eng.close()


if __name__ == "__main__":
    main()
