#!/usr/bin/env python3
"""Diagnostic: C5 power-law bounded forwarding, eager launches with per-kernel and
per-bucket stamps (AGX_STAMPS=1 in the environment)."""
import sys, pathlib, time, argparse
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000_000)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--workload", default="c5")
a = ap.parse_args()
import torch
from akka_amd import workloads as wl
from akka_amd.engine import EngineConfig, GpuEngine
if a.workload == "c5":
    w = wl.power_law_forward(a.n, ttl=15, capacity=64, throughput=5, device_graph=True)
elif a.workload == "c3":
    w = wl.zipf_fanout(a.n, k=1, ttl=15, root_every=1, capacity=1000)
elif a.workload == "c3s":  # C3 steady state at SURVEY's spec shape (ttl 64, 1/64 roots, unbounded)
    w = wl.zipf_fanout(a.n if a.n != 100_000_000 else 10_000_000, k=1, ttl=64, root_every=64, throughput=5)
elif a.workload == "c3t":  # C3 fan-out tree as benched
    w = wl.zipf_fanout(a.n if a.n != 100_000_000 else 10_000_000, k=4, ttl=3, root_every=64, capacity=1000)
elif a.workload in ("c4g", "c4o"):
    from akka_amd.engine import Kind
    w = wl.crdt_gossip(a.n if a.n != 100_000_000 else 1_000_000, Kind.GCOUNTER if a.workload == "c4g" else Kind.ORSET,
                       rounds=40)
elif a.workload in ("c4gd", "c4od"):  # delta-CRDT replication as benched
    from akka_amd.engine import Kind
    w = wl.crdt_delta(a.n if a.n != 100_000_000 else 1_000_000, Kind.GCOUNTER if a.workload == "c4gd" else Kind.ORSET,
                      rounds=40, write=True)
else:
    w = wl.ping_pong(1000, messages_per_pair=2_000_000, throughput=50)
cfg = EngineConfig(**w.gpu_kwargs())
if a.workload == "c1":
    cfg.msg_capacity = 1 << 20
if a.workload in ("c4gd", "c4od"):
    cfg.msg_capacity = 8_000_000
eng = GpuEngine(cfg)
w.apply_to(eng)
eng.run(2)
eng.profile(True)
for i in range(a.steps):
    eng.profile_reset()
    s0 = eng.stats()
    s1 = eng.run(1)
    p = eng.profile_read()
    print("step", i, "delivered", s1.delivered - s0.delivered, "dead", s1.dead_letters - s0.dead_letters,
          "in_flight", s1.in_flight, "ring_buckets", eng.ring_buckets() if hasattr(eng, "ring_buckets") else None,
          {k: round(v["total_ms"], 3) for k, v in p.items() if v["launches"]}, flush=True)
