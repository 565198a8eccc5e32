#!/usr/bin/env python3
"""Benchmark: messages delivered/sec of the batched actor dispatcher.

Workload (BASELINE.json configs[1], C2): token ring, 1M actors per GPU, every
actor holds one token (integer payload = remaining hop budget); RING behaviour
= count++, forward payload-1 to actor (self+1) mod N.  With N GPUs the ring
has N x 1M actors hash-sharded by ShardRegion's extractShardId (weak scaling),
cross-GPU mail is exchanged with RCCL once per superstep.

A "step" is one BSP superstep (one Mailbox.run round over every actor with
mail) = 1M deliveries per GPU.  Inputs are resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
N_PER_GPU = 1_000_000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--actors-per-gpu", type=int, default=N_PER_GPU)
    ap.add_argument("--hops", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--large-actors", type=int, default=100_000_000,
                    help="whole-job actor count of the second operating point (0 = skip)")
    ap.add_argument("--large-steps", type=int, default=24)
    ap.add_argument("--large-warmup", type=int, default=4)
    ap.add_argument("--cpu-hops", type=int, default=96, help="hop budget of the bounded CPU sample")
    ap.add_argument("--no-configs", action="store_true", help="skip the other BASELINE configs (N=1 only)")
    ap.add_argument("--quick-configs", action="store_true", help="C5 at 10M instead of 100M actors")
    ap.add_argument("--pmc", default=str(ROOT / "profiles" / "pmc_r06.json"),
                    help="PMC traffic summary written by profiles/collect_pmc.py")
    return ap.parse_args()


def kernel_bytes_per_msg(W: int) -> dict:
    """Algorithmic HBM bytes per message for each kernel class."""
    return {
        "bucket_apply": 12 + 12 + (16 * W + 2),  # read inbox envelope, write emitted tell, state r/w + kind/alive
        "bucket_apply_dense": 12 + 12 + (16 * W + 2),  # the same, one message per actor (k_dense_fused / _apply)
        "ring_apply": 12 + 12 + (16 * W + 2),    # the same per delivered message (bounded mailboxes, agx_ring.h)
        "chunk_downsweep": 24,                  # read + write one 12 B envelope (first radix pass)
        "sort_downsweep": 24,                   # read + write one 12 B envelope (later passes)
        "sort_upsweep": 4,                      # read key
        "chunk_rowscan": 0, "sort_rowscan": 0, "mcompact": 24, "exchange": 12,
    }


SORT_CLASSES = ("chunk_downsweep", "sort_upsweep", "sort_downsweep")
# profiling classes that are not one HBM-bound kernel: the multi-rank exchange (RCCL all-gather + send /
# receive + the slab pack / unpack kernels) is reported on its own (the line's `exchange` object)
NON_KERNEL = ("exchange",)
DENSE_FOLLOWERS = ("bucket_apply", "bucket_apply_tiny")  # (launched after k_dense_apply in one superstep)


def kernel_rooflines(prof: dict, per_msg: dict, msgs_per_launch: int, identity: bool = False) -> dict:
    """HBM roofline of every kernel class with algorithmic bytes: achieved = bytes per message x
    messages per launch / average launch time (HIP events); `dominant` = largest total time.
    identity: every profiled superstep was grouped without a radix pass -- the
    pass kernels were launched but returned at entry, so they move no bytes and get no roofline."""
    out = {}
    for k, v in prof.items():
        if identity and k in SORT_CLASSES and v["launches"]:
            out[k] = {"returned_at_entry": True, "avg_launch_ms": round(v["total_ms"] / v["launches"], 4)}
            continue
        if v["launches"] and k in NON_KERNEL:  # (RCCL + slab copies: no HBM roofline)
            out[k] = {"avg_ms": round(v["total_ms"] / v["launches"], 4), "note": "RCCL exchange, not an HBM kernel"}
            continue
        if not v["launches"] or not per_msg.get(k):
            continue
        avg_ms = v["total_ms"] / v["launches"]
        ach = per_msg[k] * msgs_per_launch / (avg_ms * 1e-3) / 1e9
        dense = prof.get("bucket_apply_dense", {})
        if k in DENSE_FOLLOWERS and dense.get("launches") and dense.get("items", 0) == dense["launches"]:
            # every profiled dense launch took every bucket (the device's dense_left flags, read back after
            # each launch: agx_profile_read items): this launch returned at entry
            out[k] = {"returned_at_entry": True, "avg_launch_ms": round(avg_ms, 4),
                      "reason": "the dense launch before it took every bucket (device dense_left flags)"}
            continue
        out[k] = {"achieved": round(ach, 1), "frac": round(ach / PEAK_HBM_GBS, 4), "avg_launch_ms": round(avg_ms, 4),
                  "alg_bytes_per_launch": per_msg[k] * msgs_per_launch}
    dom = max((k for k in prof if prof[k]["launches"] and k not in NON_KERNEL), key=lambda k: prof[k]["total_ms"],
              default=None)
    return {"bound": "hbm", "peak": PEAK_HBM_GBS, "unit": "GB/s", "dominant": dom, "kernels": out}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _fjp_rate(w, threads: int) -> dict:
    from oracle import FjpOracle
    f = FjpOracle(**w.engine_kwargs())
    w.apply_to(f)
    st = f.run(threads)
    wall = f.wall_s
    f.close()
    return {"value": st["delivered"] / wall, "delivered": st["delivered"], "dead_letters": st["dead_letters"],
            "wall_s": round(wall, 3)}


def cpu_baseline(hops: int) -> dict:
    """fjp_ref (oracle/fjp_ref.cpp: restatement of Dispatcher + Mailbox + a lock-free work-stealing
    ForkJoinPool) on the host cores, on bounded samples of each workload.  The
    headline `value` is the C2 ring sample; `configs` carries C1 (the reference's own CPU-only
    JMH config, ForkJoinActorBenchmark.pingPong), C3, C4 and C5 samples.  bsp_ref = the
    single-threaded deterministic oracle on the same ring."""
    from akka_amd import workloads as wl
    from akka_amd.engine import Kind
    from oracle import BspOracle

    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    cores = min(cores, len(os.sched_getaffinity(0)))
    ring = wl.token_ring(N_PER_GPU, hops, throughput=5)
    head = _fjp_rate(ring, cores)
    b = BspOracle(**ring.engine_kwargs())
    ring.apply_to(b)
    t0 = time.perf_counter()
    sb = b.run()
    bsp_s = time.perf_counter() - t0
    b.close()
    # C1 as the JMH config, C2 / C3 / C4 at the GPU run's full populations (C4 ORSet with
    # fewer gossip rounds: each full-state merge moves 2 KB rows, ~1 us per merge on a host core), C5 at
    # 10M actors (host RAM / run time; the GPU config is 100M)
    samples = {
        "C1_ping_pong": ("ForkJoinActorBenchmark.pingPong: 1000 pairs, throughput 50, 100 in flight per pair, "
                         "1,000,000 messages per pair (the JMH run uses 2,000,000)",
                         lambda: wl.ping_pong(1000, messages_per_pair=1_000_000, throughput=50)),
        "C3_zipf_fanout": ("10M actors (full size), Zipf(1.1) FANOUT k=1, every actor one message with ttl 15, "
                           "BoundedMailbox(1000), throughput 5, to quiescence",
                           lambda: wl.zipf_fanout(10_000_000, k=1, ttl=15, root_every=1, capacity=1000)),
        "C3_zipf_tree": ("10M actors (full size), Zipf(1.1) FANOUT k=4 ttl=3, 1/64 roots, BoundedMailbox(1000), "
                         "throughput 5, to quiescence",
                         lambda: wl.zipf_fanout(10_000_000, k=4, ttl=3, root_every=64, capacity=1000)),
        "C4_gcounter_gossip": ("1M GCounter replicas (full size), 40 rounds of full-state gossip to 2 peers "
                               "(the GPU config)",
                               lambda: wl.crdt_gossip(1_000_000, Kind.GCOUNTER, rounds=40)),
        "C4_orset_gossip": ("1M ORSet replicas (full size), 4 rounds of full-state gossip to 2 peers (the GPU "
                            "config runs 20)",
                            lambda: wl.crdt_gossip(1_000_000, Kind.ORSET, rounds=4)),
        "C4_orset_delta_gossip": ("1M delta-CRDT ORSet replicas (full size, keys of 8), 8 DeltaPropagationTicks "
                                  "with a writer update each (the GPU config runs 40)",
                                  lambda: wl.crdt_delta(1_000_000, Kind.ORSET, rounds=8, write=True)),
        "C5_power_law_bounded": ("10M actors (the GPU config: 100M), power-law R-MAT graph, FORWARD_RR ttl 15, "
                                 "BoundedMailbox(64), to quiescence",
                                 lambda: wl.power_law_forward(10_000_000, ttl=15, capacity=64, throughput=5)),
    }
    configs = {}
    for name, (desc, make) in samples.items():
        try:
            configs[name] = dict(sample=desc, unit="msg/s", **_fjp_rate(make(), cores))
        except Exception as ex:  # one sample failing must not hide the others
            configs[name] = {"sample": desc, "error": repr(ex)}
    return {"value": head["value"], "unit": "msg/s", "cores": cores, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"fjp_ref ForkJoin-dispatcher restatement (lock-free work-stealing pool, {cores} threads), "
                      f"1M-actor token ring, hops={hops} ({head['delivered']} deliveries, {head['wall_s']} s, "
                      f"throughput=5)",
            "bsp_ref_1thread_msg_s": sb["delivered"] / bsp_s, "configs": configs}


def timed_ring(n_total: int, hops: int, warmup: int, steps: int, world: int, rank: int, local: int,
               msg_capacity: int = 0, keep: bool = False):
    """Build the C2 ring over n_total actors (this rank keeps the ones it owns),
    run `warmup` untimed supersteps, then time exactly `steps` supersteps
    bracketed by barrier + device sync.  Returns (engine|None, s, delivered, supersteps)."""
    import torch
    import torch.distributed as dist
    from akka_amd import workloads as wl
    from akka_amd.engine import EngineConfig, GpuEngine

    w = wl.token_ring(n_total, hops)
    cfg = EngineConfig(device=local, n_ranks=world, rank=rank, **w.gpu_kwargs())
    cfg.msg_capacity = msg_capacity
    eng = GpuEngine(cfg)
    w.apply_to(eng)
    del w
    if world > 1:
        uid = [GpuEngine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(uid[0])
    # warmup (includes the upload of actor state, the initial tells and the graph capture)
    s0 = eng.run(warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(steps, stats=False)  # (the counters are read back after the timed region)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    s1 = eng.stats()
    if not keep:
        eng.close()
        eng = None
    return eng, t1 - t0, s1.delivered - s0.delivered, s1.supersteps - s0.supersteps


def timed_workload(w, warmup: int, steps: int, msg_capacity: int = 0) -> dict:
    """One BASELINE config on one GPU: install the workload, `warmup` untimed supersteps,
    then exactly `steps` timed supersteps (inputs resident in HBM, replayed from hipGraphs).
    The per-kernel breakdown comes from a second engine on the same workload driven through
    the SAME superstep window (warmup, then `steps` eager supersteps with HIP events around
    every kernel class): a workload's mail changes from superstep to superstep (C5's tokens die
    after 15 hops), so a window after the timed one would describe different supersteps."""
    import torch
    from akka_amd.engine import EngineConfig, GpuEngine

    def make():
        cfg = EngineConfig(**w.gpu_kwargs())
        cfg.msg_capacity = msg_capacity
        eng = GpuEngine(cfg)
        w.apply_to(eng)
        return eng

    t0 = time.perf_counter()
    eng = make()
    setup = time.perf_counter() - t0
    s0 = eng.run(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(steps, stats=False)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    s1 = eng.stats()
    rings = eng.ring_buckets()
    eng.close()
    eng = make()  # the profiled replay of the same window
    eng.run(warmup)
    eng.profile(True)
    eng.profile_reset()
    sp = eng.run(steps)
    prof = eng.profile_read()
    eng.close()
    d = s1.delivered - s0.delivered
    ss = s1.supersteps - s0.supersteps
    bytes_alg = s1.bytes_alg - s0.bytes_alg
    kms = {k: round(v["total_ms"] / max(ss, 1), 4) for k, v in prof.items() if v["launches"]}
    return {"value": d / el, "unit": "msg/s", "delivered": d, "dead_letters": s1.dead_letters - s0.dead_letters,
            "supersteps_timed": ss, "ms_per_step": el / max(ss, 1) * 1e3, "setup_s": round(setup, 2),
            "alg_bytes_per_msg": bytes_alg / max(d, 1), "ring_buckets": rings,
            "superstep_frac": bytes_alg / el / 1e9 / PEAK_HBM_GBS,
            "profiled_window_same": sp.delivered == s1.delivered and sp.supersteps == s1.supersteps,
            "kernel_ms_per_step": kms, "kernel_ms_per_step_sum": round(sum(kms.values()), 4)}


def other_configs(quick: bool, only: str = "") -> dict:
    """BASELINE.json configs other than the headline ring, each measured on one GPU
    (`only`: just that one, for tools/cfg_one.py)."""
    from akka_amd import workloads as wl
    from akka_amd.engine import Kind

    n5 = 10_000_000 if quick else 100_000_000
    specs = {
        "C5_power_law_bounded": (
            f"{n5 // 1_000_000}M actors, power-law out-degree (alpha 2.1, d<=1024) R-MAT graph, FORWARD_RR "
            "round-robin forwarding, BoundedMailbox(64) tail-drop, throughput 5, 1 message/actor",
            lambda: wl.power_law_forward(n5, ttl=15, capacity=64, throughput=5, device_graph=True), 2, 10, 0),
        "C5_power_law_cap1000": (
            f"{n5 // 1_000_000}M actors, the C5 graph and behaviour with SURVEY.md 8(d)'s second mailbox setting: "
            "the reference's default mailbox-capacity 1000 (bounded, tail-drop), throughput 5",
            lambda: wl.power_law_forward(n5, ttl=15, capacity=1000, throughput=5, device_graph=True), 2, 10, 0),
        "C3_zipf_fanout": (
            "10M actors, Zipf(1.1) destinations over a seeded permutation, FANOUT counter/sum behaviour, k=1 steady "
            "state (every actor holds one message, ttl 15), BoundedMailbox(1000) (an unbounded mailbox lets the hot "
            "actors' backlogs grow without limit at throughput 5), throughput 5",
            lambda: wl.zipf_fanout(10_000_000, k=1, ttl=15, root_every=1, capacity=1000), 2, 10, 0),
        "C3_zipf_steady_spec": (
            "10M actors, SURVEY.md 8(d)'s steady-state shape as specified: Zipf(1.1) FANOUT, k=1, ttl 64, 1/64 of "
            "the actors roots, the reference's default UNBOUNDED mailbox, throughput 5 (the hot actors' queues grow "
            "without limit; beside the bounded variant above)",
            lambda: wl.zipf_fanout(10_000_000, k=1, ttl=64, root_every=64, throughput=5), 2, 10, 0),
        "C3_zipf_tree": (
            "10M actors, Zipf(1.1) fan-out tree of SURVEY.md 8(d): 1/64 of the actors are roots, k=4 tells per "
            "message, ttl 3, BoundedMailbox(1000), throughput 5; timed from the first superstep (the burst)",
            lambda: wl.zipf_fanout(10_000_000, k=4, ttl=3, root_every=64, capacity=1000), 0, 8, 0),
        "C3_zipf_tree_spec": (
            "10M actors, SURVEY.md 8(d)'s fan-out tree as specified: Zipf(1.1) FANOUT k=4, ttl 3, 1/64 roots, the "
            "reference's default UNBOUNDED mailbox, throughput 5; timed from the first superstep (the burst)",
            lambda: wl.zipf_fanout(10_000_000, k=4, ttl=3, root_every=64, throughput=5), 0, 8, 0),
        "C4_gcounter_gossip": (
            "1M Replicator-style GCounter replicas (8 node slots), full-state gossip to 2 random peers per tick, "
            "merge = slot-wise max (akka-distributed-data GCounter.merge)",
            lambda: wl.crdt_gossip(1_000_000, Kind.GCOUNTER, rounds=40), 4, 24, 0),
        "C4_orset_gossip": (
            "1M Replicator-style ORSet replicas (64-element universe, 8 nodes, dots + version vector), full-state "
            "gossip to 2 random peers per tick, ORSet.merge",
            lambda: wl.crdt_gossip(1_000_000, Kind.ORSET, rounds=20), 2, 12, 0),
        "C4_orset_delta_gossip": (
            "1M Replicator-style ORSet replicas with delta-CRDT replication (keys of 8 replicas = 8 nodes): each "
            "DeltaPropagationTick tells the replica one writer Update (add/remove) and propagates the merged delta "
            "groups to a round-robin slice of 2 nodes (DeltaPropagationSelector, causal delivery, ORSet.mergeDelta)",
            lambda: wl.crdt_delta(1_000_000, Kind.ORSET, rounds=40, write=True), 4, 24, 8_000_000),
        "C4_gcounter_delta_gossip": (
            "1M Replicator-style GCounter replicas with delta-CRDT replication (keys of 8): each "
            "DeltaPropagationTick tells one writer increment and propagates the counter deltas to 2 nodes",
            lambda: wl.crdt_delta(1_000_000, Kind.GCOUNTER, rounds=40, write=True), 4, 24, 8_000_000),
        "C1_ping_pong": (
            "akka-bench-jmh ForkJoinActorBenchmark.pingPong shape: 1000 PingPong pairs, 100 in flight per pair, "
            "throughput 50",
            lambda: wl.ping_pong(1000, messages_per_pair=2_000_000, throughput=50), 16, 400, 1 << 20),
    }
    out = {}
    # counted HBM bytes per superstep of the same window (profiles/pmc_r06.json "configs", from the
    # rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/cfg_one.py): the fraction on the bytes the
    # kernels actually moved, beside the one on the algorithmic model (C4 ORSet's sparse rows move
    # fewer bytes than its dense-state model; C5 / C3 far more)
    try:
        counted = json.loads((ROOT / "profiles" / "pmc_r06.json").read_text()).get("configs", {})
    except Exception:
        counted = {}
    for name, (desc, make, warm, steps, mcap) in specs.items():
        if only and name != only:
            continue
        try:  # one config failing must not hide the others
            out[name] = dict(workload=desc, **timed_workload(make(), warm, steps, msg_capacity=mcap))
            c = counted.get(name)
            if c and out[name].get("ms_per_step"):
                t = out[name]["ms_per_step"] * 1e-3
                out[name]["superstep_frac_counted"] = c["counted_bytes_per_superstep"] / t / 1e9 / PEAK_HBM_GBS
                if "counted_bytes_per_superstep_raw" in c:
                    out[name]["superstep_frac_counted_raw"] = c["counted_bytes_per_superstep_raw"] / t / 1e9 / PEAK_HBM_GBS
        except Exception as ex:
            out[name] = {"workload": desc, "error": repr(ex)}
    return out


def summary(out: dict) -> dict:
    """Every reported rate in one small object (printed last)."""
    s = {"C2_1M_ring": {"msg_s": out["value"], "ms_per_step": out["ms_per_step"],
                        "apply_frac": round(out["roofline"]["frac"], 4)}}
    lg = out.get("at_100M_actors")
    if lg:
        s["ring_100M"] = {"msg_s": lg["value"], "ms_per_step": round(lg["ms_per_step"], 4),
                          "superstep_frac": round(lg["superstep_frac"], 4),
                          "identity_supersteps": lg.get("identity_supersteps")}
    for k, v in (out.get("configs") or {}).items():
        if isinstance(v, dict) and "value" in v:
            s[k] = {"msg_s": v["value"], "ms_per_step": round(v["ms_per_step"], 4),
                    "superstep_frac": round(v["superstep_frac"], 4)}
            if "superstep_frac_counted" in v:
                s[k]["superstep_frac_counted"] = round(v["superstep_frac_counted"], 4)
    cb = out.get("cpu_baseline")
    if isinstance(cb, dict) and "value" in cb:
        s["cpu_baseline"] = {"msg_s": cb["value"], "cores": cb["cores"], "kind": cb["kind"]}
    return s


def reduce_ranks(elapsed: float, delivered: int, world: int):
    """MAX elapsed and SUM delivered over ranks."""
    if world == 1:
        return elapsed, delivered
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    d = torch.tensor([delivered], dtype=torch.float64)
    dist.all_reduce(d, op=dist.ReduceOp.SUM)
    return float(t.item()), int(d.item())


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1:
        raise SystemExit("--gpus N>1 needs one process per GPU: torchrun --nproc-per-node N bench.py --gpus N")

    import torch
    import torch.distributed as dist

    import __graft_entry__ as g
    if rank == 0 or world == 1:
        g.build_native()
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist.barrier()
    torch.cuda.set_device(local)

    prof_steps = min(args.steps, 64)
    hops = max(args.hops, args.warmup + args.steps + 2 * prof_steps + 1)  # (eager profile + graph-timed replay)
    n_total = args.actors_per_gpu * world
    eng, elapsed, delivered, steps_done = timed_ring(n_total, hops, args.warmup, args.steps, world, rank, local,
                                                     msg_capacity=int(2 * args.actors_per_gpu * 1.25) if world > 1 else 0,
                                                     keep=True)

    # per-kernel HIP-event timing on the engine's stream (eager launches: the
    # event pairs bracket every kernel); kernel durations are launch-mode independent
    eng.profile(True)
    eng.profile_reset()
    eng.run(prof_steps)
    prof = eng.profile_read()
    eng.profile(False)
    # the same supersteps replayed from graphs, timed by HIP events on the engine stream (device time
    # per superstep; in the fused strict replay a superstep is the dense launch alone, plus one
    # k_replay_out per 8 supersteps): the eager per-class events above add ~3 us of event overhead
    # per launch that rocprofv3 does not see
    pi0 = eng.persist_info()
    _, graph_ms = eng.run_timed(prof_steps)
    pi1 = eng.persist_info()
    # supersteps per persistent launch in that window (0: one launch per superstep)
    persist_k = ((pi1["supersteps"] - pi0["supersteps"]) / (pi1["launches"] - pi0["launches"])
                 if pi1["launches"] > pi0["launches"] else 0)
    cfg_words = eng.cfg.n_words
    # multi-rank: the exchange beside the kernels -- its time per superstep (the eager profiled window:
    # all-gather, slab pack, send / receive, unpack) and this rank's wire bytes per superstep
    xinfo = None
    if world > 1 and prof.get("exchange", {}).get("launches"):
        xi = eng.exchange_info()
        xms = prof["exchange"]["total_ms"] / prof["exchange"]["launches"]
        wire = xi["env_bytes"] / max(xi["dev_steps"], 1)
        xinfo = {"ms_per_superstep": round(xms, 4), "wire_bytes_per_superstep": int(wire), "slab": xi["slab"],
                 "achieved_GBps": round(wire / (xms * 1e-3) / 1e9, 1) if xms > 0 else None,
                 "device_resident_supersteps": xi["dev_steps"], "host_planned_supersteps": xi["host_steps"]}
    eng.close()

    elapsed, delivered = reduce_ranks(elapsed, delivered, world)

    # the metric's second operating point: 100M actors over the whole job
    # (strong-scaled: 100M/N actors per GPU), same ring, shorter timed region
    large = None
    if args.large_actors > 0:
        n_l = args.large_actors
        per = (n_l + world - 1) // world
        steps_l = args.large_steps
        prof_l = 4
        eng_l, el_l, dl_l, sd_l = timed_ring(n_l, args.large_warmup + steps_l + prof_l + 2, args.large_warmup, steps_l,
                                             world, rank, local,
                                             msg_capacity=int(per * (2.5 if world > 1 else 1.25)) + 4096, keep=True)
        ident_l = eng_l.identity_supersteps()  # supersteps grouped without a radix pass
        # per-kernel HIP-event timing at this size (eager launches on the engine stream)
        eng_l.profile(True)
        eng_l.profile_reset()
        eng_l.run(prof_l)
        pl = eng_l.profile_read()
        prof_ident = eng_l.identity_supersteps() - ident_l == prof_l
        eng_l.close()
        roof_l = kernel_rooflines(pl, kernel_bytes_per_msg(cfg_words), per, identity=prof_ident)
        # the dense launch's fraction on COUNTED bytes beside the 42-B model (PMC, corrected as the guide
        # prescribes): at 10^8 the model over-counts what the kernel moves
        try:
            cnt_l = json.loads(pathlib.Path(args.pmc).read_text()).get("ring_100M_apply", {}).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            cnt_l = None
        kd = roof_l["kernels"].get("bucket_apply_dense", {})
        if cnt_l and kd.get("avg_launch_ms"):
            kd["counted_bytes_per_launch"] = cnt_l
            kd["frac_counted"] = round(cnt_l / (kd["avg_launch_ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
        el_l, dl_l = reduce_ranks(el_l, dl_l, world)
        large = {"actors": n_l, "actors_per_gpu": per, "steps": steps_l, "warmup": args.large_warmup,
                 "supersteps_timed": int(sd_l), "value": dl_l / el_l, "unit": "msg/s",
                 "ms_per_step": el_l / steps_l * 1e3, "scaling": "strong",
                 "superstep_frac": (12 + 12 + 16 * cfg_words + 2) * per / (el_l / steps_l) / 1e9 / PEAK_HBM_GBS,
                 "identity_supersteps": int(ident_l),
                 "roofline": roof_l}

    value = delivered / elapsed
    # roofline of the dominant kernel (largest total time in the timed region)
    per_msg = kernel_bytes_per_msg(cfg_words)
    local_msgs_per_step = args.actors_per_gpu
    dom = max((k for k in prof if prof[k]["launches"] and k not in NON_KERNEL), key=lambda k: prof[k]["total_ms"])
    avg_ms_eager = prof[dom]["total_ms"] / prof[dom]["launches"]
    # the dense launch alone per replayed superstep (C2's strict replays): its launch time is the
    # graph-timed superstep (an upper bound: 1/8 of a k_replay_out included); else the eager events
    graph_step_ms = graph_ms / max(prof_steps, 1)
    avg_ms = min(avg_ms_eager, graph_step_ms) if dom == "bucket_apply_dense" else avg_ms_eager
    alg_bytes = per_msg.get(dom, 0) * local_msgs_per_step
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = pathlib.Path(args.pmc)
    if pmc_path.exists():
        try:
            pmc = json.loads(pmc_path.read_text())
            traffic = pmc.get("kernels", {}).get(dom, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    step_time = elapsed / max(args.steps, 1)
    superstep_bytes = (12 + 12 + 16 * cfg_words + 2) * local_msgs_per_step
    out = {
        "metric": "messages delivered/sec (whole node) at 1M and 100M actors; % HBM roofline",
        "value": value,
        "unit": "msg/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_time * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (deterministic SplitMix64-seeded token ring; integer payloads)",
        "config": {"workload": "C2 token ring, 1M actors/GPU, 1 token/actor, RING behaviour, throughput=5, "
                               "unbounded mailbox" + (", hash-sharded (ShardRegion extractShardId), RCCL exchange"
                                                      if world > 1 else ""),
                   "actors": n_total, "actors_per_gpu": args.actors_per_gpu, "hop_budget": hops,
                   "supersteps_timed": int(steps_done), "profiled_supersteps": prof_steps,
                   "parallelism": f"shard{world}"},
        "kernel_ms": {k: {"total_ms": round(v["total_ms"], 4), "launches": v["launches"]} for k, v in prof.items()},
    }
    if world == 1 and not args.no_configs:
        try:
            out["configs"] = other_configs(args.quick_configs)
        except Exception as ex:  # an auxiliary config must never hide the headline number
            out["configs"] = {"error": repr(ex)}
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args.cpu_hops)
            except Exception as ex:  # the baseline must never hide the GPU number
                out["cpu_baseline"] = {"error": repr(ex)}
        # the compact objects last: a driver that keeps only the tail of the line still shows them
        out["roofline"] = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                           "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                           "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": avg_ms,
                           "avg_launch_ms_eager_events": avg_ms_eager, "graph_superstep_device_ms": graph_step_ms,
                           "superstep_frac": superstep_bytes / step_time / 1e9 / PEAK_HBM_GBS}
        if persist_k and dom == "bucket_apply_dense":
            # the replayed supersteps ran as persistent launches of persist_k supersteps each
            # (k_dense_fused<.., true>, one grid barrier between supersteps): per launch, persist_k x
            # the superstep's bytes in persist_k x its time -- the same fraction; rocprofv3 shows that
            # kernel's launches at persist_k x avg_launch_ms (profiles/)
            out["roofline"].update({"kernel": "bucket_apply_dense (persistent launch, k_dense_fused<KM, false, true>)",
                                    "supersteps_per_launch": persist_k,
                                    "alg_bytes_per_launch": alg_bytes * persist_k,
                                    "avg_launch_ms": avg_ms * persist_k,
                                    "avg_superstep_ms": avg_ms})
        if xinfo:
            out["exchange"] = xinfo
        out["at_100M_actors"] = large
        out["summary"] = summary(out)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
