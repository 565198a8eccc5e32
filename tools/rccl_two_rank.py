#!/usr/bin/env python3
"""The RCCL exchange path (agx_comm_init + run_multi_rccl) with `--world` ranks in
separate processes on the SAME device (a one-GPU box), checked bit-exactly against
the BSP oracle in the sharded canonical order.  RCCL refuses two ranks on one
device of one host ("Duplicate GPU detected"); --split-hosts gives every rank its
own NCCL_HOSTID, so the ranks look like separate hosts and exchange over RCCL's
socket transport on loopback -- the same ncclSend/ncclRecv/ncclAllGather calls as
over xGMI on a multi-GPU node.  Exit 0 = parity, 1 = mismatch, 2 = a rank failed.

    python tools/rccl_two_rank.py --split-hosts [--world 2] [--n 20000] [--hops 8]
                                  [--workload ring|mixed|orset|power|zipf] [--restage K]
--restage K: run K supersteps, stage a second burst of tells on every rank (each keeps the ones it
owns), then run to quiescence -- a staged burst between device-resident replays.
"""
import argparse
import os
import pathlib
import socket
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(a):
    from akka_amd import workloads as wl
    from akka_amd.engine import Kind
    if a.workload == "ring":
        return wl.token_ring(a.n, a.hops)
    if a.workload == "orset":  # CRDT snapshot rows travel beside the envelopes
        return wl.crdt_gossip(a.n, Kind.ORSET, rounds=a.hops, throughput=2)
    if a.workload == "orset_delta":  # delta rows (DeltaPropagation) and full-state gossips
        return wl.crdt_delta(a.n, Kind.ORSET, rounds=a.hops, ops_per_replica=2, gossip_rounds=2, throughput=2)
    if a.workload == "crdt_mixed":  # GCounter / PNCounter / ORSet rows of three pitches' kinds
        return wl.crdt_mixed(a.n, rounds=a.hops, throughput=2)
    if a.workload == "power":  # C5 shape: bounded(64) forwarding over the R-MAT graph
        return wl.power_law_forward(a.n, ttl=a.hops, capacity=64, throughput=5, device_graph=True)
    if a.workload == "zipf":
        return wl.zipf_fanout(a.n, k=4, ttl=3, root_every=16, throughput=3)
    return wl.mixed(a.n, seed=3, throughput=2, capacity=6)


def _burst(n):
    """the second staged burst of --restage: every 7th actor, payload 3 (a hop budget / an op)"""
    import numpy as np
    d = np.arange(0, n, 7, dtype=np.uint32)
    return d, np.full(d.size, 3, np.uint32)


def _rank_main(rank, world, port, a, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if a.split_hosts:
        # RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"); a distinct
        # host id per rank makes them two "hosts" that talk over the socket transport on loopback
        os.environ["NCCL_HOSTID"] = f"agx-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    import numpy as np
    import torch.distributed as dist
    from akka_amd.engine import EngineConfig, GpuEngine
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = _make(a)
        eng = GpuEngine(EngineConfig(device=0, n_ranks=world, rank=rank, **w.gpu_kwargs()))
        w.apply_to(eng)
        uid = [GpuEngine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(uid[0])
        if a.restage:
            eng.run(a.restage)
            d, pay = _burst(w.n_actors)
            eng.tell(d, pay)
        st = eng.run()
        ws, al = eng.read_state()
        xi = eng.exchange_info() if hasattr(eng.lib, "agx_exchange_info") else {}
        eng.close()
        q.put((rank, "ok", st.__dict__ if hasattr(st, "__dict__") else dict(st._asdict()), ws, al, xi))
    except Exception as ex:  # report, do not hang the peer
        q.put((rank, "error", repr(ex), None, None, None))
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--hops", type=int, default=8)
    ap.add_argument("--workload", default="ring")
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--split-hosts", action="store_true", help="one NCCL_HOSTID per rank (one-GPU box)")
    ap.add_argument("--restage", type=int, default=0, help="stage a second burst after this many supersteps")
    a = ap.parse_args()
    import numpy as np
    import torch.multiprocessing as mp
    from akka_amd.engine import owner
    from oracle import BspOracle
    world = a.world
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, a, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    errs = [r for r in res if r[1] != "ok"]
    if errs:
        print("RCCL two-rank run failed:", errs)
        sys.exit(2)
    w = _make(a)
    ref = BspOracle(n_ranks=world, **w.engine_kwargs())
    w.apply_to(ref)
    if a.restage:
        ref.run(a.restage)
        d, pay = _burst(w.n_actors)
        ref.tell(d, pay)
    so = ref.run()
    wo, ao = ref.read_state()
    wg = np.zeros_like(wo)
    ag = np.zeros_like(ao)
    own_of = np.array([owner(i, 1000, world) for i in range(w.n_actors)])
    tot = {}
    for rank, _, st, ws, al, xi in res:
        if xi:  # the exchange this rank ran, and what it sent per superstep
            steps = max(1, xi["dev_steps"] + xi["host_steps"])
            print(f"exchange rank {rank}: dev_steps={xi['dev_steps']} host_steps={xi['host_steps']} "
                  f"rows_on_host={xi['rows_on_host']} slab={xi['slab']} env_B/step={xi['env_bytes'] // steps} "
                  f"row_B/step={xi['row_bytes'] // steps}")
        own = own_of == rank
        wg[own] = ws[own]
        ag[own] = al[own]
        for k, v in st.items():
            tot[k] = tot.get(k, 0) + v
    print("gpu (sum over ranks):", {k: tot[k] for k in ("delivered", "dead_letters", "unhandled", "emitted", "staged")})
    print("oracle:", {k: so[k] for k in ("delivered", "dead_letters", "unhandled", "emitted", "staged")})
    keys = ("delivered", "dead_letters", "unhandled", "emitted", "staged")
    # (per-rank counters, or counters already reduced over the ranks)
    ok = all(tot[k] == so[k] for k in keys) or all(r[2][k] == so[k] for r in res for k in keys)
    ok = ok and np.array_equal(wg, wo) and np.array_equal(ag, ao)
    print("RCCL two-rank parity:", "OK" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
