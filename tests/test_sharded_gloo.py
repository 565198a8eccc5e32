"""N>1 path on CPU: two gloo ranks run the sharded superstep protocol of the
multi-GPU engine -- ownership by ShardRegion hashing (akka_amd.sharding /
agx_owner), per-step exchange sized by the product's agx_exchange_plan,
received mail placed after the local backlog in sender-rank order -- and the
union of their final states must equal the BSP oracle in the sharded order.
(The per-rank step here is a numpy restatement; on the GPU the same protocol
runs in akka_amd/csrc with RCCL.)"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

N, HOPS, T, C = 3000, 6, 2, 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["AKKA_AMD_NO_TORCH"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from akka_amd import sharding
    from akka_amd.engine import exchange_plan

    own = sharding.owners(N, 1000, world)
    mine = np.nonzero(own == rank)[0]                 # local order = id order
    count = {int(a): 0 for a in mine}
    backlog = []                                      # (dst, src, pay)
    # staged tells: every actor gets one token (hop budget HOPS), only owned dsts kept
    staged = [(int(a), 0xFFFFFFFF, HOPS) for a in mine]
    emitted = []                                      # (dst, src, pay) in local src order
    delivered = 0
    while True:
        # partition emissions by owner (stable)
        parts = [[e for e in emitted if own[e[0]] == r] for r in range(world)]
        vec = np.array([len(p) for p in parts] + [len(backlog), len(staged)], np.uint64)
        mats = [None] * world
        dist.all_gather_object(mats, vec.tolist())
        plan = exchange_plan(np.array(mats, np.uint64), rank)
        if plan["inflight"] == 0:
            break
        got = [None] * world
        dist.all_gather_object(got, parts)
        recv = []
        for r in range(world):                       # sender-rank order
            recv += got[r][rank]
        assert len(recv) == int(plan["recv_cnt"].sum())
        inbox = backlog + recv + staged              # backlog first, staged last
        backlog, staged, emitted = [], [], []
        order = sorted(range(len(inbox)), key=lambda i: (inbox[i][0], i))  # stable by dst
        by = {}
        for i in order:
            by.setdefault(inbox[i][0], []).append(inbox[i])
        for a in mine:                               # apply in local order
            msgs = by.get(int(a), [])
            for p, (d, s, pay) in enumerate(msgs):
                if p < T:
                    count[d] += 1
                    delivered += 1
                    if pay > 0:
                        emitted.append(((d + 1) % N, d, pay - 1))
                elif C == 0 or p < C:
                    backlog.append((d, s, pay))
    q.put((rank, count, delivered))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_oracle(built):
    from oracle import BspOracle
    from akka_amd import workloads as wl
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    counts = np.zeros(N, np.uint64)
    delivered = 0
    for _, cnt, d in res:
        delivered += d
        for a, c in cnt.items():
            counts[a] = c
    w = wl.token_ring(N, HOPS, throughput=T)
    o = BspOracle(n_ranks=world, **w.engine_kwargs())
    w.apply_to(o)
    st = o.run()
    assert delivered == st["delivered"] == N * (HOPS + 1)
    assert np.array_equal(counts, o.read_state()[0][:, 0])
