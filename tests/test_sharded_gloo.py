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


def _rank_main(rank, world, port, q, slab0=0):
    """slab0 > 0: the device-resident protocol (run_multi_rccl's replays): fixed-size per-peer slabs
    exchanged every superstep, the decision from the product's agx_mr_plan (the code k_mr_pack runs
    on the device); a count over the slab -> that superstep's exchange exactly, slabs grown to 5/4 of
    the largest count + 1024 on every rank alike; a staged burst enters through one exact superstep."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["AKKA_AMD_NO_TORCH"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    from akka_amd import sharding
    from akka_amd.engine import MR_GO, MR_OVER_SLAB, MR_QUIET, exchange_plan, mr_plan

    own = sharding.owners(N, 1000, world)
    mine = np.nonzero(own == rank)[0]                 # local order = id order
    count = {int(a): 0 for a in mine}
    backlog = []                                      # (dst, src, pay)
    # staged tells: every actor gets one token (hop budget HOPS), only owned dsts kept
    staged = [(int(a), 0xFFFFFFFF, HOPS) for a in mine]
    emitted = []                                      # (dst, src, pay) in local src order
    delivered = 0
    slab, codes = slab0, []
    while True:
        # partition emissions by owner (stable)
        parts = [[e for e in emitted if own[e[0]] == r] for r in range(world)]
        vec = np.array([len(p) for p in parts] + [len(backlog), len(staged)], np.uint64)
        mats = [None] * world
        dist.all_gather_object(mats, vec.tolist())
        mat = np.array(mats, np.uint64)
        plan = exchange_plan(mat, rank)
        if plan["inflight"] == 0:
            break
        code = None
        if slab and not staged:
            d = mr_plan(mat, rank, slab, 1 << 40)
            code = d["code"]
            codes.append(code)
            assert code != MR_QUIET and d["n_backlog"] == len(backlog)
            assert np.array_equal(d["recv_off"][:-1], plan["recv_off"] - len(backlog))
        if code == MR_GO:  # fixed-size slabs: [peer][slab][key, src, payload], zero padded
            sl = torch.zeros((world, slab, 3), dtype=torch.int64)
            for r in range(world):
                if parts[r]:
                    sl[r, :len(parts[r])] = torch.tensor(parts[r], dtype=torch.int64)
            allv = [torch.zeros_like(sl) for _ in range(world)]
            dist.all_gather(allv, sl)
            recv = []
            for r in range(world):                   # sender-rank order, counts from the matrix
                n = int(mat[r][rank])
                recv += parts[r] if r == rank else [tuple(int(x) for x in t) for t in allv[r][rank, :n].tolist()]
        else:
            got = [None] * world
            dist.all_gather_object(got, parts)
            recv = []
            for r in range(world):                   # sender-rank order
                recv += got[r][rank]
            if code == MR_OVER_SLAB:  # every rank grows alike (the same matrix)
                mx = max(int(mat[r][c]) for r in range(world) for c in range(world) if r != c)
                slab = max(slab, mx + mx // 4 + 1024)
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
    q.put((rank, count, delivered, codes))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("slab0", [0, 64])
def test_two_rank_gloo_matches_oracle(built, slab0):
    from oracle import BspOracle
    from akka_amd import workloads as wl
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q, slab0)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    counts = np.zeros(N, np.uint64)
    delivered = 0
    for _, cnt, d, codes in res:
        delivered += d
        if slab0:  # the slabs overflowed once (then grown) and carried the other supersteps
            assert codes.count(1) == 1 and codes.count(0) == len(codes) - 1 and len(codes) > 2, codes
        for a, c in cnt.items():
            counts[a] = c
    w = wl.token_ring(N, HOPS, throughput=T)
    o = BspOracle(n_ranks=world, **w.engine_kwargs())
    w.apply_to(o)
    st = o.run()
    assert delivered == st["delivered"] == N * (HOPS + 1)
    assert np.array_equal(counts, o.read_state()[0][:, 0])
