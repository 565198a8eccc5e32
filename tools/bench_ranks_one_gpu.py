#!/usr/bin/env python3
"""Rehearse `bench.py --gpus N` (the driver's torchrun launch) on a ONE-GPU box: N processes with
RANK / WORLD_SIZE / LOCAL_RANK=0 / MASTER_* set as torchrun would, each with its own NCCL_HOSTID
so RCCL accepts several ranks on one device (socket transport on loopback).  Checks that the
multi-rank bench path runs end to end and prints one JSON line; its numbers are not multi-GPU
numbers (the ranks share one GPU).

    python tools/bench_ranks_one_gpu.py --world 2 -- --steps 5 --warmup 2 --large-actors 0
"""
import os
import socket
import subprocess
import sys


def main():
    argv = sys.argv[1:]
    world = 2
    if "--world" in argv:
        i = argv.index("--world")
        world = int(argv[i + 1])
        del argv[i:i + 2]
    if argv and argv[0] == "--":
        argv = argv[1:]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NCCL_HOSTID=f"agx-bench-{r}",
                   NCCL_SOCKET_IFNAME=os.environ.get("NCCL_SOCKET_IFNAME", "lo"), NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), *argv],
                                      env=env, cwd=root))
    rc = 0
    for p in procs:
        rc = rc or p.wait(timeout=900)
    sys.exit(rc)


if __name__ == "__main__":
    main()
