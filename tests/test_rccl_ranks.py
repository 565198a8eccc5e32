"""The real multi-process RCCL path on one GPU: N ranks (processes) with one engine each,
agx_comm_init + run_multi_rccl (ncclAllGather of the count vectors, grouped
ncclSend/ncclRecv of envelopes and CRDT rows), bit-exact against the BSP oracle in the
sharded canonical order.  Every behaviour runs the device-resident replays (fixed per-peer
slabs, k_mr_pack / k_mr_unpack, no host round trip per superstep; CRDT state rows travel in row
slabs beside the envelope slabs); `env` forces the
host-planned exchange (AGX_MR_HOST) or tiny slabs (AGX_MR_SLAB: the first superstep's counts
overflow them -> the host redoes that exchange exactly, grows the slabs and the replays resume).  tools/rccl_two_rank.py gives every rank its own NCCL_HOSTID so
RCCL accepts several ranks on one device (socket transport on loopback)."""
import os
import pathlib
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("workload,world,n,hops,env", [
    ("ring", 2, 20_000, 8, {}),
    ("ring", 2, 20_000, 8, {"AGX_MR_SLAB": "64"}),      # slab overflow -> exact exchange, bigger slabs
    ("ring", 3, 20_000, 30, {"AGX_MR_SLAB": "6000"}),   # 3+ replays of 8 supersteps, budget not a multiple
    ("mixed", 3, 20_000, 8, {"AGX_MR_HOST": "1"}),      # the host-planned exchange
    ("power", 4, 60_000, 8, {"AGX_MR_SLAB": "64"}),
    ("zipf", 2, 30_000, 3, {"AGX_MR_SLAB": "2000"}),   # fan-out grows 4x: the slab overflows mid-replay
    ("ring", 2, 20_000, 12, {"RESTAGE": "5"}),         # a staged burst between device-resident replays
    # replays captured as graphs (the default), agreed by every rank, re-captured after the slabs grow,
    # and the engines destroyed after (graph before communicator) -- / the eager replay
    ("ring", 2, 20_000, 24, {"AGX_MR_DEBUG": "1", "EXPECT": r"(?s)2 of 2 ranks captured.*graph replay 1: launch"
                             r".*destroy: communicator destroyed"}),
    ("ring", 2, 20_000, 24, {"AGX_MR_GRAPH": "0", "AGX_MR_DEBUG": "1", "EXPECT": r"eager replay of 8 supersteps"}),
    ("mixed", 3, 20_000, 8, {}),
    ("orset", 2, 6_000, 6, {}),  # CRDT rows in row slabs beside the envelope slabs
    ("orset", 2, 6_000, 6, {"AGX_MR_SLAB": "64"}),     # row slabs overflow -> exact exchange, regrown
    ("orset", 3, 6_000, 6, {"AGX_MR_HOST": "1"}),      # CRDT rows over the host-planned exchange
    # row slabs over the row budget (AGX_MR_ROW_MB): every rank agrees to the host-planned exchange,
    # from the first superstep / after the slabs outgrow the budget mid-run
    ("orset", 2, 6_000, 6, {"AGX_MR_ROW_MB": "0", "EXPECT": r"dev_steps=0 host_steps=\d+ rows_on_host=True"}),
    ("orset", 3, 6_000, 6, {"AGX_MR_SLAB": "64", "AGX_MR_ROW_MB": "1", "EXPECT": r"host_steps=[1-9]\d* rows_on_host=True"}),
    ("orset_delta", 2, 4_096, 4, {}),
    ("crdt_mixed", 3, 5_000, 5, {}),
    ("power", 4, 60_000, 8, {}),
    ("zipf", 2, 30_000, 3, {}),
    ("zipf", 4, 40_000, 3, {}),     # C3 sharded over 4 ranks
    ("orset", 4, 4_000, 5, {}),     # C4 ORSet rows over 4 ranks
    # (world <= 4 on ONE device: a round-3 run of 8 ranks on the 1-GPU box stalled after communicator
    # setup and was killed at its time limit; its log was scratch output and was not kept -- see
    # DESIGN.md §7.  The 8-rank exchange is covered by agx_group_run's loopback of the same kernels,
    # test_gpu_benched.py::test_sharded_8_ranks)
])
def test_rccl_ranks_parity(built, workload, world, n, hops, env):
    env = dict(env)
    expect = env.pop("EXPECT", None)
    cmd = [sys.executable, "-u", str(ROOT / "tools" / "rccl_two_rank.py"), "--split-hosts", "--world", str(world),
           "--n", str(n), "--hops", str(hops), "--workload", workload, "--restage", env.pop("RESTAGE", "0")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280, env=dict(os.environ, **env))
    tail = (r.stdout[-1500:] + "\n" + r.stderr[-1500:])
    assert r.returncode == 0, tail
    assert "parity: OK" in r.stdout, tail
    if expect:
        assert re.search(expect, r.stderr + r.stdout), tail
