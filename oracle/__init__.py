"""TEST INFRASTRUCTURE ONLY — CPU oracles for parity checks and the CPU baseline.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product path (akka_amd/) never does.

  BspOracle  deterministic BSP restatement of Dispatcher/Mailbox (parity oracle)
  FjpOracle  multi-threaded Dispatcher/Mailbox/ForkJoinPool restatement (CPU baseline)
"""
from .oracle import BspOracle, FjpOracle, build, crdt, java_hash, shard_id  # noqa: F401
