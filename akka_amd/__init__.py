"""akka_amd — MI355X-native batched actor dispatch (Akka Dispatcher/Mailbox hot path).

Layers:
  akka_amd.engine     GpuEngine: Python host over the C ABI (include/akka_gpu.h)
  akka_amd.dispatch   the reference's plugin surface: HOCON dispatcher/mailbox
                      configurators, typed Behaviors subset, MailboxSelector
  akka_amd.sharding   ShardRegion.HashCodeMessageExtractor partition function
  akka_amd.workloads  deterministic synthetic workloads (BASELINE configs C1..C5)
The compute path is akka_amd/csrc (hand-written gfx950 HIP); there is no CPU fallback.
"""
__version__ = "0.1.0"
