"""ClusterSharding's partition function, mirrored on the host.

ShardRegion.HashCodeMessageExtractor.shardId
(akka-cluster-sharding/src/main/scala/akka/cluster/sharding/ShardRegion.scala:154-158):

    (math.abs(id.hashCode) % maxNumberOfShards).toString

with JLS String.hashCode (s[0]*31^(n-1) + ... + s[n-1], Int overflow).
math.abs(Int.MinValue) == Int.MinValue, so a shard id can be negative.
The GPU engine places shard s on rank floor-mod(s, n_ranks), which replaces
the dynamic LeastShardAllocationStrategy (SH/ShardCoordinator.scala:201-213).
"""
from __future__ import annotations

import numpy as np

INT_MIN = -(1 << 31)


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode over UTF-16 code units."""
    h = 0
    data = s.encode("utf-16-be")
    for i in range(0, len(data), 2):
        h = (h * 31 + ((data[i] << 8) | data[i + 1])) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def java_abs(x: int) -> int:
    return x if x == INT_MIN else abs(x)


def java_rem(a: int, b: int) -> int:
    """Java '%' (truncates toward zero)."""
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def shard_id(entity_id: str, max_number_of_shards: int = 1000) -> str:
    """HashCodeMessageExtractor.shardId (ShardRegion.scala:154-158)."""
    return str(java_rem(java_abs(java_string_hash(entity_id)), max_number_of_shards))


def shard_of_actor(actor_id: int, num_shards: int = 1000) -> int:
    """Shard of a GPU actor; its entityId is the decimal string of its index."""
    return int(shard_id(str(actor_id), num_shards))


def rank_of_shard(shard: int, n_ranks: int) -> int:
    return shard % n_ranks  # Python '%' is floor-mod: negative shards wrap into [0, n_ranks)


def owners(n_actors: int, num_shards: int, n_ranks: int) -> np.ndarray:
    """Vectorised owner rank of actors 0..n-1 (decimal-string Java hash)."""
    ids = np.arange(n_actors, dtype=np.int64)
    digits = np.where(ids == 0, 1, np.floor(np.log10(np.maximum(ids, 1))).astype(np.int64) + 1)
    h = np.zeros(n_actors, dtype=np.uint64)
    maxd = int(digits.max()) if n_actors else 1
    for pos in range(maxd):  # most significant digit first
        exp = digits - 1 - pos
        valid = exp >= 0
        d = (ids // (10 ** np.maximum(exp, 0))) % 10
        h = np.where(valid, (h * np.uint64(31) + (d + 48).astype(np.uint64)) & np.uint64(0xFFFFFFFF), h)
    hs = h.astype(np.int64)
    hs = np.where(hs >= (1 << 31), hs - (1 << 32), hs)
    a = np.where(hs == INT_MIN, hs, np.abs(hs))
    shard = np.sign(a) * (np.abs(a) % num_shards)
    return np.mod(shard, n_ranks).astype(np.int64)


class HashCodeMessageExtractor:
    """Typed HashCodeMessageExtractor (akka-cluster-sharding-typed/.../ShardingMessageExtractor.scala:73-79)."""

    def __init__(self, number_of_shards: int = 1000):
        self.number_of_shards = number_of_shards

    def entity_id(self, envelope) -> str:
        return envelope[0]

    def shard_id(self, entity_id: str) -> str:
        return shard_id(entity_id, self.number_of_shards)

    def unwrap_message(self, envelope):
        return envelope[1]
