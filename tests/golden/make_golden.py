#!/usr/bin/env python3
"""Writes the golden fixtures in this directory.

The reference (Scala/JVM) cannot run in this image (no java/sbt),
so the vectors are *data transcribed from the reference's own tests*, each with
the file:line it comes from, plus vectors computed from the published JLS
String.hashCode formula for the shard-id function (no shard-id KAT exists in the
reference: "parity unpinned" by reference tests, pinned by the JLS formula).

Run:  python tests/golden/make_golden.py   (rewrites *.json next to this file)
"""
import json
import pathlib

HERE = pathlib.Path(__file__).resolve().parent


def jls_hash(s: str) -> int:
    h = 0
    for ch in s:
        h = (h * 31 + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def shard(s: str, n: int) -> int:
    h = jls_hash(s)
    a = h if h == -(1 << 31) else abs(h)
    r = abs(a) % n
    return -r if a < 0 else r


def shard_vectors():
    ids = ["0", "1", "9", "10", "42", "999", "1000", "65535", "999999", "1000000", "2147483647", "4294967295",
           "polygenelubricants", "entity-1", "user-42"]
    ids += [str(i) for i in (7, 31, 961, 29791, 123456789, 987654321, 3000000000)]
    out = []
    for s in ids:
        for n in (1000, 100, 8, 7):
            out.append({"entity_id": s, "num_shards": n, "hash": jls_hash(s), "shard": shard(s, n)})
    return {
        "source": "JLS String.hashCode formula; ShardRegion.HashCodeMessageExtractor.shardId = "
                  "(math.abs(id.hashCode) % maxNumberOfShards) "
                  "(akka-cluster-sharding/src/main/scala/akka/cluster/sharding/ShardRegion.scala:154-158). "
                  "SURVEY.md §8(c) examples: '0'->48->'48', '42'->1662->'662', '999999'->1686256992->'992', "
                  "'polygenelubricants'->-2147483648->'-648'.",
        "pinned_by_reference_tests": False,
        "vectors": out,
    }


def gcounter_kats():
    # node1..3 = UniqueAddress(akka://Sys@localhost:2551..2553, uid 1..3) (GCounterSpec.scala:15-17);
    # UniqueAddress order (Member.scala:303-311) -> slots 0,1,2.
    # ops: ["inc", slot, n] applied in order to an empty counter.
    return {
        "source": "akka-distributed-data/src/test/scala/akka/cluster/ddata/GCounterSpec.scala",
        "slots": 3,
        "cases": [
            {"name": "increment each node's record by one (:21-40)",
             "ops": [["inc", 0, 1], ["inc", 0, 1], ["inc", 1, 1], ["inc", 1, 1], ["inc", 1, 1]],
             "state": [2, 3, 0]},
            {"name": "increment by arbitrary delta (:42-56)",
             "ops": [["inc", 0, 3], ["inc", 0, 4], ["inc", 1, 2], ["inc", 1, 7], ["inc", 1, 1]],
             "state": [7, 10, 0], "value": 17},
        ],
        "merges": [
            {"name": "merged with another GCounter 1 (:75-110)",
             "a_ops": [["inc", 0, 3], ["inc", 0, 4], ["inc", 1, 2], ["inc", 1, 7], ["inc", 1, 1]],
             "b_ops": [["inc", 0, 2], ["inc", 0, 2], ["inc", 1, 3], ["inc", 1, 2], ["inc", 1, 1]],
             "a_state": [7, 10, 0], "a_value": 17, "b_state": [4, 6, 0], "b_value": 10,
             "merged_state": [7, 10, 0], "merged_value": 17},
            {"name": "merged with another GCounter 2 (:112-145)",
             "a_ops": [["inc", 0, 2], ["inc", 0, 2], ["inc", 1, 2], ["inc", 1, 7], ["inc", 1, 1]],
             "b_ops": [["inc", 0, 3], ["inc", 0, 4], ["inc", 1, 3], ["inc", 1, 2], ["inc", 1, 1]],
             "a_state": [4, 10, 0], "a_value": 14, "b_state": [7, 6, 0], "b_value": 13,
             "merged_state": [7, 10, 0], "merged_value": 17},
            {"name": "unapply extractor value (:170-174)",
             "a_ops": [["inc", 0, 1], ["inc", 1, 1]], "b_ops": [],
             "a_state": [1, 1, 0], "a_value": 2, "b_state": [0, 0, 0], "b_value": 0,
             "merged_state": [1, 1, 0], "merged_value": 2},
        ],
    }


def mailbox_kats():
    """Queue semantics as engine runs on one receiver (COUNTER behaviour:
    w0 = messages invoked, w1 = sum of payloads)."""
    return {
        "source": "akka-actor-tests/src/test/scala/akka/dispatch/MailboxConfigSpec.scala",
        "cases": [
            {"name": "bounded capacity 10: the 11th enqueue is exactly one DeadLetter (:47-66)",
             "capacity": 10, "throughput": 1000, "payloads": list(range(1, 12)),
             "delivered": 10, "dead_letters": 1, "sum": 55},
            {"name": "BoundedMailbox(10, 0): enqueue 20, dequeue 10, 10 dead letters, FIFO survivors (:84-86,131-183)",
             "capacity": 10, "throughput": 1000, "payloads": list(range(1, 21)),
             "delivered": 10, "dead_letters": 10, "sum": 55},
            {"name": "unbounded single-consumer FIFO, 100 enqueued then drained (:98-116)",
             "capacity": 0, "throughput": 1000, "payloads": list(range(100)),
             "delivered": 100, "dead_letters": 0, "sum": 4950},
            {"name": "throughput 1: one message per Mailbox.run (Mailbox.scala:260-277), 5 rounds",
             "capacity": 0, "throughput": 1, "payloads": [5, 6, 7, 8, 9],
             "delivered": 5, "dead_letters": 0, "sum": 35, "supersteps": 5},
            {"name": "throughput <= 0 behaves as 1 (Mailbox.scala:261, Dispatcher.scala:27-29 comment not code)",
             "capacity": 0, "throughput": 0, "payloads": [1, 2, 3],
             "delivered": 3, "dead_letters": 0, "sum": 6, "supersteps": 3},
        ],
    }


def pingpong_kats():
    """BenchmarkActors.PingPong (akka-bench-jmh/src/main/scala/akka/actor/BenchmarkActors.scala:20-32,96-117):
    each actor starts with left = M/2, replies to every message and stops when left == 0 after
    replying once more, so each actor is invoked M/2 + 1 times; the inFlight = 2*tpt messages of
    a pair all end as dead letters at the stopped actors.  Derived from the reference code, not
    from a committed result."""
    cases = []
    for pairs, m, tpt in ((1, 20, 5), (3, 100, 5), (10, 2000, 50)):
        cases.append({"pairs": pairs, "messages_per_pair": m, "throughput": tpt, "in_flight": 2 * tpt,
                      "delivered": pairs * (m + 2), "dead_letters": pairs * 2 * tpt})
    return {"source": "derived from BenchmarkActors.PingPong", "cases": cases}


def ring_kats():
    """C2 token ring: every actor invoked H+1 times, N*(H+1) deliveries, H+1 supersteps."""
    return {"source": "BASELINE.json configs[1] / SURVEY.md §8(d) C2",
            "cases": [{"n": n, "hops": h, "delivered": n * (h + 1), "supersteps": h + 1, "count": h + 1}
                      for n, h in ((1, 0), (1, 9), (5, 3), (1000, 20), (65536, 4))]}


def main():
    files = {
        "shard_ids.json": shard_vectors(),
        "gcounter_kat.json": gcounter_kats(),
        "mailbox_kat.json": mailbox_kats(),
        "pingpong_kat.json": pingpong_kats(),
        "ring_kat.json": ring_kats(),
    }
    for name, obj in files.items():
        (HERE / name).write_text(json.dumps(obj, indent=1) + "\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
