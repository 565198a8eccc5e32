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


def pncounter_kats():
    # node1, node2 = UniqueAddress(akka://Sys@localhost:2551/2552, uid 1/2) (PNCounterSpec.scala:15-16) -> slots 0, 1.
    # ops: ["inc"|"dec", slot, n]; state = (increments slots, decrements slots).
    a_ops = [["inc", 0, 3], ["dec", 0, 2], ["inc", 1, 5], ["dec", 1, 2], ["inc", 1, 1]]
    b_ops = [["inc", 0, 2], ["dec", 0, 3], ["inc", 1, 3], ["dec", 1, 2], ["inc", 1, 1]]
    return {
        "source": "akka-distributed-data/src/test/scala/akka/cluster/ddata/PNCounterSpec.scala",
        "slots": 2,
        "cases": [
            {"name": "increment each node's record by one (:20-40)",
             "ops": [["inc", 0, 1], ["inc", 0, 1], ["inc", 1, 1], ["inc", 1, 1], ["inc", 1, 1]],
             "increments": [2, 3], "decrements": [0, 0]},
            {"name": "decrement each node's record by one (:42-60)",
             "ops": [["dec", 0, 1], ["dec", 0, 1], ["dec", 1, 1], ["dec", 1, 1], ["dec", 1, 1]],
             "increments": [0, 0], "decrements": [2, 3]},
            {"name": "increment by arbitrary delta (:62-75)",
             "ops": [["inc", 0, 3], ["inc", 0, 4], ["inc", 1, 2], ["inc", 1, 7], ["inc", 1, 1]],
             "increments": [7, 10], "decrements": [0, 0]},
            {"name": "decrement by arbitrary delta (:91-104)",
             "ops": [["dec", 0, 3], ["dec", 0, 4], ["dec", 1, 2], ["dec", 1, 7], ["dec", 1, 1]],
             "increments": [0, 0], "decrements": [7, 10]},
            {"name": "increment and decrement by arbitrary delta (:106-118,119-131)",
             "ops": a_ops, "increments_value": 9, "decrements_value": 4, "value": 5},
        ],
        "merges": [
            {"name": "history correctly merged with another counter (:133-167), both ways",
             "a_ops": a_ops, "b_ops": b_ops,
             "a_value": 5, "b_value": 1, "b_increments_value": 6, "b_decrements_value": 5,
             "merged_increments_value": 9, "merged_decrements_value": 5, "merged_value": 4},
        ],
    }


def orset_kats():
    """ORSetSpec 'ORSet unit test' vectors.  Nodes nodeA..nodeH (ORSetSpec.scala:22-29) -> 0..7,
    node1..node3 (:18-20) -> 0..2 (UniqueAddress order).  Elements are numbered in order of
    first appearance.  Dots/vvectors are {node: version}."""
    A, B, C, D, E, F, G = range(7)
    return {
        "source": "akka-distributed-data/src/test/scala/akka/cluster/ddata/ORSetSpec.scala",
        "subtract_dots": [
            {"name": "verify subtractDots (:489-495)",
             "dot": {A: 3, B: 2, D: 14, G: 22}, "vvector": {A: 4, B: 1, C: 1, D: 14, E: 5, F: 2},
             "expected": {B: 2, G: 22}},
        ],
        "merges": [
            {"name": "verify mergeCommonKeys (:497-511)",
             "this": {"elements": {"K1": {A: 3, D: 7}, "K2": {B: 5, C: 2}}, "vvector": {A: 3, B: 5, C: 2, D: 7}},
             "that": {"elements": {"K1": {A: 3}, "K2": {B: 6}}, "vvector": {A: 3, B: 6, C: 1, D: 8}},
             "expected_elements": {"K1": {A: 3}, "K2": {B: 6, C: 2}}},
            {"name": "verify mergeDisjointKeys (:513-524): keys only in `this`, against that.vvector",
             "this": {"elements": {"K3": {A: 4}, "K4": {A: 3, D: 8}, "K5": {A: 2}}, "vvector": {A: 4, D: 8}},
             "that": {"elements": {}, "vvector": {A: 3, D: 7}},
             "expected_elements": {"K3": {A: 4}, "K4": {D: 8}}},
        ],
        # replica scripts: ["new", r] | ["add", r, node, elem] | ["remove", r, elem] | ["copy", dst, src]
        # | ["merge", dst, x, y] (dst := x.merge(y)); checks: ["elements", r, [elems...]]
        "scripts": [
            {"name": "verify disjoint merge (:526-533)",
             "ops": [["new", "a1"], ["add", "a1", 0, "bar"], ["new", "b1"], ["add", "b1", 1, "baz"],
                     ["merge", "c", "a1", "b1"], ["copy", "a2", "a1"], ["remove", "a2", "bar"],
                     ["merge", "d", "a2", "c"]],
             "checks": [["elements", "d", ["baz"]]]},
            {"name": "verify removed after merge (:535-568)",
             "ops": [["new", "a"], ["add", "a", 0, "Z"], ["copy", "c", "a"], ["copy", "a2", "a"],
                     ["remove", "a2", "Z"], ["new", "b"], ["add", "b", 1, "Z"], ["merge", "a3", "b", "a2"],
                     ["copy", "b2", "b"], ["remove", "b2", "Z"],
                     ["merge", "t1", "a3", "c"], ["merge", "t1", "t1", "b2"],
                     ["merge", "t2", "a3", "b2"], ["merge", "t2", "t2", "c"],
                     ["merge", "t3", "c", "b2"], ["merge", "t3", "t3", "a3"],
                     ["merge", "t4", "c", "a3"], ["merge", "t4", "t4", "b2"],
                     ["merge", "t5", "b2", "c"], ["merge", "t5", "t5", "a3"],
                     ["merge", "t6", "b2", "a3"], ["merge", "t6", "t6", "c"]],
             "checks": [["elements", "a3", ["Z"]], ["elements", "c", ["Z"]], ["elements", "b2", []],
                        ["elements", "t1", []], ["elements", "t2", []], ["elements", "t3", []],
                        ["elements", "t4", []], ["elements", "t5", []], ["elements", "t6", []]]},
            {"name": "verify removed after merge 2 (:570-591)",
             "ops": [["new", "a"], ["add", "a", 0, "Z"], ["new", "b"], ["add", "b", 1, "Z"], ["copy", "c", "a"],
                     ["copy", "a2", "a"], ["remove", "a2", "Z"], ["merge", "a3", "a2", "b"],
                     ["copy", "b2", "b"], ["remove", "b2", "Z"], ["merge", "b3", "b2", "c"],
                     ["merge", "t1", "a3", "c"], ["merge", "t1", "t1", "b3"],
                     ["merge", "t2", "a3", "b3"], ["merge", "t2", "t2", "c"],
                     ["merge", "t3", "c", "b3"], ["merge", "t3", "t3", "a3"],
                     ["merge", "t4", "c", "a3"], ["merge", "t4", "t4", "b3"],
                     ["merge", "t5", "b3", "c"], ["merge", "t5", "t5", "a3"],
                     ["merge", "t6", "b3", "a3"], ["merge", "t6", "t6", "c"]],
             "checks": [["elements", "a3", ["Z"]], ["elements", "b3", ["Z"]],
                        ["elements", "t1", []], ["elements", "t2", []], ["elements", "t3", []],
                        ["elements", "t4", []], ["elements", "t5", []], ["elements", "t6", []]]},
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
        "pncounter_kat.json": pncounter_kats(),
        "orset_kat.json": orset_kats(),
        "mailbox_kat.json": mailbox_kats(),
        "pingpong_kat.json": pingpong_kats(),
        "ring_kat.json": ring_kats(),
    }
    for name, obj in files.items():
        (HERE / name).write_text(json.dumps(obj, indent=1) + "\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
