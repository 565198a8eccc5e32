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


def versionvector_kats():
    """VersionVectorSpec programs (node1..node4 -> 0..3).  `inc` draws the new version from one
    global counter, as VersionVector.increment does from Timestamp.counter (VersionVector.scala:277-281).
    ops: ["new", v] | ["copy", v, x] | ["inc", v, x, node] (v = x + node) | ["merge", v, x, y];
    checks: ["size", v, n] | ["contains", v, node, bool] | ["cmp", x, y, "<"|">"|"<>"|"==", bool]
    | ["gt_at", x, y, node] (x.versionAt(node) > y.versionAt(node)) | ["eq_at", x, y, node]."""
    chain1 = [["new", "a1"], ["inc", "a2", "a1", 0], ["inc", "a3", "a2", 1], ["inc", "a4", "a3", 0]]
    chain2 = [["new", "b1"], ["inc", "b2", "b1", 0], ["inc", "b3", "b2", 1], ["inc", "b4", "b3", 0]]
    five = [["new", "a1"], ["inc", "a2", "a1", 0], ["inc", "a3", "a2", 1], ["inc", "a4", "a3", 1],
            ["inc", "a5", "a4", 2]]
    merged = lambda n: [["size", "m1", n], ["size", "m2", n]] + [["contains", m, k, True] for m in ("m1", "m2")
                                                                  for k in range(n)] + \
        [["cmp", "b3", "m1", "<", True], ["cmp", "a5", "m1", "<", True], ["cmp", "b3", "m2", "<", True],
         ["cmp", "a5", "m2", "<", True], ["cmp", "m1", "m2", "==", True]]
    return {
        "source": "akka-distributed-data/src/test/scala/akka/cluster/ddata/VersionVectorSpec.scala",
        "cases": [
            {"name": "have zero versions when created (:32-35)", "ops": [["new", "v"]], "checks": [["size", "v", 0]]},
            {"name": "not happen before itself (:37-42)", "ops": [["new", "v1"], ["new", "v2"]],
             "checks": [["cmp", "v1", "v2", "<>", False]]},
            {"name": "increment correctly (:44-54)",
             "ops": [["new", "v1"], ["inc", "v2", "v1", 0], ["inc", "v3", "v2", 0], ["inc", "v4", "v3", 1]],
             "checks": [["gt_at", "v2", "v1", 0], ["gt_at", "v3", "v2", 0], ["eq_at", "v4", "v3", 0],
                        ["gt_at", "v4", "v3", 1]]},
            {"name": "misc comparison test 1 (:56-68)", "ops": chain1 + chain2,
             "checks": [["cmp", "a4", "b4", "<>", False]]},
            {"name": "misc comparison test 2 (:70-83)", "ops": chain1 + chain2 + [["inc", "b5", "b4", 2]],
             "checks": [["cmp", "a4", "b5", "<", True]]},
            {"name": "misc comparison test 3 (:85-93)",
             "ops": [["new", "a1"], ["inc", "a2", "a1", 0], ["new", "b1"], ["inc", "b2", "b1", 1]],
             "checks": [["cmp", "a2", "b2", "<>", True]]},
            {"name": "misc comparison test 4 (:95-107)",
             "ops": [["new", "a1"], ["inc", "a2", "a1", 0], ["inc", "a3", "a2", 1], ["inc", "a4", "a3", 0],
                     ["new", "b1"], ["inc", "b2", "b1", 0], ["inc", "b3", "b2", 0], ["inc", "b4", "b3", 2]],
             "checks": [["cmp", "a4", "b4", "<>", True]]},
            {"name": "misc comparison test 5 (:109-122)",
             "ops": [["new", "a1"], ["inc", "a2", "a1", 1], ["inc", "a3", "a2", 1], ["new", "b1"],
                     ["inc", "b2", "b1", 0], ["inc", "b3", "b2", 1], ["inc", "b4", "b3", 1], ["inc", "b5", "b4", 2]],
             "checks": [["cmp", "a3", "b5", "<", True], ["cmp", "b5", "a3", ">", True]]},
            {"name": "misc comparison test 6 (:124-135)",
             "ops": [["new", "a1"], ["inc", "a2", "a1", 0], ["inc", "a3", "a2", 1], ["new", "b1"],
                     ["inc", "b2", "b1", 0], ["inc", "b3", "b2", 0]],
             "checks": [["cmp", "a3", "b3", "<>", True], ["cmp", "b3", "a3", "<>", True]]},
            {"name": "misc comparison test 7 (:137-150)",
             "ops": five + [["copy", "b1", "a4"], ["inc", "b2", "b1", 1], ["inc", "b3", "b2", 1]],
             "checks": [["cmp", "a5", "b3", "<>", True], ["cmp", "b3", "a5", "<>", True]]},
            {"name": "misc comparison test 8 (:152-164)",
             "ops": [["new", "a1"], ["inc", "a2", "a1", 0], ["inc", "a3", "a2", 2], ["inc", "b1", "a3", 1],
                     ["inc", "a4", "a3", 2]],
             "checks": [["cmp", "a4", "b1", "<>", True], ["cmp", "b1", "a4", "<>", True]]},
            {"name": "correctly merge two version vectors (:166-197)",
             "ops": five + [["copy", "b1", "a4"], ["inc", "b2", "b1", 1], ["inc", "b3", "b2", 1],
                            ["merge", "m1", "b3", "a5"], ["merge", "m2", "a5", "b3"]],
             "checks": merged(3)},
            {"name": "correctly merge two disjoint version vectors (:199-232)",
             "ops": five + [["new", "b1"], ["inc", "b2", "b1", 3], ["inc", "b3", "b2", 3],
                            ["merge", "m1", "b3", "a5"], ["merge", "m2", "a5", "b3"]],
             "checks": merged(4)},
            {"name": "pass blank version vector incrementing (:234-249)",
             "ops": [["new", "v1"], ["new", "v2"], ["inc", "vv1", "v1", 0], ["inc", "vv2", "v2", 1]],
             "checks": [["cmp", "vv1", "v1", ">", True], ["cmp", "vv2", "v2", ">", True],
                        ["cmp", "vv1", "v2", ">", True], ["cmp", "vv2", "v1", ">", True],
                        ["cmp", "vv2", "vv1", ">", False], ["cmp", "vv1", "vv2", ">", False]]},
            {"name": "pass merging behavior (:251-264)",
             "ops": [["new", "a"], ["new", "b"], ["inc", "a1", "a", 0], ["inc", "b1", "b", 1], ["inc", "a2", "a1", 0],
                     ["merge", "c", "a2", "b1"], ["inc", "c1", "c", 2]],
             "checks": [["cmp", "c1", "a2", ">", True], ["cmp", "c1", "b1", ">", True]]},
        ],
    }


def orset_delta_kats():
    """ORSetSpec "ORSet deltas" programs (:230-487) and "not pollute the vvector of result during
    mergeRemoveDelta" (:588-600).  node1..node3 -> 0..2, nodeA/nodeB -> 0/1; elements numbered by
    first appearance; versions from one global counter (Timestamp.counter).
    ops: ["empty", x] | ["add", x, y, node, e] (x = y.add(node, e)) | ["remove", x, y, node, e]
    | ["clear", x, y] | ["reset", x, y] (resetDelta) | ["merge", x, y, z] | ["merge_delta", x, y, d]
    | ["delta", d, x] (x.delta.get) | ["dmerge", d, d1, d2] (d1.merge(d2));
    checks: ["elements", x, [..]] | ["absent", x, e] | ["equal", x, y] | ["vv_has", x, node, bool]
    | ["add_op", d, [..]] (asAddDeltaOp(d).underlying.elements) | ["group", d, size, last_type]
    | ["last_add", d, [..]] (the last op of a DeltaGroup is an AddDeltaOp with these elements)."""
    return {
        "source": "akka-distributed-data/src/test/scala/akka/cluster/ddata/ORSetSpec.scala",
        "cases": [
            {"name": "work for additions (:242-271)",
             "ops": [["empty", "s1"], ["add", "s2", "s1", 0, "a"], ["delta", "d2", "s2"],
                     ["merge_delta", "t1", "s1", "d2"],
                     ["reset", "r2", "s2"], ["add", "s3a", "r2", 0, "b"], ["add", "s3", "s3a", 0, "c"],
                     ["delta", "d3", "s3"], ["merge_delta", "t2", "s2", "d3"],
                     ["reset", "r3", "s3"], ["add", "s4", "r3", 1, "d"], ["delta", "d4", "s4"],
                     ["merge_delta", "t3", "s3", "d4"],
                     ["add", "s5", "r3", 0, "e"], ["merge", "s6", "s5", "s4"], ["merge_delta", "t4", "s5", "d4"],
                     ["add", "s7", "r3", 0, "d"], ["merge", "s8", "s7", "s4"], ["merge_delta", "t5", "s7", "d4"],
                     ["delta", "d7", "s7"], ["merge_delta", "t6", "s4", "d7"]],
             "checks": [["add_op", "d2", ["a"]], ["equal", "t1", "s2"], ["add_op", "d3", ["b", "c"]],
                        ["equal", "t2", "s3"], ["add_op", "d4", ["d"]], ["equal", "t3", "s4"], ["equal", "t4", "s6"],
                        ["equal", "t5", "s8"], ["equal", "t6", "s8"]]},
            {"name": "handle another concurrent add scenario (:273-285)",
             "ops": [["empty", "s1"], ["add", "s2", "s1", 0, "a"], ["add", "s3", "s2", 0, "b"],
                     ["add", "s4", "s2", 1, "c"], ["merge", "s5", "s4", "s3"], ["delta", "d3", "s3"],
                     ["merge_delta", "s6", "s4", "d3"]],
             "checks": [["elements", "s5", ["a", "b", "c"]], ["elements", "s6", ["a", "b", "c"]]]},
            {"name": "merge deltas into delta groups (:287-313)",
             "ops": [["empty", "s1"], ["add", "s2", "s1", 0, "a"], ["delta", "d2", "s2"], ["reset", "r2", "s2"],
                     ["add", "s3", "r2", 0, "b"], ["delta", "d3", "s3"], ["dmerge", "d4", "d2", "d3"],
                     ["merge_delta", "t1", "s1", "d4"], ["merge_delta", "t2", "s2", "d4"],
                     ["reset", "r3", "s3"], ["remove", "s5", "r3", 0, "b"], ["delta", "d5", "s5"],
                     ["dmerge", "d6", "d4", "d5"], ["merge_delta", "t3", "s3", "d6"],
                     ["reset", "r5", "s5"], ["add", "s7", "r5", 0, "c"], ["reset", "r7", "s7"],
                     ["add", "s8", "r7", 0, "d"], ["delta", "d7", "s7"], ["delta", "d8", "s8"],
                     ["dmerge", "d9a", "d6", "d7"], ["dmerge", "d9", "d9a", "d8"],
                     ["merge_delta", "t4", "s5", "d9"], ["merge_delta", "t5a", "s5", "d7"],
                     ["merge_delta", "t5", "t5a", "d8"]],
             "checks": [["add_op", "d4", ["a", "b"]], ["equal", "t1", "s3"], ["equal", "t2", "s3"],
                        ["group", "d6", 2, "remove"], ["equal", "t3", "s5"], ["last_add", "d9", ["c", "d"]],
                        ["group", "d9", 3, "add"], ["equal", "t4", "s8"], ["equal", "t5", "s8"]]},
            {"name": "work for removals (:315-334)",
             "ops": [["empty", "s1"], ["add", "x1", "s1", 0, "a"], ["add", "x2", "x1", 0, "b"], ["reset", "s2", "x2"],
                     ["remove", "s3", "s2", 0, "b"], ["merge", "t1", "s2", "s3"], ["delta", "d3", "s3"],
                     ["merge_delta", "t2", "s2", "d3"],
                     ["add", "x4", "s2", 1, "c"], ["reset", "s4", "x4"], ["merge", "s5", "s4", "s3"],
                     ["merge_delta", "t3", "s4", "d3"],
                     ["add", "s6", "s5", 1, "b"], ["merge_delta", "t4", "s6", "d3"]],
             "checks": [["equal", "t1", "s3"], ["equal", "t2", "s3"], ["elements", "t2", ["a"]],
                        ["elements", "s5", ["a", "c"]], ["equal", "t3", "s5"], ["equal", "t4", "s6"],
                        ["elements", "t4", ["a", "b", "c"]]]},
            {"name": "work for clear (:336-358)",
             "ops": [["empty", "s1"], ["add", "x1", "s1", 0, "a"], ["add", "s2", "x1", 0, "b"], ["reset", "r2", "s2"],
                     ["clear", "s3", "r2"], ["reset", "r3", "s3"], ["add", "s4", "r3", 0, "c"],
                     ["merge", "t1", "s2", "s3"], ["delta", "d3", "s3"], ["merge_delta", "t2", "s2", "d3"],
                     ["delta", "d4", "s4"], ["merge_delta", "t3", "s2", "d3"], ["merge_delta", "s5", "t3", "d4"],
                     ["add", "s6", "r2", 1, "d"], ["merge", "s7", "s6", "s3"], ["merge_delta", "t4", "s6", "d3"],
                     ["add", "s8", "s7", 1, "b"], ["merge_delta", "t5", "s8", "d3"]],
             "checks": [["equal", "t1", "s3"], ["equal", "t2", "s3"], ["elements", "s5", ["c"]], ["equal", "s5", "s4"],
                        ["elements", "s7", ["d"]], ["equal", "t4", "s7"], ["equal", "t5", "s8"],
                        ["elements", "t5", ["b", "d"]]]},
            {"name": "handle a mixed add/remove scenario (:360-377)",
             "ops": [["empty", "s1"], ["reset", "r1", "s1"], ["remove", "s2", "r1", 0, "e"], ["reset", "r2", "s2"],
                     ["add", "s3", "r2", 0, "b"], ["reset", "r3", "s3"], ["add", "s4", "r3", 0, "a"],
                     ["reset", "r4", "s4"], ["remove", "s5", "r4", 0, "b"], ["delta", "d3", "s3"],
                     ["delta", "d4", "s4"], ["delta", "d5", "s5"], ["dmerge", "g1a", "d3", "d4"],
                     ["dmerge", "g1", "g1a", "d5"], ["merge_delta", "s7", "s2", "g1"],
                     ["add", "s8", "r2", 1, "z"], ["merge_delta", "s9", "s8", "g1"]],
             "checks": [["elements", "s7", ["a"]], ["elements", "s9", ["a", "z"]]]},
            {"name": "handle a mixed add/remove scenario 2 (:379-399)",
             "ops": [["empty", "s1"], ["reset", "r1", "s1"], ["add", "s2", "r1", 0, "a"], ["reset", "r2", "s2"],
                     ["add", "s3", "r2", 0, "b"], ["reset", "r3", "s3"], ["add", "s4", "r3", 1, "a"],
                     ["reset", "r4", "s4"], ["remove", "s5", "r4", 0, "a"], ["delta", "d2", "s2"],
                     ["delta", "d3", "s3"], ["dmerge", "delta1", "d2", "d3"], ["delta", "delta2", "s4"],
                     ["empty", "t1"], ["merge_delta", "t2a", "t1", "delta1"], ["merge_delta", "t2", "t2a", "delta2"],
                     ["reset", "rt2", "t2"], ["add", "t3", "rt2", 2, "z"], ["delta", "d5", "s5"],
                     ["merge_delta", "t4", "t3", "d5"]],
             "checks": [["elements", "s5", ["b"]], ["elements", "t2", ["a", "b"]], ["elements", "t4", ["b", "z"]]]},
            {"name": "handle a mixed add/remove scenario 3 (:401-421)",
             "ops": [["empty", "s1"], ["reset", "r1", "s1"], ["add", "s2", "r1", 0, "a"], ["reset", "r2", "s2"],
                     ["add", "s3", "r2", 0, "b"], ["reset", "r3", "s3"], ["add", "s4", "r3", 1, "a"],
                     ["reset", "r4", "s4"], ["remove", "s5", "r4", 0, "a"], ["delta", "d2", "s2"],
                     ["delta", "d3", "s3"], ["dmerge", "delta1", "d2", "d3"], ["empty", "t1"],
                     ["merge_delta", "t2", "t1", "delta1"], ["reset", "rt2", "t2"], ["add", "t3", "rt2", 2, "a"],
                     ["delta", "d5", "s5"], ["merge_delta", "t4", "t3", "d5"]],
             "checks": [["elements", "s5", ["b"]], ["elements", "t2", ["a", "b"]], ["elements", "t4", ["b", "a"]]]},
            {"name": "not have anomalies for ORSet in complex but realistic scenario (:423-455)",
             "ops": [["empty", "e0"], ["add", "x1", "e0", 0, "q"], ["remove", "n11", "x1", 0, "q"], ["delta", "dl11", "n11"],
                     ["reset", "r11", "n11"], ["add", "x2", "r11", 0, "z"], ["remove", "n12", "x2", 0, "z"],
                     ["delta", "dl12", "n12"], ["merge_delta", "x3", "e0", "dl11"], ["reset", "x3r", "x3"],
                     ["add", "n21", "x3r", 1, "x"], ["delta", "dl21", "n21"], ["reset", "r21", "n21"],
                     ["add", "x4", "r21", 1, "a"], ["remove", "n22", "x4", 1, "a"], ["delta", "dl22", "n22"],
                     ["merge_delta", "y1", "e0", "dl11"], ["merge_delta", "y2", "y1", "dl21"],
                     ["merge_delta", "n31", "y2", "dl12"], ["merge", "m1", "n31", "n22"],
                     ["merge_delta", "m2", "n31", "dl22"]],
             "checks": [["absent", "m1", "a"], ["elements", "m2", ["x"]]]},
            {"name": "require causal delivery of deltas (:457-486)",
             "ops": [["empty", "e"], ["add", "s0", "e", 0, "a"], ["reset", "r0", "s0"], ["add", "s11", "r0", 0, "b"],
                     ["reset", "r11", "s11"], ["add", "s12", "r11", 0, "c"], ["add", "s21", "r0", 1, "d"],
                     ["delta", "d21", "s21"], ["delta", "d12", "s12"], ["delta", "d11", "s11"],
                     ["merge_delta", "x1", "s0", "d21"], ["merge_delta", "s31", "x1", "d12"],
                     ["merge_delta", "y1", "s0", "d11"], ["merge_delta", "y2", "y1", "d12"],
                     ["merge_delta", "s41", "y2", "d21"], ["merge", "s32", "s31", "s41"]],
             "checks": [["elements", "s31", ["a", "c", "d"]], ["elements", "s41", ["a", "b", "c", "d"]],
                        ["elements", "s32", ["a", "c", "d"]]]},
            {"name": "not pollute the vvector of result during mergeRemoveDelta (:588-600)",
             "ops": [["empty", "e"], ["add", "a", "e", 0, "a"], ["add", "x1", "a", 1, "b"], ["remove", "x2", "x1", 1, "b"],
                     ["reset", "x3", "x2"], ["remove", "a1", "x3", 0, "a"], ["delta", "da", "a"],
                     ["delta", "da1", "a1"], ["merge_delta", "y1", "e", "da"], ["merge_delta", "a2", "y1", "da1"]],
             "checks": [["vv_has", "a", 0, True], ["vv_has", "a", 1, False], ["vv_has", "a1", 0, True],
                        ["vv_has", "a1", 1, True], ["elements", "a2", []], ["vv_has", "a2", 1, False]]},
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
        "orset_delta_kat.json": orset_delta_kats(),
        "versionvector_kat.json": versionvector_kats(),
        "mailbox_kat.json": mailbox_kats(),
        "pingpong_kat.json": pingpong_kats(),
        "ring_kat.json": ring_kats(),
    }
    for name, obj in files.items():
        (HERE / name).write_text(json.dumps(obj, indent=1) + "\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
