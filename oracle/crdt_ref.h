/*
 * crdt_ref.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * akka-distributed-data merge semantics on the engine's fixed layouts
 * (include/akka_gpu.h "CRDT behaviours").  Used by the BSP oracle's
 * behaviour table and by the KAT tests against the reference's specs.
 *
 * Node index n in 0..AGX_CRDT_NODES-1 stands for a UniqueAddress in
 * UniqueAddress.compare order (akka-cluster/.../Member.scala:307-311);
 * version 0 = "no entry" (VersionVector Timestamp.Zero, VersionVector.scala:76-80).
 */
#ifndef AKKA_CRDT_REF_H
#define AKKA_CRDT_REF_H
#include <stdint.h>

#include "../include/akka_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* GCounter.merge (DD/GCounter.scala:113-125): slot-wise max over `slots`. */
static inline void crdt_counter_merge(uint64_t* s, const uint64_t* r, uint32_t slots) {
  for (uint32_t i = 0; i < slots; ++i)
    if (r[i] > s[i]) s[i] = r[i];
}

/* ORSet layout (u32 view of the u64 state words, little endian):
 *   dot(e, n) = u32[e * AGX_CRDT_NODES + n]            e < AGX_ORSET_ELEMS
 *   vv(n)     = u32[AGX_ORSET_ELEMS * AGX_CRDT_NODES + n]
 * An element is in the set iff any of its dot entries is non-zero.        */
static inline uint32_t* orset_dots(uint64_t* w) { return (uint32_t*)w; }
static inline uint32_t* orset_vv(uint64_t* w) { return (uint32_t*)w + AGX_ORSET_ELEMS * AGX_CRDT_NODES; }

/* ORSet.subtractDots (DD/ORSet.scala:127-160): keep entries of `dot` not
 * dominated by `vv`. */
static inline void orset_subtract_dots(uint32_t* out, const uint32_t* dot, const uint32_t* vv) {
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) out[n] = (dot[n] && dot[n] > vv[n]) ? dot[n] : 0u;
}

/* One element of ORSet.merge = dryMerge(that, addDeltaOp = false)
 * (DD/ORSet.scala:427-452) in per-node form.  For an element in both sets
 * (mergeCommonKeys, :164-229) an entry equal on both sides is a common dot
 * and kept; otherwise each side keeps what the other's vvector has not seen
 * (subtractDots) and the kept dots merge by max (VersionVector.merge,
 * VersionVector.scala:296-308,355-375).  For an element on one side only
 * (mergeDisjointKeys, :236-259) this reduces to subtractDots against the
 * other side's vvector, and a fully dominated dot drops the element. */
static inline uint32_t orset_merge_entry(uint32_t l, uint32_t r, uint32_t lvv, uint32_t rvv) {
  if (l == r) return l;
  uint32_t lk = l > rvv ? l : 0u;
  uint32_t rk = r > lvv ? r : 0u;
  return lk > rk ? lk : rk;
}

/* this := this.merge(that); both in the engine layout (AGX_ORSET_WORDS u64). */
static inline void orset_merge(uint64_t* self, const uint64_t* that) {
  uint32_t* ld = orset_dots(self);
  uint32_t* lv = orset_vv(self);
  const uint32_t* rd = (const uint32_t*)that;
  const uint32_t* rv = rd + AGX_ORSET_ELEMS * AGX_CRDT_NODES;
  for (uint32_t e = 0; e < AGX_ORSET_ELEMS; ++e)
    for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) {
      uint32_t* x = &ld[e * AGX_CRDT_NODES + n];
      *x = orset_merge_entry(*x, rd[e * AGX_CRDT_NODES + n], lv[n], rv[n]);
    }
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
    if (rv[n] > lv[n]) lv[n] = rv[n];
}

/* ORSet.add (DD/ORSet.scala:339-351): vvector + node; the element's birth dot
 * becomes (node -> new version).  Versions come from a per-replica monotonic
 * counter (the reference draws them from the JVM-wide Timestamp.counter,
 * VersionVector.scala:76-80,277-281; merges only compare them per node). */
static inline void orset_add(uint64_t* w, uint32_t node, uint32_t e) {
  uint32_t* d = orset_dots(w) + e * AGX_CRDT_NODES;
  uint32_t* vv = orset_vv(w);
  vv[node] += 1u;
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) d[n] = 0u;
  d[node] = vv[node];
}

/* ORSet.remove (:380-387): drop the element, vvector unchanged. */
static inline void orset_remove(uint64_t* w, uint32_t e) {
  uint32_t* d = orset_dots(w) + e * AGX_CRDT_NODES;
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) d[n] = 0u;
}

/* ORSet.clear (:404-412): all elements dropped, history kept. */
static inline void orset_clear(uint64_t* w) {
  uint32_t* d = orset_dots(w);
  for (uint32_t i = 0; i < AGX_ORSET_ELEMS * AGX_CRDT_NODES; ++i) d[i] = 0u;
}

/* Gossip peer j of replica `self` at countdown `round`: uniform over the
 * other n-1 actors (Replicator.selectRandomNode, DD/Replicator.scala:2063-2064,
 * with the counter RNG instead of ThreadLocalRandom). */
static inline uint32_t crdt_peer(uint64_t seed, uint32_t self, uint32_t round, uint32_t j, uint64_t n) {
  uint64_t r = ref_fanout_rand(seed, self, round | 0x08000000u, j);
  uint32_t d = (uint32_t)(r % (n - 1));
  return d >= self ? d + 1u : d;
}

#ifdef __cplusplus
}
#endif
#endif
