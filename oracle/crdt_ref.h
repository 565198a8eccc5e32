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
#include <string.h>

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

/* Delta-CRDT mode: the replicas of one key are the ids [g, g + m) with g = self & ~7 and
 * m = min(8, n - g); node = self - g.  Full-state gossip picks one of the other m - 1. */
static inline uint32_t crdt_key_size(uint32_t self, uint64_t n) {
  uint64_t g = self & ~(uint64_t)(AGX_CRDT_NODES - 1u), m = n - g;
  return m < AGX_CRDT_NODES ? (uint32_t)m : AGX_CRDT_NODES;
}
static inline uint32_t crdt_key_peer(uint64_t seed, uint32_t self, uint32_t round, uint32_t j, uint64_t n) {
  const uint32_t m = crdt_key_size(self, n), node = self % AGX_CRDT_NODES;
  uint64_t r = ref_fanout_rand(seed, self, round | 0x08000000u, j);
  uint32_t d = (uint32_t)(r % (m - 1u));
  return self - node + (d >= node ? d + 1u : d);
}

/* ------------------------------------------------------------------------
 * ORSet deltas (DD/ORSet.scala:43-120 the DeltaOp types, :339-412 add/remove/clear
 * producing them, :455-501 mergeDelta / mergeRemoveDelta).  A delta is None
 * (nops == 0), one AtomicDeltaOp (group == 0, nops == 1) or a DeltaGroup. */
#define ORSET_DOP_ADD 1u    /* AddDeltaOp       */
#define ORSET_DOP_REMOVE 2u /* RemoveDeltaOp    */
#define ORSET_DOP_FULL 3u   /* FullStateDeltaOp */
#define ORSET_DELTA_MAX_OPS 64u

typedef struct {
  uint32_t type;
  uint32_t n;                                      /* entries of the underlying elementsMap */
  uint32_t elem[AGX_ORSET_ELEMS];
  uint32_t dot[AGX_ORSET_ELEMS][AGX_CRDT_NODES];   /* elem[i] -> dot[i] (0 = no entry)       */
  uint32_t vv[AGX_CRDT_NODES];                     /* the underlying ORSet's vvector          */
} orset_dop;

typedef struct {
  uint32_t group; /* DeltaGroup (else ops[0] is one AtomicDeltaOp) */
  uint32_t nops;  /* 0 = no delta                                  */
  orset_dop ops[ORSET_DELTA_MAX_OPS];
} orset_delta;

/* ReplicatedDeltaSize.deltaSize: 1 for an AtomicDeltaOp, ops.size for a DeltaGroup (:47-53,113) */
static inline uint32_t orset_delta_size(const orset_delta* d) { return d->group ? d->nops : 1u; }

static inline void orset_dop_single(orset_dop* op, uint32_t type, uint32_t e, const uint32_t* dot, const uint32_t* vv) {
  memset(op, 0, sizeof *op);
  op->type = type;
  if (type != ORSET_DOP_FULL) {
    op->n = 1;
    op->elem[0] = e;
    memcpy(op->dot[0], dot, sizeof op->dot[0]);
  }
  memcpy(op->vv, vv, sizeof op->vv);
}

/* AddDeltaOp.merge(AddDeltaOp): concatElementsMap (that's entries win) and vvector merge (:58-74) */
static inline void orset_add_op_concat(orset_dop* a, const orset_dop* b) {
  for (uint32_t i = 0; i < b->n; ++i) {
    uint32_t k = 0;
    while (k < a->n && a->elem[k] != b->elem[i]) ++k;
    if (k == a->n) a->elem[a->n++] = b->elem[i];
    memcpy(a->dot[k], b->dot[i], sizeof a->dot[k]);
  }
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
    if (b->vv[n] > a->vv[n]) a->vv[n] = b->vv[n];
}

static inline int orset_delta_push(orset_delta* d, const orset_dop* op) {
  if (d->nops >= ORSET_DELTA_MAX_OPS) return -1;
  d->ops[d->nops++] = *op;
  return 0;
}

/* d1 := d1.merge(d2) (DeltaOp.merge: AddDeltaOp :58-68, RemoveDeltaOp :84-87, FullStateDeltaOp
 * :93-96, DeltaGroup :106-117); d1 = None takes d2 (`delta match { case None => op }`). */
static inline int orset_delta_merge(orset_delta* d1, const orset_delta* d2) {
  if (d2->nops == 0) return 0;
  if (d1->nops == 0) {
    *d1 = *d2;
    return 0;
  }
  if (!d1->group) {
    if (!d2->group && d1->ops[0].type == ORSET_DOP_ADD && d2->ops[0].type == ORSET_DOP_ADD) {
      orset_add_op_concat(&d1->ops[0], &d2->ops[0]); /* AddDeltaOp(AddDeltaOp) */
      return 0;
    }
    d1->group = 1; /* DeltaGroup(Vector(this, that)) / DeltaGroup(this +: ops) */
    for (uint32_t i = 0; i < d2->nops; ++i)
      if (orset_delta_push(d1, &d2->ops[i])) return -1;
    return 0;
  }
  if (!d2->group && d2->ops[0].type == ORSET_DOP_ADD && d1->ops[d1->nops - 1].type == ORSET_DOP_ADD) {
    orset_add_op_concat(&d1->ops[d1->nops - 1], &d2->ops[0]); /* merged into the last AddDeltaOp */
    return 0;
  }
  for (uint32_t i = 0; i < d2->nops; ++i) /* ops :+ that / ops ++ thatOps */
    if (orset_delta_push(d1, &d2->ops[i])) return -1;
  return 0;
}

static inline int orset_has(const uint32_t* d) {
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
    if (d[n]) return 1;
  return 0;
}

/* dryMerge(that, addDeltaOp) (:427-452) of `self` with an op's underlying ORSet:
 * mergeCommonKeys for elements on both sides, mergeDisjointKeys for that's unique keys
 * against this.vvector, and this's unique keys either kept (addDeltaOp) or
 * mergeDisjointKeys'd against that.vvector; vvectors merge. */
static inline void orset_dry_merge(uint64_t* self, const orset_dop* that, int add_delta_op) {
  uint32_t* ld = orset_dots(self);
  uint32_t* lv = orset_vv(self);
  uint32_t in_that[AGX_ORSET_ELEMS];
  memset(in_that, 0xFF, sizeof in_that);
  for (uint32_t i = 0; i < that->n; ++i) in_that[that->elem[i]] = i;
  for (uint32_t e = 0; e < AGX_ORSET_ELEMS; ++e) {
    uint32_t* x = &ld[e * AGX_CRDT_NODES];
    const int here = orset_has(x);
    if (in_that[e] != 0xFFFFFFFFu) {
      const uint32_t* r = that->dot[in_that[e]];
      if (here) {
        for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) x[n] = orset_merge_entry(x[n], r[n], lv[n], that->vv[n]);
      } else {
        for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) x[n] = r[n] > lv[n] ? r[n] : 0u;
      }
    } else if (here && !add_delta_op) {
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) x[n] = x[n] > that->vv[n] ? x[n] : 0u;
    }
  }
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
    if (that->vv[n] > lv[n]) lv[n] = that->vv[n];
}

/* mergeRemoveDelta (:471-501): the element goes if its dot is <= the remover's vvector on every
 * node the remover knows and has no node the remover does not know; the vvector only merges the
 * remover's own dot (ORSetSpec "not pollute the vvector of result during mergeRemoveDelta"). */
static inline void orset_merge_remove_delta(uint64_t* self, const orset_dop* rm) {
  uint32_t* x = orset_dots(self) + rm->elem[0] * AGX_CRDT_NODES;
  uint32_t* lv = orset_vv(self);
  if (orset_has(x)) {
    int del = 1;
    for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) {
      if (rm->vv[n] && x[n] > rm->vv[n]) del = 0;  /* deleteDotsAreGreater */
      if (x[n] && !rm->vv[n]) del = 0;             /* thisDot nodes within deleteDotsNodes */
    }
    if (del)
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) x[n] = 0u;
  }
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
    if (rm->dot[0][n] > lv[n]) lv[n] = rm->dot[0][n];
}

/* this := this.mergeDelta(delta) (:455-469) */
static inline void orset_merge_delta(uint64_t* self, const orset_delta* d) {
  for (uint32_t i = 0; i < d->nops; ++i) {
    const orset_dop* op = &d->ops[i];
    if (op->type == ORSET_DOP_REMOVE) orset_merge_remove_delta(self, op);
    else orset_dry_merge(self, op, op->type == ORSET_DOP_ADD);
  }
}

/* ORSet.add / remove / clear with their deltas (:339-351,380-387,404-412); `ver` is the new
 * version of `node` (VersionVector.increment draws it from Timestamp.counter,
 * VersionVector.scala:277-281; a replica uses vvector(node) + 1).  `delta` may be NULL. */
static inline void orset_add_d(uint64_t* w, orset_delta* delta, uint32_t node, uint32_t e, uint32_t ver) {
  uint32_t dot[AGX_CRDT_NODES] = {0};
  dot[node] = ver;
  uint32_t* d = orset_dots(w) + e * AGX_CRDT_NODES;
  orset_vv(w)[node] = ver;
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) d[n] = dot[n];
  if (delta) {
    orset_delta op;
    op.group = 0;
    op.nops = 1;
    orset_dop_single(&op.ops[0], ORSET_DOP_ADD, e, dot, dot);
    orset_delta_merge(delta, &op);
  }
}
static inline void orset_remove_d(uint64_t* w, orset_delta* delta, uint32_t node, uint32_t e) {
  if (delta) {
    uint32_t dot[AGX_CRDT_NODES] = {0};
    dot[node] = orset_vv(w)[node]; /* deltaDot = VersionVector(node, vvector.versionAt(node)) */
    orset_delta op;
    op.group = 0;
    op.nops = 1;
    orset_dop_single(&op.ops[0], ORSET_DOP_REMOVE, e, dot, orset_vv(w));
    orset_delta_merge(delta, &op);
  }
  orset_remove(w, e);
}
static inline void orset_clear_d(uint64_t* w, orset_delta* delta) {
  if (delta) {
    orset_delta op;
    op.group = 0;
    op.nops = 1;
    orset_dop_single(&op.ops[0], ORSET_DOP_FULL, 0, (const uint32_t*)0, orset_vv(w));
    orset_delta_merge(delta, &op);
  }
  orset_clear(w);
}

/* VersionVector.compareTo (VersionVector.scala:180-256) on the fixed layout (0 = no entry):
 * 0 Same, 1 Before (a < b), 2 After, 3 Concurrent. */
static inline uint32_t vv_compare(const uint32_t* a, const uint32_t* b) {
  int lt = 0, gt = 0;
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) {
    if (a[n] < b[n]) lt = 1;
    if (a[n] > b[n]) gt = 1;
  }
  return lt && gt ? 3u : lt ? 1u : gt ? 2u : 0u;
}

#ifdef __cplusplus
}
#endif
#endif
