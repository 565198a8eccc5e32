/*
 * behaviors_ref.h — TEST INFRASTRUCTURE ONLY.  The fixed-layout behaviour
 * table shared by the two CPU oracles (bsp_ref.c, fjp_ref.cpp).
 *
 * One call = one ActorCell.invoke of one message
 * (akka-actor/src/main/scala/akka/actor/ActorCell.scala:539-555) through the
 * typed adapter (akka-actor-typed/src/main/scala/akka/actor/typed/internal/adapter/ActorAdapter.scala:77-168),
 * returning the next-behaviour tag of ActorAdapter.next (:152-168):
 * AGX_RES_SAME (Behaviors.same), AGX_RES_STOPPED, AGX_RES_UNHANDLED.
 */
#ifndef AKKA_BEHAVIORS_REF_H
#define AKKA_BEHAVIORS_REF_H
#include <stdint.h>

#include "../include/akka_gpu.h"

#ifdef __cplusplus
#define REF_TLS thread_local
extern "C" {
#else
#define REF_TLS _Thread_local
#endif

typedef struct {
  uint64_t n;            /* global actor count */
  uint32_t W;            /* state words */
  uint32_t ring_stride;
  uint32_t fan_k;
  uint64_t fan_seed;
  const uint32_t* zipf_cdf;
  const uint32_t* zipf_perm;
  uint64_t zipf_n;
  const uint64_t* row_ptr; /* global CSR */
  const uint32_t* col;
  uint32_t gossip_f;       /* CRDT gossip fan-out */
  uint64_t gossip_seed;
  uint32_t delta_max;      /* delta-CRDT mode: Replicator max-delta-size (0 = off) */
  uint32_t error;          /* set on a delta-log overflow (engine: AGX_ECAPACITY) */
  const agx_case* bcase;   /* compiled behaviours (agx_set_behaviors) */
  const agx_act* bact;
  const uint32_t* bfirst;
  uint32_t n_beh;
} ref_params;

/* tell(dst, payload) from `self`; row != NULL = a CRDT state gossip carrying
 * `row_words` u64 of snapshot (copied by the callee). */
typedef void (*ref_emit_fn)(void* ctx, uint32_t dst, uint32_t self, uint32_t payload, const uint64_t* row,
                            uint32_t row_words);

static inline uint64_t ref_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Fan-out child randomness: a pure function of (seed, receiver, message hash, j),
 * so the fan-out tree is schedule independent (confluent). */
static inline uint64_t ref_fanout_rand(uint64_t seed, uint32_t self, uint32_t h, uint32_t j) {
  return ref_splitmix64(seed ^ ref_splitmix64(((uint64_t)self << 32) ^ ((uint64_t)h << 4) ^ (uint64_t)j));
}

/* Zipf sample: smallest i with u <= cdf[i], u = high 32 bits of r. */
static inline uint32_t ref_zipf_index(const uint32_t* cdf, uint64_t n, uint64_t r) {
  uint32_t u = (uint32_t)(r >> 32);
  uint64_t lo = 0, hi = n - 1;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (cdf[mid] >= u) hi = mid; else lo = mid + 1;
  }
  return (uint32_t)lo;
}

#include "crdt_ref.h"

static inline int ref_is_wide(uint32_t src) { return (src & AGX_WIDE_BIT) && src != AGX_NO_SENDER; }

static inline uint32_t ref_crdt_words(uint32_t kind) {
  return kind == AGX_KIND_GCOUNTER ? AGX_GCOUNTER_WORDS
         : kind == AGX_KIND_PNCOUNTER ? AGX_PNCOUNTER_WORDS
         : kind == AGX_KIND_ORSET ? AGX_ORSET_WORDS : 0u;
}

/* u64 words of a CRDT message row: the full state (+ deltaVersions in delta mode), or a
 * delta propagation (include/akka_gpu.h "delta-CRDT replication"). */
static inline uint32_t ref_row_words(uint32_t kind, uint32_t delta) {
  const uint32_t d = ref_crdt_words(kind);
  if (!d || !delta) return d;
  const uint32_t u = kind == AGX_KIND_ORSET ? AGX_ORSET_DELTA_ROW_U32 : 2u * d + AGX_CRDT_NODES;
  return (u + 1u) / 2u;
}

/* ---------------------------------------------------------------------------
 * Delta-CRDT replicas: DataEnvelope.deltaVersions + DeltaPropagationSelector state in the
 * words after the data (layout: include/akka_gpu.h).  Restates
 *   DeltaPropagationSelector.update / collectPropagations / deltaEntriesAfter
 *     (DD/DeltaPropagationSelector.scala:44-130,149-155; nodesSliceSize :65-68),
 *   Replicator.receiveUpdate's delta bookkeeping (DD/Replicator.scala:1646-1695: a modify
 *     without a delta records NoDeltaPlaceholder), createDeltaPropagation (:1357-1371),
 *   Replicator.receiveDeltaPropagation (:1965-2027) and DataEnvelope.merge of the
 *     deltaVersions (:960-1000).  Pruning (removed nodes) is out of scope: membership is static. */
static inline uint32_t* dref_env(uint64_t* w, uint32_t kind) { return (uint32_t*)(w + ref_crdt_words(kind)); }
static inline uint32_t* dref_entry(uint64_t* w, uint32_t kind, uint32_t seq) {
  return dref_env(w, kind) + 2u * AGX_DELTA_ENV_WORDS + AGX_DELTA_LOG_U32(kind == AGX_KIND_ORSET) * (seq % AGX_DELTA_LOG);
}

/* the replica's other nodes (Replicator.allNodes, sorted) and this tick's slice */
static inline uint32_t dref_slice(const ref_params* P, uint32_t a, uint32_t rr, uint32_t* out, uint32_t* nall) {
  const uint32_t m = crdt_key_size(a, P->n), node = a % AGX_CRDT_NODES;
  uint32_t all[AGX_CRDT_NODES], na = 0;
  for (uint32_t i = 0; i < m; ++i)
    if (i != node) all[na++] = i;
  *nall = na;
  if (!na) return 0;
  uint32_t s = na / 5u + 1u; /* nodesSliceSize: gossipIntervalDivisor = 5 (Replicator.scala:1349) */
  if (s < 2u) s = 2u;
  if (s > na) s = na;
  if (s > 10u) s = 10u;
  if (na <= s) {
    for (uint32_t i = 0; i < na; ++i) out[i] = all[i];
    return na;
  }
  const uint32_t i0 = rr % na;
  for (uint32_t i = 0; i < s; ++i) out[i] = all[(i0 + i) % na];
  return s;
}

/* A local ORSet update (Replicator.receiveUpdate with delta-crdt enabled): record the update's
 * delta under the next seqNr in the ring; `type` as in the log layout. */
static inline uint32_t* dref_record(ref_params* P, uint64_t* w, uint32_t kind, uint32_t a) {
  uint32_t* env = dref_env(w, kind);
  const uint32_t s = ++env[8];
  if (s > AGX_DELTA_LOG) { /* the ring slot's previous seqNr must have reached every node */
    const uint32_t m = crdt_key_size(a, P->n), node = a % AGX_CRDT_NODES;
    for (uint32_t i = 0; i < m; ++i)
      if (i != node && env[10 + i] < s - AGX_DELTA_LOG) P->error = 1;
  }
  uint32_t* e = dref_entry(w, kind, s);
  memset(e, 0, AGX_DELTA_LOG_U32(kind == AGX_KIND_ORSET) * 4u);
  e[0] = s;
  return e;
}

/* Counters' deltaEntries (include/akka_gpu.h): a delta is the updated slot's new value
 * (GCounter.scala:97-111, PNCounter.scala:161-179) and is never a ReplicatedDeltaSize, so
 * collectPropagations' reduceLeft over the entries after j is the slot-wise max of those deltas,
 * or NoDeltaPlaceholder if one lies after j (DD/DeltaPropagationSelector.scala:112-125).  A node's
 * own slots never decrease, so that max is the last delta of each slot after j: the oracle keeps
 * {seqNr, value} of each slot's last delta and the last placeholder's seqNr, for any number of
 * unsent seqNrs (the reference's map is unbounded). */
static inline void dref_record_counter(uint64_t* w, uint32_t kind, uint32_t side, uint64_t v) {
  uint32_t* env = dref_env(w, kind);
  uint32_t* e = env + 2u * AGX_DELTA_ENV_WORDS + 3u * side; /* side 0 increments, 1 decrements, 2 placeholder */
  e[0] = ++env[8];
  if (side < 2u) {
    e[1] = (uint32_t)v;
    e[2] = (uint32_t)(v >> 32);
  }
}

/* The merged delta group of seqNrs (j, ctr] (collectPropagations' reduceLeft with the
 * max-delta-size check), encoded as a DeltaPropagation row; returns 1 if it is a placeholder. */
static inline uint32_t dref_group_row(const ref_params* P, uint64_t* w, uint32_t kind, uint32_t a, uint32_t j,
                                      uint32_t* row) {
  uint32_t* env = dref_env(w, kind);
  const uint32_t ctr = env[8], node = a % AGX_CRDT_NODES;
  memset(row, 0, ref_row_words(kind, 1) * 8u);
  row[1] = node;
  row[2] = j + 1u;
  row[3] = ctr;
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) row[4 + n] = env[n];
  uint32_t ph = 0;
  if (kind != AGX_KIND_ORSET) { /* GCounter / PNCounter deltas merge by slot max (no deltaSize) */
    const uint32_t* e = env + 2u * AGX_DELTA_ENV_WORDS;
    ph = e[6] > j;
    for (uint32_t b = 0; b < 2; ++b)
      if (e[3 * b] > j) {
        row[12] |= 1u << b;
        row[13 + 2 * b] = e[3 * b + 1];
        row[14 + 2 * b] = e[3 * b + 2];
      }
  } else {
    static REF_TLS orset_delta g, d2; /* (fjp_ref runs replicas on several threads) */
    for (uint32_t s = j + 1; s <= ctr && !ph; ++s) {
      const uint32_t* e = dref_entry(w, kind, s);
      const uint32_t type = e[1] & 0xFFu, el = e[1] >> 8;
      uint32_t dot[AGX_CRDT_NODES] = {0};
      dot[node] = e[2];
      orset_delta* tgt = s == j + 1 ? &g : &d2;
      tgt->group = 0;
      tgt->nops = 1;
      orset_dop_single(&tgt->ops[0], type, el, dot, type == ORSET_DOP_ADD ? dot : e + 4);
      if (s > j + 1) {
        orset_delta_merge(&g, &d2);
        if (orset_delta_size(&g) >= P->delta_max) ph = 1;
      }
    }
    if (!ph) {
      uint32_t o = 12;
      for (uint32_t i = 0; i < g.nops; ++i) {
        const orset_dop* op = &g.ops[i];
        row[o++] = op->type | (op->n << 8);
        if (op->type == ORSET_DOP_ADD) {
          row[o++] = op->vv[node];
          for (uint32_t k = 0; k < op->n; ++k) {
            row[o++] = op->elem[k];
            row[o++] = op->dot[k][node];
          }
        } else {
          if (op->type == ORSET_DOP_REMOVE) {
            row[o++] = op->elem[0];
            row[o++] = op->dot[0][node];
          }
          for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) row[o++] = op->vv[n];
        }
      }
      row[0] = g.nops;
    }
  }
  if (ph) row[0] = 0x80000000u;
  return ph;
}

/* A received DeltaPropagation row (receiveDeltaPropagation + DataEnvelope.merge). */
static inline void dref_receive(uint64_t* w, uint32_t kind, const uint32_t* row) {
  if (row[0] & 0x80000000u) return; /* NoDeltaPlaceholder: not part of the propagation */
  uint32_t* env = dref_env(w, kind);
  const uint32_t from = row[1], lo = row[2], hi = row[3];
  if (kind != AGX_KIND_ORSET) { /* not RequiresCausalDeliveryOfDeltas: merge the sender's envelope */
    const uint32_t node_words = AGX_CRDT_NODES;
    if (row[12] & 1u) {
      const uint64_t x = ((uint64_t)row[14] << 32) | row[13];
      if (x > w[from]) w[from] = x;
    }
    if (row[12] & 2u) {
      const uint64_t x = ((uint64_t)row[16] << 32) | row[15];
      if (x > w[node_words + from]) w[node_words + from] = x;
    }
    for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
      if (row[4 + n] > env[n]) env[n] = row[4 + n];
    return;
  }
  const uint32_t cur = env[from];
  if (cur >= hi) return;     /* toSeqNr already handled */
  if (lo > cur + 1u) return; /* missing deltas between cur + 1 and fromSeqNr - 1 */
  static REF_TLS orset_delta g;
  g.group = row[0] > 1u;
  g.nops = 0;
  uint32_t o = 12;
  for (uint32_t i = 0; i < row[0]; ++i) {
    orset_dop* op = &g.ops[g.nops++];
    memset(op, 0, sizeof *op);
    op->type = row[o] & 0xFFu;
    const uint32_t cnt = row[o++] >> 8;
    if (op->type == ORSET_DOP_ADD) {
      op->vv[from] = row[o++];
      for (uint32_t k = 0; k < cnt; ++k, o += 2) { /* concatElementsMap: a later entry wins */
        uint32_t x = 0;
        while (x < op->n && op->elem[x] != row[o]) ++x;
        if (x == op->n) op->elem[op->n++] = row[o];
        memset(op->dot[x], 0, sizeof op->dot[x]);
        op->dot[x][from] = row[o + 1];
      }
    } else {
      if (op->type == ORSET_DOP_REMOVE) {
        op->n = 1;
        op->elem[0] = row[o++];
        op->dot[0][from] = row[o++];
      }
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) op->vv[n] = row[o++];
    }
  }
  orset_merge_delta(w, &g);
  env[from] = hi; /* deltaVersions.merge(VersionVector(fromNode, toSeqNr)) */
}

/* DeltaPropagationTick of replica `a` (DD/Replicator.scala:1953-1963), arg = k | AGX_DELTA_WRITE */
static inline void dref_tick(ref_params* P, uint32_t kind, uint32_t a, uint64_t* w, uint32_t arg, ref_emit_fn emit,
                             void* ctx) {
  const uint32_t k = arg & 0xFFFFu;
  if (arg & AGX_DELTA_WRITE) { /* a writer client: one seeded Update per tick, told to the replica */
    const uint64_t r = ref_fanout_rand(P->gossip_seed, a, k | 0x04000000u, 0);
    const uint32_t amount = 1u + (uint32_t)((r >> 32) & 3u);
    uint32_t op;
    if (kind == AGX_KIND_GCOUNTER) op = AGX_OP(AGX_OP_INCREMENT, amount);
    else if (kind == AGX_KIND_PNCOUNTER) op = AGX_OP((r >> 34) & 1u ? AGX_OP_DECREMENT : AGX_OP_INCREMENT, amount);
    else op = AGX_OP(((r >> 40) & 3u) ? AGX_OP_ADD : AGX_OP_REMOVE, (uint32_t)(r >> 48) % AGX_ORSET_ELEMS);
    emit(ctx, a, a, op, (const uint64_t*)0, 0u);
  }
  uint32_t* env = dref_env(w, kind);
  uint32_t sl[AGX_CRDT_NODES], na;
  const uint32_t s = dref_slice(P, a, env[9], sl, &na);
  if (na) {
    static REF_TLS uint64_t rowbuf[(AGX_ORSET_DELTA_ROW_U32 + 1) / 2];
    for (uint32_t i = 0; i < s; ++i) {
      const uint32_t j = env[10 + sl[i]];
      if (env[8] <= j) continue; /* deltaEntriesAfter(j) is empty */
      const uint32_t ph = dref_group_row(P, w, kind, a, j, (uint32_t*)rowbuf);
      env[10 + sl[i]] = env[8]; /* deltaSentToNode(node) = last seqNr, also for a placeholder */
      /* createDeltaPropagation leaves NoDeltaPlaceholder out (DD/Replicator.scala:1364) and nothing is
         sent for an empty propagation (:1957): a placeholder group is not told */
      if (!ph)
        emit(ctx, a - a % AGX_CRDT_NODES + sl[i], a, ((kind - AGX_KIND_GCOUNTER) << 30) | AGX_DELTA_ROW_BIT, rowbuf,
             ref_row_words(kind, 1));
    }
    env[9] += s; /* deltaNodeRoundRobinCounter += sliceSize */
  }
  if (k > 0) emit(ctx, a, a, AGX_OP(AGX_OP_DELTA_TICK, (k - 1u) | (arg & AGX_DELTA_WRITE)), (const uint64_t*)0, 0u);
}

/* One invoke of a CRDT replica (include/akka_gpu.h "CRDT behaviours"). */
static inline uint32_t ref_apply_crdt(ref_params* P, uint32_t kind, uint32_t a, uint64_t* w, uint32_t src,
                                      uint32_t payload, const uint64_t* row, ref_emit_fn emit, void* ctx) {
  const uint32_t node = a % AGX_CRDT_NODES;
  const uint32_t dm = P->delta_max;
  if (ref_is_wide(src)) { /* state gossip: merge (Replicator.receiveGossip -> write, DD/Replicator.scala:2118-2133) */
    if ((payload >> 30) != kind - AGX_KIND_GCOUNTER) return AGX_RES_UNHANDLED; /* another data type */
    if (payload & AGX_DELTA_ROW_BIT) {
      if (!dm) return AGX_RES_UNHANDLED;
      dref_receive(w, kind, (const uint32_t*)row);
      return AGX_RES_SAME;
    }
    if (dm) { /* DataEnvelope.merge: data and deltaVersions */
      const uint32_t* rdv = (const uint32_t*)(row + ref_crdt_words(kind));
      uint32_t* env = dref_env(w, kind);
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
        if (rdv[n] > env[n]) env[n] = rdv[n];
    }
    if ((payload >> 30) != kind - AGX_KIND_GCOUNTER) return AGX_RES_UNHANDLED; /* another data type */
    if (kind == AGX_KIND_ORSET) orset_merge(w, row);
    else crdt_counter_merge(w, row, ref_crdt_words(kind));
    return AGX_RES_SAME;
  }
  const uint32_t op = payload >> 24, arg = payload & 0xFFFFFFu;
  switch (op) {
    case AGX_OP_INCREMENT:
    case AGX_OP_DECREMENT: {
      if (kind == AGX_KIND_ORSET || (op == AGX_OP_DECREMENT && kind != AGX_KIND_PNCOUNTER)) return AGX_RES_UNHANDLED;
      const uint32_t slot = (op == AGX_OP_DECREMENT ? AGX_CRDT_NODES : 0u) + node;
      w[slot] += arg;
      if (dm) /* delta = the counter of the new slot value (GCounter.scala:97-111); n = 0: none */
        dref_record_counter(w, kind, arg ? (op == AGX_OP_DECREMENT ? 1u : 0u) : 2u, w[slot]);
      return AGX_RES_SAME;
    }
    case AGX_OP_ADD:
    case AGX_OP_REMOVE:
    case AGX_OP_CLEAR:
      if (kind != AGX_KIND_ORSET || (op != AGX_OP_CLEAR && arg >= AGX_ORSET_ELEMS)) return AGX_RES_UNHANDLED;
      if (dm) { /* AddDeltaOp (element, dot) / RemoveDeltaOp (element, deltaDot, vvector) / FullStateDeltaOp */
        uint32_t* e = dref_record(P, w, kind, a);
        e[1] = (op == AGX_OP_ADD ? ORSET_DOP_ADD : op == AGX_OP_REMOVE ? ORSET_DOP_REMOVE : ORSET_DOP_FULL) |
               (op == AGX_OP_CLEAR ? 0u : arg << 8);
        e[2] = orset_vv(w)[node] + (op == AGX_OP_ADD ? 1u : 0u);
        if (op != AGX_OP_ADD) memcpy(e + 4, orset_vv(w), AGX_CRDT_NODES * 4u);
        if (op == AGX_OP_CLEAR) e[2] = 0;
      }
      if (op == AGX_OP_ADD) orset_add(w, node, arg);
      else if (op == AGX_OP_REMOVE) orset_remove(w, arg);
      else orset_clear(w);
      return AGX_RES_SAME;
    case AGX_OP_GOSSIP:
      if (P->n > 1 && (!dm || crdt_key_size(a, P->n) > 1))
        for (uint32_t j = 0; j < P->gossip_f; ++j)
          emit(ctx, dm ? crdt_key_peer(P->gossip_seed, a, arg, j, P->n) : crdt_peer(P->gossip_seed, a, arg, j, P->n), a,
               (kind - AGX_KIND_GCOUNTER) << 30, w, ref_row_words(kind, dm));
      if (arg > 0) emit(ctx, a, a, AGX_OP(AGX_OP_GOSSIP, arg - 1u), (const uint64_t*)0, 0u);
      return AGX_RES_SAME;
    case AGX_OP_DELTA_TICK:
      if (!dm) return AGX_RES_UNHANDLED;
      dref_tick(P, kind, a, w, arg, emit, ctx);
      return AGX_RES_SAME;
    default:
      return AGX_RES_UNHANDLED;
  }
}

/* ---------------------------------------------------------------------------
 * Compiled behaviours (include/akka_gpu.h): a typed Behaviors.receiveMessage / ReceiveBuilder
 * restated as its case table.  ReceiveBuilder.receive (TY/javadsl/ReceiveBuilder.scala:209-218)
 * tries the handlers in order and takes the first whose class and predicate match; none ->
 * Behaviors.unhandled.  A become replaces the actor's behaviour for its next message
 * (TY/Behavior.scala:150 canonicalize, ActorAdapter.next TY/internal/adapter/ActorAdapter.scala:152-168). */
static inline uint64_t ref_operand(uint32_t src, uint32_t word, int64_t k, uint32_t pay, const uint64_t* w,
                                   uint32_t sender, uint32_t self) {
  uint64_t b = 0;
  if (src == AGX_V_PAYLOAD) b = pay;
  else if (src == AGX_V_TAG) b = pay >> 24;
  else if (src == AGX_V_ARG) b = pay & 0xFFFFFFu;
  else if (src == AGX_V_WORD) b = w[word];
  else if (src == AGX_V_SENDER) b = sender;
  else if (src == AGX_V_SELF) b = self;
  return b + (uint64_t)k;
}
static inline int ref_cmp(uint32_t op, uint64_t a, uint64_t b) {
  switch (op) {
    case AGX_CMP_EQ: return a == b;
    case AGX_CMP_NE: return a != b;
    case AGX_CMP_LT: return a < b;
    case AGX_CMP_LE: return a <= b;
    case AGX_CMP_GT: return a > b;
    case AGX_CMP_GE: return a >= b;
    default: return 1;
  }
}
static inline uint32_t ref_apply_compiled(const ref_params* P, uint32_t* kind, uint32_t a, uint64_t* w, uint32_t src,
                                          uint32_t pay, ref_emit_fn emit, void* ctx) {
  const uint32_t b = *kind - AGX_KIND_COMPILED;
  if (b >= P->n_beh) return AGX_RES_UNHANDLED;
  for (uint32_t c = P->bfirst[b]; c < P->bfirst[b + 1]; ++c) {
    const agx_case* C = &P->bcase[c];
    if (!ref_cmp(C->cmp1, ref_operand(C->src1, C->word1, C->k1, pay, w, src, a),
                 ref_operand(C->src2, C->word2, C->k2, pay, w, src, a)))
      continue;
    if (!ref_cmp(C->cmp2, ref_operand(C->src3, C->word3, C->k3, pay, w, src, a),
                 ref_operand(C->src4, C->word4, C->k4, pay, w, src, a)))
      continue;
    for (uint32_t i = C->act_first; i < (uint32_t)C->act_first + C->act_count; ++i) {
      const agx_act* A = &P->bact[i];
      const uint64_t v = ref_operand(A->src, A->sword, A->k, pay, w, src, a);
      if (A->op == AGX_A_SET) w[A->word] = v;
      else if (A->op == AGX_A_ADD) w[A->word] += v;
      else if (A->op == AGX_A_MAX) { if (v > w[A->word]) w[A->word] = v; }
      else if (A->op == AGX_A_MIN) { if (v < w[A->word]) w[A->word] = v; }
      else if (A->op == AGX_A_TELL) {
        uint64_t d;
        if (A->dsrc == AGX_V_SELF) {
          int64_t x = ((int64_t)a + A->dk) % (int64_t)P->n;
          d = (uint64_t)(x < 0 ? x + (int64_t)P->n : x);
        } else {
          d = ref_operand(A->dsrc, A->dword, A->dk, pay, w, src, a);
        }
        emit(ctx, d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d, a,
             A->or_mask ? ((uint32_t)v & 0xFFFFFFu) | A->or_mask : (uint32_t)v, (const uint64_t*)0, 0u);
      }
    }
    if (C->result == AGX_RES_BECOME) {
      *kind = AGX_KIND_COMPILED + C->next;
      return AGX_RES_SAME;
    }
    return C->result;
  }
  return AGX_RES_UNHANDLED;
}

/* `kind` in/out: a compiled behaviour's become changes it for the actor's next message. */
static inline uint32_t ref_apply(ref_params* P, uint32_t* kind_io, uint32_t a, uint64_t* w, uint32_t src,
                                 uint32_t payload, const uint64_t* row, ref_emit_fn emit, void* ctx) {
  const uint32_t kind = *kind_io;
  if (kind >= AGX_KIND_COMPILED) {
    if (ref_is_wide(src)) return AGX_RES_UNHANDLED;
    return ref_apply_compiled(P, kind_io, a, w, src, payload, emit, ctx);
  }
  if (kind >= AGX_KIND_GCOUNTER && kind <= AGX_KIND_ORSET)
    return ref_apply_crdt(P, kind, a, w, src, payload, row, emit, ctx);
  if (ref_is_wide(src)) return AGX_RES_UNHANDLED; /* a state gossip is not in this behaviour's protocol */
  switch (kind) {
    case AGX_KIND_COUNTER:
      w[0] += 1;
      if (P->W > 1) w[1] += payload;
      return AGX_RES_SAME;
    case AGX_KIND_RING:
      w[0] += 1;
      if (payload > 0) emit(ctx, (uint32_t)(((uint64_t)a + P->ring_stride) % P->n), a, payload - 1, 0, 0);
      return AGX_RES_SAME;
    case AGX_KIND_FANOUT: {
      w[0] += 1;
      if (P->W > 1) w[1] += payload;
      uint32_t ttl = payload >> 24, h = payload & 0x00FFFFFFu; /* ttl 8 bits, hash 24 bits */
      if (ttl > 0)
        for (uint32_t j = 0; j < P->fan_k; ++j) {
          uint64_t r = ref_fanout_rand(P->fan_seed, a, h, j);
          uint32_t d = P->zipf_perm[ref_zipf_index(P->zipf_cdf, P->zipf_n, r)];
          emit(ctx, d, a, ((ttl - 1) << 24) | ((uint32_t)r & 0x00FFFFFFu), 0, 0);
        }
      return AGX_RES_SAME;
    }
    case AGX_KIND_FORWARD_RR:
      w[0] += 1;
      if (payload > 0 && P->row_ptr) {
        uint64_t b = P->row_ptr[a], deg = P->row_ptr[a + 1] - b;
        if (deg) {
          uint64_t e = b + (w[1] % deg);
          w[1] += 1;
          emit(ctx, P->col[e], a, payload - 1, 0, 0);
        }
      }
      return AGX_RES_SAME;
    case AGX_KIND_STOP_AFTER:
      w[0] += 1;
      return (w[0] >= w[1]) ? AGX_RES_STOPPED : AGX_RES_SAME;
    case AGX_KIND_PINGPONG: {
      /* BenchmarkActors.PingPong (akka-bench-jmh/src/main/scala/akka/actor/BenchmarkActors.scala:20-32):
       *   if (left == 0) { latch.countDown(); context.stop(self) }
       *   sender() ! Message; left -= 1                                       */
      uint32_t res = (w[0] == 0) ? AGX_RES_STOPPED : AGX_RES_SAME;
      if (P->W > 1) w[1] += 1;
      emit(ctx, src, a, payload, 0, 0);
      w[0] -= 1;
      return res;
    }
    case AGX_KIND_EVEN:
      if (payload & 1u) return AGX_RES_UNHANDLED; /* Behaviors.unhandled */
      w[0] += 1;
      return AGX_RES_SAME;
    default:
      return AGX_RES_SAME;
  }
}

#ifdef __cplusplus
}
#endif
#endif
