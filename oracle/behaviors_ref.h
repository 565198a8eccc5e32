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
extern "C" {
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

/* One invoke of a CRDT replica (include/akka_gpu.h "CRDT behaviours"). */
static inline uint32_t ref_apply_crdt(const ref_params* P, uint32_t kind, uint32_t a, uint64_t* w, uint32_t src,
                                      uint32_t payload, const uint64_t* row, ref_emit_fn emit, void* ctx) {
  const uint32_t node = a % AGX_CRDT_NODES;
  if (ref_is_wide(src)) { /* state gossip: merge (Replicator.receiveGossip -> write, DD/Replicator.scala:2118-2133) */
    if ((payload >> 30) != kind - AGX_KIND_GCOUNTER) return AGX_RES_UNHANDLED; /* another data type */
    if (kind == AGX_KIND_ORSET) orset_merge(w, row);
    else crdt_counter_merge(w, row, ref_crdt_words(kind));
    return AGX_RES_SAME;
  }
  const uint32_t op = payload >> 24, arg = payload & 0xFFFFFFu;
  switch (op) {
    case AGX_OP_INCREMENT:
      if (kind == AGX_KIND_ORSET) return AGX_RES_UNHANDLED;
      w[node] += arg;
      return AGX_RES_SAME;
    case AGX_OP_DECREMENT:
      if (kind != AGX_KIND_PNCOUNTER) return AGX_RES_UNHANDLED;
      w[AGX_CRDT_NODES + node] += arg;
      return AGX_RES_SAME;
    case AGX_OP_ADD:
    case AGX_OP_REMOVE:
    case AGX_OP_CLEAR:
      if (kind != AGX_KIND_ORSET || (op != AGX_OP_CLEAR && arg >= AGX_ORSET_ELEMS)) return AGX_RES_UNHANDLED;
      if (op == AGX_OP_ADD) orset_add(w, node, arg);
      else if (op == AGX_OP_REMOVE) orset_remove(w, arg);
      else orset_clear(w);
      return AGX_RES_SAME;
    case AGX_OP_GOSSIP:
      if (P->n > 1)
        for (uint32_t j = 0; j < P->gossip_f; ++j)
          emit(ctx, crdt_peer(P->gossip_seed, a, arg, j, P->n), a, (kind - AGX_KIND_GCOUNTER) << 30, w,
               ref_crdt_words(kind));
      if (arg > 0) emit(ctx, a, a, AGX_OP(AGX_OP_GOSSIP, arg - 1u), (const uint64_t*)0, 0u);
      return AGX_RES_SAME;
    default:
      return AGX_RES_UNHANDLED;
  }
}

static inline uint32_t ref_apply(const ref_params* P, uint32_t kind, uint32_t a, uint64_t* w, uint32_t src,
                                 uint32_t payload, const uint64_t* row, ref_emit_fn emit, void* ctx) {
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
