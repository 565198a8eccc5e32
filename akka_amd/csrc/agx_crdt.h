// agx_crdt.h — Replicator-style CRDT replicas on the device (BASELINE C4):
// GCounter / PNCounter / ORSet actors that merge full-state gossips and
// gossip their own state on GOSSIP ticks (include/akka_gpu.h "CRDT behaviours").
//
//   GCounter.increment / merge      DD/GCounter.scala:97-125
//   PNCounter.change / merge        DD/PNCounter.scala:161-179
//   ORSet.add / remove / clear      DD/ORSet.scala:339-351,380-387,404-412
//   ORSet.merge (dryMerge)          DD/ORSet.scala:427-452 with mergeCommonKeys
//                                   (:164-229), mergeDisjointKeys (:236-259),
//                                   subtractDots (:127-160), VersionVector.merge
//   GossipTick -> gossipTo          DD/Replicator.scala:1316,2029-2064
//
// State lives in the actor SoA (word-major u64, coalesced across the lanes of
// a wave that drain consecutive actors).  A state gossip carries a handle to
// an immutable snapshot row (row-major, 16-B vector loads per lane).  Rows are
// allocated per superstep in heap[step & 1] and read in the next superstep
// from heap[(step - 1) & 1]; a gossip that stays queued beyond the
// throughput cap has its row copied forward (see bucket_finish).
#pragma once
#include "agx_device.h"

namespace agx {

// state gossip payload = (data type << 30) | handle; handles index heap rows, then rx rows
constexpr uint32_t kHandleMask = 0x3FFFFFFFu;

__device__ __forceinline__ bool is_wide(uint32_t src) { return (src & AGX_WIDE_BIT) && src != AGX_NO_SENDER; }
__device__ __forceinline__ bool is_crdt(uint32_t kind) {
  return kind - (uint32_t)AGX_KIND_GCOUNTER <= (uint32_t)(AGX_KIND_ORSET - AGX_KIND_GCOUNTER);
}
__device__ __forceinline__ uint32_t crdt_words(uint32_t kind) {
  return kind == AGX_KIND_GCOUNTER ? AGX_GCOUNTER_WORDS : kind == AGX_KIND_PNCOUNTER ? AGX_PNCOUNTER_WORDS : AGX_ORSET_WORDS;
}

// heap rows of the superstep being executed (write) and of the previous one (read)
struct CrdtHeap {
  uint32_t* wr;
  const uint32_t* rd;
  const uint32_t* rx;
  uint32_t* top;
  uint32_t rows, pw;
  __device__ __forceinline__ const uint32_t* row(uint32_t h) const {
    return h < rows ? rd + (size_t)h * pw : rx + (size_t)(h - rows) * pw;
  }
  __device__ __forceinline__ uint32_t* wrow(uint32_t h) const { return wr + (size_t)h * pw; }
};
__device__ __forceinline__ CrdtHeap crdt_heap(const DevParams& P) {
  const uint32_t s = *P.step;
  const size_t half = (size_t)P.heap_rows * P.pw;
  return {P.heap + (s & 1u) * half, P.heap + ((s + 1u) & 1u) * half, P.rx, P.heap_top + (s & 1u), P.heap_rows, P.pw};
}

// copy a row (pw u32, multiple of 4, 16-B aligned)
__device__ __forceinline__ void copy_row(uint32_t* dst, const uint32_t* src, uint32_t pw) {
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(dst);
  for (uint32_t i = 0; i < pw / 4; ++i) d[i] = s[i];
}

// Gossip peer j of `self` at countdown `round` (Replicator.selectRandomNode with the counter RNG)
__device__ __forceinline__ uint32_t crdt_peer(uint64_t seed, uint32_t self, uint32_t round, uint32_t j, uint32_t n) {
  const uint64_t r = fanout_rand(seed, self, round | 0x08000000u, j);
  const uint32_t d = (uint32_t)(r % (uint64_t)(n - 1u));
  return d >= self ? d + 1u : d;
}

// Phase A: tells and snapshot rows one message will produce (no state access).
__device__ __forceinline__ uint32_t crdt_count(const DevParams& P, uint32_t src, uint32_t pay, uint32_t* rows) {
  if (is_wide(src) || (pay >> 24) != AGX_OP_GOSSIP) return 0;
  const uint32_t f = P.n_global > 1 ? P.gossip_f : 0u;
  *rows += f ? 1u : 0u;
  return f + ((pay & 0xFFFFFFu) > 0 ? 1u : 0u);
}

__device__ __forceinline__ uint32_t orset_merge_entry(uint32_t l, uint32_t r, uint32_t lvv, uint32_t rvv) {
  if (l == r) return l;
  const uint32_t lk = l > rvv ? l : 0u, rk = r > lvv ? r : 0u;
  return lk > rk ? lk : rk;
}

// Phase B: one invoke of a CRDT replica.  `emit(dst, pay)` / `emit_wide(dst, handle)`.
// CM: the CRDT kinds present (one bit = a single-kind population, whose merge is specialised:
// the other kinds' code and registers vanish).  Merges issue all loads of a batch before its
// stores (the row and the state may alias as far as the compiler knows, so a load-store-load
// chain would serialise one memory round trip per element).
template <uint32_t CM, typename Emit>
__device__ __forceinline__ uint32_t crdt_apply(const DevParams& P, const CrdtHeap& H, uint32_t kind, uint32_t self,
                                               uint32_t l, uint32_t src, uint32_t pay, uint32_t& row_cursor,
                                               Emit& em) {
  if constexpr (CM == (1u << AGX_KIND_GCOUNTER)) kind = AGX_KIND_GCOUNTER;
  if constexpr (CM == (1u << AGX_KIND_PNCOUNTER)) kind = AGX_KIND_PNCOUNTER;
  if constexpr (CM == (1u << AGX_KIND_ORSET)) kind = AGX_KIND_ORSET;
  const size_t nl = P.n_local;
  uint64_t* st = P.state + l;  // word w at st[w * nl]
  const uint32_t node = self % AGX_CRDT_NODES;
  if (is_wide(src)) {
    if ((pay >> 30) != kind - (uint32_t)AGX_KIND_GCOUNTER) return AGX_RES_UNHANDLED;  // another data type
    const uint32_t* row = H.row(pay & kHandleMask);
    if (kind != AGX_KIND_ORSET) {  // slot-wise max, 8 words per batch
      const uint32_t nw = crdt_words(kind);
      for (uint32_t i0 = 0; i0 < nw; i0 += 8) {
        uint4 v[4];
        uint64_t s[8];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(row + 2 * i0 + 4 * u);
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u] = st[(i0 + u) * nl];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint64_t r0 = ((uint64_t)v[u].y << 32) | v[u].x, r1 = ((uint64_t)v[u].w << 32) | v[u].z;
          if (r0 > s[2 * u]) st[(i0 + 2 * u) * nl] = r0;
          if (r1 > s[2 * u + 1]) st[(i0 + 2 * u + 1) * nl] = r1;
        }
      }
      return AGX_RES_SAME;
    }
    // ORSet.merge: dots per (element, node), then vvector max
    uint32_t lvv[AGX_CRDT_NODES], rvv[AGX_CRDT_NODES];
    const uint32_t vw = AGX_ORSET_ELEMS * AGX_CRDT_NODES / 2;  // first vvector word
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t s = st[(vw + k) * nl];
      lvv[2 * k] = (uint32_t)s;
      lvv[2 * k + 1] = (uint32_t)(s >> 32);
      rvv[2 * k] = row[2 * (vw + k)];
      rvv[2 * k + 1] = row[2 * (vw + k) + 1];
    }
#ifndef AGX_ORSET_BATCH
#define AGX_ORSET_BATCH 2
#endif
    constexpr uint32_t kE = AGX_ORSET_BATCH;  // elements per batch (8 row words + 4 state words each)
    for (uint32_t e0 = 0; e0 < AGX_ORSET_ELEMS; e0 += kE) {
      uint4 ra[kE], rb[kE];
      uint64_t s[kE][4];
#pragma unroll
      for (uint32_t u = 0; u < kE; ++u) {
        ra[u] = *reinterpret_cast<const uint4*>(row + 8 * (e0 + u));
        rb[u] = *reinterpret_cast<const uint4*>(row + 8 * (e0 + u) + 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) s[u][k] = st[(size_t)(4 * (e0 + u) + k) * nl];
      }
#pragma unroll
      for (uint32_t u = 0; u < kE; ++u) {
        const uint32_t r[8] = {ra[u].x, ra[u].y, ra[u].z, ra[u].w, rb[u].x, rb[u].y, rb[u].z, rb[u].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint64_t sv = s[u][k];
          const uint32_t o0 = orset_merge_entry((uint32_t)sv, r[2 * k], lvv[2 * k], rvv[2 * k]);
          const uint32_t o1 = orset_merge_entry((uint32_t)(sv >> 32), r[2 * k + 1], lvv[2 * k + 1], rvv[2 * k + 1]);
          const uint64_t o = ((uint64_t)o1 << 32) | o0;
          if (o != sv) st[(size_t)(4 * (e0 + u) + k) * nl] = o;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a = max(lvv[2 * k], rvv[2 * k]), b = max(lvv[2 * k + 1], rvv[2 * k + 1]);
      st[(vw + k) * nl] = ((uint64_t)b << 32) | a;
    }
    return AGX_RES_SAME;
  }
  const uint32_t op = pay >> 24, arg = pay & 0xFFFFFFu;
  switch (op) {
    case AGX_OP_INCREMENT:
      if (kind == AGX_KIND_ORSET) return AGX_RES_UNHANDLED;
      st[node * nl] += arg;
      return AGX_RES_SAME;
    case AGX_OP_DECREMENT:
      if (kind != AGX_KIND_PNCOUNTER) return AGX_RES_UNHANDLED;
      st[(AGX_CRDT_NODES + node) * nl] += arg;
      return AGX_RES_SAME;
    case AGX_OP_ADD:
    case AGX_OP_REMOVE:
    case AGX_OP_CLEAR: {
      if (kind != AGX_KIND_ORSET || (op != AGX_OP_CLEAR && arg >= AGX_ORSET_ELEMS)) return AGX_RES_UNHANDLED;
      if (op == AGX_OP_CLEAR) {
        for (uint32_t w = 0; w < AGX_ORSET_ELEMS * AGX_CRDT_NODES / 2; ++w) st[w * nl] = 0;
        return AGX_RES_SAME;
      }
      uint64_t dots[4] = {0, 0, 0, 0};
      if (op == AGX_OP_ADD) {  // vvector + node; birth dot (node -> new version)
        const size_t vwi = (size_t)(AGX_ORSET_ELEMS * AGX_CRDT_NODES / 2 + node / 2) * nl;
        uint64_t vv = st[vwi];
        const uint32_t sh = (node & 1u) * 32u;
        const uint32_t ver = (uint32_t)(vv >> sh) + 1u;
        vv = (vv & ~(0xFFFFFFFFull << sh)) | ((uint64_t)ver << sh);
        st[vwi] = vv;
        dots[node / 2] = (uint64_t)ver << sh;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) st[(size_t)(4 * arg + k) * nl] = dots[k];
      return AGX_RES_SAME;
    }
    case AGX_OP_GOSSIP: {
      const uint32_t f = P.n_global > 1 ? P.gossip_f : 0u;
      if (f) {
        const uint32_t h = row_cursor++;
        if (h < H.rows) {  // snapshot of the current state, shared by the f gossips
          uint32_t* row = H.wrow(h);
          const uint32_t nw = crdt_words(kind);  // 8 | 16 | 260 words: batches of 4 (loads first)
          for (uint32_t i0 = 0; i0 < nw; i0 += 4) {
            uint64_t s[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) s[u] = st[(i0 + u) * nl];
#pragma unroll
            for (int u = 0; u < 2; ++u)
              *reinterpret_cast<uint4*>(row + 2 * i0 + 4 * u) =
                  make_uint4((uint32_t)s[2 * u], (uint32_t)(s[2 * u] >> 32), (uint32_t)s[2 * u + 1],
                             (uint32_t)(s[2 * u + 1] >> 32));
          }
        }
        const uint32_t tagged = ((kind - (uint32_t)AGX_KIND_GCOUNTER) << 30) | h;
        for (uint32_t j = 0; j < f; ++j) em.wide(crdt_peer(P.gossip_seed, self, arg, j, P.n_global), tagged);
      }
      if (arg > 0) em(self, AGX_OP(AGX_OP_GOSSIP, arg - 1u));
      return AGX_RES_SAME;
    }
    default:
      return AGX_RES_UNHANDLED;
  }
}

}  // namespace agx
