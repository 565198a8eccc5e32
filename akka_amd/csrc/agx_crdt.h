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
//   delta-CRDT replication (agx_set_delta_crdt):
//     receiveUpdate delta bookkeeping DD/Replicator.scala:1646-1695
//     DeltaPropagationSelector        DD/DeltaPropagationSelector.scala:44-155
//     receiveDeltaPropagation         DD/Replicator.scala:1965-2027 (causal delivery for ORSet)
//     ORSet.mergeDelta / mergeRemoveDelta / DeltaOp.merge  DD/ORSet.scala:43-120,455-501
//
// A CRDT engine keeps the state actor-major (wide_state: a replica's words are one contiguous
// row of P.pitch u64, 128-B aligned), so a replica's 2 KB of ORSet dots are whole cache lines
// however its lanes diverge; plain engines keep the word-major SoA.  A state gossip carries a handle to
// an immutable snapshot row (counters: the state words; ORSet: sparse, kOrRow* below).  Rows are
// allocated per superstep in heap[step & 1] and read in the next superstep
// from heap[(step - 1) & 1]; a gossip that stays queued beyond the
// throughput cap has its row copied forward (see bucket_finish).
#pragma once
#include "agx_device.h"

namespace agx {

// state gossip payload = (data type << 30) | (DeltaPropagation << 29) | handle; handles index
// heap rows, then rx rows
constexpr uint32_t kHandleMask = AGX_DELTA_ROW_BIT - 1u;

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

// Gossip peer j of `self` at countdown `round` (Replicator.selectRandomNode with the counter RNG)
__device__ __forceinline__ uint32_t crdt_peer(uint64_t seed, uint32_t self, uint32_t round, uint32_t j, uint32_t n) {
  const uint64_t r = fanout_rand(seed, self, round | 0x08000000u, j);
  const uint32_t d = (uint32_t)(r % (uint64_t)(n - 1u));
  return d >= self ? d + 1u : d;
}

__device__ __forceinline__ uint32_t orset_merge_entry(uint32_t l, uint32_t r, uint32_t lvv, uint32_t rvv) {
  if (l == r) return l;
  const uint32_t lk = l > rvv ? l : 0u, rk = r > lvv ? r : 0u;
  return lk > rk ? lk : rk;
}

// Delta-CRDT mode: the replicas of a key are [self & ~7, +m), m = min(8, n - (self & ~7)); the
// full-state gossip peer is uniform over the other m - 1 (Replicator.selectRandomNode).
__device__ __forceinline__ uint32_t key_size(uint32_t self, uint32_t n) {
  const uint32_t m = n - (self & ~(AGX_CRDT_NODES - 1u));
  return m < AGX_CRDT_NODES ? m : AGX_CRDT_NODES;
}
__device__ __forceinline__ uint32_t crdt_key_peer(uint64_t seed, uint32_t self, uint32_t round, uint32_t j, uint32_t n) {
  const uint32_t m = key_size(self, n), node = self % AGX_CRDT_NODES;
  const uint32_t d = (uint32_t)(fanout_rand(seed, self, round | 0x08000000u, j) % (uint64_t)(m - 1u));
  return self - node + (d >= node ? d + 1u : d);
}

// u32 view of one actor's word-major state (u32 i = half i & 1 of word i >> 1)
struct St32 {
  uint64_t* st;
  size_t nl;
  __device__ __forceinline__ uint32_t ld(uint32_t i) const {
    const uint64_t v = st[(size_t)(i >> 1) * nl];
    return (i & 1u) ? (uint32_t)(v >> 32) : (uint32_t)v;
  }
  __device__ __forceinline__ void put(uint32_t i, uint32_t x) const {
    reinterpret_cast<uint32_t*>(st + (size_t)(i >> 1) * nl)[i & 1u] = x;
  }
};

// Envelope / selector area and delta log (include/akka_gpu.h "delta-CRDT replication"), u32 indices
__device__ __forceinline__ uint32_t dl_env(uint32_t kind) { return 2u * crdt_words(kind); }

// ORSet-only full-state populations (the wave path: orset_protocol + k_orset_merge, which writes and
// reads every snapshot row of such an engine) keep their snapshot rows sparse: a converged set holds
// a few non-zero dots per element (one per writer node that added it), so the row carries only
// those and the receiver rebuilds the zeros.  u32 layout: [0, 8) version vector, [16, 32) node masks
// (64 x u8, element e's byte: bit n = dot (e, n) non-zero), [32, ...) the non-zero dots in
// (element, node) order -- 32 + 512 u32 at most, within the 544-u32 row pitch.  Same merge results
// as the dense row; C4 rows shrink from 2080 B to 128 B + 4 B per live dot.  (Populations that mix
// CRDT kinds or run delta-CRDT replication go through crdt_apply and keep dense rows: the sparse form
// there failed the multi-pass mixed-CRDT parity test -- a wrong emitted counter, cause not found --
// so it was taken out again.  The two row forms never meet in one engine.)
constexpr uint32_t kOrRowVV = 0, kOrRowDV = 8, kOrRowMask = 16, kOrRowDots = 32;
static_assert(kOrRowDots + AGX_ORSET_ELEMS * AGX_CRDT_NODES <= 544u, "sparse ORSet row within the row pitch");
#ifdef AGX_SPARSE_SERIAL
// (diagnostic build knob: the round-4 serial sparse form in crdt_apply, for every ORSet population)
constexpr bool kSparseSerial = true;
#else
constexpr bool kSparseSerial = false;
#endif
// where a full-state gossip row keeps the sender's deltaVersions (delta-CRDT mode)
__device__ __forceinline__ uint32_t row_dv(uint32_t kind) {
  return kSparseSerial && kind == AGX_KIND_ORSET ? kOrRowDV : 2u * crdt_words(kind);
}
__device__ __forceinline__ uint32_t dl_entry(uint32_t kind, uint32_t seq) {
  return dl_env(kind) + 2u * AGX_DELTA_ENV_WORDS + AGX_DELTA_LOG_U32(kind == AGX_KIND_ORSET) * (seq % AGX_DELTA_LOG);
}
// DeltaPropagationSelector.nodesSliceSize over the na = m - 1 other nodes (gossipIntervalDivisor 5)
__device__ __forceinline__ uint32_t dl_slice_size(uint32_t na) {
  uint32_t s = na / 5u + 1u;
  s = s < 2u ? 2u : s;
  const uint32_t cap = na < 10u ? na : 10u;
  return s < cap ? s : cap;
}
// i-th node of this tick's round-robin slice (Replicator.allNodes sorted, self excluded)
__device__ __forceinline__ uint32_t dl_slice_node(uint32_t node, uint32_t na, uint32_t s, uint32_t rr, uint32_t i) {
  const uint32_t k = na <= s ? i : (rr % na + i) % na;
  return k >= node ? k + 1u : k;
}

// Phase A of a delta replica's drain: the selector state the ticks of this drain will see.
struct DeltaSim {
  bool on;
  uint32_t ctr, rr;
  uint32_t sent[AGX_CRDT_NODES];
};

// Does this op record a delta (a valid local update of this kind)?
__device__ __forceinline__ bool dl_records(uint32_t kind, uint32_t op, uint32_t arg) {
  if (op == AGX_OP_INCREMENT) return kind != AGX_KIND_ORSET;
  if (op == AGX_OP_DECREMENT) return kind == AGX_KIND_PNCOUNTER;
  if (op == AGX_OP_ADD || op == AGX_OP_REMOVE) return kind == AGX_KIND_ORSET && arg < AGX_ORSET_ELEMS;
  if (op == AGX_OP_CLEAR) return kind == AGX_KIND_ORSET;
  return false;
}

// Phase A: tells and snapshot rows one message will produce.  Delta replicas simulate the
// selector (deltaCounter, deltaSentToNode, round robin) over the drain, so a DeltaPropagationTick
// counts exactly the propagations phase B will tell.
template <uint32_t CM>
__device__ __forceinline__ uint32_t crdt_count(const DevParams& P, uint32_t kind, uint32_t self, uint32_t l,
                                               uint32_t src, uint32_t pay, uint32_t* rows, DeltaSim& ds) {
  if (is_wide(src)) return 0;
  const uint32_t op = pay >> 24, arg = pay & 0xFFFFFFu;
  const bool dm = (CM & kDeltaKM) != 0 && P.delta_max != 0;
  if (dm && (op == AGX_OP_DELTA_TICK || dl_records(kind, op, arg)) && !ds.on) {
    const St32 s{wide_state(P, l), wide_nl(P)};
    const uint32_t e0 = dl_env(kind);
    ds.on = true;
    ds.ctr = s.ld(e0 + 8);
    ds.rr = s.ld(e0 + 9);
#pragma unroll
    for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) ds.sent[n] = s.ld(e0 + 10 + n);
  }
  if (op == AGX_OP_GOSSIP) {
    const uint32_t f = P.n_global > 1 && (!dm || key_size(self, P.n_global) > 1) ? P.gossip_f : 0u;
    *rows += f ? 1u : 0u;
    return f + (arg > 0 ? 1u : 0u);
  }
  if (!dm) return 0;
  if (dl_records(kind, op, arg)) {
    ++ds.ctr;
    return 0;
  }
  if (op != AGX_OP_DELTA_TICK) return 0;
  uint32_t t = (arg & AGX_DELTA_WRITE) ? 1u : 0u;
  const uint32_t node = self % AGX_CRDT_NODES, na = key_size(self, P.n_global) - 1u;
  if (na) {
    const uint32_t sz = dl_slice_size(na);
    const uint32_t s = na <= sz ? na : sz;
    for (uint32_t i = 0; i < s; ++i) {
      const uint32_t x = dl_slice_node(node, na, sz, ds.rr, i);
      uint32_t sx = 0;
#pragma unroll
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) sx = n == x ? ds.sent[n] : sx;
      if (ds.ctr > sx) {
        ++t;
        ++*rows;
#pragma unroll
        for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) ds.sent[n] = n == x ? ds.ctr : ds.sent[n];
      }
    }
    ds.rr += sz;
  }
  return t + ((arg & 0xFFFFu) > 0 ? 1u : 0u);
}

// A local update with delta-crdt on: the next seqNr's log entry (DeltaPropagationSelector.update).
// ORSet: the ring slot it overwrites must have been sent to every other node of the key, else the
// engine reports AGX_ECAPACITY.
__device__ __forceinline__ uint32_t dl_record(const DevParams& P, const St32& s, uint32_t kind, uint32_t self) {
  const uint32_t e0 = dl_env(kind);
  const uint32_t q = s.ld(e0 + 8) + 1u;
  s.put(e0 + 8, q);
  if (q > AGX_DELTA_LOG) {
    const uint32_t m = key_size(self, P.n_global), node = self % AGX_CRDT_NODES;
    bool lost = false;
    for (uint32_t n = 0; n < m; ++n) lost |= n != node && s.ld(e0 + 10 + n) < q - AGX_DELTA_LOG;
    if (lost) atomicOr(P.err, 1ull);  // kErrCapacity
  }
  const uint32_t x = dl_entry(kind, q);
  s.put(x, q);
  return x;
}
// Counters: a delta is the updated slot's new value, and slot-max merging of the deltas after j
// (they are never a ReplicatedDeltaSize) is the last delta of each slot after j, or a placeholder
// when a no-delta update lies after j -- the own slots never decrease, so the deltas of a slot grow
// with their seqNr.  The log is therefore {seqNr, value} of each slot's last delta and the last
// placeholder's seqNr (AGX_COUNTER_DELTA_U32): exact for any number of unsent seqNrs, like the
// reference's unbounded deltaEntries map.  side: 0 increments, 1 decrements, 2 placeholder.
__device__ __forceinline__ void dl_record_counter(const St32& s, uint32_t kind, uint32_t side, uint64_t v) {
  const uint32_t e0 = dl_env(kind), x = e0 + 2u * AGX_DELTA_ENV_WORDS + 3u * side;
  const uint32_t q = s.ld(e0 + 8) + 1u;
  s.put(e0 + 8, q);
  s.put(x, q);
  if (side < 2u) {
    s.put(x + 1, (uint32_t)v);
    s.put(x + 2, (uint32_t)(v >> 32));
  }
}

// DeltaPropagation row of seqNrs (j, ctr]: collectPropagations' merged group (DeltaOp.merge: runs of
// AddDeltaOps coalesce) or a NoDeltaPlaceholder (max-delta-size reached / a no-delta update).
__device__ __forceinline__ bool dl_group_row(const DevParams& P, const St32& s, uint32_t kind, uint32_t node, uint32_t j,
                                             uint32_t* row) {
  const uint32_t e0 = dl_env(kind), ctr = s.ld(e0 + 8);
  row[0] = 0;  // (rows are recycled: every field the receiver reads is written)
  row[1] = node;
  row[2] = j + 1u;
  row[3] = ctr;
#pragma unroll
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) row[4 + n] = s.ld(e0 + n);
  bool ph = false;
  if (kind != AGX_KIND_ORSET) {  // GCounter / PNCounter: slot max over the range (dl_record_counter)
    const uint32_t x = e0 + 2u * AGX_DELTA_ENV_WORDS;
    const uint32_t q0 = s.ld(x), q1 = s.ld(x + 3);
    ph = s.ld(x + 6) > j;
    row[12] = (q0 > j ? 1u : 0u) | (q1 > j ? 2u : 0u);
    row[13] = q0 > j ? s.ld(x + 1) : 0u;
    row[14] = q0 > j ? s.ld(x + 2) : 0u;
    row[15] = q1 > j ? s.ld(x + 4) : 0u;
    row[16] = q1 > j ? s.ld(x + 5) : 0u;
  } else {
    uint32_t o = 12, nops = 0, hdr = 0, cnt = 0, vmax = 0;
    bool last_add = false;
    // the range's entries four at a time, their (type, version) words loaded together: the row stores
    // between entries would otherwise order one log round trip per seqNr
    constexpr uint32_t kQ = 4;
    for (uint32_t q0 = j + 1; q0 <= ctr && !ph; q0 += kQ) {
      uint32_t tev[kQ], verv[kQ];
#pragma unroll
      for (uint32_t u = 0; u < kQ; ++u) {
        const uint32_t x = dl_entry(kind, q0 + u);
        tev[u] = q0 + u <= ctr ? s.ld(x + 1) : 0u;
        verv[u] = q0 + u <= ctr ? s.ld(x + 2) : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < kQ; ++u) {
        const uint32_t q = q0 + u;
        if (ph || q > ctr) break;
        const uint32_t x = dl_entry(kind, q), te = tev[u], t = te & 0xFFu, ver = verv[u];
        if (t == 1u && last_add) {  // AddDeltaOp.merge(AddDeltaOp): one more (element, version)
          if (nops >= P.delta_max) {  // (max-delta-size 1: even one coalesced AddDeltaOp is too large)
            ph = true;
            break;
          }
          row[o++] = te >> 8;
          row[o++] = ver;
          ++cnt;
          vmax = ver;
          continue;
        }
        if (last_add) row[hdr] = 1u | (cnt << 8), row[hdr + 1] = vmax;  // close the add run
        if (q > j + 1 && nops + 1u >= P.delta_max) {  // deltaSize >= maxDeltaSize
          ph = true;
          break;
        }
        ++nops;
        last_add = t == 1u;
        if (last_add) {
          hdr = o;
          o += 2;
          row[o++] = te >> 8;
          row[o++] = ver;
          cnt = 1;
          vmax = ver;
        } else {
          row[o++] = t | ((t == 2u ? 1u : 0u) << 8);
          if (t == 2u) {
            row[o++] = te >> 8;
            row[o++] = ver;
          }
          uint32_t vv[AGX_CRDT_NODES];
#pragma unroll
          for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) vv[n] = s.ld(x + 4 + n);
#pragma unroll
          for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) row[o++] = vv[n];
        }
      }
    }
    if (!ph && last_add) row[hdr] = 1u | (cnt << 8), row[hdr + 1] = vmax;
    row[0] = nops;
    if (!ph) row[P.pw - 1] = o;  // the row's used length (a queued group's row is copied forward that far)
  }
  if (ph) row[0] = 0x80000000u;
  return ph;
}

// ORSet: apply one received DeltaPropagation group (mergeDelta, DD/ORSet.scala:455-501).  lvv: the
// replica's vvector, loaded by the caller with the row's header.  Loads are issued in batches before
// the stores they precede (state and row may alias as far as the compiler knows: a load after a store
// would cost one memory round trip per element).
__device__ __forceinline__ void orset_merge_delta_row(const St32& s, const uint32_t* row, uint32_t from,
                                                      uint32_t (&lvv)[AGX_CRDT_NODES]) {
  constexpr uint32_t vb = AGX_ORSET_ELEMS * AGX_CRDT_NODES;  // u32 index of the vvector
  constexpr uint32_t kB = 4;                                 // elements per batch
  const uint32_t nops = row[0];
  uint32_t o = 12;
  for (uint32_t i = 0; i < nops; ++i) {
    const uint32_t h = row[o], t = h & 0xFFu, cnt = h >> 8;
    if (t == 1u) {  // dryMerge(addDeltaOp = true): the run's elements only, the last pair of an element wins
      const uint32_t vf = row[o + 1];
      const uint32_t p0 = o + 2;
      uint64_t seen = 0;
      for (uint32_t k1 = cnt; k1 > 0;) {  // batches of pairs from the run's end
        const uint32_t k0 = k1 > kB ? k1 - kB : 0u;
        uint32_t pe[kB], pv[kB];
#pragma unroll
        for (uint32_t u = 0; u < kB; ++u) {
          pe[u] = k0 + u < k1 ? row[p0 + 2 * (k0 + u)] : 0u;
          pv[u] = k0 + u < k1 ? row[p0 + 2 * (k0 + u) + 1] : 0u;
        }
        bool keep[kB];
#pragma unroll
        for (uint32_t u = kB; u-- > 0;) {  // (descending: a later pair of the batch wins)
          keep[u] = k0 + u < k1 && !((seen >> pe[u]) & 1ull);
          if (keep[u]) seen |= 1ull << pe[u];
        }
        uint64_t dw[kB][4];
#pragma unroll
        for (uint32_t u = 0; u < kB; ++u)
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) dw[u][k] = keep[u] ? s.st[(size_t)(4 * pe[u] + k) * s.nl] : 0ull;
#pragma unroll
        for (uint32_t u = 0; u < kB; ++u) {
          if (!keep[u]) continue;
          const uint32_t e = pe[u], ver = pv[u];
          bool here = false;
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) here |= dw[u][k] != 0ull;
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) {
            uint32_t x2[2];
#pragma unroll
            for (uint32_t h2 = 0; h2 < 2; ++h2) {
              const uint32_t n = 2 * k + h2, d = (uint32_t)(dw[u][k] >> (32 * h2));
              const uint32_t r = n == from ? ver : 0u, rvv = n == from ? vf : 0u;
              x2[h2] = here ? orset_merge_entry(d, r, lvv[n], rvv) : (r > lvv[n] ? r : 0u);
            }
            const uint64_t nw = ((uint64_t)x2[1] << 32) | x2[0];
            if (nw != dw[u][k]) s.st[(size_t)(4 * e + k) * s.nl] = nw;
          }
        }
        k1 = k0;
      }
#pragma unroll
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
        if (n == from && vf > lvv[n]) {
          lvv[n] = vf;
          s.put(vb + n, vf);
        }
      o = p0 + 2 * cnt;
    } else if (t == 2u) {  // mergeRemoveDelta
      const uint32_t e = row[o + 1], ver = row[o + 2];
      const uint32_t* rvv = row + o + 3;
      uint32_t d[AGX_CRDT_NODES];
      bool here = false, del = true;
#pragma unroll
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) {
        d[n] = s.ld(e * AGX_CRDT_NODES + n);
        here |= d[n] != 0u;
        del &= d[n] <= rvv[n];  // covered on every node (an unknown node has rvv 0)
      }
      if (here && del)
#pragma unroll
        for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
          if (d[n]) s.put(e * AGX_CRDT_NODES + n, 0u);
#pragma unroll
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
        if (n == from && ver > lvv[n]) {
          lvv[n] = ver;
          s.put(vb + n, ver);
        }
      o += 11;
    } else {  // FullStateDeltaOp: dryMerge(addDeltaOp = false) with an empty elementsMap
      uint32_t rvv[AGX_CRDT_NODES];
#pragma unroll
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) rvv[n] = row[o + 1 + n];
      for (uint32_t e0 = 0; e0 < AGX_ORSET_ELEMS; e0 += kB) {
        uint64_t dw[kB][4];
#pragma unroll
        for (uint32_t u = 0; u < kB; ++u)
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) dw[u][k] = s.st[(size_t)(4 * (e0 + u) + k) * s.nl];
#pragma unroll
        for (uint32_t u = 0; u < kB; ++u)
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) {
            uint32_t x2[2];
#pragma unroll
            for (uint32_t h2 = 0; h2 < 2; ++h2) {
              const uint32_t n = 2 * k + h2, x = (uint32_t)(dw[u][k] >> (32 * h2));
              x2[h2] = x && x <= rvv[n] ? 0u : x;
            }
            const uint64_t nw = ((uint64_t)x2[1] << 32) | x2[0];
            if (nw != dw[u][k]) s.st[(size_t)(4 * (e0 + u) + k) * s.nl] = nw;
          }
      }
#pragma unroll
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n)
        if (rvv[n] > lvv[n]) {
          lvv[n] = rvv[n];
          s.put(vb + n, rvv[n]);
        }
      o += 9;
    }
  }
}

// a received DeltaPropagation (receiveDeltaPropagation + DataEnvelope.merge)
__device__ __forceinline__ void dl_receive(const St32& s, uint32_t kind, const uint32_t* row) {
  if (kind == AGX_KIND_ORSET) {  // header, sender's deltaVersion and the vvector in one round trip
    constexpr uint32_t vb = AGX_ORSET_ELEMS * AGX_CRDT_NODES;
    const uint32_t e0 = dl_env(kind);
    const uint32_t h0 = row[0], from = row[1], lo = row[2], hi = row[3];
    uint32_t lvv[AGX_CRDT_NODES], dv[AGX_CRDT_NODES];
#pragma unroll
    for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) {
      lvv[n] = s.ld(vb + n);
      dv[n] = s.ld(e0 + n);
    }
    if (h0 & 0x80000000u) return;  // NoDeltaPlaceholder: not part of the propagation
    uint32_t cur = 0;
#pragma unroll
    for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) cur = n == from ? dv[n] : cur;
    if (cur >= hi || lo > cur + 1u) return;  // already handled / a seqNr is missing
    orset_merge_delta_row(s, row, from, lvv);
    s.put(e0 + from, hi);  // deltaVersions.merge(VersionVector(fromNode, toSeqNr))
    return;
  }
  if (row[0] & 0x80000000u) return;  // NoDeltaPlaceholder: not part of the propagation
  const uint32_t e0 = dl_env(kind), from = row[1];
  // not RequiresCausalDeliveryOfDeltas: merge the sender's envelope
  for (uint32_t b = 0; b < 2; ++b)
    if (row[12] & (1u << b)) {
      uint64_t* slot = s.st + (size_t)(b * AGX_CRDT_NODES + from) * s.nl;
      const uint64_t x = ((uint64_t)row[14 + 2 * b] << 32) | row[13 + 2 * b];
      if (x > *slot) *slot = x;
    }
#pragma unroll
  for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) {
    const uint32_t c = s.ld(e0 + n);
    if (row[4 + n] > c) s.put(e0 + n, row[4 + n]);
  }
}

// DeltaPropagationTick (DD/Replicator.scala:1953-1963); returns the row cursor advance
template <typename Emit>
__device__ __forceinline__ void dl_tick(const DevParams& P, const CrdtHeap& H, uint32_t kind, uint32_t self,
                                        const St32& s, uint32_t arg, uint32_t& row_cursor, Emit& em) {
  const uint32_t k = arg & 0xFFFFu;
  if (arg & AGX_DELTA_WRITE) {  // a writer client: one seeded Update told to the replica
    const uint64_t r = fanout_rand(P.gossip_seed, self, k | 0x04000000u, 0);
    const uint32_t amount = 1u + (uint32_t)((r >> 32) & 3u);
    uint32_t op;
    if (kind == AGX_KIND_GCOUNTER) op = AGX_OP(AGX_OP_INCREMENT, amount);
    else if (kind == AGX_KIND_PNCOUNTER) op = AGX_OP(((r >> 34) & 1u) ? AGX_OP_DECREMENT : AGX_OP_INCREMENT, amount);
    else op = AGX_OP(((r >> 40) & 3u) ? AGX_OP_ADD : AGX_OP_REMOVE, (uint32_t)(r >> 48) % AGX_ORSET_ELEMS);
    em(self, op);
  }
  const uint32_t node = self % AGX_CRDT_NODES, na = key_size(self, P.n_global) - 1u;
  if (na) {
    const uint32_t e0 = dl_env(kind), rr = s.ld(e0 + 9), ctr = s.ld(e0 + 8);
    const uint32_t sz = dl_slice_size(na), cnt = na <= sz ? na : sz;
    const uint32_t tag = ((kind - (uint32_t)AGX_KIND_GCOUNTER) << 30) | AGX_DELTA_ROW_BIT;
    for (uint32_t i = 0; i < cnt; ++i) {
      const uint32_t x = dl_slice_node(node, na, sz, rr, i);
      const uint32_t j = s.ld(e0 + 10 + x);
      if (ctr <= j) continue;  // deltaEntriesAfter(j) is empty
      const uint32_t h = row_cursor++;
      const bool ph = h < H.rows && dl_group_row(P, s, kind, node, j, H.wrow(h));
      s.put(e0 + 10 + x, ctr);  // deltaSentToNode(node) = last seqNr (also for a placeholder)
      // createDeltaPropagation leaves NoDeltaPlaceholder out (DD/Replicator.scala:1364) and nothing is
      // sent for an empty propagation (:1957): the group's slot (counted by phase A) stays void and
      // is compacted out of the bucket's tells (bucket_finish)
      if (ph) em.void_slot();
      else em.wide(self - node + x, tag | h);
    }
    s.put(e0 + 9, rr + sz);  // deltaNodeRoundRobinCounter += sliceSize
  }
  if (k > 0) em(self, AGX_OP(AGX_OP_DELTA_TICK, (k - 1u) | (arg & AGX_DELTA_WRITE)));
}


// Phase B message classes for the wave's schedule (bucket_finish, kCrdtSched): 0 a DeltaPropagation,
// 1 a full-state gossip, 2 a DeltaPropagationTick, 3 a GossipTick, 4 any other op (an update)
#ifndef AGX_CRDT_SCHED
#define AGX_CRDT_SCHED 1
#endif
constexpr bool kCrdtSched = AGX_CRDT_SCHED != 0;
__device__ __forceinline__ uint32_t crdt_class(uint32_t src, uint32_t pay) {
  if (is_wide(src)) return (pay & AGX_DELTA_ROW_BIT) ? 0u : 1u;
  const uint32_t op = pay >> 24;
  return op == AGX_OP_DELTA_TICK ? 2u : op == AGX_OP_GOSSIP ? 3u : 4u;
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
  if constexpr ((CM & ~kDeltaKM) == (1u << AGX_KIND_GCOUNTER)) kind = AGX_KIND_GCOUNTER;
  if constexpr ((CM & ~kDeltaKM) == (1u << AGX_KIND_PNCOUNTER)) kind = AGX_KIND_PNCOUNTER;
  if constexpr ((CM & ~kDeltaKM) == (1u << AGX_KIND_ORSET)) kind = AGX_KIND_ORSET;
  const size_t nl = wide_nl(P);
  uint64_t* st = wide_state(P, l);  // word w at st[w * nl] (actor-major row, or word-major: AGX_CRDT_WORDMAJOR)
  const uint32_t node = self % AGX_CRDT_NODES;
  const bool dm = (CM & kDeltaKM) != 0 && P.delta_max != 0;  // (the engine launches kDeltaKM variants then)
  const St32 s32{st, nl};
  if (is_wide(src)) {
    if ((pay >> 30) != kind - (uint32_t)AGX_KIND_GCOUNTER) return AGX_RES_UNHANDLED;  // another data type
    const uint32_t* row = H.row(pay & kHandleMask);
    if (pay & AGX_DELTA_ROW_BIT) {  // a DeltaPropagation
      if (!dm) return AGX_RES_UNHANDLED;
      dl_receive(s32, kind, row);
      return AGX_RES_SAME;
    }
    if (dm) {  // DataEnvelope.merge: the deltaVersions after the data words
      const uint32_t e0 = dl_env(kind), r0 = row_dv(kind);
#pragma unroll
      for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) {
        const uint32_t c = s32.ld(e0 + n), r = row[r0 + n];
        if (r > c) s32.put(e0 + n, r);
      }
    }
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
      rvv[2 * k] = row[kSparseSerial ? kOrRowVV + 2 * k : 2 * (vw + k)];
      rvv[2 * k + 1] = row[kSparseSerial ? kOrRowVV + 2 * k + 1 : 2 * (vw + k) + 1];
    }
#ifndef AGX_ORSET_BATCH
#define AGX_ORSET_BATCH 2
#endif
    constexpr uint32_t kE = AGX_ORSET_BATCH;  // elements per batch (8 row words + 4 state words each)
    uint32_t ro = kOrRowDots;                 // (kSparseSerial) next live dot of the sparse row
    for (uint32_t e0 = 0; e0 < AGX_ORSET_ELEMS; e0 += kE) {
      uint4 ra[kE], rb[kE];
      uint32_t rm[kE];
      uint64_t s[kE][4];
#pragma unroll
      for (uint32_t u = 0; u < kE; ++u) {
        if (kSparseSerial) {
          rm[u] = reinterpret_cast<const uint8_t*>(row + kOrRowMask)[e0 + u];
        } else {
          ra[u] = *reinterpret_cast<const uint4*>(row + 8 * (e0 + u));
          rb[u] = *reinterpret_cast<const uint4*>(row + 8 * (e0 + u) + 4);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) s[u][k] = st[(size_t)(4 * (e0 + u) + k) * nl];
      }
#pragma unroll
      for (uint32_t u = 0; u < kE; ++u) {
        uint32_t r[8];
        if (kSparseSerial) {
#pragma unroll
          for (int n = 0; n < 8; ++n) r[n] = (rm[u] >> n) & 1u ? row[ro++] : 0u;
        } else {
          r[0] = ra[u].x, r[1] = ra[u].y, r[2] = ra[u].z, r[3] = ra[u].w;
          r[4] = rb[u].x, r[5] = rb[u].y, r[6] = rb[u].z, r[7] = rb[u].w;
        }
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
    case AGX_OP_DECREMENT: {
      if (kind == AGX_KIND_ORSET || (op == AGX_OP_DECREMENT && kind != AGX_KIND_PNCOUNTER)) return AGX_RES_UNHANDLED;
      const uint32_t w = (op == AGX_OP_DECREMENT ? AGX_CRDT_NODES : 0u) + node;
      const uint64_t v = st[w * nl] + arg;
      if (v < arg) atomicOr(P.err, 2ull);  // kErrRange: the reference's BigInt slot would not wrap
      st[w * nl] = v;
      if (dm)  // delta = the counter of the new slot value; an update by 0 has none (placeholder)
        dl_record_counter(s32, kind, arg ? (op == AGX_OP_DECREMENT ? 1u : 0u) : 2u, v);
      return AGX_RES_SAME;
    }
    case AGX_OP_ADD:
    case AGX_OP_REMOVE:
    case AGX_OP_CLEAR: {
      if (kind != AGX_KIND_ORSET || (op != AGX_OP_CLEAR && arg >= AGX_ORSET_ELEMS)) return AGX_RES_UNHANDLED;
      if (dm) {  // AddDeltaOp (element, dot) / RemoveDeltaOp (element, deltaDot, vvector) / FullStateDeltaOp
        constexpr uint32_t vb = AGX_ORSET_ELEMS * AGX_CRDT_NODES;
        const uint32_t x = dl_record(P, s32, kind, self);
        const uint32_t vn = s32.ld(vb + node);
        s32.put(x + 1, (op == AGX_OP_ADD ? 1u : op == AGX_OP_REMOVE ? 2u : 3u) | (op == AGX_OP_CLEAR ? 0u : arg << 8));
        s32.put(x + 2, op == AGX_OP_ADD ? vn + 1u : op == AGX_OP_REMOVE ? vn : 0u);
        s32.put(x + 3, 0u);
        if (op != AGX_OP_ADD)
#pragma unroll
          for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) s32.put(x + 4 + n, s32.ld(vb + n));
      }
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
    case AGX_OP_DELTA_TICK:
      if (!dm) return AGX_RES_UNHANDLED;
      dl_tick(P, H, kind, self, s32, arg, row_cursor, em);
      return AGX_RES_SAME;
    case AGX_OP_GOSSIP: {
      const uint32_t f = P.n_global > 1 && (!dm || key_size(self, P.n_global) > 1) ? P.gossip_f : 0u;
      if (f) {
        const uint32_t h = row_cursor++;
        if (kSparseSerial && h < H.rows && kind == AGX_KIND_ORSET) {  // sparse snapshot (kOrRow*)
          uint32_t* row = H.wrow(h);
          const uint32_t vw = AGX_ORSET_ELEMS * AGX_CRDT_NODES / 2;
          uint32_t o = kOrRowDots;
          for (uint32_t e0 = 0; e0 < AGX_ORSET_ELEMS; e0 += 4) {  // four elements' dots (one mask word) per batch
            uint64_t d[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int k = 0; k < 4; ++k) d[u][k] = st[(size_t)(4 * (e0 + u) + k) * nl];
            uint32_t mw = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int n = 0; n < 8; ++n) {
                const uint32_t x = (uint32_t)(d[u][n >> 1] >> (32 * (n & 1)));
                if (x) {
                  row[o++] = x;
                  mw |= 1u << (8 * u + n);
                }
              }
            row[kOrRowMask + e0 / 4] = mw;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint64_t v = st[(vw + k) * nl];
            row[kOrRowVV + 2 * k] = (uint32_t)v;
            row[kOrRowVV + 2 * k + 1] = (uint32_t)(v >> 32);
          }
          if (dm)
#pragma unroll
            for (uint32_t n = 0; n < AGX_CRDT_NODES; ++n) row[kOrRowDV + n] = s32.ld(dl_env(kind) + n);
        } else if (h < H.rows) {  // snapshot of the current state (+ deltaVersions), shared by the f gossips
          uint32_t* row = H.wrow(h);
          const uint32_t nw = crdt_words(kind) + (dm ? AGX_CRDT_NODES / 2u : 0u);  // batches of 4 (loads first)
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
        for (uint32_t j = 0; j < f; ++j)
          em.wide(dm ? crdt_key_peer(P.gossip_seed, self, arg, j, P.n_global) : crdt_peer(P.gossip_seed, self, arg, j, P.n_global),
                  tagged);
      }
      if (arg > 0) em(self, AGX_OP(AGX_OP_GOSSIP, arg - 1u));
      return AGX_RES_SAME;
    }
    default:
      return AGX_RES_UNHANDLED;
  }
}

// ORSet-only populations with full-state gossip: one replica's drain run (nd messages in order)
// in two passes.  orset_protocol (one lane per replica): emissions and snapshot-row allocation in
// message order, the unhandled count.  orset_merge_wave (the whole wave on one replica, lane e =
// element e of the 64-element universe): the replica's 2 KB of dots, every merged row and every
// snapshot row move as whole contiguous rows (one 32-B slice per lane), and each message of the run
// is applied to all elements at once -- message q sees the state left by messages < q (per element;
// the version-vector chain is uniform across the lanes).  Same results as nd calls of
// crdt_apply<kb(ORSET)>.
constexpr uint32_t kOrMerge = 1, kOrAdd = 2, kOrRemove = 3, kOrClear = 4, kOrSnap = 5;
__device__ __forceinline__ uint32_t orset_code(uint32_t sv, uint32_t pv) {
  if (is_wide(sv)) return (pv >> 30) == (uint32_t)(AGX_KIND_ORSET - AGX_KIND_GCOUNTER) && !(pv & AGX_DELTA_ROW_BIT) ? kOrMerge : 0u;
  const uint32_t op = pv >> 24, arg = pv & 0xFFFFFFu;
  if (op == AGX_OP_ADD) return arg < AGX_ORSET_ELEMS ? kOrAdd : 0u;
  if (op == AGX_OP_REMOVE) return arg < AGX_ORSET_ELEMS ? kOrRemove : 0u;
  if (op == AGX_OP_CLEAR) return kOrClear;
  if (op == AGX_OP_GOSSIP) return kOrSnap;
  return 0u;
}

// pass 1 (per lane): returns the unhandled count; *state_work: the run reads or writes the state
template <typename Emit, typename Src, typename Pay>
__device__ __forceinline__ uint32_t orset_protocol(const DevParams& P, uint32_t self, uint32_t s0, uint32_t nd,
                                                   const Src& isrc, const Pay& ipay, uint32_t& row_cursor, Emit& em,
                                                   bool* state_work) {
  const uint32_t f = P.n_global > 1 ? P.gossip_f : 0u;
  uint32_t nunh = 0, nmod = 0;
  const uint32_t rc0 = row_cursor;
  for (uint32_t q = 0; q < nd; ++q) {
    const uint32_t sv = isrc(s0 + q), pv = ipay(s0 + q);
    const uint32_t c = orset_code(sv, pv);
    if (c == 0) {
      ++nunh;
      continue;
    }
    if (c != kOrSnap) {
      ++nmod;
      continue;
    }
    const uint32_t arg = pv & 0xFFFFFFu;
    if (f) {
      const uint32_t tagged = ((uint32_t)(AGX_KIND_ORSET - AGX_KIND_GCOUNTER) << 30) | row_cursor++;
      for (uint32_t j = 0; j < f; ++j) em.wide(crdt_peer(P.gossip_seed, self, arg, j, P.n_global), tagged);
    }
    if (arg > 0) em(self, AGX_OP(AGX_OP_GOSSIP, arg - 1u));
  }
  *state_work = nmod != 0 || row_cursor != rc0;
  return nunh;
}

// pass 2 (wave-uniform arguments, all 64 lanes converged): the run's state effects, rows from rc0
template <typename Src, typename Pay>
__device__ __forceinline__ void orset_merge_wave(const DevParams& P, const CrdtHeap& H, uint32_t l, uint32_t node,
                                                 uint32_t s0, uint32_t nd, uint32_t rc0, const Src& isrc,
                                                 const Pay& ipay) {
  static_assert(AGX_ORSET_ELEMS == kWave, "one lane per ORSet element");
  constexpr uint32_t vw = AGX_ORSET_ELEMS * AGX_CRDT_NODES / 2;  // first vvector word
  const uint32_t e = lane_id();
  const uint32_t f = P.n_global > 1 ? P.gossip_f : 0u;
  uint64_t* st = wide_state(P, l);
  uint4* se = reinterpret_cast<uint4*>(st + 4 * e);  // element e: 8 u32 dots = 2 x 16 B
  const uint4* sv4 = reinterpret_cast<const uint4*>(st + vw);
  const uint4 a0 = se[0], a1 = se[1], v0 = sv4[0], v1 = sv4[1];
  uint32_t d[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  const uint32_t vv0[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  uint32_t cur[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) cur[n] = vv0[n];
  bool dirty = false;
  uint32_t h = rc0;
  for (uint32_t q = 0; q < nd; ++q) {
    const uint32_t sv = isrc(s0 + q), pv = ipay(s0 + q);
    const uint32_t c = orset_code(sv, pv);
    const uint32_t arg = pv & 0xFFFFFFu;
    if (c == kOrMerge) {  // ORSet.merge: dots per (element, node) against both vvectors, then vvector max
      const uint32_t* row = H.row(pv & kHandleMask);
      // sparse row: element e's live dots start after the earlier elements' (a wave prefix count)
      const uint32_t rm = reinterpret_cast<const uint8_t*>(row + kOrRowMask)[e];
      const uint32_t rc = __popc(rm);
      uint32_t ro = kOrRowDots + wave_incl_sum(rc) - rc;
      const uint4 va = *reinterpret_cast<const uint4*>(row + kOrRowVV), vb = *reinterpret_cast<const uint4*>(row + kOrRowVV + 4);
      uint32_t r[8];
#pragma unroll
      for (int n = 0; n < 8; ++n) r[n] = (rm >> n) & 1u ? row[ro++] : 0u;
      const uint32_t rvv[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        const uint32_t o = orset_merge_entry(d[n], r[n], cur[n], rvv[n]);
        dirty |= o != d[n];
        d[n] = o;
      }
#pragma unroll
      for (int n = 0; n < 8; ++n) cur[n] = max(cur[n], rvv[n]);
    } else if (c == kOrAdd || c == kOrRemove || c == kOrClear) {
      uint32_t ver = 0;
      if (c == kOrAdd) {  // vvector + node; birth dot (node -> new version)
#pragma unroll
        for (uint32_t n = 0; n < 8; ++n)
          if (n == node) ver = cur[n] = cur[n] + 1u;
      }
      if (c == kOrClear || arg == e) {
#pragma unroll
        for (uint32_t n = 0; n < 8; ++n) d[n] = (c == kOrAdd && n == node) ? ver : 0u;
        dirty = true;
      }
    } else if (c == kOrSnap && f) {  // snapshot row: element e per lane, the vvector from lane 0
      const uint32_t hr = h++;
      if (hr < H.rows) {  // sparse row (kOrRow*): lane e's node mask byte and its live dots
        uint32_t* row = H.wrow(hr);
        uint32_t m = 0;
#pragma unroll
        for (int n = 0; n < 8; ++n) m |= d[n] ? 1u << n : 0u;
        const uint32_t cnt = __popc(m);
        uint32_t o = kOrRowDots + wave_incl_sum(cnt) - cnt;
        reinterpret_cast<uint8_t*>(row + kOrRowMask)[e] = (uint8_t)m;
#pragma unroll
        for (int n = 0; n < 8; ++n)
          if (d[n]) row[o++] = d[n];
        if (e == 0) {
          *reinterpret_cast<uint4*>(row + kOrRowVV) = make_uint4(cur[0], cur[1], cur[2], cur[3]);
          *reinterpret_cast<uint4*>(row + kOrRowVV + 4) = make_uint4(cur[4], cur[5], cur[6], cur[7]);
        }
      }
    }
  }
  if (dirty) {
    se[0] = make_uint4(d[0], d[1], d[2], d[3]);
    se[1] = make_uint4(d[4], d[5], d[6], d[7]);
  }
  bool vch = false;
#pragma unroll
  for (int n = 0; n < 8; ++n) vch |= cur[n] != vv0[n];
  if (vch && e == 0) {
    uint4* vo = reinterpret_cast<uint4*>(st + vw);
    vo[0] = make_uint4(cur[0], cur[1], cur[2], cur[3]);
    vo[1] = make_uint4(cur[4], cur[5], cur[6], cur[7]);
  }
}

}  // namespace agx
