// agx_kernels.h — the superstep kernels (gfx950, wave64, integer only, no MFMA).
//
// One BSP superstep replaces one round of Mailbox.run/processMailbox over every
// scheduled mailbox (akka-actor/src/main/scala/akka/dispatch/Mailbox.scala:227-277).
// Actors are grouped in buckets of 2^bb consecutive local ids (bb <= kBucketBits, chosen per
// engine: agx_cfg.bucket_actors); one bucket's inbox up to one LDS tile takes the fast path.
//
//   k_bucket_apply     per bucket: stable in-bucket counting sort of its mail by
//                      actor (LDS wave multisplit), segmented drain with the
//                      throughput cap and bounded-mailbox tail-drop, behaviour
//                      apply (ActorCell.invoke), scan-compacted emission of the
//                      next step's tells into a per-bucket chunk, and the chunk's
//                      digit histogram for the next step's first radix pass.
//   k_chunk_rowscan    per digit: exclusive prefix of the chunk histograms.
//   k_chunk_downsweep  stable LSD radix pass that reads the chunk list
//                      [backlog chunks][tell chunks][host-staged tells] directly
//                      (no separate compaction) and groups mail by bucket.
//   k_sort_upsweep / k_sort_rowscan / k_sort_downsweep
//                      the same pass over a dense array (later digits, and the
//                      multi-GPU path after the RCCL exchange).
//   k_dense_fused / k_dense_apply
//                      (round 5) buckets with at most one message per actor, applied from
//                      registers in actor order with no in-bucket sort (fused superstep /
//                      multi-pass); every other bucket is marked for k_bucket_apply.
//   k_tiny_apply       one wave per bucket with a few messages (multi-pass, sparse supersteps).
//
// Envelopes are SoA u32 {key, src, payload} = 12 B.
#pragma once
#include "agx_crdt.h"
#include "agx_device.h"

namespace agx {

// ---------------------------------------------------------------- geometry
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr int kIpt = 8;
constexpr int kTile = kThreads * kIpt;  // 2048 envelopes per sort tile

constexpr int kBucketBits = 11;            // widest bucket (the LDS per-actor arrays' size)
constexpr int kBucket = 1 << kBucketBits;  // max actors per bucket = messages per apply tile
constexpr int kMinBucketBits = 5;

constexpr int kRadixBits = 9;  // max digit width of one pass
constexpr int kRadix = 1 << kRadixBits;

constexpr int kScanThreads = 1024;
constexpr int kStagedChunks = 256;  // host-staged tells are split over this many chunks

// stats slots (u64) on device
enum { ST_DELIVERED = 0, ST_DEAD = 1, ST_UNHANDLED = 2, ST_EMITTED = 3, ST_STEPS = 4, ST_ERROR = 5, ST_ACTIVE = 6,
       ST_IDENT = 7, ST_N = 8 };
constexpr uint64_t kErrCapacity = 1;
constexpr uint64_t kErrRange = 2;  // a counter slot wrapped past 2^64 - 1 (AGX_ERANGE)
constexpr uint64_t kErrBarrier = 4;  // a persistent superstep launch's grid barrier timed out (AGX_EDEVICE)
// per-block counters of k_bucket_apply: delivered, dead, unhandled, emitted, active
constexpr int kBStats = 5;
constexpr uint32_t kMaxApplyGrid = 4096;

struct Msgs {
  uint32_t* key;
  uint32_t* src;
  uint32_t* pay;
};
struct CMsgs {
  const uint32_t* key;
  const uint32_t* src;
  const uint32_t* pay;
};

__device__ __forceinline__ uint32_t div_up(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// A new superstep begins: bump the step counter and reset the snapshot rows of
// heap[step & 1] (their gossips were consumed or copied forward two steps ago).
__device__ __forceinline__ void begin_step(uint32_t* step, uint32_t* heap_top) {
  if (threadIdx.x == 0 && step) {
    const uint32_t s = *step + 1u;
    *step = s;
    heap_top[s & 1u] = 0u;
  }
}

// Commit Behaviors.stopped results of the previous apply: alive[l] = 0.
// (k_bucket_apply never writes `alive`, so every block classifies against the
// alive-at-step-start value — deterministic across block schedules.)
__device__ __forceinline__ void commit_stops(uint8_t* alive, const uint32_t* stopq, uint32_t* nstop) {
  const uint32_t ns = *nstop;
  for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) alive[stopq[i]] &= 0xFEu;  // (bits 1..3: mailbox class)
  __syncthreads();
  if (threadIdx.x == 0) *nstop = 0;
}
static __global__ void __launch_bounds__(kScanThreads) k_commit_stops(uint8_t* alive, const uint32_t* stopq, uint32_t* nstop) {
  commit_stops(alive, stopq, nstop);
}

// Chunk list written by k_bucket_apply (nb buckets):
//   chunk b          backlog of bucket b        (in the bl arena)
//   chunk nb + b     tells emitted by bucket b  (in the em arena)
//   chunk 2nb        host-staged tells          (staging buffer)
struct Chunks {
  CMsgs bl, em, st;
  const uint32_t* off;
  const uint32_t* cnt;
  uint32_t nb;
  __device__ __forceinline__ const CMsgs& arena(uint32_t c) const { return c < nb ? bl : (c < 2 * nb ? em : st); }
};

// =========================================================================
// Wave-level multisplit: rank of this lane's item among the wave's earlier
// items with the same digit (ballot match over the digit bits); `hist` is the
// wave's running per-digit count in LDS.
// =========================================================================
template <typename HT>
__device__ __forceinline__ uint32_t wave_rank(bool valid, uint32_t d, uint32_t bits, HT* hist, uint64_t lt_mask) {
  const uint64_t vm = __ballot(valid);
  if (vm == 0) return 0;  // uniform: no valid lane in this wave
  // lowest valid lane's digit; when every valid lane has it (local topologies), the match
  // mask is the valid mask and the per-bit ballots are skipped
  const uint32_t first = __builtin_amdgcn_readlane(d, vm ? (int)__builtin_ctzll(vm) : 0);
  uint64_t m = vm;
  if (__ballot(valid && d != first) != 0)
    for (uint32_t b = 0; b < bits; ++b) {
      const uint32_t bit = (d >> b) & 1u;
      const uint64_t bal = __ballot(bit);
      m &= bit ? bal : ~bal;
    }
  const uint32_t before = (uint32_t)__popcll(m & lt_mask);
  const uint32_t c = (uint32_t)__popcll(m);
  uint32_t old = 0;
  if (valid) old = hist[d];
  __builtin_amdgcn_wave_barrier();
  if (valid && before == 0) hist[d] = (HT)(old + c);
  __builtin_amdgcn_wave_barrier();
  return old + before;
}

// a wave-uniform pointer forced into SGPRs
template <typename T>
__device__ __forceinline__ T* sgpr_ptr(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}

// load through a global (address space 1) pointer: global_load, not flat_load, once the
// compiler has lost track of where a laundered pointer points
__device__ __forceinline__ uint32_t ldg(const uint32_t* p, uint32_t i) {
  return ((const __attribute__((address_space(1))) uint32_t*)p)[i];
}

// state words 0/1 (index < 2^29: n_local < 2^28) through a 32-bit byte offset from an SGPR base
__device__ __forceinline__ uint64_t ldg64(const uint64_t* base, uint32_t i) {
  return *(const __attribute__((address_space(1))) uint64_t*)((const __attribute__((address_space(1))) char*)base + (i << 3));
}
__device__ __forceinline__ void stg64(uint64_t* base, uint32_t i, uint64_t v) {
  *(__attribute__((address_space(1))) uint64_t*)((__attribute__((address_space(1))) char*)base + (i << 3)) = v;
}

// streaming (non-temporal) vector stores for the dense launches' state and tell stores (AGX_NT=0 A/B
// build knob: plain stores).  Same-box A/B, 1M ring: superstep 16.0 -> 14.7 us -- the bucket's
// write-once results stream out during the kernel instead of sitting dirty in L2 until its end
#ifndef AGX_NT
#define AGX_NT 1
#endif
__device__ __forceinline__ void st64x(uint64_t* base, uint32_t i, uint64_t v) {
  if constexpr (AGX_NT != 0)
    __builtin_nontemporal_store(v, (__attribute__((address_space(1))) uint64_t*)((__attribute__((address_space(1))) char*)base + (i << 3)));
  else
    stg64(base, i, v);
}
__device__ __forceinline__ void st32x(uint32_t* p, uint64_t i, uint32_t v) {
  if constexpr (AGX_NT != 0)
    __builtin_nontemporal_store(v, (__attribute__((address_space(1))) uint32_t*)p + i);
  else
    p[i] = v;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const uint32_t lane = lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// h[d] += 1 from every active lane.  When all active lanes share the digit (local
// topologies: a whole wave's tells go to one destination bucket) one lane adds the
// popcount instead of 64 serialised LDS atomics on one address.
__device__ __forceinline__ void lds_hist_inc(uint32_t* h, uint32_t d) {
  const uint64_t act = __ballot(1);
  const uint32_t first = __builtin_amdgcn_readfirstlane(d);
  if (__ballot(d == first) == act) {
    if (lane_id() == (uint32_t)__builtin_ctzll(act)) atomicAdd(&h[first], (uint32_t)__popcll(act));
  } else {
    atomicAdd(&h[d], 1u);
  }
}

// =========================================================================
// Stable multisplit of one tile (<= kTile items) by a radix digit: wave ballot
// ranks, LDS staging, coalesced scatter.  `S.base[d]` is the output position of
// the next item of digit d and is advanced by this tile's digit counts.
// =========================================================================
struct SplitLds {
  uint32_t* whist;            // [NT/64][kRadix] per-wave digit counts
  uint32_t* base;             // [kRadix] running output position per digit
  uint32_t* ldig;             // [kRadix] tile-local digit starts
  uint32_t* gadj;             // [kRadix] base - ldig
  uint32_t* scratch;          // NT/64 + 1
  uint32_t *key, *src, *pay;  // [kTile]
};

// `loc(q)` is the index in `src` of item q < cnt of the tile.  Every item is located first (LDS /
// arithmetic only), then all 3 x IPT loads are issued back to back with no branch around them (items
// past cnt read index 0 and are masked) -- a per-item locate-then-load left the compiler waiting for
// each item's loads before the next item's search.
template <int NT, class Loc>
__device__ __forceinline__ void split_tile_ld(const CMsgs& src, const Loc& loc, uint32_t cnt, const Msgs& out,
                                              uint32_t shift, uint32_t bits, const SplitLds& S) {
  constexpr int NW = NT / kWave, IPT = kTile / NT, DPT = kRadix / NT;
  const int tid = threadIdx.x, w = tid / kWave;
  const uint32_t lane = lane_id();
  const uint32_t mask = (1u << bits) - 1u, nd = 1u << bits;
  const uint64_t ltm = lanemask_lt();
  for (int i = tid; i < NW * kRadix; i += NT) S.whist[i] = 0;
  const uint32_t wbase = w * (IPT * kWave);
  uint32_t k[IPT], sv[IPT], pv[IPT], rk[IPT], ix[IPT];
#pragma unroll
  for (int r = 0; r < IPT; ++r) {
    const uint32_t q = wbase + r * kWave + lane;
    ix[r] = q < cnt ? loc(q) : 0u;
  }
  const uint32_t *Kp = sgpr_ptr(src.key), *Sp = sgpr_ptr(src.src), *Pp = sgpr_ptr(src.pay);
#pragma unroll
  for (int r = 0; r < IPT; ++r) {
    k[r] = ldg(Kp, ix[r]);
    sv[r] = ldg(Sp, ix[r]);
    pv[r] = ldg(Pp, ix[r]);
  }
#pragma unroll
  for (int r = 0; r < IPT; ++r)
    if (wbase + r * kWave + lane >= cnt) k[r] = 0xFFFFFFFFu;
  __syncthreads();  // (the histogram clear above is visible before the ranks' LDS updates)
#pragma unroll
  for (int r = 0; r < IPT; ++r) {
    const uint32_t q = wbase + r * kWave + lane;
    rk[r] = wave_rank(q < cnt, (k[r] >> shift) & mask, bits, S.whist + w * kRadix, ltm);
  }
  __syncthreads();
  uint32_t cd[DPT];
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const uint32_t d = tid + j * NT;
    uint32_t run = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const uint32_t c2 = S.whist[q * kRadix + d];
      S.whist[q * kRadix + d] = run;
      run += c2;
    }
    cd[j] = d < nd ? run : 0u;
    S.ldig[d] = cd[j];
  }
  __syncthreads();
  {  // tile-local digit starts: exclusive scan over kRadix digits, DPT per thread (blocked)
    uint32_t v[DPT], tot = 0;
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      v[j] = S.ldig[tid * DPT + j];
      tot += v[j];
    }
    __syncthreads();
    uint32_t t2;
    uint32_t ex = block_excl_sum<NT>(tot, S.scratch, &t2);
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      S.ldig[tid * DPT + j] = ex;
      ex += v[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const uint32_t d = tid + j * NT;
    if (d < nd) {
      S.gadj[d] = S.base[d] - S.ldig[d];
      S.base[d] += cd[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < IPT; ++r) {
    const uint32_t q = wbase + r * kWave + lane;
    if (q < cnt) {
      const uint32_t d = (k[r] >> shift) & mask;
      const uint32_t lp = S.ldig[d] + S.whist[w * kRadix + d] + rk[r];
      S.key[lp] = k[r];
      S.src[lp] = sv[r];
      S.pay[lp] = pv[r];
    }
  }
  __syncthreads();
  for (uint32_t lp = tid; lp < cnt; lp += NT) {
    const uint32_t kk = S.key[lp];
    const uint32_t g = S.gadj[(kk >> shift) & mask] + lp;
    out.key[g] = kk;
    out.src[g] = S.src[lp];
    out.pay[g] = S.pay[lp];
  }
  __syncthreads();
}

template <int NT>
__device__ __forceinline__ void split_tile(const CMsgs& in, uint32_t base, uint32_t cnt, const Msgs& out,
                                           uint32_t shift, uint32_t bits, const SplitLds& S) {
  split_tile_ld<NT>(in, [&](uint32_t q) -> uint32_t { return base + q; }, cnt, out, shift, bits, S);
}

// digit bases: s_dbase[d] = exclusive scan of tot[d] over digits; returns the total
__device__ __forceinline__ uint32_t digit_bases(const uint32_t* tot, uint32_t nd, uint32_t* s_dbase, uint32_t* scratch) {
  const int tid = threadIdx.x;
  for (uint32_t d = tid; d < kRadix; d += kThreads) s_dbase[d] = d < nd ? tot[d] : 0u;
  __syncthreads();
  const uint32_t v0 = s_dbase[2 * tid], v1 = s_dbase[2 * tid + 1];
  __syncthreads();
  uint32_t t;
  const uint32_t ex = block_excl_sum<kThreads>(v0 + v1, scratch, &t);
  s_dbase[2 * tid] = ex;
  s_dbase[2 * tid + 1] = ex + v0;
  __syncthreads();
  return t;
}

// Exclusive prefix, in place, of one digit row of a histogram table (len entries,
// row 16-byte aligned): 16 consecutive entries per thread per round, their four uint4 loads in
// flight together before the block scan (a row of up to 4096 entries -- the first pass's units at
// 10^7 actors -- is one round trip, not four).  Returns the row total.
__device__ __forceinline__ uint32_t scan_row(uint32_t* row, uint32_t len, uint32_t* scratch) {
  constexpr uint32_t kPer = 16;
  const int tid = threadIdx.x;
  uint32_t run = 0;
  for (uint32_t base = 0; base < len; base += kPer * kThreads) {
    const uint32_t i0 = base + kPer * tid;
    uint4 v[kPer / 4];
#pragma unroll
    for (uint32_t q = 0; q < kPer / 4; ++q) {
      const uint32_t j = i0 + 4 * q;
      v[q] = make_uint4(0, 0, 0, 0);
      if (j + 3 < len) {
        v[q] = reinterpret_cast<const uint4*>(row)[j / 4];
      } else if (j < len) {
        v[q].x = row[j];
        if (j + 1 < len) v[q].y = row[j + 1];
        if (j + 2 < len) v[q].z = row[j + 2];
      }
    }
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < kPer / 4; ++q) sum += v[q].x + v[q].y + v[q].z + v[q].w;
    uint32_t t;
    uint32_t ex = run + block_excl_sum<kThreads>(sum, scratch, &t);
#pragma unroll
    for (uint32_t q = 0; q < kPer / 4; ++q) {
      const uint32_t j = i0 + 4 * q;
      const uint4 o = make_uint4(ex, ex + v[q].x, ex + v[q].x + v[q].y, ex + v[q].x + v[q].y + v[q].z);
      ex += v[q].x + v[q].y + v[q].z + v[q].w;
      if (j + 3 < len) {
        reinterpret_cast<uint4*>(row)[j / 4] = o;
      } else if (j < len) {
        row[j] = o.x;
        if (j + 1 < len) row[j + 1] = o.y;
        if (j + 2 < len) row[j + 2] = o.z;
      }
    }
    run += t;
  }
  return run;
}

// =========================================================================
// First radix pass, reading the chunk list left by k_bucket_apply.
// Histogram columns ("units") group G consecutive buckets' chunks:
//   unit u <  ng        backlog chunks of buckets [uG, uG+G)
//   unit ng + u         tell chunks of buckets [uG, uG+G)
//   unit 2ng + c        host-staged chunk c
// k_bucket_apply adds its digit counts into its unit's column; the rowscan turns
// each digit row into an exclusive prefix over units; the downsweep block of unit
// u places that unit's chunks in order (canonical order preserved).
// =========================================================================
// Exclusive scan, in one block, of a table of `rows` rows x `len` entries (row stride
// `stride`) flattened row-major; each thread owns one contiguous range of the flattened
// index (all of its loads in flight before the block scan).  Writes the prefixes to `out`
// (same layout) and row r's first prefix to rbase[r] (LDS, rows + 1 entries).  Returns the total.
template <int NT>
__device__ __forceinline__ uint64_t block_scan_table(const uint32_t* in, uint32_t* out, uint32_t rows, uint32_t len,
                                                     uint32_t stride, uint32_t* scratch, uint32_t* rbase,
                                                     uint32_t* total = nullptr) {
  const uint32_t tid = threadIdx.x, L = rows * len, per = (L + NT - 1) / NT;
  const uint32_t i0 = min(L, tid * per), i1 = min(L, i0 + per);
  uint32_t sum = 0;
  {
    uint32_t r = len ? i0 / len : 0u, c = i0 - r * len;
    for (uint32_t i = i0; i < i1; ++i) {
      sum += in[(size_t)r * stride + c];
      if (++c == len) { c = 0; ++r; }
    }
  }
  uint32_t t;
  uint32_t run = block_excl_sum<NT>(sum, scratch, &t);
  {
    uint32_t r = len ? i0 / len : 0u, c = i0 - r * len;
    for (uint32_t i = i0; i < i1; ++i) {
      const size_t x = (size_t)r * stride + c;
      const uint32_t v = in[x];
      out[x] = run;
      if (c == 0 && rbase) rbase[r] = run;
      run += v;
      if (++c == len) { c = 0; ++r; }
    }
  }
  if (tid == 0 && rbase) rbase[rows] = t;
  if (tid == 0 && total) *total = t;
  __syncthreads();
  return t;
}

constexpr uint32_t kMaxUnitChunks = kThreads - 4;  // chunks per histogram unit (G) — one per thread (252: the
                                                   // chunk downsweep's LDS stays within 40 KB, 4 workgroups/CU)
constexpr uint32_t kBlSlice = kThreads * 8;     // backlog-prefix slice (buckets per rowscan block)
constexpr uint32_t kMaxBlSlices = kWave;        // nb <= 2^17 (n_local < 2^28): one wave sums the slices

struct ChunkSortArgs {
  Chunks ch;
  Msgs out;
  uint32_t* hist;      // digit-major [nbins][stride]: per-unit digit counts -> exclusive prefix
  uint32_t* tot;       // [nbins] digit totals
  uint32_t* d_n;       // out: total messages
  uint32_t* bstart;    // out: exclusive scan of digit totals (bucket starts when one pass)
  uint64_t* stats;
  uint8_t* alive;      // stop commit
  const uint32_t* stopq;
  uint32_t* nstop;
  uint32_t* step;      // CRDT heap parity (null when no CRDT kind is registered)
  uint32_t* heap_top;
  uint32_t* skew_n;    // skew list of the coming apply: reset here
  uint32_t* blpre;     // bypass: [nb] slice-local exclusive scan of the backlog chunk counts (rowscan blocks >= nd)
  uint32_t* bl_stot;   // bypass: [slices] backlog total per slice of kBlSlice buckets
  uint32_t* bl_sbase;  // bypass: out: [slices] exclusive scan of bl_stot (downsweep block 0)
  uint32_t* d_ninbox;  // bypass: out: messages in this superstep's inboxes (sorted + backlog + rings)
  const unsigned long long* ring_total;  // bypass: messages held in bounded-mailbox rings (null: none)
  uint64_t cap;
  uint32_t stride, nunits, ng, G, shift, bits;
  uint32_t bypass;     // backlog chunks are read in place by the apply (not sorted; units < ng skipped)
  // identity grouping (single-rank multi-pass; null = off): per tell chunk the apply's key summary
  // {first, last, descents, descent position}; the rowscan's extra blocks reduce it per slice of
  // kBlSlice chunks into slsum, k_ident_combine decides, ident[0..2] = {on, rotation, total}
  const uint4* emmeta;
  uint32_t* slsum;     // [kMaxBlSlices + 1][kSlSum]; row kMaxBlSlices = the host-staged total
  uint32_t* ident;
  uint64_t* istats;    // stats[ST_IDENT]: supersteps grouped by identity
  // launch split (identity grouping with > 1 pass): part 1 = the slice summaries only (then
  // k_ident_combine), part 2 = stops + digit rows + backlog slices, the digit rows skipped when the
  // superstep is grouped by identity (nothing reads them: k_bucket_bounds finds the bucket starts
  // in place); part 0 = every block in one launch
  uint32_t part;
};
constexpr uint32_t kSlSum = 8;  // per slice: total, flags, delta, descents, position, first key, last key, -

// ---- identity grouping (single-rank multi-pass).  If the previous apply's tell chunks, read in
// bucket order, are already in key order -- up to one rotation -- and lie densely at [0, total) of
// its tell arena, that arena IS the sorted new mail: no radix pass runs, k_bucket_bounds searches
// it in place and the apply reads it there (InView).  Bucket d's inbox then holds exactly the mail
// for d, each actor's in (sender bucket, sender, emission) order -- the canonical order of a stable
// sort.  The rotation case (a ring's wrap-around: the last sender bucket's tells to actor 0) needs
// the wrapped keys strictly below the first key, so no actor receives from both ends.
// SURVEY.md §7 hard part 2: skipping the sort for a static topology is legitimate if the inbox
// order is identical (akka-actor/src/main/scala/akka/dispatch/Mailbox.scala:89 enqueue order).
// (scratch: 2 * (kWaves + 1) u32)
__device__ __forceinline__ void ident_slice(const ChunkSortArgs& a, uint32_t sl, uint32_t nsl, uint32_t* scratch) {
  __shared__ uint32_t s_tlast[kThreads], s_tfirst[kThreads];
  __shared__ int s_iscr[kWaves + 1];
  __shared__ uint32_t s_red[4];  // delta min / max, first / last thread with a non-empty chunk
  const uint32_t tid = threadIdx.x;
  if (sl >= nsl) {  // host-staged tells this superstep (any -> no identity)
    uint32_t v = 0;
    for (uint32_t i = tid; i < kStagedChunks; i += kThreads) v += a.ch.cnt[2 * a.ch.nb + i];
    uint32_t t;
    block_excl_sum<kThreads>(v, scratch, &t);
    if (tid == 0) a.slsum[kMaxBlSlices * kSlSum] = t;
    return;
  }
  if (tid == 0) {
    s_red[0] = 0xFFFFFFFFu;
    s_red[1] = 0u;
    s_red[2] = 0xFFFFFFFFu;
    s_red[3] = 0u;
  }
  const uint32_t c0 = sl * kBlSlice + tid * 8, nb = a.ch.nb;
  uint32_t cnt[8], off[8], sum = 0;
  uint4 m[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t c = c0 + j;
    cnt[j] = c < nb ? a.ch.cnt[nb + c] : 0u;
    off[j] = c < nb ? a.ch.off[nb + c] : 0u;
    sum += cnt[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) m[j] = cnt[j] ? a.emmeta[c0 + j] : make_uint4(0, 0, 0, 0);
  uint32_t tot;
  uint32_t p = block_excl_sum<kThreads>(sum, scratch, &tot);  // slice-local stream position (syncs s_red)
  uint32_t dmin = 0xFFFFFFFFu, dmax = 0, nd = 0, pos = 0, tfirst = 0, tlast = 0, fpos = 0;
  bool thas = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (cnt[j]) {
      const uint32_t dv = off[j] - p;  // dense: off == slice base + position, for every chunk
      dmin = min(dmin, dv);
      dmax = max(dmax, dv);
      if (m[j].z) pos = p + m[j].w;  // an internal descent (its position, used when it is the only one)
      nd += min(m[j].z, 2u);
      if (thas && m[j].x < tlast) {  // a descent where this chunk starts
        ++nd;
        pos = p;
      }
      if (!thas) {
        tfirst = m[j].x;
        fpos = p;
      }
      thas = true;
      tlast = m[j].y;
    }
    p += cnt[j];
  }
  s_tlast[tid] = tlast;
  s_tfirst[tid] = tfirst;
  if (thas) {
    atomicMin(&s_red[0], dmin);
    atomicMax(&s_red[1], dmax);
    atomicMin(&s_red[2], tid);
    atomicMax(&s_red[3], tid);
  }
  const int prev = block_excl_max<kThreads>(thas ? (int)tid : -1, s_iscr);  // (syncs: s_tlast, s_red)
  if (thas && prev >= 0 && tfirst < s_tlast[prev]) {  // a descent between the previous thread's chunks and ours
    ++nd;
    pos = fpos;
  }
  uint32_t tnd, tpos;
  block_excl_sum2<kThreads>(min(nd, 2u), nd ? pos : 0u, scratch, &tnd, &tpos);  // (tpos valid when tnd == 1)
  if (tid == 0) {
    uint32_t* o = a.slsum + (size_t)sl * kSlSum;
    const bool ne = s_red[2] != 0xFFFFFFFFu;
    o[0] = tot;
    o[1] = (ne ? 1u : 0u) | (ne && s_red[0] == s_red[1] ? 2u : 0u);
    o[2] = s_red[0];  // every non-empty chunk sits at (this delta) + its stream position
    o[3] = min(tnd, 2u);
    o[4] = tpos;
    o[5] = ne ? s_tfirst[s_red[2]] : 0u;
    o[6] = ne ? s_tlast[s_red[3]] : 0u;
  }
}

// The superstep's decision, one wave over the <= kMaxBlSlices slice summaries: ident = {on, rotation,
// total}.  On iff no host-staged tells, every non-empty chunk at (stream position) in the arena
// (dense from 0), and the stream in key order up to one descent whose wrapped keys stay strictly
// below the first key (then sorted item i is stream item (i + rotation) mod total).
static __global__ void __launch_bounds__(kWave) k_ident_combine(const uint32_t* slsum, uint32_t nsl, uint32_t* ident,
                                                               unsigned long long* istats) {
  const uint32_t s = lane_id();
  const bool in = s < nsl;
  const uint32_t* S = slsum + (size_t)(in ? s : 0u) * kSlSum;
  const uint32_t tot = in ? S[0] : 0u, fl = in ? S[1] : 0u, s2 = S[2], s3 = S[3], s4 = S[4], s5 = S[5], s6 = S[6];
  const bool ne = (fl & 1u) != 0;
  const uint32_t inc = wave_incl_sum(tot), base = inc - tot;
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, kWave - 1);
  const bool dense = !ne || ((fl & 2u) != 0 && s2 == base);
  uint32_t nd = ne ? s3 : 0u, pos = ne && s3 ? base + s4 : 0u;
  const uint64_t nem = __ballot(ne);
  const uint64_t before = nem & lanemask_lt();
  const int prev = before ? 63 - __clzll((long long)before) : 0;
  const uint32_t plast = (uint32_t)__shfl((int)s6, prev, kWave);
  if (ne && before && s5 < plast) {  // a descent where this slice's mail starts
    ++nd;
    pos = base;
  }
  nd = min(nd, 2u);
  const uint32_t ndt = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(nd), kWave - 1);
  const uint32_t post = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(nd ? pos : 0u), kWave - 1);
  const bool all_dense = __ballot(!dense) == 0;
  const int fl0 = nem ? __builtin_ctzll(nem) : 0, fl1 = nem ? 63 - __clzll((long long)nem) : 0;
  const uint32_t first_key = (uint32_t)__shfl((int)s5, fl0, kWave), last_key = (uint32_t)__shfl((int)s6, fl1, kWave);
  if (s == 0) {
    const uint32_t staged = slsum[kMaxBlSlices * kSlSum];
    const bool on = all_dense && staged == 0 && total > 0 && (ndt == 0 || (ndt == 1 && last_key < first_key));
    ident[0] = on ? 1u : 0u;
    ident[1] = on && ndt ? post : 0u;
    ident[2] = total;
    if (on) atomicAdd(istats, 1ull);
  }
}

// one block per digit: exclusive prefix over units (in place) + digit total;
// block 0 also commits the previous step's stops.
static __global__ void __launch_bounds__(kThreads) k_chunk_rowscan(ChunkSortArgs a) {
  __shared__ uint32_t scratch[2 * (kWaves + 1)];  // (block_excl_sum2 in ident_slice needs both halves)
  if (a.part == 1) {
    ident_slice(a, blockIdx.x, (a.ch.nb + kBlSlice - 1) / kBlSlice, scratch);
    return;
  }
  if (blockIdx.x == 0) {
    begin_step(a.step, a.heap_top);
    commit_stops(a.alive, a.stopq, a.nstop);
    if (threadIdx.x == 0) {
      a.skew_n[0] = 0u;
    }
  }
  const uint32_t d = blockIdx.x;
  const uint32_t nsl = (a.ch.nb + kBlSlice - 1) / kBlSlice;
  if (a.emmeta && d >= (1u << a.bits) + nsl) {  // identity grouping: tell-chunk slices, then the staged total
    ident_slice(a, d - (1u << a.bits) - nsl, nsl, scratch);
    return;
  }
  if (d >= (1u << a.bits) && a.bypass) {  // extra blocks: backlog prefix, one slice of kBlSlice buckets each
    const uint32_t sl = d - (1u << a.bits), i0 = sl * kBlSlice + threadIdx.x * 8;
    uint32_t v[8], sum = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = i0 + j < a.ch.nb ? a.ch.cnt[i0 + j] : 0u;
      sum += v[j];
    }
    uint32_t t;
    uint32_t ex = block_excl_sum<kThreads>(sum, scratch, &t);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i0 + j < a.ch.nb) a.blpre[i0 + j] = ex;  // slice-local; + bl_sbase[slice] in the apply
      ex += v[j];
    }
    if (threadIdx.x == 0) a.bl_stot[sl] = t;
    return;
  }
  if (d >= (1u << a.bits)) return;
  if (a.part == 2 && a.ident[0]) return;  // identity: no pass reads the digit prefixes
  const uint32_t t = scan_row(a.hist + (size_t)d * a.stride, a.nunits, scratch);
  if (threadIdx.x == 0) a.tot[d] = t;
}

static __global__ void __launch_bounds__(kThreads) k_chunk_downsweep(ChunkSortArgs a) {
  // 40 KB of LDS or less (four workgroups per CU, not three): the digit bases stay in registers
  // (thread t owns digits t and t + kThreads), the block scans' scratch lives in s_gadj's first
  // words (as in k_sort_downsweep), the chunk prefix keeps its total at index nc
  static_assert(kRadix == 2 * kThreads, "two digit bases per thread");
  __shared__ uint32_t whist[kWaves][kRadix];
  __shared__ uint32_t s_base[kRadix], s_ldig[kRadix], s_gadj[kRadix];
  __shared__ uint32_t s_key[kTile], s_src[kTile], s_pay[kTile];
  __shared__ uint32_t s_cpre[kMaxUnitChunks + 1], s_coff[kMaxUnitChunks];
  uint32_t* const scratch = s_gadj;
  const SplitLds S{&whist[0][0], s_base, s_ldig, s_gadj, scratch, s_key, s_src, s_pay};
  const int tid = threadIdx.x;
  const uint32_t nd = 1u << a.bits;
  const bool idn = a.ident && a.ident[0];  // identity grouping: nothing to move (histogram columns still zeroed)
  // (split launch: the digit rows were not scanned -- the total is the identity stream's, and
  // k_bucket_bounds writes the bucket starts)
  const bool idsk = idn && a.part == 2;
  const uint32_t total = idsk ? a.ident[2] : digit_bases(a.tot, nd, s_base, scratch);
  const uint32_t db0 = idsk ? 0u : s_base[tid], db1 = idsk ? 0u : s_base[tid + kThreads];  // digit bases
  const bool over = total > a.cap;  // the sorted mail must fit A (the apply checks mail + backlog)
  if (blockIdx.x == 0) {
    if (!idsk) {
      if ((uint32_t)tid < nd) a.bstart[tid] = db0;
      if ((uint32_t)tid + kThreads < nd) a.bstart[tid + kThreads] = db1;
    }
    if (tid == 0) {
      a.bstart[nd] = total;
      *a.d_n = over ? 0u : total;
      if (over) atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
    }
    if (a.bypass && tid < kWave) {  // backlog (read in place by the apply): slice bases, inbox total
      const uint32_t nsl = (a.ch.nb + kBlSlice - 1) / kBlSlice;
      const uint32_t v = (uint32_t)tid < nsl ? a.bl_stot[tid] : 0u;
      const uint32_t inc = wave_incl_sum(v);
      if ((uint32_t)tid < nsl) a.bl_sbase[tid] = inc - v;
      if (tid == kWave - 1) {  // (rings: clamped, only "any mail at all" is read from it)
        const unsigned long long rt = a.ring_total ? *a.ring_total : 0ull;
        *a.d_ninbox = over ? 0u : total + inc + (uint32_t)(rt < (1ull << 30) ? rt : (1ull << 30));
      }
    }
  }
  if (over) return;
  if (idsk) {  // nothing moves: zero the apply's histogram columns for the next superstep, row by row
    for (uint32_t d = blockIdx.x; d < nd; d += gridDim.x)
      for (uint32_t u = tid; u < a.nunits; u += kThreads) a.hist[(size_t)d * a.stride + u] = 0u;
    return;
  }

  for (uint32_t u = blockIdx.x; u < a.nunits; u += gridDim.x) {
    if (a.bypass && u < a.ng) continue;  // backlog units: nothing counted, nothing to move
    // chunk range of this unit
    uint32_t c0, c1;
    if (u < a.ng) {
      c0 = u * a.G;
      c1 = min(a.ch.nb, c0 + a.G);
    } else if (u < 2 * a.ng) {
      c0 = a.ch.nb + (u - a.ng) * a.G;
      c1 = a.ch.nb + min(a.ch.nb, (u - a.ng + 1) * a.G);
    } else {
      c0 = 2 * a.ch.nb + (u - 2 * a.ng);
      c1 = c0 + 1;
    }
    // this unit's per-digit prefix (from the rowscan); the column is then zeroed so
    // that the next k_bucket_apply can accumulate fresh counts without a memset
    __syncthreads();  // (the previous unit's tiles are done with s_base; digit_bases' reads of it too)
#pragma unroll
    for (uint32_t j = 0; j < 2; ++j) {
      const uint32_t d = tid + j * kThreads;
      if (d < nd) {
        uint32_t* hp = a.hist + (size_t)d * a.stride + u;
        s_base[d] = (j ? db1 : db0) + *hp;
        *hp = 0u;
      }
    }
    if (idn) continue;
    // the unit's chunks as one stream (tiles cross chunk boundaries: small chunks — skewed
    // or sparse supersteps — do not cost a tile each); chunk j of the unit holds stream
    // items [s_cpre[j], s_cpre[j+1])
    const uint32_t nc = c1 - c0;  // <= kMaxUnitChunks
    {
      const uint32_t j = tid;
      const uint32_t v = j < nc ? a.ch.cnt[c0 + j] : 0u;
      if (j < nc) s_coff[j] = a.ch.off[c0 + j];
      uint32_t t;
      const uint32_t ex = block_excl_sum<kThreads>(v, scratch, &t);
      if (j <= nc) s_cpre[j] = ex;  // (s_cpre[nc] = the unit's total)
      if (j == 0) s_cpre[nc] = t;
    }
    __syncthreads();
    const uint32_t ntot = s_cpre[nc];
    const CMsgs& src = a.ch.arena(c0);  // one arena per unit
    if (ntot >= nc * (uint32_t)(kTile / 2)) {  // large chunks: tile by tile, direct addressing
      for (uint32_t j = 0; j < nc; ++j) {
        const uint32_t cnt = s_cpre[j + 1] - s_cpre[j];
        for (uint32_t sub = 0; sub < cnt; sub += kTile)
          split_tile<kThreads>(src, s_coff[j] + sub, min((uint32_t)kTile, cnt - sub), a.out, a.shift, a.bits, S);
      }
      continue;
    }
    for (uint32_t t0 = 0; t0 < ntot; t0 += kTile) {
      const auto loc = [&](uint32_t q) -> uint32_t {
        const uint32_t i = t0 + q;
        uint32_t lo = 0, hi = nc - 1;  // last chunk whose start <= i
        while (lo < hi) {
          const uint32_t mid = (lo + hi + 1) >> 1;
          if (s_cpre[mid] <= i) lo = mid; else hi = mid - 1;
        }
        return s_coff[lo] + (i - s_cpre[lo]);
      };
      split_tile_ld<kThreads>(src, loc, min((uint32_t)kTile, ntot - t0), a.out, a.shift, a.bits, S);
    }
  }
}

// =========================================================================
// Dense radix pass (reduce-then-scan) over "super-tiles" of kSub tiles: one
// histogram column per super-tile keeps the digit-major tables small.
// =========================================================================
constexpr int kSub = 8;
constexpr uint32_t kSuper = (uint32_t)kTile * kSub;

struct SortArgs {
  CMsgs in;
  Msgs out;
  const uint32_t* d_n;
  uint32_t* hist;  // digit-major [nbins][stride]
  uint32_t* tot;
  uint32_t* bstart;  // out (block 0 of the downsweep): exclusive scan of digit totals
  uint32_t stride;
  uint32_t shift, bits;
  uint32_t maxsub;  // largest super-tile, in tiles (1..kSub): sized from the message capacity
  const uint32_t* ident;  // single-rank multi-pass: [0] != 0 = identity grouping this superstep (no pass runs)
};

// Envelopes per super-tile of THIS pass, from its input size n (on the device, so a graph-captured
// pass adapts to each superstep's mail): about 1024 super-tiles, 1..maxsub tiles each.  A sparse
// superstep (C3: ~4e5 messages against a capacity of 4e7) gets one-tile super-tiles on ~200
// workgroups instead of ~25 workgroups walking 8 tiles each.
__device__ __forceinline__ uint32_t pass_super(const SortArgs& a, uint32_t n) {
  const uint32_t sub = n / ((uint32_t)kTile * 1024u);
  return (uint32_t)kTile * (sub < 1u ? 1u : sub > a.maxsub ? a.maxsub : sub);
}

// Digit counts of four keys into a wave's LDS histogram.  Sorted-by-lower-bits input
// (the ring after the first pass) gives whole waves of one digit: those cost one LDS
// atomic instead of 256 conflicting ones.
__device__ __forceinline__ void count4(uint32_t* h, const uint4& v, uint32_t shift, uint32_t mask) {
  const uint32_t d0 = (v.x >> shift) & mask, d1 = (v.y >> shift) & mask, d2 = (v.z >> shift) & mask,
                 d3 = (v.w >> shift) & mask;
  const bool same4 = d0 == d1 && d0 == d2 && d0 == d3;
  const uint32_t first = __builtin_amdgcn_readfirstlane(d0);
  const uint64_t act = __ballot(1);
  if (__ballot(same4 && d0 == first) == act) {
    if (lane_id() == (uint32_t)__builtin_ctzll(act)) atomicAdd(&h[first], 4u * (uint32_t)__popcll(act));
  } else if (same4) {
    atomicAdd(&h[d0], 4u);
  } else {
    atomicAdd(&h[d0], 1u);
    atomicAdd(&h[d1], 1u);
    atomicAdd(&h[d2], 1u);
    atomicAdd(&h[d3], 1u);
  }
}

static __global__ void __launch_bounds__(kThreads) k_sort_upsweep(SortArgs a) {
  if (a.ident && a.ident[0]) return;  // identity grouping: the mail is already in key order
  __shared__ uint32_t h[kWaves][kRadix];
  const uint32_t n = *a.d_n, super = pass_super(a, n), nt = div_up(n, super);
  const int tid = threadIdx.x, w = tid / kWave;
  const uint32_t mask = (1u << a.bits) - 1u, nd = 1u << a.bits;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    for (int i = tid; i < kWaves * kRadix; i += kThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint32_t b0 = t * super, b1 = min(n, b0 + super);
    const uint32_t nfull = (b1 - b0) / (4 * kThreads);  // full rounds of one uint4 per thread
    const uint4* k4 = reinterpret_cast<const uint4*>(a.in.key + b0);
    uint32_t j = 0;
    for (; j + 8 <= nfull; j += 8) {  // eight loads in flight per thread before the LDS updates
      uint4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = k4[(j + u) * kThreads + tid];
      asm volatile("" ::: "memory");  // keep the loads ahead of the LDS atomics (issued together)
#pragma unroll
      for (int u = 0; u < 8; ++u) count4(h[w], v[u], a.shift, mask);
    }
    for (; j < nfull; ++j) count4(h[w], k4[j * kThreads + tid], a.shift, mask);
    for (uint32_t i = b0 + nfull * 4 * kThreads + tid; i < b1; i += kThreads)
      atomicAdd(&h[w][(a.in.key[i] >> a.shift) & mask], 1u);
    __syncthreads();
    for (uint32_t d = tid; d < nd; d += kThreads) {
      uint32_t s = 0;
#pragma unroll
      for (int q = 0; q < kWaves; ++q) s += h[q][d];
      a.hist[(size_t)d * a.stride + t] = s;
    }
    __syncthreads();
  }
}

static __global__ void __launch_bounds__(kThreads) k_sort_rowscan(SortArgs a) {
  if (a.ident && a.ident[0]) return;
  __shared__ uint32_t scratch[kWaves + 1];
  const uint32_t d = blockIdx.x;
  if (d >= (1u << a.bits)) return;
  const uint32_t n = *a.d_n;
  const uint32_t t = scan_row(a.hist + (size_t)d * a.stride, div_up(n, pass_super(a, n)), scratch);
  if (threadIdx.x == 0) a.tot[d] = t;
}

static __global__ void __launch_bounds__(kThreads) k_sort_downsweep(SortArgs a) {
  if (a.ident && a.ident[0]) return;
  __shared__ uint32_t whist[kWaves][kRadix];
  __shared__ uint32_t s_dbase[kRadix], s_base[kRadix], s_ldig[kRadix], s_gadj[kRadix];
  __shared__ uint32_t s_key[kTile], s_src[kTile], s_pay[kTile];
  // the block scans' scratch lives in s_gadj's first kWaves + 1 words: digit_bases runs before any
  // tile, and a tile scans its digit starts before it writes s_gadj (and after the previous tile's
  // scatter, which read it, has passed its barrier) -- 40 KB of LDS exactly: four workgroups per CU
  uint32_t* const scratch = s_gadj;
  const SplitLds S{&whist[0][0], s_base, s_ldig, s_gadj, scratch, s_key, s_src, s_pay};
  const int tid = threadIdx.x;
  const uint32_t n = *a.d_n, super = pass_super(a, n), nt = div_up(n, super);
  if (blockIdx.x >= nt && blockIdx.x != 0) return;  // (no super-tile: the grid is sized for the capacity)
  const uint32_t nd = 1u << a.bits;
  const uint32_t total = digit_bases(a.tot, nd, s_dbase, scratch);
  if (blockIdx.x == 0) {
    for (uint32_t d = tid; d < nd; d += kThreads) a.bstart[d] = s_dbase[d];
    if (tid == 0) a.bstart[nd] = total;
  }
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    for (uint32_t d = tid; d < nd; d += kThreads) s_base[d] = s_dbase[d] + a.hist[(size_t)d * a.stride + t];
    __syncthreads();
    const uint32_t b0 = t * super, b1 = min(n, b0 + super);
    for (uint32_t base = b0; base < b1; base += kTile)
      split_tile<kThreads>(a.in, base, min((uint32_t)kTile, b1 - base), a.out, a.shift, a.bits, S);
  }
}

// =========================================================================
// Bucket apply: in-bucket sort + segmented drain + behaviour + emission
// =========================================================================
constexpr uint32_t kVoidKey = 0xFFFFFFFFu;  // never a key: local ids < 2^28 - 1, owners < 16

template <bool kWrite>
struct Emitter {
  const DevParams* P;
  Msgs out;
  uint64_t pos;       // next write position (kWrite)
  uint32_t self;      // sender id (global)
  uint32_t n_valid;   // tells to a known actor
  uint32_t n_all;     // all tells
  uint32_t* nh;       // next-pass digit histogram (LDS)
  uint32_t nh_shift, nh_mask;
  __device__ __forceinline__ void operator()(uint32_t dst, uint32_t pay) {
    if (dst >= P->n_global) {  // a host-side actor (the reply path: outbox) or an unknown ref -> deadLetters
      if (!outbound_tell(*P, dst, self, pay, kWrite)) ++n_all;
      return;
    }
    ++n_all;
    ++n_valid;
    if (kWrite) {
      const uint32_t key = (P->R > 1) ? P->route[dst] : dst;
      out.key[pos] = key;
      out.src[pos] = self;
      out.pay[pos] = pay;
      ++pos;
      lds_hist_inc(nh, (key >> nh_shift) & nh_mask);
    }
  }
  // CRDT state gossip to a known actor: the sender field carries the wide tag, payload = row handle
  __device__ __forceinline__ void wide(uint32_t dst, uint32_t h) {
    ++n_all;
    ++n_valid;
    if (kWrite) {
      const uint32_t key = (P->R > 1) ? P->route[dst] : dst;
      out.key[pos] = key;
      out.src[pos] = self | AGX_WIDE_BIT;
      out.pay[pos] = h;
      ++pos;
      lds_hist_inc(nh, (key >> nh_shift) & nh_mask);
    }
  }
  __device__ __forceinline__ void count(uint32_t k) {
    n_all += k;
    n_valid += k;
  }
  // delta-CRDT: a NoDeltaPlaceholder group's slot (phase A counted it): a void tell, compacted out
  // of the bucket's tells after phase B (compact_void); not emitted, not in the next-pass histogram
  uint32_t n_void = 0;
  __device__ __forceinline__ void void_slot() {
    ++n_void;
    if (kWrite) {
      out.key[pos] = kVoidKey;
      ++pos;
    }
  }
};

// Remove the void tells (kVoidKey) from a bucket's tell chunk [base, base + n) in place, keeping the
// sender order (tile by tile: every write lands at or below the positions still to be read).
__device__ __forceinline__ uint32_t compact_void(const Msgs& m, uint64_t base, uint32_t n, uint32_t* scratch) {
  constexpr uint32_t NT = 512, IPT = 4;
  uint32_t out = 0;
  for (uint32_t t0 = 0; t0 < n; t0 += NT * IPT) {
    uint32_t k[IPT], sv[IPT], pv[IPT], c = 0;
#pragma unroll
    for (uint32_t r = 0; r < IPT; ++r) {
      const uint32_t i = t0 + threadIdx.x * IPT + r;
      k[r] = i < n ? m.key[base + i] : kVoidKey;
      if (k[r] != kVoidKey) {
        sv[r] = m.src[base + i];
        pv[r] = m.pay[base + i];
        ++c;
      }
    }
    uint32_t tot;
    uint32_t o = out + block_excl_sum<NT>(c, scratch, &tot);  // (barriers: every load of the tile is done)
#pragma unroll
    for (uint32_t r = 0; r < IPT; ++r)
      if (k[r] != kVoidKey) {
        m.key[base + o] = k[r];
        m.src[base + o] = sv[r];
        m.pay[base + o] = pv[r];
        ++o;
      }
    out += tot;
    __syncthreads();
  }
  return out;
}

constexpr int kBThreads = 512;                 // bucket_apply block: 8 waves
constexpr int kBWaves = kBThreads / kWave;
constexpr int kBIpt = kBucket / kBThreads;      // items per thread per sub-tile (4)
#ifndef AGX_PING_PAR
#define AGX_PING_PAR 1
#endif
constexpr bool kPingPar = AGX_PING_PAR != 0;  // PingPong drains message-parallel (bucket_finish)
constexpr int kBAct = kBucket / kBThreads;      // actors per thread (4)
static_assert(kBAct == 4 && kBIpt == 4, "bucket_apply assumes 4 actors and 4 inbox items per thread");
#ifndef AGX_NO_MONO
constexpr bool kMonoShortcut = true;
#else
constexpr bool kMonoShortcut = false;
#endif
#ifndef AGX_PF
#define AGX_PF 4
#endif
#ifndef AGX_COMPACT_DRAIN
#define AGX_COMPACT_DRAIN 1
#endif
// single-pass drains of the actors with mail, one actor per thread (bucket_finish kCompact; A/B build knob)
constexpr bool kCompactDrain = AGX_COMPACT_DRAIN != 0;
#ifndef AGX_FWD_PRE
#define AGX_FWD_PRE 4
#endif
constexpr uint32_t kFwdPre = AGX_FWD_PRE;  // FORWARD_RR destinations loaded before a compacted drain
constexpr int kPF = AGX_PF;                     // apply prefetch window (messages in global scratch)

// Tell staging in LDS (single-pass path): tells overwrite consumed inbox slots of the same actor.
struct EmitterLds {
  const DevParams* P;
  uint32_t* key;
  uint32_t* src;
  uint32_t* pay;
  uint32_t slot;      // next LDS slot
  uint32_t self;
  uint32_t n_valid, n_all;
  uint32_t* nh;
  uint32_t nh_shift, nh_mask;
  __device__ __forceinline__ void operator()(uint32_t dst, uint32_t p) {
    if (dst >= P->n_global) {  // a host-side actor (the reply path: outbox) or an unknown ref -> deadLetters
      if (!outbound_tell(*P, dst, self, p, true)) ++n_all;
      return;
    }
    ++n_all;
    ++n_valid;
    const uint32_t k = (P->R > 1) ? P->route[dst] : dst;
    key[slot] = k;
    src[slot] = self;
    pay[slot] = p;
    ++slot;
    lds_hist_inc(nh, (k >> nh_shift) & nh_mask);
  }
};

// Fused superstep (single rank, one radix digit covers every bucket): k_bucket_apply
// gathers its inbox straight from the tell chunks of the previous superstep, which
// were written grouped by destination bucket, so no separate sort kernel runs.
// Arenas and tables are double-buffered by superstep parity (step & 1).
struct GatherArgs {
  Msgs bl[2];              // backlog of bucket b at [lo_b, +blc) (parity)
  Msgs eg[2];              // tells grouped by destination bucket (parity)
  CMsgs stg;               // host-staged tells, grouped by bucket on the host
  uint32_t* tcnt[2];       // [nd][tstride]: tells from chunk c to bucket d (zeroed by the reader)
  uint32_t* toff[2];       // [nd][tstride]: their offset in eg[parity]
  uint32_t* blo[2];        // [nb] backlog offset / count per bucket
  uint32_t* blc[2];
  uint32_t* emc[2];        // [nb] tells emitted per bucket (in-flight accounting)
  uint32_t* stg_off;       // [nb] staged tells per bucket (count zeroed by the reader)
  uint32_t* stg_cnt;
  Msgs inb;                // skewed buckets: gathered inbox copy at [lo, lo+cnt)
  uint32_t* ovf;           // [2] overflow-region cursor per parity (inboxes larger than `region`)
  uint32_t* cntb;          // [slot][nb] inbox size per bucket, one row per superstep of a replay
                           // (the host sums them: quiescence, superstep count — no shared counter)
  uint32_t* heap_top;      // CRDT heap tops [2] (null when no CRDT kind is registered)
  uint64_t cap;
  uint32_t tstride;
  uint32_t region;         // bucket b's inbox lives at [b*region, ...) unless larger (overflow region)
};

struct BucketArgs {
  DevParams P;
  GatherArgs g;
  CMsgs in;                // mail sorted by bucket (local key >> bb)
  const uint32_t* d_n;
  const uint32_t* bstart;  // bucket starts [nb + 1]
  Msgs scr;                // general path: bucket-local sorted copy (index space of `in`)
  Msgs bl, em;             // chunk arenas: backlog of bucket b at [lo, lo+cnt), tells at [lo*kmax, (lo+cnt)*kmax)
  uint32_t* chunk_off;
  uint32_t* chunk_cnt;
  uint32_t* nhist;         // next step's first-pass histogram, digit-major [nbins][nhist_stride]
  uint32_t nhist_stride, nx_shift, nx_bits;
  uint32_t G, ng;          // histogram units: G buckets per column, ng units per arena
  uint32_t nb, kmax;
  uint32_t bb;             // bucket bits: bucket b = local actors [b << bb, (b + 1) << bb), bb <= kBucketBits
  uint64_t cap;            // bypass: message capacity of the inbox index space
  const uint32_t* pstep;   // bypass (single-rank multi-pass): superstep counter; backlog arena parity = step & 1
  const uint32_t* blpre;   // bypass: backlog prefix (bucket b's inbox index space starts at bstart[b] +
  const uint32_t* bl_sbase;  // blpre[b] + bl_sbase[b / kBlSlice]); chunk_off/cnt[b] locate its backlog in g.bl[par ^ 1]
  const uint32_t* d_ninbox;  // bypass: sorted + backlog messages of this superstep
  uint32_t par;            // fused: parity of this superstep (arenas/tables written; read = par ^ 1)
  uint32_t slot;           // fused: index of this superstep within its graph replay (row of g.cntb)
  uint32_t* skew_list;     // buckets whose inbox exceeds one LDS tile (appended by the fast launch)
  uint32_t* skew_n;        // their count (reset by the first kernel of the next superstep)
  uint64_t* stats;
  unsigned long long* bstats;  // [gridDim][kBStats] per-block counters (summed by k_stats_reduce)
  unsigned long long* dbg;  // diagnostic build only (AGX_STAMPS): per-block phase timestamps
  // fused graphs without skew launches ("strict" replays, null otherwise): [parity] -> 1 + the replay
  // slot of a superstep that deferred a skewed bucket; every later superstep is a no-op that
  // passes the mark on, and the host runs the deferred skew launch and resumes (run_single)
  uint32_t* abort;
  uint32_t tiny_max;       // bypass: inboxes of at most this many messages take the wave path (0 = off)
  // bypass, plain behaviours: [nb] marks of the buckets k_tiny_apply left to the block launch
  // (non-null: the block launch skips the unmarked ones)
  uint32_t* blist;
  uint32_t dense_first;    // bypass: k_dense_apply ran first -- k_tiny_apply takes only the buckets it marked
  uint32_t dense_alone;    // fused strict replay: k_dense_fused is the whole superstep (a bucket it leaves aborts)
  // persistent fused launch (k_dense_fused<.., kPersist>): psteps supersteps in one launch, one block
  // per bucket, a grid barrier between supersteps; pbar = {arrivals, generation, timed out}
  uint32_t psteps;
  uint32_t* pbar;
  uint32_t* dense_left;    // [2] by superstep parity: the dense launch left a bucket to the wave / block launches
                           // (they return at entry when it did not); null: no such shortcut
  // bypass, plain behaviours: skewed buckets pre-partitioned by k_skew_* (see there); [i] = skew index
  const uint32_t* sk_rec;  // [i][kSkRec] bucket, bounds, parts, drained and queued totals
  const uint32_t* sk_act;  // [i][3][kBucket] per actor: admitted, drained-segment start, backlog start
  // single-rank multi-pass, identity grouping (k_ident_combine): when ident[0] != 0 the sorted new mail
  // is the previous apply's tell arena in_alt itself, rotated by ident[1] (n = ident[2]); emmeta
  // (non-null in this mode) receives this superstep's per-chunk key summary for the next decision
  const uint32_t* ident;
  CMsgs in_alt;
  uint4* emmeta;
  // bounded-mailbox rings (single-rank multi-pass, plain behaviours, every mailbox class bounded;
  // null = off).  A bucket that reaches the skew path takes a pool slot (k_skew_plan) for good: its
  // actors' queued messages then stay in per-actor rings of ring_c slots -- a queued message is
  // written once and read once, when it is drained (AbstractBoundedNodeQueue.java:92-113: a queued
  // node does not move) -- instead of being copied forward every superstep.
  uint32_t* ring_of;        // [nb] pool slot + 1 (0 = the bucket's backlog is in the bl arena)
  uint32_t* ring_state;     // [slots][kBucket] head | len << 16
  uint32_t* ring_src;       // [slots][kBucket][ring_c]
  uint32_t* ring_pay;
  uint32_t* ring_next;      // [0] pool slots handed out, [1] released slots on the free stack
  uint32_t* ring_free;      // [slots] free stack (slots of buckets that cooled down)
  // ORSet-only full-state populations: the state effects of each replica's run are left to
  // k_orset_merge (a lean kernel, lane = element): one item per replica with work, and its run
  uint4* orw;               // [n_local] {l, node, message offset, first snapshot row}
  uint2* orm;               // [cap] (src, payload) of the runs
  uint32_t* orw_n;          // [0] items, [1] messages (reset before the apply)
  unsigned long long* ring_total;  // messages held in rings (in flight)
  // device-resident multi-rank replays: halt[0] != 0 stops every later kernel of the replay (k_mr_pack)
  const uint32_t* halt;
  uint32_t ring_slots, ring_c, ring_t;
  uint32_t ring_lo0;        // drain scratch / tell slice of slot k: ring_lo0 + k * kBucket * ring_t
};

// The sorted new mail of a single-rank multi-pass superstep: the radix passes' output, or --
// identity grouping -- the previous apply's tell arena in place, whose concatenated chunks were
// already in key order up to one rotation (a ring's wrap-around: sorted item i at (i + rot) mod n).
struct InView {
  CMsgs m;
  uint32_t rot, n;
  __device__ __forceinline__ uint32_t at(uint32_t i) const {
    const uint32_t j = i + rot;
    return j >= n ? j - n : j;
  }
};
__device__ __forceinline__ InView in_view(const BucketArgs& a) {
  if (a.ident && a.ident[0]) return InView{a.in_alt, a.ident[1], a.ident[2]};
  return InView{a.in, 0u, 0xFFFFFFFFu};
}

#define AGX_STAMP(a, idx)                                                                         \
  do {                                                                                            \
    if ((a).dbg && threadIdx.x == 0) (a).dbg[blockIdx.x * 16 + (idx)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
// (diagnostic, with AGX_STAMPS) the device-wide 100 MHz clock at a block's start / end, slots 13 / 14:
// when blocks start and finish within a launch (s_memtime is per-XCD and cannot be compared across blocks)
#define AGX_RTSTAMP(a, idx)                                                                        \
  do {                                                                                            \
    if ((a).dbg && threadIdx.x == 0) (a).dbg[blockIdx.x * 16 + (idx)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

struct BucketLds {
  uint32_t* key;   // fast path: sorted items (LDS); general path: run / tmp scratch
  uint32_t* src;
  uint32_t* pay;
  uint64_t* U;     // time-shared: whist (u16 [kBWaves][kBucket]) / blpre (u32) / w0,w1 (u64)
  uint32_t* seg;   // [kBucket + 4] segment starts
  uint32_t* ecnt;  // [kBucket] emission counts -> offsets
  uint8_t* alive;
  uint8_t* kind;
  uint32_t* nh;    // [kRadix]
  uint32_t* scratch;
  unsigned long long* stat;
  uint32_t* rowtop;  // snapshot rows taken from this bucket's heap region (CRDT kinds)
};

// After the in-bucket sort: classification, queued copy, behaviour apply, emission.
// kLds: sorted items are in LDS (fast path) or in the global scratch copy.
// Tells of one bucket in sender order -> grouped by destination digit in eg[w] at
// [embase, embase+emtot), plus this chunk's column of the parity-w tables.  Every
// destination's run is contiguous and in sender order (stable multisplit).  The digit is
// (key >> nx_shift) & (2^nx_bits - 1): the destination bucket (fused, single rank) or the
// owner rank (multi-rank: the chunk's tells leave grouped by the GPU that owns them).
template <bool kFromLds>
__device__ __forceinline__ void group_tells(const BucketArgs& a, const BucketLds& L, uint32_t b, uint32_t w,
                                            uint64_t embase, uint32_t emtot, const Msgs& src) {
  const GatherArgs& g = a.g;
  const int tid = threadIdx.x;
  const uint32_t nd = 1u << a.nx_bits;
  uint32_t* whist = L.key;             // [kBWaves][kRadix] u32 = 16 KB over key+src (free now)
  uint32_t* dbase = L.ecnt;            // [kRadix]
  uint32_t* base = L.ecnt + kRadix;    // [kRadix] running positions (multi-tile)
  uint32_t* ldig = L.ecnt + 2 * kRadix;
  uint32_t* gadj = L.ecnt + 3 * kRadix;
  {  // destination bases inside the chunk: exclusive scan of the per-destination counts
    const uint32_t v = (uint32_t)tid < nd ? L.nh[tid] : 0u;
    uint32_t t;
    const uint32_t ex = block_excl_sum<kBThreads>(v, L.scratch, &t);
    dbase[tid] = (uint32_t)embase + ex;
    base[tid] = (uint32_t)embase + ex;
    if ((uint32_t)tid < nd && v) {
      g.tcnt[w][(size_t)tid * g.tstride + b] = v;
      g.toff[w][(size_t)tid * g.tstride + b] = (uint32_t)embase + ex;
    }
  }
  __syncthreads();
  if (kFromLds) {  // <= kBucket tells, compacted in sender order in U: ranks + direct scatter
    const uint32_t* ukey = reinterpret_cast<const uint32_t*>(L.U);
    const uint32_t* usrc = ukey + kBucket;
    const uint32_t* upay = usrc + kBucket;
    const int wv = tid / kWave;
    const uint32_t lane = lane_id();
    const uint64_t ltm = lanemask_lt();
    uint32_t k[kBIpt], d[kBIpt], rk[kBIpt];
    int mono = 1;  // destinations non-decreasing in sender order (local topologies): already grouped
#pragma unroll
    for (int r = 0; r < kBIpt; ++r) {
      const uint32_t i = wv * (kBIpt * kWave) + r * kWave + lane;
      k[r] = i < emtot ? ukey[i] : 0u;
      d[r] = (k[r] >> a.nx_shift) & (nd - 1);
      if (i < emtot && i > 0) mono &= ((ukey[i - 1] >> a.nx_shift) & (nd - 1)) <= d[r];
    }
    if (kMonoShortcut && __syncthreads_and(mono)) {  // every tell's slot is embase + its sender-order index
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) {
        const uint32_t i = wv * (kBIpt * kWave) + r * kWave + lane;
        if (i < emtot) {
          g.eg[w].key[embase + i] = k[r];
          g.eg[w].src[embase + i] = usrc[i];
          g.eg[w].pay[embase + i] = upay[i];
        }
      }
      if (tid == 0 && g.emc[w]) g.emc[w][b] = emtot;
      return;
    }
    for (int i = tid; i < kBWaves * kRadix; i += kBThreads) whist[i] = 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kBIpt; ++r) {
      const uint32_t i = wv * (kBIpt * kWave) + r * kWave + lane;
      rk[r] = wave_rank(i < emtot, d[r], a.nx_bits, whist + wv * kRadix, ltm);
    }
    __syncthreads();
    if ((uint32_t)tid < nd) {  // per destination: prefix over waves
      uint32_t run = 0;
#pragma unroll
      for (int q = 0; q < kBWaves; ++q) {
        const uint32_t c2 = whist[q * kRadix + tid];
        whist[q * kRadix + tid] = run;
        run += c2;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kBIpt; ++r) {
      const uint32_t i = wv * (kBIpt * kWave) + r * kWave + lane;
      if (i < emtot) {
        const uint32_t o = dbase[d[r]] + whist[wv * kRadix + d[r]] + rk[r];
        g.eg[w].key[o] = k[r];
        g.eg[w].src[o] = usrc[i];
        g.eg[w].pay[o] = upay[i];
      }
    }
  } else if (__syncthreads_or((uint32_t)tid < nd && emtot > 0 && L.nh[tid] == emtot)) {
    // every tell goes to one destination bucket: the sender order is already grouped
    for (uint32_t i = tid; i < emtot; i += kBThreads) {
      g.eg[w].key[embase + i] = src.key[embase + i];
      g.eg[w].src[embase + i] = src.src[embase + i];
      g.eg[w].pay[embase + i] = src.pay[embase + i];
    }
  } else {  // tells in sender order in the em scratch arena: tile-wise stable multisplit
    uint32_t* U32 = reinterpret_cast<uint32_t*>(L.U);
    const SplitLds S{whist, base, ldig, gadj, L.scratch, U32, U32 + kTile, U32 + 2 * kTile};
    const CMsgs in{src.key, src.src, src.pay};
    for (uint32_t sub = 0; sub < emtot; sub += kTile)
      split_tile<kBThreads>(in, (uint32_t)embase + sub, min((uint32_t)kTile, emtot - sub), g.eg[w], a.nx_shift,
                            a.nx_bits, S);
  }
  if (tid == 0 && g.emc[w]) g.emc[w][b] = emtot;
}

#ifdef AGX_ACC_SHADOW
// diagnostic build knob (the round-4 sparse-row counter fault): each wave also
// keeps its emitted count in LDS, reduced from the same per-bucket nall values the acc[3]
// registers add up.  AGX_ACC_SHADOW=1 flushes the LDS shadow as the emitted counter, =2 flushes the
// registers (same code and layout otherwise): which of the two is right tells where the count is lost.
__device__ __forceinline__ uint32_t* acc_shadow() {
  __shared__ uint32_t s[kBWaves];
  return s;
}
#define AGX_SHADOW_ADD(nall)                                                   \
  do {                                                                         \
    const uint32_t sv_ = wave_incl_sum(nall);                                  \
    if (lane_id() == kWave - 1) acc_shadow()[threadIdx.x / kWave] += sv_;      \
  } while (0)
#else
#define AGX_SHADOW_ADD(nall) ((void)0)
#endif

// the block's counters -> its own slot of the per-block stats (summed by k_stats_reduce)
__device__ __forceinline__ void flush_stats(const BucketArgs& a, const uint32_t (&acc)[kBStats]) {
#ifdef AGX_DEBUG_EMIT
  if (acc[3] > (1u << 22) || acc[0] > (1u << 22) || acc[1] > (1u << 22))
    printf("[agx dbg flush] block %u tid %u acc %u %u %u %u %u\n", blockIdx.x, threadIdx.x, acc[0], acc[1], acc[2], acc[3],
           acc[4]);
#endif
  uint32_t v[kBStats];
#pragma unroll
  for (int i = 0; i < kBStats; ++i) v[i] = wave_incl_sum(acc[i]);
#if defined(AGX_ACC_SHADOW) && AGX_ACC_SHADOW == 1
  v[3] = acc_shadow()[threadIdx.x / kWave];  // (lane kWave - 1 flushes: the wave's LDS shadow)
#endif
  if (lane_id() == kWave - 1) {
    unsigned long long* bs = a.bstats + (size_t)blockIdx.x * kBStats;
#pragma unroll
    for (int i = 0; i < kBStats; ++i)
      if (v[i]) atomicAdd(&bs[i], (unsigned long long)v[i]);
  }
}

// bl_given != ~0: the backlog of this bucket was already written (pre-partitioned skewed bucket:
// the inbox holds only the drained messages) and holds bl_given messages.
constexpr uint32_t kWaveRowU32 = 64;  // (multi-rank packing) rows of at least this many u32 are copied by a whole wave


template <bool kLds, bool kWide, uint32_t KM, bool kGather, bool kOwner>
__device__ __forceinline__ void bucket_finish(const BucketArgs& a, const BucketLds& L, uint32_t b, uint32_t lo,
                                              uint32_t cnt, uint32_t a0, uint32_t na, uint32_t w, uint32_t ndead0,
                                              uint32_t (&acc)[kBStats], uint32_t bl_given = 0xFFFFFFFFu,
                                              const uint64_t* pre0 = nullptr, const uint64_t* pre1 = nullptr) {
  const DevParams& P = a.P;
  const int tid = threadIdx.x;
  const uint32_t nhmask = (1u << a.nx_bits) - 1u;
  auto ikey = [&](uint32_t q) -> uint32_t { return kLds ? L.key[q] : a.scr.key[lo + q]; };
  auto isrc = [&](uint32_t q) -> uint32_t { return kLds ? L.src[q] : a.scr.src[lo + q]; };
  auto ipay = [&](uint32_t q) -> uint32_t { return kLds ? L.pay[q] : a.scr.pay[lo + q]; };
  uint32_t* blpre = reinterpret_cast<uint32_t*>(L.U);
  uint64_t* w0s = L.U;
  uint64_t* w1s = L.U + kBucket;
  CrdtHeap H{};
  if (kWide) H = crdt_heap(P);
  // Snapshot rows of bucket b (one lane allocates for its wave / block): the bucket's own heap
  // region [b << bb, (b+1) << bb) (one row per actor) through an LDS cursor, then the overflow
  // area after all regions through the shared cursor — no contended atomic for the common case.
  auto alloc_rows = [&](uint32_t n) -> uint32_t {
    const uint32_t r = atomicAdd(L.rowtop, n);
    if (r + n <= (1u << a.bb)) return (b << a.bb) + r;
    return (a.nb << a.bb) + atomicAdd(H.top, n);
  };

  AGX_STAMP(a, 3);
  // ---- classification per actor (blocked): drained / queued (backlog) / dead letters
  uint32_t nbl_t = 0, ndead = ndead0, blc[kBAct];  // ndead0: this thread's actors' arrivals dropped before the sort
#pragma unroll
  for (int j = 0; j < kBAct; ++j) {
    const uint32_t la = tid * kBAct + j;
    const uint32_t len = L.seg[la + 1] - L.seg[la];
    uint32_t q = 0;
    if (len) {
      const uint32_t ab = L.alive[la];
      if (!(ab & 1u)) {
        ndead += len;
      } else {
        uint32_t C, T;
        mbox_limits(P, ab, C, T);
        const uint32_t keep = (C == 0 || len < C) ? len : C;  // admitted (tail-drop beyond C)
        ndead += len - keep;
        q = keep > T ? keep - T : 0u;
      }
    }
    blc[j] = q;
    nbl_t += q;
  }
  uint32_t bltot;
  uint32_t blex = block_excl_sum<kBThreads>(nbl_t, L.scratch, &bltot);
  constexpr bool kBypass = !kGather && !kOwner;
  const Msgs blw = (kGather || kBypass) ? a.g.bl[w] : a.bl;  // backlog arena written by this superstep
  if (tid == 0) {
    if constexpr (kGather) {
      a.g.blo[w][b] = lo;
      a.g.blc[w][b] = bltot;
    } else {
      a.chunk_off[b] = lo;
      a.chunk_cnt[b] = bl_given != 0xFFFFFFFFu ? bl_given : bltot;
    }
  }
  if (bltot) {
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      blpre[tid * kBAct + j] = blex;
      blex += blc[j];
    }
    __syncthreads();
    // ORSet populations (2 KB rows): wave-uniform trip count, the row copies below take the whole
    // wave; counters (64-128 B rows): a lane per message, as before
    constexpr bool kBigRows = kWide && (KM & kb(AGX_KIND_ORSET)) != 0;
    const uint32_t qstart = kBigRows ? (uint32_t)tid - lane_id() : (uint32_t)tid;
    for (uint32_t qb = qstart; qb < cnt; qb += kBThreads) {  // queued messages, in actor order
      const uint32_t q = kBigRows ? qb + lane_id() : qb;
      const bool valid = q < cnt;
      const uint32_t key = valid ? ikey(q) : 0u;
      const uint32_t la = key & ((1u << a.bb) - 1u);
      const uint32_t p = q - L.seg[la];
      const uint32_t len = L.seg[la + 1] - L.seg[la];
      const uint32_t ab = L.alive[la];
      uint32_t C, T;
      mbox_limits(P, ab, C, T);
      const uint32_t keep = (C == 0 || len < C) ? len : C;
      const bool queued = valid && (ab & 1u) && p >= T && p < keep;
      const uint32_t sv = valid ? isrc(q) : 0u;
      uint32_t pv = valid ? ipay(q) : 0u;
      if (kWide) {  // a queued state gossip outlives its row's superstep: copy the row forward
        const bool need = queued && is_wide(sv);
        const uint64_t m = __ballot(need);
        if (m) {
          const uint32_t lane = lane_id(), leader = (uint32_t)__builtin_ctzll(m);
          uint32_t base = 0;
          if (lane == leader) base = alloc_rows((uint32_t)__popcll(m));
          base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);
          const uint32_t h = base + (uint32_t)__popcll(m & lanemask_lt());
          if (need && h >= H.rows) atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
          if (!kBigRows && need && h < H.rows) {  // counter rows: each lane its own
            const uint4* s = reinterpret_cast<const uint4*>(H.row(pv & kHandleMask));
            uint4* d = reinterpret_cast<uint4*>(H.wrow(h));
            for (uint32_t k2 = 0; k2 < H.pw / 4; ++k2) d[k2] = s[k2];
          }
          // ORSet rows (2 KB): the wave copies them one after the other, 16 B per lane -- whole
          // lines per instruction instead of each lane walking its own row in a load-store chain
          // (same-box A/B: C4 ORSet +10 %, ORSet delta +18 %)
          for (uint64_t mm = kBigRows ? m : 0ull; mm; mm &= mm - 1) {
            const int i = __builtin_ctzll(mm);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)h, i);
            const uint32_t pi = (uint32_t)__builtin_amdgcn_readlane((int)pv, i), si = pi & kHandleMask;
            if (hi < H.rows) {
              const uint4* s = reinterpret_cast<const uint4*>(H.row(si));
              uint4* d = reinterpret_cast<uint4*>(H.wrow(hi));
              const uint32_t q4 = H.pw / 4;
              uint32_t n4 = q4;
              if (pi & AGX_DELTA_ROW_BIT) {  // a DeltaPropagation: its used length (dl_group_row), not the pitch
                const uint32_t used = reinterpret_cast<const uint32_t*>(s)[H.pw - 1];
                n4 = min(q4, (used + 3u) / 4u);
                if (lane == 0 && n4 < q4) d[q4 - 1] = s[q4 - 1];  // (the length word travels too)
              }
              for (uint32_t k2 = lane; k2 < n4; k2 += kWave) d[k2] = s[k2];
            }
          }
          if (need) pv = (pv & ~kHandleMask) | h;
        }
      }
      if (queued) {
        const uint32_t o = lo + blpre[la] + (p - T);
        blw.key[o] = key;
        blw.src[o] = sv;
        blw.pay[o] = pv;
      }
    }
    // (single rank: the backlog stays in place for the next apply — not part of the next sort)
  }
  __syncthreads();

  AGX_STAMP(a, 4);
  // ---- FANOUT with one tell per message (C3): every drained message's Zipf destination is looked
  // up here, the four items of a thread in lockstep (index range, then each binary-search step's
  // loads together, then the permutation), instead of ~5 dependent loads per message inside the
  // serial per-actor drain.  The destination replaces the message's sender in LDS (FANOUT does not
  // read it); the drain emits exactly what apply_msg would (same hash, same lookup).
  constexpr bool kFanPre = !kWide && kLds && KM == kb(AGX_KIND_FANOUT);
  const bool fan_pre = kFanPre && P.fan_k == 1 && a.kmax == 1;
  if (kFanPre && fan_pre) {
    uint32_t qi[kBIpt], lo[kBIpt], hi[kBIpt], uu[kBIpt];
    bool need[kBIpt];
    bool dir[kBIpt];
#pragma unroll
    for (int r = 0; r < kBIpt; ++r) {
      const uint32_t q = r * kBThreads + tid;
      qi[r] = q;
      need[r] = false;
      uu[r] = 0;
      if (q < cnt) {
        const uint32_t la = L.key[q] & ((1u << a.bb) - 1u), s0 = L.seg[la], len = L.seg[la + 1] - s0;
        const uint32_t ab = L.alive[la], pv = L.pay[q];
        uint32_t Ca, Ta;
        mbox_limits(P, ab, Ca, Ta);
        if (la < na && (ab & 1u) && q - s0 < min(len, Ta) && (pv >> 24) > 0) {
          const uint32_t l = a0 + la, self = P.R > 1 ? P.gid[l] : l;
          const uint64_t rr = fanout_rand(P.fan_seed, self, pv & 0x00FFFFFFu, 0);
          need[r] = true;
          uu[r] = (uint32_t)(rr >> 32);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kBIpt; ++r) {
      const uint32_t t = uu[r] >> (32 - kZipfBits);
      const uint2 z = need[r] ? P.zipf_ent[t] : make_uint2(0u, 0u);
      dir[r] = z.y == kZipfDirect;  // (the Zipf head: the destination itself, no search)
      lo[r] = z.x;
      hi[r] = dir[r] ? z.x : z.y;
    }
    for (;;) {  // zipf_dest's binary search, one step of every item per round
      bool more = false;
      uint32_t c[kBIpt];
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) c[r] = lo[r] < hi[r] ? P.zipf_cdf[(lo[r] + hi[r]) >> 1] : 0u;
#pragma unroll
      for (int r = 0; r < kBIpt; ++r)
        if (lo[r] < hi[r]) {
          const uint32_t mid = (lo[r] + hi[r]) >> 1;
          if (c[r] >= uu[r]) hi[r] = mid; else lo[r] = mid + 1;
          more |= lo[r] < hi[r];
        }
      if (!more) break;
    }
    uint32_t d[kBIpt];
#pragma unroll
    for (int r = 0; r < kBIpt; ++r) d[r] = need[r] ? (dir[r] ? lo[r] : P.zipf_perm[lo[r]]) : 0u;
#pragma unroll
    for (int r = 0; r < kBIpt; ++r)
      if (need[r]) L.src[qi[r]] = d[r];
    __syncthreads();
  }
  // ---- prefetch kind + state words 0/1 of actors with mail (striped: coalesced).  All loads
  // are issued before the LDS stores (the stores go through generic pointers).
  // FORWARD_RR (C5) single pass: each actor's out-edge row and the destination of its next
  // round-robin edge are fetched here for all four actors at once, instead of two dependent
  // loads (row_ptr, then col) per message inside the serial drain (fdeg = kNoHint: no hint).
  constexpr bool kFwd = !kWide && KM == kb(AGX_KIND_FORWARD_RR);
  constexpr bool kUnrollActors = KM == kb(AGX_KIND_RING);  // single pass: see sp_actor below
  // single pass, behaviours other than the ring: the actors with mail are drained one per thread
  // (a compacted list) instead of four fixed actors per thread one after the other -- a sparse
  // bucket (C5: ~150 of 2048 actors with mail) then costs one actor's drain, not up to four
  // (FORWARD_RR populations only: C5 3.19e9 vs 2.76e9 without it; C1 ping-pong, every actor active,
  // pays the list build for nothing: 2.41e9 with it, 2.50e9 without; C3 tree within noise)
  constexpr bool kCompact = !kWide && !kUnrollActors && kCompactDrain && KM == kb(AGX_KIND_FORWARD_RR);
  constexpr bool kFwdHint = kFwd && !kCompact;  // (the compacted drain loads its hints itself)
  constexpr uint32_t kNoHint = 0xFFFFFFFFu;
  uint64_t frb[kBAct];
  uint32_t fdeg[kBAct], fdst[kBAct];
  {
    uint32_t kd[kBAct];
    uint64_t x0[kBAct], x1[kBAct], fre[kBAct];
    constexpr bool kKindNeeded = kWide || (KM & (KM - 1)) != 0 || (KM & kb(AGX_KIND_COMPILED)) != 0;
    if constexpr (!kGather) {  // (multi-pass: the branchy form measured 6 % faster at 10^8 actors)
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        const uint32_t la = j * kBThreads + tid;
        const bool has = la < na && (L.alive[la] & 1u) && L.seg[la + 1] != L.seg[la];
        const uint32_t l = a0 + la;
        kd[j] = has && kKindNeeded ? P.kind[l] : 0u;  // single-kind variants never read it
        if constexpr (kWide) {  // (CRDT engines: actor-major rows, wide_state)
          x0[j] = has ? wide_state(P, l)[0] : 0ull;
          x1[j] = has && P.W > 1 ? wide_state(P, l)[wide_nl(P)] : 0ull;
        } else {
          x0[j] = has ? ldg64(P.state, sidx(P, l, 0)) : 0ull;  // (32-bit offsets: one VGPR per address)
          x1[j] = has && P.W > 1 ? ldg64(P.state, sidx(P, l, 1)) : 0ull;
        }
        if constexpr (kFwdHint) {
          frb[j] = has ? P.row_ptr[l] : 0ull;
          fre[j] = has ? P.row_ptr[l + 1] : ~0ull;  // (no mail: deg out of range -> no hint)
        }
      }
    } else {
    uint32_t hasm = 0, li[kBAct];  // actors with mail; their local ids (0 for the others)
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      const uint32_t la = j * kBThreads + tid;
      const bool has = la < na && (L.alive[la] & 1u) && L.seg[la + 1] != L.seg[la];
      hasm |= has ? 1u << j : 0u;
      li[j] = has ? a0 + la : 0u;
    }
    // fused: every load issued unconditionally, back to back (actors without mail read actor 0's
    // words: one cached line, no traffic), then masked -- no branch around a load, no wait between
    // them (fused RING spills 11 -> 2 VGPRs; 1M apply -3.6 %, same-box A/B)
    const uint32_t w1off = P.W > 1 ? P.sw : 0u;
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      kd[j] = kKindNeeded ? P.kind[li[j]] : 0u;  // single-kind variants never read it
      if (pre0) {  // (fused fast path: loaded at the start of the bucket, beside the table row)
        x0[j] = pre0[j];
        x1[j] = pre1[j];
      } else if constexpr (kWide) {
        x0[j] = wide_state(P, li[j])[0];
        x1[j] = wide_state(P, li[j])[w1off ? wide_nl(P) : 0];
      } else {
        x0[j] = ldg64(P.state, li[j] * P.sa);  // (32-bit offsets: one VGPR per address)
        x1[j] = ldg64(P.state, li[j] * P.sa + w1off);
      }
      if constexpr (kFwdHint) {
        frb[j] = P.row_ptr[li[j]];
        fre[j] = P.row_ptr[li[j] + 1];
      }
    }
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      const bool has = (hasm >> j) & 1u;
      kd[j] = has ? kd[j] : 0u;
      x0[j] = has ? x0[j] : 0ull;
      x1[j] = has && P.W > 1 ? x1[j] : 0ull;
      if constexpr (kFwdHint) {
        frb[j] = has ? frb[j] : 0ull;
        fre[j] = has ? fre[j] : ~0ull;  // (no mail: deg out of range -> no hint)
      }
    }
    }  // fused
    if constexpr (kFwdHint) {
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        const uint64_t deg = fre[j] - frb[j];
        const bool ok = deg < kNoHint && x1[j] <= 0xFFFFFFFFull;
        fdeg[j] = ok ? (uint32_t)deg : kNoHint;
        fdst[j] = ok && deg ? P.col[frb[j] + (uint32_t)x1[j] % (uint32_t)deg] : 0u;
      }
    }
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      const uint32_t la = j * kBThreads + tid;
      L.ecnt[la] = 0;
      L.kind[la] = (uint8_t)kd[j];
      w0s[la] = x0[j];
      w1s[la] = x1[j];
    }
  }
  uint32_t ndel = 0, nunh = 0, nall = 0, nact = 0, emtot = 0;
  const uint64_t embase = (uint64_t)lo * a.kmax;  // this bucket's slice of the tell arena
  if (!kWide && a.kmax == 1) {
    // ---- single pass (each message emits <= 1 tell): drain + apply; tells are staged over the
    // actor's own, already consumed, inbox slots (tell e of an actor <= message index q that made it):
    // in LDS (fast path) or in the bucket's scratch copy (skew launch)
    uint32_t* const stk = kLds ? L.key : a.scr.key + lo;
    uint32_t* const sts = kLds ? L.src : a.scr.src + lo;
    uint32_t* const stp = kLds ? L.pay : a.scr.pay + lo;
    uint32_t ecl[kBAct];
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    uint32_t alist[kBAct];  // kCompact: this thread's actors with mail (active index x * kBThreads + tid)
    if constexpr (kCompact) {
      uint32_t c = 0;
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        const uint32_t la = j * kBThreads + tid;
        c += la < na && L.seg[la + 1] != L.seg[la] && (L.alive[la] & 1u) ? 1u : 0u;
      }
      uint32_t nactive;
      uint32_t pos = block_excl_sum<kBThreads>(c, L.scratch, &nactive);  // (syncs: LDS state stores done)
      uint32_t* const actl = L.key;  // (the inbox keys are not read any more: the drains read src / pay)
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        const uint32_t la = j * kBThreads + tid;
        if (la < na && L.seg[la + 1] != L.seg[la] && (L.alive[la] & 1u)) actl[pos++] = la;
      }
      __syncthreads();
#pragma unroll
      for (int x = 0; x < kBAct; ++x) {
        const uint32_t i = x * kBThreads + tid;
        alist[x] = i < nactive ? actl[i] : kNone;
      }
      __syncthreads();  // (every entry read before the drains stage tells over L.key)
    }
    auto act_of = [&](int j) -> uint32_t { return kCompact ? alist[j] : (uint32_t)(j * kBThreads + tid); };
    // PingPong populations (C1): a drain's messages are independent -- each replies (sender,
    // payload) and the state is a count -- so an actor's run needs no serial loop: per actor the
    // closed form (k = the messages processed up to and including the stopping one, w0 -= k, w1 += k),
    // then every inbox position writes its own reply in place, the block's 512 threads at once
    // (a bucket of 32 ping-pong actors draining 50 messages each otherwise runs on 32 lanes of one
    // wave, one message after the other).  Only when every sender in the inbox is an actor of the
    // population (a host-side sender's reply goes through the outbox: the serial path).
    // (Populations with PingPong actors run the all-kinds variant: the bucket takes this drain when
    // every actor with mail in it is a PingPong actor.)
    constexpr bool kPPar = kLds && !kWide && (KM & kb(AGX_KIND_PINGPONG)) != 0 &&
                           (KM & kb(AGX_KIND_COMPILED)) == 0 && kPingPar;
    bool ppar = false;
    if constexpr (kPPar) {
      bool bad = false;
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) {
        const uint32_t q = r * kBThreads + tid;
        bad |= q < cnt && L.src[q] >= P.n_global;
      }
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        const uint32_t la = j * kBThreads + tid;
        bad |= la < na && L.seg[la + 1] != L.seg[la] && (L.alive[la] & 1u) && (KM & (KM - 1)) != 0 &&
               L.kind[la] != AGX_KIND_PINGPONG;  // (a single-kind variant leaves L.kind unread)
      }
      __syncthreads();
      if (tid == 0) L.scratch[0] = 0u;
      __syncthreads();
      if (bad) L.scratch[0] = 1u;
      __syncthreads();
      ppar = L.scratch[0] == 0u;
    }
    auto sp_actor = [&](int j) {
      const uint32_t la = act_of(j);
      ecl[j] = 0;
      if (kCompact && la == kNone) return;
      const uint32_t s0 = L.seg[la], len = L.seg[la + 1] - s0;
      if (la >= na || !len || !(L.alive[la] & 1u)) return;
      const uint32_t l = a0 + la;
      const uint32_t self = P.R > 1 ? P.gid[l] : l;
      EmitterLds em{&P, stk, sts, stp, s0, self, 0, 0, L.nh, a.nx_shift, nhmask};
      uint64_t wv[2] = {w0s[la], w1s[la]};
      uint32_t Ca, Ta;
      mbox_limits(P, L.alive[la], Ca, Ta);
      const uint32_t nd = min(len, Ta);
      uint32_t kcur = L.kind[la];  // (a compiled behaviour's become changes it)
      ++nact;
      if constexpr (kPPar) {
        if (ppar) {  // apply_msg's PINGPONG over the run: message w0 (if drained) is the stopping one
          const uint64_t w0 = wv[0];
          const bool stops = w0 < nd;
          const uint32_t k = stops ? (uint32_t)w0 + 1u : nd;
          wv[0] -= k;
          wv[1] += k;
          ndel += k;
          nall += k;
          if (stops) {
            if constexpr (kGather) P.alive[l] = L.alive[la] & 0xFEu;
            else P.stopq[atomicAdd(P.nstop, 1u)] = l;
            ndead += nd - k;  // drained-but-unprocessed after the stop
          }
          stg64(P.state, sidx(P, l, 0), wv[0]);
          if (P.W > 1) stg64(P.state, sidx(P, l, 1), wv[1]);
          ecl[j] = k;
          L.ecnt[la] = k;
          return;
        }
      }
      uint64_t hb = 0;
      uint32_t hdeg = kNoHint, hdst = 0;
      bool fresh = true;  // no forward yet: the next edge is fdst
      uint32_t fpre[kFwdPre], nfw = 0;  // (kCompact) the first kFwdPre forwards' destinations, forwards so far
      if constexpr (kFwdHint) {  // (j is wave-uniform)
        hb = j == 0 ? frb[0] : j == 1 ? frb[1] : j == 2 ? frb[2] : frb[3];
        hdeg = j == 0 ? fdeg[0] : j == 1 ? fdeg[1] : j == 2 ? fdeg[2] : fdeg[3];
        hdst = j == 0 ? fdst[0] : j == 1 ? fdst[1] : j == 2 ? fdst[2] : fdst[3];
      }
      if constexpr (kFwd && kCompact) {
        // this actor's out-edge row, then the destinations of its next kFwdPre round-robin edges in
        // one round trip (forward m of the drain takes edge (cursor + m) mod deg: apply_msg's
        // arithmetic), so a drain of up to kFwdPre forwards has no dependent global load
        const uint64_t rb = P.row_ptr[l], deg = P.row_ptr[l + 1] - rb;
        if (deg < kNoHint && wv[1] + kFwdPre <= 0xFFFFFFFFull) {
          hb = rb;
          hdeg = (uint32_t)deg;
          uint32_t e = deg ? (uint32_t)wv[1] % (uint32_t)deg : 0u;
#pragma unroll
          for (uint32_t m = 0; m < kFwdPre; ++m) {
            fpre[m] = deg && m < nd ? P.col[rb + e] : 0u;
            e = e + 1u == (uint32_t)deg ? 0u : e + 1u;
          }
        }
      }
      for (uint32_t q = 0; q < nd; ++q) {
        const uint32_t sv = sts[s0 + q], pv = stp[s0 + q];
        uint32_t r;
        if (kFanPre && fan_pre) {  // apply_msg's FANOUT with the destination looked up above (in sv)
          wv[0] += 1;
          wv[1] += pv;
          const uint32_t ttl = pv >> 24;
          if (ttl > 0) {
            const uint64_t rr = fanout_rand(P.fan_seed, self, pv & 0x00FFFFFFu, 0);
            em(sv, ((ttl - 1) << 24) | ((uint32_t)rr & 0x00FFFFFFu));
          }
          r = AGX_RES_SAME;
        } else if (kFwd && hdeg != kNoHint && wv[1] <= 0xFFFFFFFFull) {
          // apply_msg's FORWARD_RR with the prefetched row (same cursor arithmetic)
          wv[0] += 1;
          if (pv > 0 && hdeg) {
            uint32_t d;
            if constexpr (kCompact) {
              d = 0u;
#pragma unroll
              for (uint32_t m = 0; m < kFwdPre; ++m) d = nfw == m ? fpre[m] : d;
              if (nfw >= kFwdPre) d = P.col[hb + (uint32_t)wv[1] % hdeg];
              ++nfw;
            } else {
              d = fresh ? hdst : P.col[hb + (uint32_t)wv[1] % hdeg];
              fresh = false;
            }
            wv[1] += 1;
            em(d, pv - 1);
          }
          r = AGX_RES_SAME;
        } else {
          r = apply_msg<KM>(P, kcur, self, l, wv, sv, pv, em);
        }
        ++ndel;
        if (r == AGX_RES_UNHANDLED) ++nunh;
        if (r == AGX_RES_STOPPED) {
          if constexpr (kGather) P.alive[l] = L.alive[la] & 0xFEu;  // fused: only this block reads this bucket's flags
          else P.stopq[atomicAdd(P.nstop, 1u)] = l;
          ndead += nd - q - 1;  // drained-but-unprocessed after the stop
          break;
        }
      }
      stg64(P.state, sidx(P, l, 0), wv[0]);
      if (P.W > 1) stg64(P.state, sidx(P, l, 1), wv[1]);
      if constexpr ((KM & kb(AGX_KIND_COMPILED)) != 0)
        if (kcur != L.kind[la]) P.kind[l] = (uint8_t)kcur;
      nall += em.n_all;
      ndead += em.n_all - em.n_valid;
      ecl[j] = em.n_valid;
      L.ecnt[la] = em.n_valid;
    };
    // the ring's single-message actors: four independent drains (their LDS and state latencies
    // overlap); other behaviours keep one serial loop (measured: C5 FORWARD_RR is 9 % slower unrolled)
    if constexpr (kUnrollActors) {
      sp_actor(0); sp_actor(1); sp_actor(2); sp_actor(3);
    } else {
#pragma unroll 1
      for (int j = 0; j < kBAct; ++j) sp_actor(j);
    }
    __syncthreads();
    AGX_STAMP(a, 5);
    {  // exclusive scan of tell counts in actor (= sender) order
      uint32_t ec[kBAct], run = 0;
      const uint4 v = reinterpret_cast<const uint4*>(L.ecnt)[tid];
      ec[0] = v.x; ec[1] = v.y; ec[2] = v.z; ec[3] = v.w;
#pragma unroll
      for (int j = 0; j < kBAct; ++j) run += ec[j];
      uint32_t ex = block_excl_sum<kBThreads>(run, L.scratch, &emtot);
      uint32_t o[kBAct];
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        o[j] = ex;
        ex += ec[j];
      }
      reinterpret_cast<uint4*>(L.ecnt)[tid] = make_uint4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
    AGX_STAMP(a, 6);
    // PingPong message-parallel drain: every processed message's reply straight to its place in
    // sender order (tell q of an actor = its message q, at the actor's scanned offset + q): U (the
    // grouped paths) or the bucket's tell chunk, with the destination histogram
    auto ppar_write = [&](auto put) {
      const uint32_t amask = (1u << a.bb) - 1u;
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) {
        const uint32_t q = r * kBThreads + tid;
        if (q >= cnt) continue;
        const uint32_t la = L.key[q] & amask, e = q - L.seg[la], o = L.ecnt[la];
        const uint32_t oend = la + 1u < (uint32_t)kBucket ? L.ecnt[la + 1] : emtot;
        if (o + e >= oend) continue;  // (after the stopping message / beyond the throughput cap)
        const uint32_t d = L.src[q], l = a0 + la;
        const uint32_t k = P.R > 1 ? P.route[d] : d;
        put(o + e, k, P.R > 1 ? P.gid[l] : l, L.pay[q]);
        lds_hist_inc(L.nh, (k >> a.nx_shift) & nhmask);
      }
    };
    if constexpr ((kGather || kOwner) && kLds) {
      // compact the staged tells in sender order into U (free: state was written back), then
      // group them by destination straight into this superstep's tell arena
      uint32_t* ukey = reinterpret_cast<uint32_t*>(L.U);
      auto compact = [&](int j) {
        if (ppar || !ecl[j]) return;
        const uint32_t la = act_of(j);
        const uint32_t s0 = L.seg[la], o = L.ecnt[la];
        for (uint32_t e = 0; e < ecl[j]; ++e) {
          ukey[o + e] = L.key[s0 + e];
          ukey[kBucket + o + e] = L.src[s0 + e];
          ukey[2 * kBucket + o + e] = L.pay[s0 + e];
        }
      };
      if constexpr (kUnrollActors) {
        compact(0); compact(1); compact(2); compact(3);
      } else {
#pragma unroll 1
        for (int j = 0; j < kBAct; ++j) compact(j);
      }
      if constexpr (kPPar)
        if (ppar)
          ppar_write([&](uint32_t i, uint32_t k, uint32_t sv, uint32_t pv) {
            ukey[i] = k;
            ukey[kBucket + i] = sv;
            ukey[2 * kBucket + i] = pv;
          });
      __syncthreads();
      group_tells<true>(a, L, b, w, embase, emtot, a.em);
    } else {
      // compact the staged tells into the bucket's tell chunk (lane-consecutive actors: coalesced)
      constexpr bool kMeta = !kGather && !kOwner && kLds;  // bypass fast path: the chunk's key summary
      uint32_t* const ck = reinterpret_cast<uint32_t*>(L.U);  // (free: the state was written back)
      auto compact = [&](int j) {
        if (ppar || !ecl[j]) return;
        const uint32_t la = act_of(j);
        const uint32_t s0 = L.seg[la], o = L.ecnt[la];
        for (uint32_t e = 0; e < ecl[j]; ++e) {
          a.em.key[embase + o + e] = stk[s0 + e];
          a.em.src[embase + o + e] = sts[s0 + e];
          a.em.pay[embase + o + e] = stp[s0 + e];
          if constexpr (kMeta) ck[o + e] = stk[s0 + e];
        }
      };
      if constexpr (kUnrollActors) {
        compact(0); compact(1); compact(2); compact(3);
      } else {
#pragma unroll 1
        for (int j = 0; j < kBAct; ++j) compact(j);
      }
      if constexpr (kPPar)
        if (ppar)
          ppar_write([&](uint32_t i, uint32_t k, uint32_t sv, uint32_t pv) {
            a.em.key[embase + i] = k;
            a.em.src[embase + i] = sv;
            a.em.pay[embase + i] = pv;
            if constexpr (kMeta) ck[i] = k;
          });
      if constexpr (kGather || kOwner) {  // (skew launch) grouped by destination from the em arena
        __syncthreads();
        group_tells<false>(a, L, b, w, embase, emtot, a.em);
      }
      if constexpr (kMeta) {
        // identity grouping (k_ident_combine): first / last key of the chunk and its descents
        // (positions i with key[i] < key[i - 1]) in sender order
        if (a.emmeta) {
          __syncthreads();
          uint32_t nd = 0, dp = 0;
#pragma unroll
          for (uint32_t i = 4 * tid; i < 4 * tid + 4; ++i)
            if (i > 0 && i < emtot && ck[i] < ck[i - 1]) {
              ++nd;
              dp = i;
            }
          uint32_t tnd, tdp;
          block_excl_sum2<kBThreads>(nd, nd ? dp : 0u, L.scratch, &tnd, &tdp);  // (tdp is THE position if tnd == 1)
          if (tid == 0) a.emmeta[b] = make_uint4(emtot ? ck[0] : 0u, emtot ? ck[emtot - 1] : 0u, tnd, tdp);
        }
      } else if constexpr (!kGather && !kOwner) {
        if (a.emmeta && tid == 0) a.emmeta[b] = make_uint4(0u, 0u, 2u, 0u);  // (not summarised: forces a sort)
      }
    }
  } else {
  uint32_t nrows_t = 0;  // snapshot rows this thread's actors will write (kWide)
  uint32_t nvoid = 0;    // delta-CRDT: void tells (NoDeltaPlaceholder groups) this thread left
  // ---- phase A: emissions per actor (drain min(len, T) messages in order)
  #pragma unroll 1
    for (int j = 0; j < kBAct; ++j) {
      const uint32_t la = j * kBThreads + tid;
      const uint32_t s0 = L.seg[la], len = L.seg[la + 1] - s0;
      if (la >= na || !len || !(L.alive[la] & 1u)) continue;
      const uint32_t l = a0 + la;
      const uint32_t self = P.R > 1 ? P.gid[l] : l;
      Emitter<false> em{&P, {}, 0, self, 0, 0, L.nh, a.nx_shift, nhmask};
      uint64_t wv[2] = {w0s[la], w1s[la]};  // behaviours read/write state words 0-1 only
      uint32_t Ca, Ta;
      mbox_limits(P, L.alive[la], Ca, Ta);
      const uint32_t nd = min(len, Ta);
      uint32_t kd = L.kind[la];
      if (kWide && is_crdt(kd)) {
        DeltaSim ds;
        ds.on = false;
        for (uint32_t q = 0; q < nd; ++q)
          em.count(crdt_count<KM>(P, kd, self, l, isrc(s0 + q), ipay(s0 + q), &nrows_t, ds));
      } else if constexpr (!kLds) {  // messages in global scratch: loads issued kPF at a time
        bool stop = false;
        for (uint32_t q0 = 0; q0 < nd && !stop; q0 += kPF) {
          uint32_t svb[kPF], pvb[kPF];
#pragma unroll
          for (int u = 0; u < kPF; ++u)
            if (q0 + u < nd) {
              svb[u] = isrc(s0 + q0 + u);
              pvb[u] = ipay(s0 + q0 + u);
            }
#pragma unroll
          for (int u = 0; u < kPF; ++u) {
            if (stop || q0 + u >= nd) continue;
            if (kWide && is_wide(svb[u])) continue;  // not in this behaviour's protocol: unhandled, no tells
            if (apply_msg<KM>(P, kd, self, l, wv, svb[u], pvb[u], em) == AGX_RES_STOPPED) stop = true;
          }
        }
      } else {
        for (uint32_t q = 0; q < nd; ++q) {
          const uint32_t sv = isrc(s0 + q);
          if (kWide && is_wide(sv)) continue;  // not in this behaviour's protocol: unhandled, no tells
          const uint32_t r = apply_msg<KM>(P, kd, self, l, wv, sv, ipay(s0 + q), em);
          if (r == AGX_RES_STOPPED) break;
        }
      }
      L.ecnt[la] = em.n_valid;
    }
    __syncthreads();
    AGX_STAMP(a, 5);
    // ---- exclusive scan of emission counts in actor (= sender) order
      {
      uint32_t ec[kBAct], run = 0;
      const uint4 v = reinterpret_cast<const uint4*>(L.ecnt)[tid];
      ec[0] = v.x; ec[1] = v.y; ec[2] = v.z; ec[3] = v.w;
  #pragma unroll
      for (int j = 0; j < kBAct; ++j) run += ec[j];
      uint32_t ex = block_excl_sum<kBThreads>(run, L.scratch, &emtot);
      uint32_t o[kBAct];
  #pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        o[j] = ex;
        ex += ec[j];
      }
      reinterpret_cast<uint4*>(L.ecnt)[tid] = make_uint4(o[0], o[1], o[2], o[3]);
    }
    uint32_t row_cursor = 0;
    if (kWide) {  // this block's snapshot rows: one heap allocation, thread ranges by scan
      uint32_t rtot;
      const uint32_t rex = block_excl_sum<kBThreads>(nrows_t, L.scratch, &rtot);
      if (tid == 0) {
        const uint32_t base = rtot ? alloc_rows(rtot) : 0u;
        if (base + rtot > H.rows) atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
        L.scratch[kBWaves] = base;
      }
      __syncthreads();
      row_cursor = L.scratch[kBWaves] + rex;
    }
    __syncthreads();
  
    AGX_STAMP(a, 6);
    // ---- phase B: apply for real, write tells (sender order) and state
    // (ORSet-only full-state variant: the state effects of each replica's run are applied by
    // k_orset_merge after the apply; L.ecnt[la] = the run's first snapshot row, or ~0)
    constexpr bool kOrWave = kWide && KM == kb(AGX_KIND_ORSET);
  #pragma unroll 1
    for (int j = 0; j < kBAct; ++j) {
      const uint32_t la = j * kBThreads + tid;
      const uint32_t s0 = L.seg[la], len = L.seg[la + 1] - s0;
      if (la >= na || !len || !(L.alive[la] & 1u)) {
        if constexpr (kOrWave) L.ecnt[la] = 0xFFFFFFFFu;
        continue;
      }
      const uint32_t l = a0 + la;
      const uint32_t self = P.R > 1 ? P.gid[l] : l;
      Emitter<true> em{&P, a.em, embase + L.ecnt[la], self, 0, 0, L.nh, a.nx_shift, nhmask};
      uint64_t wv[2] = {w0s[la], w1s[la]};  // behaviours read/write state words 0-1 only
      uint32_t Ca, Ta;
      mbox_limits(P, L.alive[la], Ca, Ta);
      const uint32_t nd = min(len, Ta);
      uint32_t kd = L.kind[la];
      ++nact;
      if (kWide && is_crdt(kd)) {
        if constexpr (kOrWave) {  // protocol here, state effects by k_orset_merge (agx_crdt.h)
          bool work = false;
          const uint32_t rc0 = row_cursor;
          nunh += orset_protocol(P, self, s0, nd, isrc, ipay, row_cursor, em, &work);
          ndel += nd;
          L.ecnt[la] = work ? rc0 : 0xFFFFFFFFu;  // (this actor's tell offset is no longer needed)
        } else if (kCrdtSched) {
          // the wave's lanes are 64 replicas, each with its own mix of messages (delta mode: a tick, an
          // update, DeltaPropagations): instead of the q-th message of every lane together (the wave
          // walks every kind's path each step), each step applies the next message of the lanes whose
          // next message is of the class most lanes have next -- a lane still applies its messages in
          // order, and its tells and rows go where phase A counted them
          uint32_t q = 0;
          for (;;) {
            const uint32_t sv = q < nd ? isrc(s0 + q) : 0u, pv = q < nd ? ipay(s0 + q) : 0u;
            const uint32_t cls = q >= nd ? 7u : crdt_class(sv, pv);
            uint32_t best = 7u, bn = 0;
#pragma unroll
            for (uint32_t c = 0; c < 5; ++c) {
              const uint32_t m = (uint32_t)__popcll(__ballot(cls == c));
              if (m > bn) bn = m, best = c;
            }
            if (best == 7u) break;
            if (cls == best) {
              const uint32_t r = crdt_apply<KM>(P, H, kd, self, l, sv, pv, row_cursor, em);
              ++ndel;
              if (r == AGX_RES_UNHANDLED) ++nunh;
              ++q;
            }
          }
        } else {
          for (uint32_t q = 0; q < nd; ++q) {
            const uint32_t r = crdt_apply<KM>(P, H, kd, self, l, isrc(s0 + q), ipay(s0 + q), row_cursor, em);
            ++ndel;
            if (r == AGX_RES_UNHANDLED) ++nunh;
          }
        }
      } else {
        bool stop = false;
        constexpr uint32_t kW = kLds ? 1u : (uint32_t)kPF;  // global scratch: loads issued kPF at a time
        for (uint32_t q0 = 0; q0 < nd && !stop; q0 += kW) {
          uint32_t svb[kW], pvb[kW];
#pragma unroll
          for (uint32_t u = 0; u < kW; ++u)
            if (q0 + u < nd) {
              svb[u] = isrc(s0 + q0 + u);
              pvb[u] = ipay(s0 + q0 + u);
            }
#pragma unroll
          for (uint32_t u = 0; u < kW; ++u) {
            if (stop || q0 + u >= nd) continue;
            ++ndel;
            if (kWide && is_wide(svb[u])) {
              ++nunh;
              continue;
            }
            const uint32_t r = apply_msg<KM>(P, kd, self, l, wv, svb[u], pvb[u], em);
            if (r == AGX_RES_UNHANDLED) ++nunh;
            if (r == AGX_RES_STOPPED) {
              if constexpr (kGather) P.alive[l] = L.alive[la] & 0xFEu;  // fused: only this block reads this bucket's flags
              else P.stopq[atomicAdd(P.nstop, 1u)] = l;
              ndead += nd - (q0 + u) - 1;  // drained-but-unprocessed after the stop
              stop = true;
            }
          }
        }
        if constexpr (kWide) {
          wide_state(P, l)[0] = wv[0];
          if (P.W > 1) wide_state(P, l)[wide_nl(P)] = wv[1];
        } else {
          stg64(P.state, sidx(P, l, 0), wv[0]);
          if (P.W > 1) stg64(P.state, sidx(P, l, 1), wv[1]);
        }
        if constexpr ((KM & kb(AGX_KIND_COMPILED)) != 0)
          if (kd != L.kind[la]) P.kind[l] = (uint8_t)kd;
        if constexpr (kOrWave) L.ecnt[la] = 0xFFFFFFFFu;
      }
      nall += em.n_all;
      ndead += em.n_all - em.n_valid;
      nvoid += em.n_void;
#ifdef AGX_DEBUG_EMIT
      if (em.n_all > 4096u || nall > (1u << 22))
        printf("[agx dbg actor] b %u la %u kind %u nd %u n_all %u n_valid %u nall %u pos %llu base %llu\n", b, la, kd, nd,
               em.n_all, em.n_valid, nall, (unsigned long long)em.pos, (unsigned long long)(embase + L.ecnt[la]));
#endif
    }
    if constexpr (kOrWave) {  // the runs with state work -> k_orset_merge's list (wave-aggregated slots)
      const uint32_t lane = lane_id();
  #pragma unroll 1
      for (int j = 0; j < kBAct; ++j) {
        const uint32_t la = j * kBThreads + tid;
        const uint32_t rc0 = L.ecnt[la];
        const bool work = rc0 != 0xFFFFFFFFu;
        uint32_t nd = 0;
        if (work) {
          uint32_t Ca, Ta;
          mbox_limits(P, L.alive[la], Ca, Ta);
          nd = min(L.seg[la + 1] - L.seg[la], Ta);
        }
        const uint64_t m = __ballot(work);
        if (!m) continue;
        const uint32_t mi = wave_incl_sum(nd), mtot = (uint32_t)__builtin_amdgcn_readlane((int)mi, kWave - 1);
        uint32_t ib = 0, mb = 0;
        if (lane == 0) {
          ib = atomicAdd(&a.orw_n[0], (uint32_t)__popcll(m));
          mb = atomicAdd(&a.orw_n[1], mtot);
        }
        ib = (uint32_t)__builtin_amdgcn_readlane((int)ib, 0) + (uint32_t)__popcll(m & lanemask_lt());
        mb = (uint32_t)__builtin_amdgcn_readlane((int)mb, 0) + mi - nd;
        if (work) {
          const uint32_t l = a0 + la, self = P.R > 1 ? P.gid[l] : l, s0 = L.seg[la];
          a.orw[ib] = make_uint4(l, (self % AGX_CRDT_NODES) | (nd << 8), mb, rc0);
          for (uint32_t q = 0; q < nd; ++q) a.orm[mb + q] = make_uint2(isrc(s0 + q), ipay(s0 + q));
        }
      }
    }
    if constexpr ((KM & kDeltaKM) != 0) {  // NoDeltaPlaceholder groups are not told: drop their void slots
      uint32_t tv;
      block_excl_sum<kBThreads>(nvoid, L.scratch, &tv);
      if (tv) emtot = compact_void(a.em, embase, emtot, L.scratch);
    }
    if constexpr (kGather || kOwner) {
      __syncthreads();  // phase B's tells are in the em scratch arena (sender order)
      group_tells<false>(a, L, b, w, embase, emtot, a.em);
    }
  }
  if (!kGather && tid == 0) {
    a.chunk_off[a.nb + b] = (uint32_t)embase;
    a.chunk_cnt[a.nb + b] = emtot;
    if (!kOwner && !(!kWide && a.kmax == 1) && a.emmeta) a.emmeta[b] = make_uint4(0u, 0u, 2u, 0u);  // (phase A/B path)
  }
  __syncthreads();
  AGX_STAMP(a, 7);
  // next first-pass histogram column of this bucket's tell chunk (zeroed by the chunk downsweep)
  if (!kGather && !kOwner)
    for (uint32_t d = tid; d < (1u << a.nx_bits); d += kBThreads)
      if (L.nh[d]) atomicAdd(&a.nhist[(size_t)d * a.nhist_stride + a.ng + b / a.G], L.nh[d]);
  // block stats: per-thread sums over the block's buckets, flushed once at the end of the kernel
  // (flush_stats): no reduction, LDS atomics or barrier per bucket
  if constexpr (kOwner || (kGather && !kLds)) {
    // multi-rank and fused skew variants: per bucket through LDS (a flush at the end of the kernel
    // made these variants spill: 3 -> 14 VGPRs for the multi-rank RING apply)
    const uint32_t lane = lane_id();
    const uint32_t v0 = wave_incl_sum(ndel), v1 = wave_incl_sum(ndead), v2 = wave_incl_sum(nunh),
                   v3 = wave_incl_sum(nall), v4 = wave_incl_sum(nact);
    if (lane == kWave - 1) {
      atomicAdd(&L.stat[0], (unsigned long long)v0);
      atomicAdd(&L.stat[1], (unsigned long long)v1);
      atomicAdd(&L.stat[2], (unsigned long long)v2);
      atomicAdd(&L.stat[3], (unsigned long long)v3);
      atomicAdd(&L.stat[4], (unsigned long long)v4);
    }
    __syncthreads();
    if (tid < kBStats && L.stat[tid])  // this block's own slot (no contention; no load round trip)
      atomicAdd(&a.bstats[(size_t)blockIdx.x * kBStats + tid], L.stat[tid]);
  } else {
    acc[0] += ndel;
    acc[1] += ndead;
    acc[2] += nunh;
    acc[3] += nall;
    acc[4] += nact;
    AGX_SHADOW_ADD(nall);
  }
  __syncthreads();  // (L.nh and the other per-bucket LDS arrays are reset by the next bucket)
  AGX_STAMP(a, 8);
  if (a.dbg && tid == 0) {  // diagnostic: slowest bucket of this block (cycles, bucket, inbox size)
    const unsigned long long dur = a.dbg[blockIdx.x * 16 + 8] - a.dbg[blockIdx.x * 16 + 0];
    if (dur > a.dbg[blockIdx.x * 16 + 10]) {
      a.dbg[blockIdx.x * 16 + 10] = dur;
      a.dbg[blockIdx.x * 16 + 11] = b;
      a.dbg[blockIdx.x * 16 + 12] = cnt;
    }
  }
}

// ---- Dense buckets: at most one message per actor.
// When a bucket's inbox keys are strictly increasing in inbox order (a token ring, a stencil, any
// one-to-one topology), every actor holds at most one message, and bucket_finish's rule for len = 1
// is: admitted (C = 0 or C >= 1), drained (T >= 1), nothing queued (AD/Mailbox.scala:261,551-565).
// Each message is then applied by the thread that holds it, straight from registers, and its tell
// (max_emit 1) goes to its rank among the bucket's tells -- sender order = inbox order = actor
// order, exactly where bucket_finish's per-actor scan would put it.  What this skips: the in-bucket
// counting sort (segment counts and scan), the classification and backlog scans, the LDS round of
// the state words and the per-actor drain loop -- about half of the barriers of a bucket.
struct RegEmitter {  // at most one tell per message (max_emit 1), kept in registers
  const DevParams* P;
  uint32_t self, key, pay, n_valid, n_all;
  __device__ __forceinline__ void operator()(uint32_t dst, uint32_t p) {
    if (dst >= P->n_global) {  // a host-side actor (the reply path: outbox) or an unknown ref -> deadLetters
      if (!outbound_tell(*P, dst, self, p, true)) ++n_all;
      return;
    }
    ++n_all;
    ++n_valid;
    key = (P->R > 1) ? P->route[dst] : dst;
    pay = p;
  }
  __device__ __forceinline__ void wide(uint32_t, uint32_t) {}
};

// Items: the bucket's inbox in LDS (L.key / L.src / L.pay, inbox order); item q is handled by thread
// q % kBThreads as its r = q / kBThreads -- the actor mapping of the fused early state loads
// (pre0 / pre1: actor r * kBThreads + tid), so a full bucket (item q = actor q) uses them directly.
template <uint32_t KM, bool kGather, bool kOwner>
__device__ __forceinline__ void dense_finish(const BucketArgs& a, const BucketLds& L, uint32_t b, uint32_t lo,
                                             uint32_t cnt, uint32_t a0, uint32_t w, uint32_t (&acc)[kBStats],
                                             const uint64_t* pre0, const uint64_t* pre1) {
  const DevParams& P = a.P;
  const int tid = threadIdx.x;
  const uint32_t lane = lane_id(), wv = (uint32_t)tid / kWave;
  const uint64_t ltm = lanemask_lt();
  const uint32_t amask = (1u << a.bb) - 1u, nhmask = (1u << a.nx_bits) - 1u;
  constexpr bool kKindNeeded = (KM & (KM - 1)) != 0 || (KM & kb(AGX_KIND_COMPILED)) != 0;
  constexpr bool kBypass = !kGather && !kOwner;
  AGX_STAMP(a, 3);
  // ---- items, their actors' flags and state words (all loads issued together)
  uint32_t sv[kBIpt], pv[kBIpt], l[kBIpt], ab[kBIpt], kd[kBIpt];
  uint64_t x0[kBIpt], x1[kBIpt];
  bool on[kBIpt];
#pragma unroll
  for (int r = 0; r < kBIpt; ++r) {
    const uint32_t q = r * kBThreads + tid;
    on[r] = q < cnt;
    const uint32_t la = on[r] ? L.key[q] & amask : 0u;
    sv[r] = on[r] ? L.src[q] : 0u;
    pv[r] = on[r] ? L.pay[q] : 0u;
    ab[r] = on[r] ? L.alive[la] : 0u;
    l[r] = a0 + la;
  }
  const uint32_t w1off = P.W > 1 ? P.sw : 0u;
#pragma unroll
  for (int r = 0; r < kBIpt; ++r) {
    kd[r] = kKindNeeded ? P.kind[l[r]] : 0u;
    const bool early = pre0 && l[r] == a0 + r * kBThreads + tid;  // (fused: loaded at the bucket's start)
    x0[r] = early ? pre0[r] : ldg64(P.state, l[r] * P.sa);
    x1[r] = early ? pre1[r] : ldg64(P.state, l[r] * P.sa + w1off);
  }
  // ---- apply (one message per actor: admitted and drained, bucket_finish with len = 1)
  uint32_t ndel = 0, ndead = 0, nunh = 0, nall = 0, nact = 0;
  uint32_t tk[kBIpt], ts[kBIpt], tp[kBIpt];
  bool tv[kBIpt];
#pragma unroll
  for (int r = 0; r < kBIpt; ++r) {
    tv[r] = false;
    tk[r] = ts[r] = tp[r] = 0u;
    if (!on[r]) continue;
    if (!(ab[r] & 1u)) {  // to a stopped actor: a dead letter
      ++ndead;
      continue;
    }
    const uint32_t self = P.R > 1 ? P.gid[l[r]] : l[r];
    RegEmitter em{&P, self, 0u, 0u, 0u, 0u};
    uint64_t wv2[2] = {x0[r], x1[r]};
    uint32_t kc = kd[r];
    ++nact;
    ++ndel;
    const uint32_t res = apply_msg<KM>(P, kc, self, l[r], wv2, sv[r], pv[r], em);
    if (res == AGX_RES_UNHANDLED) ++nunh;
    if (res == AGX_RES_STOPPED) {
      if constexpr (kGather) P.alive[l[r]] = (uint8_t)(ab[r] & 0xFEu);  // fused: only this block reads the bucket's flags
      else P.stopq[atomicAdd(P.nstop, 1u)] = l[r];
    }
    stg64(P.state, l[r] * P.sa, wv2[0]);
    if (P.W > 1) stg64(P.state, l[r] * P.sa + w1off, wv2[1]);
    if constexpr ((KM & kb(AGX_KIND_COMPILED)) != 0)
      if (kc != kd[r]) P.kind[l[r]] = (uint8_t)kc;
    nall += em.n_all;
    ndead += em.n_all - em.n_valid;
    tv[r] = em.n_valid != 0u;
    tk[r] = em.key;
    ts[r] = self;
    tp[r] = em.pay;
  }
#pragma unroll
  for (int r = 0; r < kBIpt; ++r)
    if (tv[r]) lds_hist_inc(L.nh, (tk[r] >> a.nx_shift) & nhmask);
  AGX_STAMP(a, 5);
  // ---- each tell's rank in item order: per (row r, wave) counts, one block-wide exclusive scan
  uint32_t rk[kBIpt];
#pragma unroll
  for (int r = 0; r < kBIpt; ++r) {
    const uint64_t m = __ballot(tv[r]);
    rk[r] = (uint32_t)__popcll(m & ltm);
    if (lane == 0) L.seg[r * kBWaves + wv] = (uint32_t)__popcll(m);  // (L.seg: no segments on this path)
  }
  __syncthreads();
  uint32_t emtot = 0;
  {
    uint32_t run = 0;
#pragma unroll
    for (int r = 0; r < kBIpt; ++r)
#pragma unroll
      for (int x = 0; x < kBWaves; ++x) {
        const uint32_t c = L.seg[r * kBWaves + x];
        if (x == (int)wv) rk[r] += run;
        run += c;
      }
    emtot = run;
  }
  const uint64_t embase = (uint64_t)lo * a.kmax;  // this bucket's slice of the tell arena
  if (tid == 0) {  // nothing queued: the bucket's backlog is empty
    if constexpr (kGather) {
      a.g.blo[w][b] = lo;
      a.g.blc[w][b] = 0u;
    } else {
      a.chunk_off[b] = lo;
      a.chunk_cnt[b] = 0u;
    }
  }
  if constexpr (kGather || kOwner) {
    // compacted in sender order into U, then grouped by destination (bucket / owner rank)
    uint32_t* ukey = reinterpret_cast<uint32_t*>(L.U);
#pragma unroll
    for (int r = 0; r < kBIpt; ++r)
      if (tv[r]) {
        ukey[rk[r]] = tk[r];
        ukey[kBucket + rk[r]] = ts[r];
        ukey[2 * kBucket + rk[r]] = tp[r];
      }
    __syncthreads();
    group_tells<true>(a, L, b, w, embase, emtot, a.em);
  } else {
    uint32_t* const ck = reinterpret_cast<uint32_t*>(L.U);
#pragma unroll
    for (int r = 0; r < kBIpt; ++r)
      if (tv[r]) {
        a.em.key[embase + rk[r]] = tk[r];
        a.em.src[embase + rk[r]] = ts[r];
        a.em.pay[embase + rk[r]] = tp[r];
        ck[rk[r]] = tk[r];
      }
    if (a.emmeta) {  // identity grouping (k_ident_combine): first / last key and descents, sender order
      __syncthreads();
      uint32_t nd = 0, dp = 0;
#pragma unroll
      for (uint32_t i = 4 * tid; i < 4 * tid + 4; ++i)
        if (i > 0 && i < emtot && ck[i] < ck[i - 1]) {
          ++nd;
          dp = i;
        }
      uint32_t tnd, tdp;
      block_excl_sum2<kBThreads>(nd, nd ? dp : 0u, L.scratch, &tnd, &tdp);
      if (tid == 0) a.emmeta[b] = make_uint4(emtot ? ck[0] : 0u, emtot ? ck[emtot - 1] : 0u, tnd, tdp);
    }
  }
  if (!kGather && tid == 0) {  // the bucket's tell chunk (multi-pass and multi-rank: in-flight accounting)
    a.chunk_off[a.nb + b] = (uint32_t)embase;
    a.chunk_cnt[a.nb + b] = emtot;
  }
  __syncthreads();
  AGX_STAMP(a, 7);
  if constexpr (kBypass)  // next first-pass histogram column of this bucket's tell chunk
    for (uint32_t d = tid; d < (1u << a.nx_bits); d += kBThreads)
      if (L.nh[d]) atomicAdd(&a.nhist[(size_t)d * a.nhist_stride + a.ng + b / a.G], L.nh[d]);
  if constexpr (kOwner) {  // multi-rank: per bucket through LDS (as bucket_finish)
    const uint32_t v0 = wave_incl_sum(ndel), v1 = wave_incl_sum(ndead), v2 = wave_incl_sum(nunh),
                   v3 = wave_incl_sum(nall), v4 = wave_incl_sum(nact);
    if (lane == kWave - 1) {
      atomicAdd(&L.stat[0], (unsigned long long)v0);
      atomicAdd(&L.stat[1], (unsigned long long)v1);
      atomicAdd(&L.stat[2], (unsigned long long)v2);
      atomicAdd(&L.stat[3], (unsigned long long)v3);
      atomicAdd(&L.stat[4], (unsigned long long)v4);
    }
    __syncthreads();
    if (tid < kBStats && L.stat[tid]) atomicAdd(&a.bstats[(size_t)blockIdx.x * kBStats + tid], L.stat[tid]);
  } else {
    acc[0] += ndel;
    acc[1] += ndead;
    acc[2] += nunh;
    acc[3] += nall;
    acc[4] += nact;
    AGX_SHADOW_ADD(nall);
  }
  __syncthreads();  // (the per-bucket LDS arrays are reset by the next bucket)
  AGX_STAMP(a, 8);
  if (a.dbg && tid == 0) {  // diagnostic: slowest bucket of this block (cycles, bucket, inbox size)
    const unsigned long long dur = a.dbg[blockIdx.x * 16 + 8] - a.dbg[blockIdx.x * 16 + 0];
    if (dur > a.dbg[blockIdx.x * 16 + 10]) {
      a.dbg[blockIdx.x * 16 + 10] = dur;
      a.dbg[blockIdx.x * 16 + 11] = b;
      a.dbg[blockIdx.x * 16 + 12] = cnt;
    }
  }
}

// Inbox of one bucket in fused mode: [backlog][tell segments, sender-bucket order][staged].
struct GatherView {
  const uint32_t* segp;  // [nseg + 1] inbox position of each non-empty tell segment; [nseg] = staged start
  const uint32_t* sego;  // [nseg] its offset in eg[r]
  uint32_t nseg, blc, blo, sto;
  // arena pointers are re-read from the kernel arguments at each use (scalar loads): holding
  // them here would pin 18 VGPRs across the whole bucket
  __device__ __forceinline__ uint32_t key(const GatherArgs& g, uint32_t r, uint32_t q) const {
    if (q < blc) return g.bl[r].key[blo + q];
    uint32_t lo = 0, hi = nseg;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (segp[mid] <= q) lo = mid; else hi = mid - 1;
    }
    return lo < nseg ? g.eg[r].key[sego[lo] + (q - segp[lo])] : g.stg.key[sto + (q - segp[nseg])];
  }
  // where inbox item q lives: sel 0 = backlog (bl[r]), 1 = a tell segment (eg[r]), 2 = staged (stg);
  // LDS reads only, so a caller can issue every item's global loads back to back
  __device__ __forceinline__ uint32_t locate(uint32_t q, uint32_t& sel) const {
    if (q < blc) {
      sel = 0;
      return blo + q;
    }
    uint32_t lo = 0, hi = nseg;  // last segment start <= q
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (segp[mid] <= q) lo = mid; else hi = mid - 1;
    }
    sel = lo < nseg ? 1u : 2u;
    return lo < nseg ? sego[lo] + (q - segp[lo]) : sto + (q - segp[nseg]);
  }
  __device__ __forceinline__ void load(const GatherArgs& g, uint32_t r, uint32_t q, uint32_t& k, uint32_t& sv,
                                       uint32_t& pv) const {
    if (q < blc) {
      const uint32_t i = blo + q;
      k = g.bl[r].key[i];
      sv = g.bl[r].src[i];
      pv = g.bl[r].pay[i];
      return;
    }
    uint32_t lo = 0, hi = nseg;  // last segment start <= q
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (segp[mid] <= q) lo = mid; else hi = mid - 1;
    }
    if (lo < nseg) {
      const uint32_t i = sego[lo] + (q - segp[lo]);
      k = g.eg[r].key[i];
      sv = g.eg[r].src[i];
      pv = g.eg[r].pay[i];
    } else {
      const uint32_t i = sto + (q - segp[nseg]);
      k = g.stg.key[i];
      sv = g.stg.src[i];
      pv = g.stg.pay[i];
    }
  }
};

// =========================================================================
// Wave-per-bucket path (single-rank multi-pass, plain and compiled behaviours): a bucket whose
// inbox holds at most kTinyMax messages -- most buckets of a sparse superstep at 10^7+ actors
// (C3, C5) -- is drained by one wave with no workgroup barrier, so the 8 waves of a block
// finish 8 such buckets in the time the block path spends on one (its ~30 barriers and 4-6
// dependent round trips are per bucket, not per message).  Same semantics as the block path:
// stable order by actor (inbox order within an actor), tail-drop at C, drain min(len, T), the
// rest queued in order, Behaviors.stopped / unhandled, tells in sender (= actor) order.
#ifndef AGX_TINY_IPL
#define AGX_TINY_IPL 2  // (4 = 256-message wave path: measured slower, C3 -18 %, C5 -4 %: the rank loop is
#endif                  // quadratic in the inbox and the bypass apply spills 44 -> 84 B/lane)
constexpr uint32_t kTinyIpl = AGX_TINY_IPL;      // inbox items per lane
constexpr uint32_t kTinyMax = kTinyIpl * kWave;  // 128
struct TinyLds {                                 // one per wave (2.5 KB)
  uint32_t key[kTinyMax], src[kTinyMax], pay[kTinyMax];
  uint16_t st[kTinyMax], len[kTinyMax];
};
static_assert(kBWaves * sizeof(TinyLds) <= 2 * kBucket * sizeof(uint64_t), "the waves' TinyLds live in the apply's U");

// Tells of the wave path: into the bucket's tell chunk, next-pass histogram column updated
// directly (the block path stages it in LDS).
struct TinyEmitter {
  const DevParams* P;
  const BucketArgs* a;
  uint64_t pos;
  uint32_t self, col, nhmask;
  uint32_t n_valid, n_all;
  __device__ __forceinline__ void operator()(uint32_t dst, uint32_t pay) {
    if (dst >= P->n_global) {  // the reply path (outbox) or an unknown ref -> deadLetters
      if (!outbound_tell(*P, dst, self, pay, true)) ++n_all;
      return;
    }
    ++n_all;
    ++n_valid;
    a->em.key[pos] = dst;  // (single rank: key = local id = global id)
    a->em.src[pos] = self;
    a->em.pay[pos] = pay;
    ++pos;
    atomicAdd(&a->nhist[(size_t)((dst >> a->nx_shift) & nhmask) * a->nhist_stride + col], 1u);
  }
  __device__ __forceinline__ void wide(uint32_t, uint32_t) {}
};

// max_emit 1: a message's tell is staged in LDS over the actor's already consumed inbox slots
struct TinyStageEmitter {
  const DevParams* P;
  TinyLds* T;
  uint32_t slot, self;
  uint32_t n_valid, n_all;
  __device__ __forceinline__ void operator()(uint32_t dst, uint32_t pay) {
    if (dst >= P->n_global) {  // the reply path (outbox) or an unknown ref -> deadLetters
      if (!outbound_tell(*P, dst, self, pay, true)) ++n_all;
      return;
    }
    ++n_all;
    ++n_valid;
    T->key[slot] = dst;
    T->src[slot] = self;
    T->pay[slot] = pay;
    ++slot;
  }
  __device__ __forceinline__ void wide(uint32_t, uint32_t) {}
};

template <uint32_t KM>
__device__ __forceinline__ void tiny_bucket(const BucketArgs& a, const InView& iv, TinyLds& T, uint32_t b, uint32_t lo,
                                            uint32_t cnt, uint32_t xblc, uint32_t xblo, uint32_t xbst, uint32_t rpar,
                                            uint32_t wpar) {
  const DevParams& P = a.P;
  const uint32_t lane = lane_id();
  const uint32_t amask = (1u << a.bb) - 1u, a0 = b << a.bb;
  // ---- items, and their stable rank by (actor, inbox position) over the whole inbox
  uint32_t k[kTinyIpl], sv[kTinyIpl], pv[kTinyIpl], la[kTinyIpl];
  {  // all loads back to back (selected SGPR bases, no branch around the loads)
    const uint32_t *Bk = sgpr_ptr(a.g.bl[rpar].key), *Bs = sgpr_ptr(a.g.bl[rpar].src), *Bp = sgpr_ptr(a.g.bl[rpar].pay);
#pragma unroll
    for (uint32_t r = 0; r < kTinyIpl; ++r) {
      const uint32_t q = r * kWave + lane;
      const bool bl = q < xblc, ok = q < cnt;
      const uint32_t i = !ok ? 0u : bl ? xblo + q : iv.at(xbst + q - xblc);
      k[r] = ldg(bl || !ok ? Bk : iv.m.key, i);
      sv[r] = ldg(bl || !ok ? Bs : iv.m.src, i);
      pv[r] = ldg(bl || !ok ? Bp : iv.m.pay, i);
    }
#pragma unroll
    for (uint32_t r = 0; r < kTinyIpl; ++r) la[r] = r * kWave + lane < cnt ? k[r] & amask : 0xFFFFFFFFu;
  }
  uint32_t rank[kTinyIpl] = {}, st[kTinyIpl] = {}, len[kTinyIpl] = {};
#pragma unroll
  for (uint32_t r2 = 0; r2 < kTinyIpl; ++r2) {  // item j = r2 * 64 + jj, held by lane jj in la[r2]
    const uint32_t jn = cnt > r2 * kWave ? min(cnt - r2 * kWave, (uint32_t)kWave) : 0u;
    for (uint32_t jj = 0; jj < jn; ++jj) {  // (uniform loop; v_readlane with a scalar lane, no LDS crossbar)
      const uint32_t lj = (uint32_t)__builtin_amdgcn_readlane((int)la[r2], (int)jj), j = r2 * kWave + jj;
#pragma unroll
      for (uint32_t r = 0; r < kTinyIpl; ++r) {
        const bool lt = lj < la[r], eq = lj == la[r];
        st[r] += lt;
        len[r] += eq;
        rank[r] += lt || (eq && j < r * kWave + lane);
      }
    }
  }
#pragma unroll
  for (uint32_t r = 0; r < kTinyIpl; ++r)
    if (r * kWave + lane < cnt) {
      T.key[rank[r]] = k[r];
      T.src[rank[r]] = sv[r];
      T.pay[rank[r]] = pv[r];
      T.st[rank[r]] = (uint16_t)st[r];
      T.len[rank[r]] = (uint16_t)len[r];
    }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // ---- per actor (the head of its run of sorted positions; lane l owns positions 2l, 2l + 1,
  // so lane order is actor order)
  uint32_t hl[kTinyIpl], hlen[kTinyIpl], hkeep[kTinyIpl], hkind[kTinyIpl], nd[kTinyIpl], hab[kTinyIpl],
      hT[kTinyIpl];
  uint64_t hw0[kTinyIpl], hw1[kTinyIpl];
  bool head[kTinyIpl], hal[kTinyIpl];
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i) {
    const uint32_t p = lane * kTinyIpl + i;
    head[i] = p < cnt && T.st[p] == p;
    hl[i] = head[i] ? a0 + (T.key[p] & amask) : 0u;
    hlen[i] = head[i] ? T.len[p] : 0u;
  }
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i) {  // (all loads in flight together)
    hab[i] = head[i] ? P.alive[hl[i]] : 0u;
    hkind[i] = head[i] ? P.kind[hl[i]] : 0u;
    hw0[i] = head[i] ? ldg64(P.state, sidx(P, hl[i], 0)) : 0ull;
    hw1[i] = head[i] && P.W > 1 ? ldg64(P.state, sidx(P, hl[i], 1)) : 0ull;
  }
  uint32_t ndead = 0, nq = 0;
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i) {
    uint32_t C, Tt;
    mbox_limits(P, hab[i], C, Tt);
    hal[i] = (hab[i] & 1u) != 0;
    const uint32_t keep = !hal[i] ? 0u : (C == 0 || hlen[i] < C) ? hlen[i] : C;  // tail-drop beyond C
    hkeep[i] = keep;
    hT[i] = Tt;
    ndead += hlen[i] - keep;
    nd[i] = hal[i] ? min(hlen[i], Tt) : 0u;
    nq += keep > Tt ? keep - Tt : 0u;
  }
  const uint64_t embase = (uint64_t)lo * a.kmax;
  const Msgs blw = a.g.bl[wpar];
  const uint32_t qinc = wave_incl_sum(nq), bltot = (uint32_t)__builtin_amdgcn_readlane((int)qinc, kWave - 1);
  uint32_t qoff = qinc - nq;
  uint32_t ndel = 0, nunh = 0, nall = 0, nact = 0, emtot = 0;
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i) {  // queued beyond the throughput cap, in order
    const uint32_t p0 = lane * kTinyIpl + i;
    for (uint32_t q = hT[i]; q < hkeep[i]; ++q, ++qoff) {
      blw.key[lo + qoff] = T.key[p0 + q];
      blw.src[lo + qoff] = T.src[p0 + q];
      blw.pay[lo + qoff] = T.pay[p0 + q];
    }
  }
  // FANOUT with one tell per message: every drained position's Zipf destination first, the lane's
  // positions in lockstep, into the position's sender slot (as the block path does)
  constexpr bool kFanPre = KM == kb(AGX_KIND_FANOUT);
  const bool fan_pre = kFanPre && P.fan_k == 1 && a.kmax == 1;
  if (kFanPre && fan_pre) {
    uint32_t uu[kTinyIpl], lo2[kTinyIpl], hi2[kTinyIpl];
    bool need[kTinyIpl];
    bool dir[kTinyIpl];
#pragma unroll
    for (uint32_t i = 0; i < kTinyIpl; ++i) {
      const uint32_t p = lane * kTinyIpl + i;
      need[i] = false;
      uu[i] = 0;
      if (p < cnt) {
        const uint32_t lp = a0 + (T.key[p] & amask), pv = T.pay[p], ab = P.alive[lp];
        uint32_t C, Tt;
        mbox_limits(P, ab, C, Tt);
        if ((ab & 1u) && p - T.st[p] < min((uint32_t)T.len[p], Tt) && (pv >> 24) > 0) {
          need[i] = true;
          uu[i] = (uint32_t)(fanout_rand(P.fan_seed, lp, pv & 0x00FFFFFFu, 0) >> 32);
        }
      }
    }
#pragma unroll
    for (uint32_t i = 0; i < kTinyIpl; ++i) {
      const uint32_t t = uu[i] >> (32 - kZipfBits);
      const uint2 z = need[i] ? P.zipf_ent[t] : make_uint2(0u, 0u);
      dir[i] = z.y == kZipfDirect;  // (the Zipf head: the destination itself, no search)
      lo2[i] = z.x;
      hi2[i] = dir[i] ? z.x : z.y;
    }
    for (;;) {
      bool more = false;
      uint32_t c[kTinyIpl];
#pragma unroll
      for (uint32_t i = 0; i < kTinyIpl; ++i) c[i] = lo2[i] < hi2[i] ? P.zipf_cdf[(lo2[i] + hi2[i]) >> 1] : 0u;
#pragma unroll
      for (uint32_t i = 0; i < kTinyIpl; ++i)
        if (lo2[i] < hi2[i]) {
          const uint32_t mid = (lo2[i] + hi2[i]) >> 1;
          if (c[i] >= uu[i]) hi2[i] = mid; else lo2[i] = mid + 1;
          more |= lo2[i] < hi2[i];
        }
      if (!more) break;
    }
    uint32_t dd[kTinyIpl];
#pragma unroll
    for (uint32_t i = 0; i < kTinyIpl; ++i) dd[i] = need[i] ? (dir[i] ? lo2[i] : P.zipf_perm[lo2[i]]) : 0u;
#pragma unroll
    for (uint32_t i = 0; i < kTinyIpl; ++i)
      if (need[i]) T.src[lane * kTinyIpl + i] = dd[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // drain + apply.  Every message emits <= 1 tell (max_emit 1): one pass, tells staged over the
  // actor's consumed inbox slots, then compacted in actor order.  Otherwise: count the tells on
  // copies of the state first (phase A), then apply for real.
  auto drain = [&](uint32_t i, auto& em) {
    const uint32_t p0 = lane * kTinyIpl + i, l = hl[i];
    ++nact;
    uint64_t wv[2] = {hw0[i], hw1[i]};
    uint32_t kd = hkind[i];
    for (uint32_t q = 0; q < nd[i]; ++q) {
      ++ndel;
      uint32_t r;
      if (kFanPre && fan_pre) {  // apply_msg's FANOUT with the destination looked up above
        const uint32_t pv = T.pay[p0 + q], ttl = pv >> 24;
        wv[0] += 1;
        wv[1] += pv;
        if (ttl > 0) em(T.src[p0 + q], ((ttl - 1) << 24) | ((uint32_t)fanout_rand(P.fan_seed, l, pv & 0x00FFFFFFu, 0) & 0x00FFFFFFu));
        r = AGX_RES_SAME;
      } else {
        r = apply_msg<KM>(P, kd, l, l, wv, T.src[p0 + q], T.pay[p0 + q], em);
      }
      if (r == AGX_RES_UNHANDLED) ++nunh;
      if (r == AGX_RES_STOPPED) {
        P.stopq[atomicAdd(P.nstop, 1u)] = l;
        ndead += nd[i] - q - 1;  // drained-but-unprocessed after the stop
        break;
      }
    }
    P.state[sidx(P, l, 0)] = wv[0];
    if (P.W > 1) P.state[sidx(P, l, 1)] = wv[1];
    if constexpr ((KM & kb(AGX_KIND_COMPILED)) != 0)
      if (kd != hkind[i]) P.kind[l] = (uint8_t)kd;
    nall += em.n_all;
    ndead += em.n_all - em.n_valid;
  };
  const uint32_t col = a.ng + b / a.G, nhmask = (1u << a.nx_bits) - 1u;
  if (a.kmax == 1) {
    uint32_t ecl[kTinyIpl], ncount = 0;
#pragma unroll
    for (uint32_t i = 0; i < kTinyIpl; ++i) {
      ecl[i] = 0;
      if (!nd[i]) continue;
      TinyStageEmitter em{&P, &T, lane * kTinyIpl + i, hl[i], 0, 0};
      drain(i, em);
      ecl[i] = em.n_valid;
      ncount += em.n_valid;
    }
    const uint32_t tinc = wave_incl_sum(ncount);
    emtot = (uint32_t)__builtin_amdgcn_readlane((int)tinc, kWave - 1);
    uint32_t toff = tinc - ncount;
#pragma unroll
    for (uint32_t i = 0; i < kTinyIpl; ++i)
      for (uint32_t e = 0; e < ecl[i]; ++e, ++toff) {
        const uint32_t p = lane * kTinyIpl + i + e, d = T.key[p];
        a.em.key[embase + toff] = d;
        a.em.src[embase + toff] = T.src[p];
        a.em.pay[embase + toff] = T.pay[p];
        atomicAdd(&a.nhist[(size_t)((d >> a.nx_shift) & nhmask) * a.nhist_stride + col], 1u);
      }
  } else {
    uint32_t ncount = 0;
#pragma unroll
    for (uint32_t i = 0; i < kTinyIpl; ++i) {
      if (!nd[i]) continue;
      const uint32_t p0 = lane * kTinyIpl + i;
      Emitter<false> em{&P, {}, 0, hl[i], 0, 0, nullptr, 0, 0};
      uint64_t wv[2] = {hw0[i], hw1[i]};
      uint32_t kd = hkind[i];
      for (uint32_t q = 0; q < nd[i]; ++q)
        if (apply_msg<KM>(P, kd, hl[i], hl[i], wv, T.src[p0 + q], T.pay[p0 + q], em) == AGX_RES_STOPPED) break;
      ncount += em.n_valid;
    }
    const uint32_t tinc = wave_incl_sum(ncount);
    emtot = (uint32_t)__builtin_amdgcn_readlane((int)tinc, kWave - 1);
    uint32_t toff = tinc - ncount;
#pragma unroll
    for (uint32_t i = 0; i < kTinyIpl; ++i) {
      if (!nd[i]) continue;
      TinyEmitter em{&P, &a, embase + toff, hl[i], col, nhmask, 0, 0};
      drain(i, em);
      toff += em.n_valid;
    }
  }
  if (lane == 0) {
    a.chunk_off[b] = lo;
    a.chunk_cnt[b] = bltot;
    a.chunk_off[a.nb + b] = (uint32_t)embase;
    a.chunk_cnt[a.nb + b] = emtot;
    if (a.emmeta) a.emmeta[b] = make_uint4(0u, 0u, 2u, 0u);  // (wave path: not summarised, forces a sort)
  }
  const uint32_t v0 = wave_incl_sum(ndel), v1 = wave_incl_sum(ndead), v2 = wave_incl_sum(nunh),
                 v3 = wave_incl_sum(nall), v4 = wave_incl_sum(nact);
  if (lane == kWave - 1) {
    unsigned long long* bs = a.bstats + (size_t)blockIdx.x * kBStats;
    if (v0) atomicAdd(&bs[0], (unsigned long long)v0);
    if (v1) atomicAdd(&bs[1], (unsigned long long)v1);
    if (v2) atomicAdd(&bs[2], (unsigned long long)v2);
    if (v3) atomicAdd(&bs[3], (unsigned long long)v3);
    if (v4) atomicAdd(&bs[4], (unsigned long long)v4);
  }
}

// Wave-per-bucket launch (single-rank multi-pass, plain and compiled behaviours): every bucket whose
// inbox -- backlog in place plus sorted new mail -- holds at most tiny_max messages is drained by one
// wave (tiny_bucket); the others are marked for the block launch that follows (k_bucket_apply over
// the a.blist marks).  A separate kernel so that its residency is set by the wave path's own registers and
// 10 KB of LDS, not by the block path's 80 KB: all of a sparse superstep's buckets (C3: 4883, most
// with a few dozen messages) are in flight at once instead of one or two waves of each of 512
// resident 8-wave blocks (the rest of such a block idled while its wave drained).
constexpr int kTinyThreads = 256;
constexpr int kTinyWaves = kTinyThreads / kWave;
template <uint32_t KM>
static __global__ void __launch_bounds__(kTinyThreads) k_tiny_apply(BucketArgs a) {
  __shared__ TinyLds T[kTinyWaves];
  const uint32_t w = threadIdx.x / kWave, lane = lane_id();
  const uint32_t wpar = *a.pstep & 1u, rpar = wpar ^ 1u;
  const InView iv = in_view(a);
  const uint32_t nw = gridDim.x * kTinyWaves;
  if (a.dense_first && a.dense_left && a.dense_left[wpar] == 0u) return;  // (the dense launch took every bucket)
  for (uint32_t bw = blockIdx.x * kTinyWaves + w; bw < a.nb; bw += nw) {
    if (a.dense_first && __builtin_amdgcn_readfirstlane(a.blist[bw]) == 0u) continue;  // (done by k_dense_apply)
    uint32_t bs = 0, lo_w = 0, hi_w = 0, blc = 0, blo = 0;
    if (lane == 0) {  // (k_bucket_apply's bypass bounds)
      bs = a.bstart[bw];
      const uint32_t be = a.bstart[bw + 1], bp = a.blpre[bw] + a.bl_sbase[bw / kBlSlice];
      blc = a.chunk_cnt[bw];
      blo = a.chunk_off[bw];
      lo_w = bs + bp;
      hi_w = lo_w + blc + (be - bs);
    }
    bs = (uint32_t)__builtin_amdgcn_readlane((int)bs, 0);
    lo_w = (uint32_t)__builtin_amdgcn_readlane((int)lo_w, 0);
    hi_w = (uint32_t)__builtin_amdgcn_readlane((int)hi_w, 0);
    blc = (uint32_t)__builtin_amdgcn_readlane((int)blc, 0);
    blo = (uint32_t)__builtin_amdgcn_readlane((int)blo, 0);
    const bool tiny = hi_w - lo_w <= a.tiny_max && (uint64_t)hi_w <= a.cap &&  // (over capacity: the block path reports it)
                      !(a.ring_of && a.ring_of[bw]);                         // (a ring bucket: skew path)
    if (tiny)
      tiny_bucket<KM>(a, iv, T[w], bw, lo_w, hi_w - lo_w, blc, blo, bs, rpar, wpar);
    if (lane == 0) a.blist[bw] = tiny ? 0u : 1u;  // (the block launch's work marks)
  }
}

// ---- Dense-bucket launch (single-rank multi-pass, plain and compiled behaviours, max_emit 1).
// A bucket whose inbox -- backlog in place, then the sorted new mail -- has strictly increasing keys
// holds at most one message per actor, so bucket_finish's rule reduces to: every message to a live
// actor is admitted and drained (len = 1: C = 0 or >= 1, T >= 1), nothing is queued, a message to a
// stopped actor is a dead letter (AD/Mailbox.scala:261,551-565).  This kernel applies such buckets
// straight from registers -- item q of the inbox by thread q % kDenseThreads, its tell written at its
// rank among the bucket's tells (sender order = inbox order = actor order) -- and marks every other
// bucket for the block launch (a.blist, as k_tiny_apply does).  It keeps no inbox tile in LDS (10 KB
// in all) and few registers, so several blocks share a CU and their buckets' memory round trips
// overlap, where the block kernel (80 KB of LDS) runs two.  The token ring -- every actor one token
// -- is all dense buckets.
constexpr int kDenseThreads = 512;
constexpr int kDenseWaves = kDenseThreads / kWave;
constexpr int kDenseIpt = kBucket / kDenseThreads;  // inbox items per thread (4)
#ifndef AGX_DENSE_WPE
#define AGX_DENSE_WPE 6  // minimum waves per SIMD (3 workgroups of 512 per CU; A/B build knob)
#endif
template <uint32_t KM>
static __global__ void __launch_bounds__(kDenseThreads, AGX_DENSE_WPE) k_dense_apply(BucketArgs a) {
  __shared__ uint32_t s_ck[kBucket];                   // tell keys in sender order (identity summary)
  __shared__ uint32_t s_nh[kRadix];                    // next first-pass digit histogram of the bucket's tells
  __shared__ uint32_t s_last[kDenseIpt * kDenseWaves];  // last key of each (row, wave): the strictness check
  __shared__ uint32_t s_cnt[kDenseIpt * kDenseWaves];   // tells of each (row, wave): their ranks
  __shared__ uint32_t scratch[2 * (kDenseWaves + 1)];
  __shared__ uint32_t s_bad;
  const DevParams& P = a.P;
  const uint32_t tid = threadIdx.x, w = tid / kWave, lane = lane_id();
  const uint64_t ltm = lanemask_lt();
  const uint32_t amask = (1u << a.bb) - 1u, nhmask = (1u << a.nx_bits) - 1u;
  const uint32_t wpar = *a.pstep & 1u, rpar = wpar ^ 1u;
  const InView iv = in_view(a);
  constexpr bool kKindNeeded = (KM & (KM - 1)) != 0 || (KM & kb(AGX_KIND_COMPILED)) != 0;
  const uint32_t w1off = P.W > 1 ? P.sw : 0u;
  uint32_t acc[kBStats] = {0u, 0u, 0u, 0u, 0u};
  if (a.dense_left && blockIdx.x == 0 && tid == 0) a.dense_left[rpar] = 0u;  // (the next superstep's flag)
  for (uint32_t d = tid; d < kRadix; d += kDenseThreads) s_nh[d] = 0;
  if (tid == 0) s_bad = 0;
  __syncthreads();
  for (uint32_t b = blockIdx.x; b < a.nb; b += gridDim.x) {
    // ---- bounds (k_bucket_apply's bypass bounds; uniform loads)
    const uint32_t bs = a.bstart[b], be = a.bstart[b + 1], bp = a.blpre[b] + a.bl_sbase[b / kBlSlice];
    const uint32_t blc = a.chunk_cnt[b], blo = a.chunk_off[b];
    const uint32_t lo = bs + bp, cnt = blc + (be - bs);
    if (cnt > (uint32_t)kBucket || (uint64_t)lo + cnt > a.cap) {  // (over capacity: the block path reports it)
      if (tid == 0) {
        a.blist[b] = 1u;
        if (a.dense_left) a.dense_left[wpar] = 1u;
      }
      continue;
    }
    const uint32_t a0 = b << a.bb;
    // ---- items: backlog (in place, g.bl[rpar]) then the sorted new mail; one round trip
    uint32_t k[kDenseIpt], sv[kDenseIpt], pv[kDenseIpt];
    {
      const uint32_t *Bk = sgpr_ptr(a.g.bl[rpar].key), *Bs = sgpr_ptr(a.g.bl[rpar].src), *Bp = sgpr_ptr(a.g.bl[rpar].pay);
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r) {
        const uint32_t q = r * kDenseThreads + tid;
        const bool bl = q < blc, ok = q < cnt;
        const uint32_t i = !ok ? 0u : bl ? blo + q : iv.at(bs + q - blc);
        k[r] = ldg(bl || !ok ? Bk : iv.m.key, i);
        sv[r] = ldg(bl || !ok ? Bs : iv.m.src, i);
        pv[r] = ldg(bl || !ok ? Bp : iv.m.pay, i);
      }
    }
    // ---- strictly increasing keys?  item q - 1 is lane - 1 of the same row and wave, or the last
    // item of the previous wave / row (through LDS)
    uint32_t bad = 0;
    {
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r)
        if (lane == kWave - 1) s_last[r * kDenseWaves + w] = k[r] & amask;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r) {
        const uint32_t q = r * kDenseThreads + tid, cur = k[r] & amask;
        uint32_t prev = (uint32_t)__shfl_up((int)cur, 1, kWave);
        if (lane == 0) {
          const int x = r * kDenseWaves + (int)w - 1;
          prev = x >= 0 ? s_last[x] : 0u;
        }
        if (q > 0 && q < cnt && prev >= cur) bad = 1;
      }
    }
    if (bad) atomicOr(&s_bad, 1u);
    __syncthreads();
    const bool dense = s_bad == 0;
    __syncthreads();  // (every thread read s_bad)
    if (!dense) {
      if (tid == 0) {
        a.blist[b] = 1u;
        if (a.dense_left) a.dense_left[wpar] = 1u;
        s_bad = 0;
      }
      continue;  // (uniform)
    }
    // ---- apply: one message per actor (admitted, drained; a stopped actor's message is a dead letter)
    uint32_t l[kDenseIpt], ab[kDenseIpt], kd[kDenseIpt];
    uint64_t x0[kDenseIpt], x1[kDenseIpt];
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r) {
      const uint32_t q = r * kDenseThreads + tid;
      l[r] = a0 + (q < cnt ? k[r] & amask : 0u);
    }
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r) {  // (all loads in flight together)
      ab[r] = P.alive[l[r]];
      kd[r] = kKindNeeded ? P.kind[l[r]] : 0u;
      x0[r] = ldg64(P.state, l[r] * P.sa);
      x1[r] = P.W > 1 ? ldg64(P.state, l[r] * P.sa + w1off) : 0ull;
    }
    uint32_t tk[kDenseIpt], tp[kDenseIpt];  // (a tell's sender is the item's actor, l[r])
    bool tv[kDenseIpt];
    if constexpr (KM == kb(AGX_KIND_RING)) {
      // RING-only populations: apply_msg<RING> through RegEmitter, branch-free (as in k_dense_fused)
      const uint32_t stride = P.ring_stride, ng = P.n_global;
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r) {
        const uint32_t q = r * kDenseThreads + tid;
        const bool has = q < cnt, live = (ab[r] & 1u) != 0u, on = has && live;
        const bool em = on && pv[r] > 0u;
        acc[0] += on ? 1u : 0u;
        acc[4] += on ? 1u : 0u;
        acc[1] += has && !live ? 1u : 0u;
        acc[3] += em ? 1u : 0u;
        uint32_t d = l[r] + stride;  // (single rank: local id = global id)
        d = d >= ng ? d - ng : d;
        tv[r] = em;
        tk[r] = em ? d : 0u;
        tp[r] = em ? pv[r] - 1u : 0u;
        if (on) st64x(P.state, l[r] * P.sa, x0[r] + 1ull);
      }
    } else {
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r) {
      const uint32_t q = r * kDenseThreads + tid;
      tv[r] = false;
      tk[r] = tp[r] = 0u;
      if (q >= cnt) continue;
      if (!(ab[r] & 1u)) {  // to a stopped actor: a dead letter
        ++acc[1];
        continue;
      }
      const uint32_t self = l[r];  // (single rank: local id = global id)
      RegEmitter em{&P, self, 0u, 0u, 0u, 0u};
      uint64_t wv2[2] = {x0[r], x1[r]};
      uint32_t kc = kd[r];
      ++acc[4];
      ++acc[0];
      const uint32_t res = apply_msg<KM>(P, kc, self, l[r], wv2, sv[r], pv[r], em);
      if (res == AGX_RES_UNHANDLED) ++acc[2];
      if (res == AGX_RES_STOPPED) P.stopq[atomicAdd(P.nstop, 1u)] = l[r];
      st64x(P.state, l[r] * P.sa, wv2[0]);
      if (P.W > 1) st64x(P.state, l[r] * P.sa + w1off, wv2[1]);
      if constexpr ((KM & kb(AGX_KIND_COMPILED)) != 0)
        if (kc != kd[r]) P.kind[l[r]] = (uint8_t)kc;
      acc[3] += em.n_all;
      acc[1] += em.n_all - em.n_valid;
      tv[r] = em.n_valid != 0u;
      tk[r] = em.key;
      tp[r] = em.pay;
    }
    }
    // ---- tells: rank in item order (per (row, wave) counts), chunk stores, next-pass histogram
    uint32_t rk[kDenseIpt];
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r) {
      const uint64_t m = __ballot(tv[r]);
      rk[r] = (uint32_t)__popcll(m & ltm);
      if (lane == 0) s_cnt[r * kDenseWaves + w] = (uint32_t)__popcll(m);
      if (tv[r]) lds_hist_inc(s_nh, (tk[r] >> a.nx_shift) & nhmask);
    }
    __syncthreads();
    uint32_t emtot = 0;
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r)
#pragma unroll
      for (int x = 0; x < kDenseWaves; ++x) {
        const uint32_t c = s_cnt[r * kDenseWaves + x];
        if (x == (int)w) rk[r] += emtot;
        emtot += c;
      }
    const uint64_t embase = (uint64_t)lo * a.kmax;
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r)
      if (tv[r]) {
        st32x(a.em.key, embase + rk[r], tk[r]);
        st32x(a.em.src, embase + rk[r], l[r]);
        st32x(a.em.pay, embase + rk[r], tp[r]);
        s_ck[rk[r]] = tk[r];
      }
    __syncthreads();  // (s_ck, s_nh complete; s_cnt read)
    if (a.emmeta) {  // identity grouping (k_ident_combine): first / last key and descents, sender order
      uint32_t nd = 0, dp = 0;
#pragma unroll
      for (uint32_t i = kDenseIpt * tid; i < kDenseIpt * tid + kDenseIpt; ++i)
        if (i > 0 && i < emtot && s_ck[i] < s_ck[i - 1]) {
          ++nd;
          dp = i;
        }
      uint32_t tnd, tdp;
      block_excl_sum2<kDenseThreads>(nd, nd ? dp : 0u, scratch, &tnd, &tdp);
      if (tid == 0) a.emmeta[b] = make_uint4(emtot ? s_ck[0] : 0u, emtot ? s_ck[emtot - 1] : 0u, tnd, tdp);
    }
    for (uint32_t d = tid; d < (1u << a.nx_bits); d += kDenseThreads)
      if (s_nh[d]) {
        atomicAdd(&a.nhist[(size_t)d * a.nhist_stride + a.ng + b / a.G], s_nh[d]);
        s_nh[d] = 0;
      }
    if (tid == 0) {
      a.chunk_off[b] = lo;  // nothing queued: the bucket's backlog is empty
      a.chunk_cnt[b] = 0u;
      a.chunk_off[a.nb + b] = (uint32_t)embase;
      a.chunk_cnt[a.nb + b] = emtot;
      a.blist[b] = 0u;
    }
    __syncthreads();  // (s_nh reset, s_ck read before the next bucket)
  }
  if (blockIdx.x < a.nb) flush_stats(a, acc);
}

// ---- Dense-bucket launch of the fused superstep (one rank, <= 2^20 actors, max_emit 1).
// The fused block kernel walks every bucket through the general pipeline: table row -> inbox loads
// -> LDS copy and sortedness check -> per-actor segments -> classification -> drain -> emission
// scatter, a dozen barriers and three dependent memory round trips per bucket; at 1M actors every
// bucket is one block's only work, so that chain IS the kernel time (stamps: ~30 K cycles per
// bucket).  A bucket whose inbox -- no backlog, no staged tells, <= kBucket tells -- holds at most one
// message per actor needs none of it: every message is admitted and drained (AD/Mailbox.scala:261,
// 551-565, len = 1), nothing is queued.  This kernel reads the bucket's row of the tell tables,
// gathers the tells, scatters them to their actors' LDS slots (an LDS hit count per actor finds a
// second message -> the bucket is left to the block launch, a.blist), and applies actor la =
// r * kDenseThreads + tid from registers: its flags, kind and state words were loaded beside the
// table row, before the inbox was known.  The tells leave in actor order (= the block path's
// drain order) through group_tells, so the next superstep's tables, tell arena, backlog entries and
// counters are exactly the block path's.  The token ring's buckets are all dense (the wrap-around
// tell arrives after its bucket's own tells: distinct actors, not increasing keys).
#ifndef AGX_EARLY_ROW
#define AGX_EARLY_ROW 1
#endif
constexpr bool kEarlyRow = AGX_EARLY_ROW != 0;
// Grid barrier of the persistent fused launch (every block resident: the host launches it only when
// nb blocks fit the device at once, agx_engine.hip persist_ok).  Thread 0 of each block releases the
// block's stores device-wide (__threadfence: L2 write-back), arrives, and the last arrival bumps the
// generation the others wait on; then acquires (L2 invalidate) before any of the block reads the
// next superstep's tables and tells.  Every wait is bounded: a barrier that times out (a block that
// never became resident) sets pbar[2] and the error word, and every block leaves -- the launch
// always drains; the host reports AGX_EDEVICE and stops using the persistent launch.
__device__ __forceinline__ bool grid_barrier(uint32_t* bar, uint32_t nblocks, uint32_t& gen, uint32_t* s_ok,
                                             uint64_t* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    // release once (L2 write-back), poll RELAXED (an acquire poll invalidates the XCD's L2 on every
    // iteration: 6x slower supersteps, measured), acquire once (L2 invalidate) after the wait
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    uint32_t ok = 1u;
    if (__hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1u) {
      __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&bar[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      uint32_t it = 0;
      while (__hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        __builtin_amdgcn_s_sleep(1);
        if ((++it & 1023u) == 0u &&
            (it > (1u << 22) || __hip_atomic_load(&bar[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          ok = 0u;
          atomicOr(&bar[2], 1u);
          atomicOr((unsigned long long*)err, (unsigned long long)kErrBarrier);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    gen += 1u;
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0u;
}

template <uint32_t KM, bool kOwner, bool kPersist = false>
static __global__ void __launch_bounds__(kDenseThreads, kPersist ? 4 : 2) k_dense_fused(BucketArgs a) {
  static_assert(!(kOwner && kPersist), "persistent launches are single-rank fused supersteps");
  __shared__ __attribute__((aligned(16))) uint32_t s_ks[2 * kBucket];   // per-actor src / pay; group_tells' histogram
  __shared__ __attribute__((aligned(16))) uint64_t U[3 * kBucket / 2];  // segment list; then the tells, sender order
  __shared__ __attribute__((aligned(16))) uint32_t s_hit[4 * kRadix];   // messages per actor; group_tells' bases
  __shared__ uint32_t s_nh[kRadix];                                     // tells per destination bucket
  __shared__ uint32_t scratch[2 * (kDenseWaves + 1)];
  __shared__ uint32_t s_cnt[kDenseIpt * kDenseWaves];
  // (owner mode) tells per (owner class, row, wave), class-major -> their exclusive prefix
  __shared__ uint32_t s_oc[kOwner ? AGX_MAX_RANKS * kDenseIpt * kDenseWaves : 1];
  __shared__ uint32_t s_g[2], s_bad, s_dmin, s_dmax, s_ok;
  static_assert(4 * kRadix >= kBucket && kDenseThreads == kBThreads && kDenseIpt == kBIpt, "group_tells' shapes");
  const BucketLds L{s_ks, s_ks + kBucket, nullptr, U, nullptr, s_hit, nullptr, nullptr, s_nh, scratch, nullptr, nullptr};
  const DevParams& P = a.P;
  const GatherArgs& g = a.g;
  const uint32_t tid = threadIdx.x, w = tid / kWave, lane = lane_id();
  const uint64_t ltm = lanemask_lt();
  const uint32_t amask = (1u << a.bb) - 1u, nhmask = (1u << a.nx_bits) - 1u;
  // Parities.  Persistent launches: the superstep's parity and replay slot advance inside the launch;
  // the host passes the parity-indexed POINTER arrays (g.eg / tcnt / toff / blo / blc / emc) swapped so
  // that index 0 is the first superstep's write parity, and the loop below is unrolled by two with
  // literal parities -- so the compiler selects each pointer at compile time instead of keeping both
  // parities' pointers live -- while the small [2] device words (abort, dense_left, cursors) keep
  // their physical index: logical parity ^ pflip.
  const uint32_t pflip = kPersist ? a.par : 0u;
  uint32_t wpar = kOwner ? 0u : kPersist ? 0u : a.par, rpar = wpar ^ 1u, slot = a.slot;
  if (kOwner && a.halt && a.halt[0]) return;  // (device-resident multi-rank replay stopped)
  // strict replay (this kernel alone is the superstep): an earlier superstep that left a bucket
  // voids this one.  The word is read here and tested after the first bucket's row / state loads are
  // issued (AGX_EARLY_ROW), so its round trip overlaps theirs instead of preceding them; nothing is
  // stored before the test.
  uint32_t ab_in = (!kOwner && a.abort) ? a.abort[rpar ^ pflip] : 0u;
  bool tested = !kEarlyRow;
  const auto abort_test = [&]() -> bool {
    if (ab_in) {
      if (tid == 0) a.abort[wpar ^ pflip] = ab_in;  // (pass it on: the next superstep reads this parity)
      return true;
    }
    if (!kOwner && blockIdx.x == 0 && tid == 0) {  // the cursors the NEXT superstep uses (as k_bucket_apply's fused launch)
      const uint32_t rp = rpar ^ pflip;
      if (a.dense_left) a.dense_left[rp] = 0u;
      g.ovf[rp] = 0u;
      a.skew_n[rp] = 0u;
      if (g.heap_top) g.heap_top[rp] = 0u;
    }
    return false;
  };
  if (!kEarlyRow && abort_test()) return;
  constexpr bool kKindNeeded = (KM & (KM - 1)) != 0 || (KM & kb(AGX_KIND_COMPILED)) != 0;
  const uint32_t w1off = P.W > 1 ? P.sw : 0u;
  uint32_t acc[kBStats] = {0u, 0u, 0u, 0u, 0u};
  if (tid == 0) s_bad = 0;

  // one bucket's superstep; true = the replay is void (return).  With a grid of >= nb blocks (the
  // fused launch: nb <= kDenseThreads) it runs once, outside a loop: the waitcnt pass then has no back
  // edge whose pending loads it must assume, and the row / flag / state loads issue back to back
  const auto bucket = [&](const uint32_t b) -> bool {
    AGX_RTSTAMP(a, 13);
    AGX_STAMP(a, 0);
    const uint32_t a0 = b << a.bb, na = min(1u << a.bb, P.n_local - a0);
    uint32_t* const segp = reinterpret_cast<uint32_t*>(U);  // [nseg + 1] inbox start of each tell segment
    uint32_t* const sego = segp + kRadix + 2;                // [nseg] its offset in eg[rpar]
    // ---- the bucket's row of the tell tables (sender bucket c = tid) and, in the same round trip,
    // this thread's actors' flags, kind and state words
    uint32_t v = 0, o = 0;
    uint32_t* tc = nullptr;  // (the row entry, cleared when consumed: tested on v there, not here -- no wait)
    // (owner: the inbox is the bucket's range of the sorted input, backlog included)
    const uint32_t ib = kOwner ? a.bstart[b] : 0u, ie = kOwner ? a.bstart[b + 1] : 0u;
    if (!kOwner && tid < a.nb) {
      tc = g.tcnt[rpar] + (size_t)b * g.tstride + tid;
      v = *tc;
      o = g.toff[rpar][(size_t)b * g.tstride + tid];
    }
    // (the bucket's backlog / staged counts: issued before the state loads, so waiting for them
    // does not wait for those)
    uint32_t blc0 = 0u, stg0 = 0u;
    if (!kOwner && tid == 0) {
      blc0 = g.blc[rpar][b];
      stg0 = g.stg_cnt[b];
    }
    uint32_t ab[kDenseIpt], kd[kDenseIpt], gs[kDenseIpt];
    uint64_t x0[kDenseIpt], x1[kDenseIpt];
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r) {
      const uint32_t la = r * kDenseThreads + tid, l = a0 + (la < na ? la : 0u);
      ab[r] = P.alive[l];  // (l clamped: unconditional, so no wait between the loads; la >= na is skipped below)
      kd[r] = kKindNeeded ? P.kind[l] : 0u;
      gs[r] = kOwner ? P.gid[l] : l;  // the actor's global id (its tells' sender)
      x0[r] = ldg64(P.state, l * P.sa);
      x1[r] = ldg64(P.state, l * P.sa + w1off);  // (W = 1: word 0 again, zeroed at the apply; no branch between loads)
    }
    if (!tested) {  // (uniform; first bucket of the block)
      tested = true;
      if (abort_test()) return true;
    }
    if (tid == 0) {
      s_g[0] = blc0;
      s_g[1] = stg0;
      s_dmin = 0xFFFFFFFFu;  // (the min / max digit of the bucket's tells to other buckets, below)
      s_dmax = 0u;
    }
    for (uint32_t i = tid; i < kBucket; i += kDenseThreads) s_hit[i] = 0;
    for (uint32_t d = tid; d < kRadix; d += kDenseThreads) s_nh[d] = 0;
    uint32_t cnt, ns;
    const uint2 exix = block_excl_sum2<kDenseThreads>(v, v ? 1u : 0u, scratch, &cnt, &ns);  // (syncs: s_g visible)
    if (kOwner) cnt = ie - ib;
    AGX_STAMP(a, 1);
    if (s_g[0] != 0u || s_g[1] != 0u || cnt > (uint32_t)kBucket) {  // (uniform) backlog / staged / big: block path
      if (tid == 0) {
        a.blist[b] = 1u;
        if (a.dense_left) a.dense_left[wpar ^ pflip] = 1u;
        if (a.dense_alone) a.abort[wpar ^ pflip] = slot + 1u;  // strict replay: the rest of it is void (run_single recovers)
      }
      __syncthreads();  // (s_g is rewritten by the next bucket)
      return false;
    }
    if (!kOwner) {
      if (v) {
        segp[exix.y] = exix.x;
        sego[exix.y] = o;
      }
      if (tid == 0) segp[ns] = cnt;
      __syncthreads();
    }
    // ---- the inbox (tell segments in sender-bucket order), one round trip; each tell to its actor's slot
    uint32_t bad = 0;
    {
      const uint32_t *Ek = sgpr_ptr(kOwner ? a.in.key : g.eg[rpar].key), *Es = sgpr_ptr(kOwner ? a.in.src : g.eg[rpar].src),
                     *Ep = sgpr_ptr(kOwner ? a.in.pay : g.eg[rpar].pay);
      uint32_t idx[kDenseIpt], k[kDenseIpt], sv[kDenseIpt], pv[kDenseIpt];
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r) {
        const uint32_t q = r * kDenseThreads + tid;
        idx[r] = kOwner ? ib + (q < cnt ? q : 0u) : 0u;
        if (!kOwner && q < cnt) {
          uint32_t lo = 0, hi = ns - 1;  // last segment start <= q
          while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (segp[mid] <= q) lo = mid; else hi = mid - 1;
          }
          idx[r] = sego[lo] + (q - segp[lo]);
        }
      }
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r) {
        k[r] = ldg(Ek, idx[r]);
        sv[r] = ldg(Es, idx[r]);
        pv[r] = ldg(Ep, idx[r]);
      }
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r)
        if (r * kDenseThreads + tid < cnt) {
          const uint32_t la = k[r] & amask;
          if (atomicAdd(&s_hit[la], 1u)) bad = 1;  // a second message to the same actor
          s_ks[la] = sv[r];
          s_ks[kBucket + la] = pv[r];
        }
    }
    if (bad) atomicOr(&s_bad, 1u);
    __syncthreads();
    AGX_STAMP(a, 2);
    AGX_STAMP(a, 3);
    AGX_STAMP(a, 4);
    if (s_bad) {  // (uniform) not dense: the block path, row untouched
      __syncthreads();  // (every thread read s_bad)
      if (tid == 0) {
        s_bad = 0;
        a.blist[b] = 1u;
        if (a.dense_left) a.dense_left[wpar ^ pflip] = 1u;
        if (a.dense_alone) a.abort[wpar ^ pflip] = slot + 1u;
      }
      return false;
    }
    if (v) *tc = 0u;  // row consumed
    // (fused: cnt <= kBucket = region, the bucket's own inbox region; owner: its sorted range)
    const uint32_t lo = kOwner ? ib : b * g.region;
    if (tid == 0) {  // nothing queued: the bucket's backlog is empty
      if constexpr (kOwner) {
        a.chunk_off[b] = lo;
        a.chunk_cnt[b] = 0u;
      } else {
        g.cntb[(size_t)slot * a.nb + b] = cnt;
        g.blo[wpar][b] = lo;
        g.blc[wpar][b] = 0u;
      }
    }
    // ---- apply, actor order (one message per actor: admitted, drained; to a stopped actor: a dead letter)
    uint32_t tk[kDenseIpt], tp[kDenseIpt];
    bool tv[kDenseIpt];
    // every actor's hit count, sender and payload in one LDS round trip (la < kBucket: in bounds)
    uint32_t hv[kDenseIpt], svv[kDenseIpt], pvv[kDenseIpt];
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r) {
      const uint32_t la = r * kDenseThreads + tid;
      hv[r] = s_hit[la];
      svv[r] = s_ks[la];
      pvv[r] = s_ks[kBucket + la];
    }
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r)  // (pinned here: the compiler would sink each read into its use, one wait each)
      asm volatile("" : "+v"(hv[r]), "+v"(svv[r]), "+v"(pvv[r]));
    if constexpr (KM == kb(AGX_KIND_RING)) {
      // RING-only populations (the C2 token ring): apply_msg<RING> through RegEmitter, branch-free --
      // w[0] += 1, Behaviors.same, one tell to self + stride while hops are left.  Its destination is
      // always in range (self < n_global, stride pre-reduced), so never a host actor or a dead letter;
      // an actor that is not alive gets a dead letter.  (The generic per-actor dispatch below issued
      // ~200 instructions per actor -- exec-mask branches, kernel-argument reloads -- and made this
      // phase the block's longest: 4.6 K of 16 K cycles.)  Word 1 is untouched, so not stored.
      const uint32_t stride = P.ring_stride, ng = P.n_global;
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r) {
        const uint32_t la = r * kDenseThreads + tid, l = a0 + la;
        const bool has = la < na && hv[r] != 0u, live = (ab[r] & 1u) != 0u, on = has && live;
        const bool em = on && pvv[r] > 0u;
        acc[0] += on ? 1u : 0u;
        acc[4] += on ? 1u : 0u;
        acc[1] += has && !live ? 1u : 0u;
        acc[3] += em ? 1u : 0u;
        uint32_t d = gs[r] + stride;
        d = d >= ng ? d - ng : d;
        tv[r] = em;
        tk[r] = em ? (kOwner ? P.route[d] : d) : 0u;
        tp[r] = em ? pvv[r] - 1u : 0u;
        if (on) st64x(P.state, l * P.sa, x0[r] + 1ull);
      }
    } else {
#pragma unroll
    for (int r = 0; r < kDenseIpt; ++r) {
      const uint32_t la = r * kDenseThreads + tid, l = a0 + la;
      tv[r] = false;
      tk[r] = tp[r] = 0u;
      if (la >= na || !hv[r]) continue;
      if (!(ab[r] & 1u)) {
        ++acc[1];
        continue;
      }
      RegEmitter em{&P, gs[r], 0u, 0u, 0u, 0u};
      uint64_t wv2[2] = {x0[r], P.W > 1 ? x1[r] : 0ull};
      uint32_t kc = kd[r];
      ++acc[4];
      ++acc[0];
      const uint32_t res = apply_msg<KM>(P, kc, gs[r], l, wv2, svv[r], pvv[r], em);
      if (res == AGX_RES_UNHANDLED) ++acc[2];
      if (res == AGX_RES_STOPPED) {
        if constexpr (kOwner) P.stopq[atomicAdd(P.nstop, 1u)] = l;  // (committed by the next superstep)
        else P.alive[l] = (uint8_t)(ab[r] & 0xFEu);  // (fused: only this block reads the bucket's flags)
      }
      st64x(P.state, l * P.sa, wv2[0]);
      if (P.W > 1) st64x(P.state, l * P.sa + w1off, wv2[1]);
      if constexpr ((KM & kb(AGX_KIND_COMPILED)) != 0)
        if (kc != kd[r]) P.kind[l] = (uint8_t)kc;
      acc[3] += em.n_all;
      acc[1] += em.n_all - em.n_valid;
      tv[r] = em.n_valid != 0u;
      tk[r] = em.key;
      tp[r] = em.pay;
    }
    }
    if constexpr (kOwner) {
      // ---- (multi-rank) tells in actor order, grouped by OWNER rank (digit = key >> kOwnerShift, at most
      // AGX_MAX_RANKS classes): per (class, row, wave) ballot counts, one block scan in class-major /
      // sender order, each tell written at its slot straight from registers -- the stable owner
      // partition that group_tells' staged multisplit produced, without the LDS staging and
      // histogram passes (hash-sharded mail goes to every owner: the two-class shortcut below never
      // applies)
      const uint32_t nd = 1u << a.nx_bits;
      uint32_t dg[kDenseIpt], rk[kDenseIpt];
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r) {
        dg[r] = (tk[r] >> a.nx_shift) & nhmask;
        rk[r] = 0u;
        for (uint32_t c = 0; c < nd; ++c) {
          const uint64_t m = __ballot(tv[r] && dg[r] == c);
          if (dg[r] == c) rk[r] = (uint32_t)__popcll(m & ltm);
          if (lane == 0) s_oc[(c * kDenseIpt + r) * kDenseWaves + w] = (uint32_t)__popcll(m);
        }
      }
      __syncthreads();
      static_assert(AGX_MAX_RANKS * kDenseIpt * kDenseWaves <= kDenseThreads, "one (class, row, wave) entry per thread");
      const uint32_t ent = nd * kDenseIpt * kDenseWaves;
      const uint32_t v = tid < ent ? s_oc[tid] : 0u;
      uint32_t emtot;
      const uint32_t ex = block_excl_sum<kDenseThreads>(v, scratch, &emtot);  // (syncs: every v read)
      if (tid < ent) s_oc[tid] = ex;
      __syncthreads();
      const uint64_t embase = (uint64_t)ib * a.kmax;
      constexpr uint32_t kPer = kDenseIpt * kDenseWaves;  // entries per class
      if (tid < nd) {  // this bucket's run for owner tid (only non-zero entries: k_mcompact_copy clears them)
        const uint32_t b0 = s_oc[tid * kPer], b1 = tid + 1 < nd ? s_oc[(tid + 1) * kPer] : emtot;
        if (b1 > b0) {
          g.tcnt[wpar][(size_t)tid * g.tstride + b] = b1 - b0;
          g.toff[wpar][(size_t)tid * g.tstride + b] = (uint32_t)embase + b0;
        }
      }
#pragma unroll
      for (int r = 0; r < kDenseIpt; ++r)
        if (tv[r]) {
          const uint64_t o = embase + s_oc[(dg[r] * kDenseIpt + r) * kDenseWaves + w] + rk[r];
          st32x(g.eg[wpar].key, o, tk[r]);
          st32x(g.eg[wpar].src, o, gs[r]);
          st32x(g.eg[wpar].pay, o, tp[r]);
        }
      if (tid == 0 && g.emc[wpar]) g.emc[wpar][b] = emtot;
      if (tid == 0) {  // the bucket's tell chunk (in-flight accounting)
        a.chunk_off[a.nb + b] = (uint32_t)embase;
        a.chunk_cnt[a.nb + b] = emtot;
      }
    } else {
      // ---- tells in actor order, grouped by destination bucket.  Two classes: digit X (this bucket's
      // own index) and the rest.  Ranks of both from one packed scan of per (row, wave) ballot counts;
      // when the rest share ONE digit (a ring, a stencil: the bucket's tells go to itself and one
      // neighbour) each tell's grouped slot follows directly -- no LDS staging, no multisplit; any
      // other mix stages the tells in sender order and takes group_tells (the block path's grouping).
      const uint32_t X = b & nhmask;
      uint32_t dg[kDenseIpt], rkA[kDenseIpt], rkB[kDenseIpt];
  #pragma unroll
      for (int r = 0; r < kDenseIpt; ++r) {
        dg[r] = (tk[r] >> a.nx_shift) & nhmask;
        const uint64_t ma = __ballot(tv[r] && dg[r] == X), mb = __ballot(tv[r] && dg[r] != X);
        rkA[r] = (uint32_t)__popcll(ma & ltm);
        rkB[r] = (uint32_t)__popcll(mb & ltm);
        if (lane == 0) s_cnt[r * kDenseWaves + w] = (uint32_t)__popcll(ma) | ((uint32_t)__popcll(mb) << 16);
        if (tv[r] && dg[r] != X) {
          atomicMin(&s_dmin, dg[r]);
          atomicMax(&s_dmax, dg[r]);
        }
      }
      __syncthreads();
      AGX_STAMP(a, 5);
      AGX_STAMP(a, 6);
      static_assert(kDenseIpt * kDenseWaves <= kWave, "one lane per (row, wave) count");
      const uint32_t c = lane < (uint32_t)(kDenseIpt * kDenseWaves) ? s_cnt[lane] : 0u;
      const uint32_t inc = wave_incl_sum(c);  // (packed halves: each class <= kBucket < 2^16, no carry)
      const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, kWave - 1);
      const uint32_t totA = tot & 0xFFFFu, totB = tot >> 16, emtot = totA + totB;
      uint32_t preA[kDenseIpt], preB[kDenseIpt];
  #pragma unroll
      for (int r = 0; r < kDenseIpt; ++r) {
        const int gi = r * kDenseWaves + (int)w;  // (wave-uniform lane index)
        const uint32_t ex = (uint32_t)__builtin_amdgcn_readlane((int)(inc - c), gi);
        preA[r] = ex & 0xFFFFu;
        preB[r] = ex >> 16;
      }
      const uint32_t dmin = s_dmin, dmax = s_dmax;
      const uint64_t embase = (uint64_t)lo * a.kmax;
      if (totB == 0 || dmin == dmax) {  // (uniform) at most two destination buckets
        const bool bfirst = totB && dmin < X;  // grouped runs in digit order
        const uint32_t baseA = bfirst ? totB : 0u, baseB = bfirst ? 0u : totA;
  #pragma unroll
        for (int r = 0; r < kDenseIpt; ++r)
          if (tv[r]) {
            const uint64_t o = embase + (dg[r] == X ? baseA + preA[r] + rkA[r] : baseB + preB[r] + rkB[r]);
            st32x(g.eg[wpar].key, o, tk[r]);
            st32x(g.eg[wpar].src, o, gs[r]);
            st32x(g.eg[wpar].pay, o, tp[r]);
          }
        if (tid == 0 && totA) {
          g.tcnt[wpar][(size_t)X * g.tstride + b] = totA;
          g.toff[wpar][(size_t)X * g.tstride + b] = (uint32_t)embase + baseA;
        }
        if (tid == 1 && totB) {
          g.tcnt[wpar][(size_t)dmin * g.tstride + b] = totB;
          g.toff[wpar][(size_t)dmin * g.tstride + b] = (uint32_t)embase + baseB;
        }
        if (tid == 0 && g.emc[wpar]) g.emc[wpar][b] = emtot;
      } else {  // sender order (rank among all tells) in U, per-destination counts, group_tells
        uint32_t* const ukey = reinterpret_cast<uint32_t*>(U);
  #pragma unroll
        for (int r = 0; r < kDenseIpt; ++r)
          if (tv[r]) {
            const uint32_t q = preA[r] + rkA[r] + preB[r] + rkB[r];
            ukey[q] = tk[r];
            ukey[kBucket + q] = gs[r];
            ukey[2 * kBucket + q] = tp[r];
            lds_hist_inc(s_nh, dg[r]);
          }
        __syncthreads();
        group_tells<true>(a, L, b, wpar, embase, emtot, a.em);
      }
    }
    AGX_STAMP(a, 7);
    if (tid == 0) a.blist[b] = 0u;
    __syncthreads();  // (the bucket's LDS arrays are reset by the next one)
    AGX_RTSTAMP(a, 14);
    AGX_STAMP(a, 8);
    return false;
  };
  if constexpr (kPersist) {
    // psteps supersteps, one bucket per block (grid = nb), a grid barrier between them.  A superstep
    // that meets a non-dense bucket marks abort[wpar] (as the graph's launch would); the next one
    // reads the mark after the barrier, passes it on and the launch ends -- the state the graph of
    // separate launches leaves, so run_single's recovery is the same.
    const uint32_t b = blockIdx.x;
    uint32_t gen = 0u;
    if (tid == 0) gen = __hip_atomic_load(&a.pbar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // superstep s + 1 after superstep s: barrier, then the mark superstep s may have left
    const auto next = [&](uint32_t wp) -> bool {
      if (!grid_barrier(a.pbar, a.nb, gen, &s_ok, (uint64_t*)&a.stats[ST_ERROR])) return false;
      wpar = wp;
      rpar = wp ^ 1u;
      ++slot;
      ab_in = a.abort ? __hip_atomic_load(&a.abort[rpar ^ pflip], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      tested = !kEarlyRow;
      return kEarlyRow || !abort_test();
    };
    // (the bucket index is made opaque each superstep: every address derived from it would otherwise
    // be hoisted out of the loop and held in registers across it -- 105 -> 164 VGPRs)
    const auto opaque = [](uint32_t x) {
      asm volatile("" : "+s"(x));
      return x;
    };
    for (uint32_t s = 0; s < a.psteps; s += 2) {  // (two supersteps per trip: literal parities 0, 1)
      if (s > 0 && !next(0u)) break;
      if (bucket(opaque(b))) break;
      if (s + 1 >= a.psteps || !next(1u)) break;
      if (bucket(opaque(b))) break;
    }
    flush_stats(a, acc);
  } else {
    if (gridDim.x >= a.nb) {
      if (blockIdx.x < a.nb && bucket(blockIdx.x)) return;
    } else {
      for (uint32_t b = blockIdx.x; b < a.nb; b += gridDim.x)
        if (bucket(b)) return;
    }
    if (blockIdx.x < a.nb) flush_stats(a, acc);
  }
}

// kSkew = false: every bucket whose inbox fits one LDS tile (<= kBucket messages); larger
// inboxes are appended to the skew list.  kSkew = true (launched right after): the listed
// buckets, general path — separate instantiation, so its register pressure never reaches
// the fast path.
// kOwner (multi-rank): tells leave grouped by owner rank into g.eg[0] + g.tcnt/toff[0]
// (digit = key >> kOwnerShift) instead of the chunk arena + next-pass histogram.
// (One launch with both paths spills ~20 VGPRs and measured 13% slower at 1M.)
// =========================================================================
// Skewed buckets across workgroups (single-rank multi-pass, plain and compiled behaviours).
// A bucket whose inbox exceeds one LDS tile -- R-MAT / Zipf hot buckets of C5 / C3 hold 10^4 -
// 10^5 arrivals plus their backlog -- is cut into parts of `span` inbox positions, one
// workgroup each, in three launches before the skew launch:
//   k_skew_plan     bucket bounds of every skewed bucket, parts per bucket (one block)
//   k_skew_count    per part: arrivals per actor                     -> pc[part][actor]
//   k_skew_scan     per bucket: exclusive prefix of pc over parts (in place), length, admission
//                   keep = alive ? min(len, C) : 0 (tail-drop, AD/Mailbox.scala:551-565), drained
//                   = min(keep, T) (:261), queued = keep - drained, and their segment starts
//   k_skew_scatter  per part: stable rank of each arrival among its actor's arrivals (the part's
//                   prefix + in-part wave ranks; a part of the previous backlog, which is already
//                   grouped by actor in actor order, takes the rank from its run start -- a
//                   streaming copy); admitted drained messages go to the scratch copy
//                   at lo + dseg[actor] + rank, queued ones straight to the backlog arena at
//                   lo + blp[actor] + rank - T (the canonical order of bucket_finish's copy)
// The skew launch then drains each bucket from the scratch copy (<= T messages per actor), so no
// workgroup walks a hot bucket's whole inbox alone (Mailbox.run semantics unchanged).
// =========================================================================
#ifndef AGX_EARLY_STATE
#define AGX_EARLY_STATE 1
#endif
#ifndef AGX_DENSE
#define AGX_DENSE 1
#endif
constexpr bool kDenseBuckets = AGX_DENSE != 0;  // dense buckets (one message per actor) skip the sort (A/B build knob)
constexpr bool kEarlyState = AGX_EARLY_STATE != 0;  // fused fast path: state loads at bucket start (A/B build knob)
#ifndef AGX_LATE_ALIVE
#define AGX_LATE_ALIVE 1
#endif
constexpr bool kLateAlive = AGX_LATE_ALIVE != 0;  // alive flags stored to LDS after the inbox loads issue (A/B knob)  // multi-pass: block path reuses the wave check's bounds (A/B knob)
constexpr uint32_t kSkRec = 12;    // b, lo, cnt, blc, blo, bst, pbase, np, ndrain, bltot, npb, -
constexpr uint32_t kSkSpan = 4 * kBucket;  // minimum inbox positions per part
constexpr uint32_t kRingMaxC = 4096;  // bounded-mailbox rings: largest mailbox capacity they hold (16-bit head / length)
constexpr uint32_t kRingMaxT = 64;   // largest throughput with rings (drain scratch of kBucket x T per slot)
constexpr uint32_t kRingSlots = 8192;  // the pool size the tests and A/B runs use (AGX_RING_SLOTS=8192; default off)
constexpr unsigned long long kRingPoolBytes = 16ull << 30;  // ring pool budget (AGX_RING_MB; <= free HBM / 4)
constexpr uint32_t kSkActPlanes = 4;       // per actor of a skewed bucket: admitted, drained start, backlog start, drain limit

struct SkewArgs {
  uint32_t* rec;      // [nb][kSkRec]
  uint32_t* act;      // [nb][kSkActPlanes][kBucket]: keep, dseg, blp, drain limit (its mailbox class)
  uint32_t* pc;       // [max_parts][kBucket] arrivals per actor -> prefix over the bucket's parts
  uint32_t* meta;     // [0] parts, [1] span
  uint32_t budget;    // target number of parts (the span grows beyond kSkSpan to stay near it)
  uint32_t max_parts; // rows of pc: budget + 2 x (skewed buckets) (a bucket's backlog and new-mail parts are
                      // rounded up separately: at most two parts beyond the budget each)
};

__device__ __forceinline__ uint32_t sk_key(const BucketArgs& a, const InView& iv, const uint32_t* r, uint32_t rpar,
                                           uint32_t q) {
  return q < r[3] ? a.g.bl[rpar].key[r[4] + q] : iv.m.key[iv.at(r[5] + q - r[3])];
}

static __global__ void __launch_bounds__(kScanThreads) k_skew_plan(BucketArgs a, SkewArgs k) {
  __shared__ uint32_t scratch[kScanThreads / kWave + 1];
  __shared__ unsigned long long s_tot;
  const uint32_t n = *a.skew_n, tid = threadIdx.x;
  if (tid == 0) s_tot = 0;
  __syncthreads();
  unsigned long long part = 0;
  // ring pool slots for skewed buckets without one: the free stack first, then fresh slots
  const uint32_t nfree = a.ring_of ? a.ring_next[1] : 0u, nnext = a.ring_of ? a.ring_next[0] : 0u;
  uint32_t taken = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += kScanThreads) {
    const uint32_t i = i0 + tid;
    const uint32_t b = i < n ? a.skew_list[i] : 0u;
    uint32_t rs = i < n && a.ring_of ? a.ring_of[b] : 0u;  // ring pool slot + 1
    const bool need = i < n && a.ring_of && !rs;
    uint32_t tn;
    const uint32_t g = taken + block_excl_sum<kScanThreads>(need ? 1u : 0u, scratch, &tn);
    taken += tn;
    if (need) {
      if (g < nfree) rs = a.ring_free[nfree - 1u - g] + 1u;
      else if (nnext + (g - nfree) < a.ring_slots) rs = nnext + (g - nfree) + 1u;
      if (rs) a.ring_of[b] = rs;
    }
    if (i >= n) continue;
    const uint32_t bs = a.bstart[b], be = a.bstart[b + 1], bp = a.blpre[b] + a.bl_sbase[b / kBlSlice];
    const uint32_t blc = a.chunk_cnt[b], blo = a.chunk_off[b];
    uint32_t* r = k.rec + (size_t)i * kSkRec;
    r[0] = b;
    r[1] = rs ? a.ring_lo0 + (rs - 1u) * (uint32_t)kBucket * a.ring_t : bs + bp;
    r[11] = rs;
    r[2] = blc + (be - bs);
    r[3] = blc;
    r[4] = blo;
    r[5] = bs;
    part += blc + (be - bs);
  }
  atomicAdd(&s_tot, part);
  if (tid == 0 && a.ring_of && taken) {
    const uint32_t fu = min(taken, nfree);
    a.ring_next[1] = nfree - fu;
    a.ring_next[0] = min(a.ring_slots, nnext + (taken - fu));
  }
  __syncthreads();
  // parts of at least kSkSpan positions, sum over buckets of ceil(cnt / span) <= budget + n
  const unsigned long long tot = s_tot;
  const uint32_t bud = k.budget;
  uint32_t span = kSkSpan;
  if (tot > (unsigned long long)span * bud)
    span = (uint32_t)(((tot + bud - 1) / bud + kBucket - 1) / kBucket * kBucket);
  uint32_t carry = 0;
  for (uint32_t i0 = 0; i0 < n; i0 += kScanThreads) {
    const uint32_t i = i0 + tid;
    uint32_t np = 0, npb = 0;
    if (i < n) {  // backlog parts, then parts of the new mail (a part never mixes the two)
      const uint32_t c = k.rec[(size_t)i * kSkRec + 2], blc = k.rec[(size_t)i * kSkRec + 3];
      npb = (blc + span - 1) / span;
      np = npb + (c - blc + span - 1) / span;
    }
    uint32_t t;
    const uint32_t ex = block_excl_sum<kScanThreads>(np, scratch, &t);
    if (i < n) {
      k.rec[(size_t)i * kSkRec + 6] = carry + ex;
      k.rec[(size_t)i * kSkRec + 7] = np;
      k.rec[(size_t)i * kSkRec + 10] = npb;
    }
    carry += t;
  }
  if (tid == 0) {
    k.meta[0] = carry;
    k.meta[1] = span;
  }
}

// part t -> (skew index, first inbox position, end) (binary search over the part bases)
__device__ __forceinline__ bool sk_part(const BucketArgs& a, const SkewArgs& k, uint32_t t, uint32_t* s_q) {
  if (threadIdx.x == 0) {
    uint32_t lo = 0, hi = *a.skew_n;  // last i with pbase[i] <= t
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) / 2;
      if (k.rec[(size_t)mid * kSkRec + 6] <= t) lo = mid;
      else hi = mid;
    }
    const uint32_t* r = k.rec + (size_t)lo * kSkRec;
    const uint32_t span = k.meta[1], p = t - r[6], npb = r[10], blc = r[3];
    s_q[0] = lo;
    if (p < npb) {
      s_q[1] = p * span;
      s_q[2] = min(blc, (p + 1) * span);
    } else {
      s_q[1] = blc + (p - npb) * span;
      s_q[2] = min(r[2], blc + (p - npb + 1) * span);
    }
  }
  __syncthreads();
  return true;
}

static __global__ void __launch_bounds__(kBThreads) k_skew_count(BucketArgs a, SkewArgs k) {
  __shared__ uint32_t s_c[kBucket];
  __shared__ uint32_t s_q[3];
  const uint32_t tid = threadIdx.x, nparts = k.meta[0], rpar = (*a.pstep & 1u) ^ 1u, amask = (1u << a.bb) - 1u;
  if (nparts > k.max_parts) {  // (plan and buffer disagree: never launched so; report, do nothing)
    if (blockIdx.x == 0 && tid == 0) atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
    return;
  }
  const InView iv = in_view(a);
  for (uint32_t t = blockIdx.x; t < nparts; t += gridDim.x) {
    for (uint32_t i = tid; i < kBucket; i += kBThreads) s_c[i] = 0;
    sk_part(a, k, t, s_q);
    const uint32_t* r = k.rec + (size_t)s_q[0] * kSkRec;
    const uint32_t q0 = s_q[1], q1 = s_q[2];
    for (uint32_t q = q0 + tid; q < q1; q += 8 * kBThreads) {  // 8 loads in flight
      uint32_t kk[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) kk[j] = q + j * kBThreads < q1 ? sk_key(a, iv, r, rpar, q + j * kBThreads) : 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (q + j * kBThreads < q1) lds_hist_inc(s_c, kk[j] & amask);
    }
    __syncthreads();
    uint32_t* pc = k.pc + (size_t)t * kBucket;
    for (uint32_t i = tid; i < kBucket; i += kBThreads) pc[i] = s_c[i];  // (all rows: zero past the bucket)
    __syncthreads();
  }
}

static __global__ void __launch_bounds__(kBThreads) k_skew_scan(BucketArgs a, SkewArgs k) {
  __shared__ uint32_t scratch[2 * (kBWaves + 1)];
  const DevParams& P = a.P;
  const uint32_t tid = threadIdx.x, n = *a.skew_n;
  if (k.meta[0] > k.max_parts) return;  // (plan and buffer disagree: k_skew_count reported it; no pc access)
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    uint32_t* r = k.rec + (size_t)i * kSkRec;
    const uint32_t b = r[0], pb = r[6], np = r[7];
    const uint32_t a0 = b << a.bb, na = min(1u << a.bb, P.n_local - a0);
    uint32_t len[kBAct] = {0, 0, 0, 0};
    const uint32_t la0 = tid * kBAct;
    for (uint32_t p = 0; p < np; ++p) {  // per actor: exclusive prefix over the parts, in place
      uint4* row = reinterpret_cast<uint4*>(k.pc + (size_t)(pb + p) * kBucket) + tid;
      const uint4 v = *row;
      *row = make_uint4(len[0], len[1], len[2], len[3]);
      len[0] += v.x; len[1] += v.y; len[2] += v.z; len[3] += v.w;
    }
    uint32_t keep[kBAct], dr[kBAct], qd[kBAct], tl[kBAct], sd = 0, sq = 0, ndead = 0;
    const uint32_t rs = r[11];  // ring bucket: its queued messages stay in the per-actor rings
    if (rs) {
      // ring of actor la: head h, length Lr (messages queued earlier, in arrival order, ahead of this
      // superstep's arrivals).  Tail-drop over the concatenation ring ++ arrivals, as bucket_finish:
      // keep = alive ? min(Lr + arr, C) : 0; Lk = min(Lr, keep) ring messages stay, keep - Lk arrivals
      // are admitted; drained = min(keep, T): the first rr = min(Lk, drained) from the ring, then
      // drained - rr arrivals; the other admitted arrivals are appended to the ring.
      // Planes: [0] arrivals admitted, [1] drained segment start, [2] ring slot of the first queued
      // arrival, [3] arrivals drained (the scatter's drain limit).
      const uint32_t cs = a.ring_c, sbase = (rs - 1u) * (uint32_t)kBucket;
      uint32_t* st = a.ring_state + sbase;
      uint32_t hd[kBAct], rr[kBAct], nl[kBAct];
      int dl = 0;
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        const uint32_t la = la0 + j;
        const uint32_t ab = la < na ? P.alive[a0 + la] : 0u;
        uint32_t C, T;
        mbox_limits(P, ab, C, T);
        const uint32_t sv = st[la], h = sv & 0xFFFFu, lr = sv >> 16, tot = lr + len[j];
        const uint32_t kp = (ab & 1u) ? ((C == 0 || tot < C) ? tot : C) : 0u;
        const uint32_t lk = min(lr, kp), drn = min(kp, T);
        rr[j] = min(lk, drn);
        hd[j] = h;
        keep[j] = kp - lk;          // arrivals admitted
        tl[j] = drn - rr[j];        // arrivals drained
        dr[j] = drn;
        qd[j] = h + lk < cs ? h + lk : h + lk - cs;  // ring slot of the first queued arrival
        nl[j] = kp - drn;           // ring length after this superstep
        ndead += tot - kp;
        dl += (int)nl[j] - (int)lr;
        sd += drn;
      }
      uint32_t td, tl2;
      uint32_t nlt = 0, arr = 0;
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        nlt += nl[j];
        arr += len[j];
      }
      const uint2 ex2 = block_excl_sum2<kBThreads>(sd, nlt, scratch, &td, &tl2);
      uint32_t ed = ex2.x;
      uint32_t ta;
      block_excl_sum<kBThreads>(arr, scratch, &ta);
      if (tid == 0 && tl2 == 0 && ta <= (uint32_t)kBucket) {
        // cooled down: rings empty and this superstep's mail fits one tile -- the slot goes back to
        // the pool (the drain scratch / tell slice is still this superstep's; the next plan reuses it)
        a.ring_of[b] = 0u;
        a.ring_free[atomicAdd(&a.ring_next[1], 1u)] = rs - 1u;
      }
      uint32_t* act = k.act + (size_t)i * kSkActPlanes * kBucket;
      uint32_t ds[kBAct];
      const uint32_t lo = r[1];
      const uint32_t* __restrict__ rsrc = a.ring_src + (size_t)sbase * cs;
      const uint32_t* __restrict__ rpay = a.ring_pay + (size_t)sbase * cs;
      uint32_t rmax = 0;
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        const uint32_t la = la0 + j;
        ds[j] = ed;
        ed += dr[j];
        rmax = max(rmax, rr[j]);
        uint32_t h2 = hd[j] + rr[j];
        h2 = h2 < cs ? h2 : h2 - cs;
        st[la] = (nl[j] ? h2 : 0u) | nl[j] << 16;
      }
      // the rings' drained heads -> the drain scratch (first in each actor's segment): the four
      // actors' loads of one ring position are issued together, then stored (a round trip per
      // position, not per message: the stores could alias the ring as far as the compiler knows)
      for (uint32_t q = 0; q < rmax; ++q) {
        uint32_t sv[kBAct], pv[kBAct];
#pragma unroll
        for (int j = 0; j < kBAct; ++j) {
          uint32_t x = hd[j] + q;
          x = x < cs ? x : x - cs;
          const size_t o = (size_t)(la0 + j) * cs + (q < rr[j] ? x : 0u);
          sv[j] = rsrc[o];
          pv[j] = rpay[o];
        }
#pragma unroll
        for (int j = 0; j < kBAct; ++j)
          if (q < rr[j]) {
            a.scr.key[lo + ds[j] + q] = a0 + la0 + j;
            a.scr.src[lo + ds[j] + q] = sv[j];
            a.scr.pay[lo + ds[j] + q] = pv[j];
          }
      }
      reinterpret_cast<uint4*>(act)[tid] = make_uint4(keep[0], keep[1], keep[2], keep[3]);
      reinterpret_cast<uint4*>(act + kBucket)[tid] = make_uint4(ds[0], ds[1], ds[2], ds[3]);
      reinterpret_cast<uint4*>(act + 2 * kBucket)[tid] = make_uint4(qd[0], qd[1], qd[2], qd[3]);
      reinterpret_cast<uint4*>(act + 3 * kBucket)[tid] = make_uint4(tl[0], tl[1], tl[2], tl[3]);
      if (tid == 0) {
        r[8] = td;
        r[9] = 0u;  // (nothing in the backlog arena)
      }
      const uint32_t wd = wave_incl_sum(ndead);
      if (lane_id() == kWave - 1 && wd) atomicAdd(&a.bstats[(size_t)blockIdx.x * kBStats + 1], (unsigned long long)wd);
      // ring length change of the block (two's complement into the u64 total)
      const uint32_t gp = wave_incl_sum(dl > 0 ? (uint32_t)dl : 0u), gn = wave_incl_sum(dl < 0 ? (uint32_t)-dl : 0u);
      if (lane_id() == kWave - 1 && gp != gn)
        atomicAdd(a.ring_total, (unsigned long long)((long long)gp - (long long)gn));
      continue;
    }
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      const uint32_t la = la0 + j;
      const uint32_t ab = la < na ? P.alive[a0 + la] : 0u;
      uint32_t C, T;
      mbox_limits(P, ab, C, T);
      keep[j] = (ab & 1u) ? ((C == 0 || len[j] < C) ? len[j] : C) : 0u;
      ndead += len[j] - keep[j];
      tl[j] = T;
      dr[j] = min(keep[j], T);
      qd[j] = keep[j] - dr[j];
      sd += dr[j];
      sq += qd[j];
    }
    uint32_t td, tq;
    const uint2 ex = block_excl_sum2<kBThreads>(sd, sq, scratch, &td, &tq);
    uint32_t* act = k.act + (size_t)i * kSkActPlanes * kBucket;
    uint32_t ds[kBAct], bs[kBAct], ed = ex.x, eq = ex.y;
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      ds[j] = ed;
      bs[j] = eq;
      ed += dr[j];
      eq += qd[j];
    }
    reinterpret_cast<uint4*>(act)[tid] = make_uint4(keep[0], keep[1], keep[2], keep[3]);
    reinterpret_cast<uint4*>(act + kBucket)[tid] = make_uint4(ds[0], ds[1], ds[2], ds[3]);
    reinterpret_cast<uint4*>(act + 2 * kBucket)[tid] = make_uint4(bs[0], bs[1], bs[2], bs[3]);
    reinterpret_cast<uint4*>(act + 3 * kBucket)[tid] = make_uint4(tl[0], tl[1], tl[2], tl[3]);
    if (tid == 0) {
      r[8] = td;
      r[9] = tq;
    }
    const uint32_t wd = wave_incl_sum(ndead);  // admission drops: dead letters (block stats slot)
    if (lane_id() == kWave - 1 && wd) atomicAdd(&a.bstats[(size_t)blockIdx.x * kBStats + 1], (unsigned long long)wd);
  }
}

static __global__ void __launch_bounds__(kBThreads) k_skew_scatter(BucketArgs a, SkewArgs k) {
  // (80 KB of LDS or less: two workgroups per CU -- with a per-actor totals array beside these it
  // was 82 KB, one workgroup per CU)
  __shared__ __attribute__((aligned(16))) uint16_t whist[kBWaves * kBucket];  // 32 KB
  __shared__ uint32_t s_run[kBucket], s_keep[kBucket], s_ds[kBucket + 1], s_bs[kBucket], s_T[kBucket];
  // backlog parts (no ranking): first position of each actor's run in the part, over whist
  uint32_t* const s_first = reinterpret_cast<uint32_t*>(whist);
  __shared__ uint32_t s_q[3];
  const DevParams& P = a.P;
  const uint32_t tid = threadIdx.x, w = tid / kWave, lane = lane_id(), nparts = k.meta[0];
  const uint32_t wpar = *a.pstep & 1u, rpar = wpar ^ 1u, amask = (1u << a.bb) - 1u;
  const uint64_t ltm = lanemask_lt();
  const Msgs blw = a.g.bl[wpar];
  if (nparts > k.max_parts) return;
  const InView iv = in_view(a);
  for (uint32_t t = blockIdx.x; t < nparts; t += gridDim.x) {
    sk_part(a, k, t, s_q);
    const uint32_t i = s_q[0], q0 = s_q[1], q1 = s_q[2];
    const uint32_t* r = k.rec + (size_t)i * kSkRec;
    const uint32_t lo = r[1], blc = r[3], blo = r[4], bst = r[5], rs = r[11];
    const uint32_t* act = k.act + (size_t)i * kSkActPlanes * kBucket;
    const uint32_t* pc = k.pc + (size_t)t * kBucket;
    for (uint32_t la = tid; la < kBucket; la += kBThreads) {
      s_run[la] = pc[la];
      s_keep[la] = act[la];
      s_ds[la] = act[kBucket + la];
      s_bs[la] = act[2 * kBucket + la];
      s_T[la] = act[3 * kBucket + la];  // the actor's drain limit (mailbox class; ring: arrivals drained)
    }
    if (tid == 0) s_ds[kBucket] = r[8];
    __syncthreads();
    // an admitted arrival of rank `rank` among its actor's arrivals: drained (the scratch copy, in
    // canonical order) or queued (the backlog arena at the canonical position; ring bucket: the
    // actor's ring, behind the messages it already holds)
    const uint32_t cs = a.ring_c;
    const size_t rbase = rs ? (size_t)(rs - 1u) * kBucket * cs : 0;
    auto place = [&](uint32_t la, uint32_t rank, uint32_t kv, uint32_t sv, uint32_t pv) {
      const uint32_t T = s_T[la];
      if (rank < T) {
        const uint32_t pos = rs ? lo + s_ds[la + 1] - T + rank : lo + s_ds[la] + rank;  // (ring: after its drained head)
        a.scr.key[pos] = kv;
        a.scr.src[pos] = sv;
        a.scr.pay[pos] = pv;
      } else if (rs) {
        uint32_t x = s_bs[la] + rank - T;
        x = x < cs ? x : x - cs;
        a.ring_src[rbase + (size_t)la * cs + x] = sv;
        a.ring_pay[rbase + (size_t)la * cs + x] = pv;
      } else {
        const uint32_t pos = lo + s_bs[la] + rank - T;
        blw.key[pos] = kv;
        blw.src[pos] = sv;
        blw.pay[pos] = pv;
      }
    };
    if (q1 <= blc) {  // a part of the previous backlog: grouped by actor, every item admitted unless
                      // its actor stopped; rank = earlier parts' count + distance to the run start
      // (every load of a sub-tile -- keys, the previous keys, senders, payloads -- is issued before the
      // run-start barrier: one round trip per sub-tile instead of two)
      const uint32_t *Bk = sgpr_ptr(a.g.bl[rpar].key), *Bs = sgpr_ptr(a.g.bl[rpar].src),
                     *Bp = sgpr_ptr(a.g.bl[rpar].pay);
      for (uint32_t sub = q0; sub < q1; sub += kBucket) {
        const uint32_t wbase = sub + w * (kBIpt * kWave);
        uint32_t kk[kBIpt], kp[kBIpt], sv[kBIpt], pv[kBIpt];
#pragma unroll
        for (int u = 0; u < kBIpt; ++u) {
          const uint32_t q = wbase + u * kWave + lane;
          const uint32_t i = q < q1 ? blo + q : blo, ip = q < q1 && q > q0 ? blo + q - 1 : blo;
          kk[u] = ldg(Bk, i);
          kp[u] = ldg(Bk, ip);
          sv[u] = ldg(Bs, i);
          pv[u] = ldg(Bp, i);
        }
#pragma unroll
        for (int u = 0; u < kBIpt; ++u) {
          const uint32_t q = wbase + u * kWave + lane;
          if (q < q1 && (q == q0 || (kp[u] & amask) != (kk[u] & amask))) s_first[kk[u] & amask] = q;
        }
        __syncthreads();  // (a run start written in a later sub-tile belongs to another actor)
#pragma unroll
        for (int u = 0; u < kBIpt; ++u) {
          const uint32_t q = wbase + u * kWave + lane, la = kk[u] & amask;
          if (q >= q1) continue;
          const uint32_t rank = s_run[la] + (q - s_first[la]);
          if (rank >= s_keep[la]) continue;
          place(la, rank, kk[u], sv[u], pv[u]);
        }
      }
      __syncthreads();
      continue;
    }
    for (uint32_t sub = q0; sub < q1; sub += kBucket) {
      const uint32_t wbase = sub + w * (kBIpt * kWave);
      uint32_t kk[kBIpt], sv[kBIpt], pv[kBIpt], rk[kBIpt];
      bool live[kBIpt];
      int any = 0;
#pragma unroll
      for (int u = 0; u < kBIpt; ++u) {
        const uint32_t q = wbase + u * kWave + lane;
        kk[u] = q < q1 ? sk_key(a, iv, r, rpar, q) : 0u;
      }
#pragma unroll
      for (int u = 0; u < kBIpt; ++u) {
        const uint32_t q = wbase + u * kWave + lane, la = kk[u] & amask;
        live[u] = q < q1 && s_run[la] < s_keep[la];  // actor not yet full: rank it
        any |= live[u];
      }
      if (!__syncthreads_or(any)) continue;  // every arrival of this sub-tile is a dead letter
      for (uint32_t x = tid; x < kBWaves * kBucket / 2; x += kBThreads) reinterpret_cast<uint32_t*>(whist)[x] = 0;
#pragma unroll
      for (int u = 0; u < kBIpt; ++u) {
        const uint32_t q = wbase + u * kWave + lane;
        if (live[u]) {
          if (q < blc) {
            sv[u] = a.g.bl[rpar].src[blo + q];
            pv[u] = a.g.bl[rpar].pay[blo + q];
          } else {
            const uint32_t x = iv.at(bst + q - blc);
            sv[u] = iv.m.src[x];
            pv[u] = iv.m.pay[x];
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < kBIpt; ++u) rk[u] = wave_rank(live[u], kk[u] & amask, a.bb, whist + w * kBucket, ltm);
      __syncthreads();
      uint32_t tot[kBucket / kBThreads];  // this thread's actors' arrivals in the sub-tile
#pragma unroll
      for (uint32_t i = 0; i < kBucket / kBThreads; ++i) {
        const uint32_t la = i * kBThreads + tid;
        uint32_t run = 0;
#pragma unroll
        for (int x = 0; x < kBWaves; ++x) {
          const uint32_t c2 = whist[x * kBucket + la];
          whist[x * kBucket + la] = (uint16_t)run;
          run += c2;
        }
        tot[i] = run;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < kBIpt; ++u) {
        if (!live[u]) continue;
        const uint32_t la = kk[u] & amask;
        const uint32_t rank = s_run[la] + whist[w * kBucket + la] + rk[u];  // among this actor's arrivals
        if (rank < s_keep[la]) place(la, rank, kk[u], sv[u], pv[u]);
      }
      __syncthreads();
#pragma unroll
      for (uint32_t i = 0; i < kBucket / kBThreads; ++i) s_run[i * kBThreads + tid] += tot[i];
      __syncthreads();
    }
  }
}

#ifndef AGX_WIDE_WPE
#define AGX_WIDE_WPE 4  // CRDT (wide) variants: minimum waves per SIMD (4: 128 VGPRs; 2: 256, one block per CU)
#endif
template <bool kWide, uint32_t KM, bool kGather, bool kSkew, bool kOwner = false>
static __global__ void __launch_bounds__(kBThreads, kWide ? AGX_WIDE_WPE : 4) k_bucket_apply(BucketArgs a) {
  constexpr bool kDefer = !kSkew;  // large inboxes are appended to the skew list
  if (kOwner && a.halt && a.halt[0]) return;  // (device-resident multi-rank replay stopped)
  // key/src/pay carved from one array: group_tells reuses key+src as a 16 KB histogram
  __shared__ __attribute__((aligned(16))) uint32_t s_ksp[3 * kBucket];
  uint32_t* const s_key = s_ksp;
  uint32_t* const s_src = s_ksp + kBucket;
  uint32_t* const s_pay = s_ksp + 2 * kBucket;
  __shared__ __attribute__((aligned(16))) uint64_t U[2 * kBucket];  // 32 KB
  __shared__ __attribute__((aligned(16))) uint32_t s_seg[kBucket + 4];
  __shared__ __attribute__((aligned(16))) uint32_t s_ecnt[kBucket];
  __shared__ uint8_t s_alive[kBucket];
  __shared__ uint8_t s_kind[kBucket];
  __shared__ uint32_t s_nh[kRadix];
  __shared__ uint32_t scratch[2 * (kBWaves + 1)];
  __shared__ uint32_t s_lo, s_hi, s_g[6], s_rowtop, s_flags;
  __shared__ unsigned long long s_stat[5];
  const BucketLds L{s_key, s_src, s_pay, U, s_seg, s_ecnt, s_alive, s_kind, s_nh, scratch, s_stat, &s_rowtop};
  uint16_t* whist = reinterpret_cast<uint16_t*>(U);  // [kBWaves][kBucket]

  const DevParams& P = a.P;
  const int tid = threadIdx.x, w = tid / kWave;
  const uint32_t lane = lane_id();
  const uint64_t ltm = lanemask_lt();
  const uint32_t amask = (1u << a.bb) - 1u;  // actor index within the bucket
  const GatherArgs& g = a.g;
  // (kBypass: single-rank multi-pass — the previous backlog is read in place, not sorted)
  constexpr bool kBypass = !kGather && !kOwner;
  const InView iv = kBypass ? in_view(a) : InView{a.in, 0u, 0xFFFFFFFFu};  // (identity grouping: rotated tells)
  // fused / bypass: write parity w, read parity w ^ 1
  const uint32_t wpar = kGather ? a.par : kBypass ? (*a.pstep & 1u) : 0u, rpar = wpar ^ 1u;
  uint32_t* const skew_n = a.skew_n + (kGather ? wpar : 0u);  // (non-fused: one list, reset by the sort)
  if (kGather && !kSkew && a.abort) {
    const uint32_t ab = a.abort[rpar];  // an earlier superstep of this replay deferred a bucket
    if (ab) {
      if (tid == 0) a.abort[wpar] = ab;  // (pass it on: the next superstep reads this parity)
      return;
    }
  }
  if (kGather && !kSkew && blockIdx.x == 0 && tid == 0) {
    // reset the per-parity cursors that the NEXT superstep (parity rpar) will use (the previous
    // superstep, which used them, is complete)
    g.ovf[rpar] = 0u;
    a.skew_n[rpar] = 0u;
    if (g.heap_top) g.heap_top[rpar] = 0u;
  }
  if (!kGather && !kSkew && blockIdx.x == 0) {
    if (tid == 0 && *(kBypass ? a.d_ninbox : a.d_n) > 0) atomicAdd((unsigned long long*)&a.stats[ST_STEPS], 1ull);
    for (uint32_t i = tid; i < kStagedChunks; i += kBThreads) a.chunk_cnt[2 * a.nb + i] = 0;  // staged consumed
  }

  // single-rank multi-pass, plain behaviours, after k_tiny_apply / k_dense_apply (fused: after
  // k_dense_fused): a.blist[b] != 0 marks the buckets the earlier launch left to this one.  A block takes kListBatch of its grid-stride buckets at a time:
  // wave 0 reads their marks in one round trip, the ballot is the batch's work mask (no list, no
  // atomics; the bucket -> block assignment stays the grid-stride one)
  constexpr uint32_t kListBatch = 32;
  const bool listed = !kSkew && !kWide && a.blist != nullptr;  // (fused / owner: k_dense_fused's marks)
  __shared__ uint32_t s_todo;
  uint32_t acc[kBStats] = {0u, 0u, 0u, 0u, 0u};  // this thread's counters over the block's buckets
#ifdef AGX_ACC_SHADOW
  if (lane == kWave - 1) acc_shadow()[w] = 0u;  // (each wave's own slot: no barrier needed)
#endif
  // (listed after a dense launch that took every bucket: nothing to do past the per-launch work above)
  const uint32_t nwork = kSkew ? *skew_n : (listed && a.dense_left && a.dense_left[wpar] == 0u) ? 0u : a.nb;
  const uint32_t istride = listed ? kListBatch * gridDim.x : gridDim.x;
  for (uint32_t it = blockIdx.x; it < nwork; it += istride) {
    uint32_t bfirst = kSkew ? a.skew_list[it] : it, nblk = 1, todo = 1u, bstep = 0;
    if (listed) {
      nblk = kListBatch;
      bstep = gridDim.x;
      if (w == 0) {
        const uint32_t bw = it + lane * bstep;
        const uint64_t m = __ballot(lane < kListBatch && bw < a.nb && a.blist[bw] != 0u);
        if (lane == 0) s_todo = (uint32_t)m;
      }
      __syncthreads();
      todo = s_todo;
      __syncthreads();  // (s_todo is rewritten by the next batch)
    }
    for (uint32_t j = 0; j < nblk; ++j) {
    if (!((todo >> j) & 1u)) continue;
    const uint32_t b = bfirst + j * bstep;
    AGX_STAMP(a, 0);
    const uint32_t a0 = b << a.bb;
    const uint32_t na = min(1u << a.bb, P.n_local - a0);
    if (tid < 5) s_stat[tid] = 0;
    if (tid == 0) s_rowtop = 0;
    if (tid == 0) s_flags = 0;
    for (uint32_t d = tid; d < kRadix; d += kBThreads) s_nh[d] = 0;
    uint32_t* my_tc = nullptr;  // (fused) this thread's table entry, zeroed once the bucket is processed
    // fused fast path, plain behaviours: state words 0 / 1 of the bucket's actors are loaded here,
    // beside the table row, so their round trip overlaps the gather instead of following the sort
    // (actors past n_local read actor 0's words; bucket_finish masks actors without mail)
    constexpr bool kEarly = kGather && kDefer && !kWide && kEarlyState;
    // (dense_finish: at most one message per actor; not in the fused superstep, where it measured slower:
    // 1M ring 24.0 -> 25.1 us -- that variant then spills 12 VGPRs)
    constexpr bool kDense = !kWide && !kGather && kDenseBuckets;
    uint64_t ex0[kBAct] = {}, ex1[kBAct] = {};
    uint32_t alive4 = 0;        // alive flags of actors 4*tid..4*tid+3, loaded first (a0 is a multiple of 32)
    {
      const uint32_t la0 = tid * 4;
      // one u32 load, no branch (the flags array is padded to whole buckets); bytes past na masked
      alive4 = *reinterpret_cast<const uint32_t*>(P.alive + a0 + la0);
      if (la0 + 4 > na) alive4 &= la0 >= na ? 0u : 0xFFFFFFFFu >> (8 * (4 - (na - la0)));
    }
    if (!kGather) {
      if (tid == 0) {
        if constexpr (kBypass) {  // inbox = [previous backlog, in place][sorted new mail]
          {
            const uint32_t bs = a.bstart[b], be = a.bstart[b + 1], bp = a.blpre[b] + a.bl_sbase[b / kBlSlice];
            const uint32_t blc = a.chunk_cnt[b], blo = a.chunk_off[b];
            s_g[0] = blc;
            s_g[1] = blo;
            s_g[3] = bs;
            s_lo = bs + bp;
            s_hi = bs + bp + blc + (be - bs);
          }
          if ((uint64_t)s_hi > a.cap) {  // mail + backlog over the message capacity: report, drop
            atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
            s_lo = s_hi = 0u;
          }
        } else {
          s_lo = a.bstart[b];
          s_hi = a.bstart[b + 1];
        }
        s_g[5] = s_hi - s_lo > (uint32_t)kBucket || (kBypass && a.ring_of && a.ring_of[b]);  // (a ring bucket: skew path)
        if (kDefer && s_g[5]) a.skew_list[atomicAdd(skew_n, 1u)] = b;
      }
    } else {
      // fused: this bucket's row of the tell tables (chunk c = sender bucket c), its backlog,
      // its host-staged tells; rows are zeroed once read (the writers only set non-zero entries)
      uint32_t* segp = s_pay;  // segment list (read by the loads; s_pay is rewritten only after a barrier)
      uint32_t* sego = segp + kRadix + 2;
      const uint32_t c = tid;
      uint32_t v = 0, o = 0;
      if (c < a.nb) {  // count and offset in one round trip (the offset is stale when the count is 0)
        uint32_t* tc = g.tcnt[rpar] + (size_t)b * g.tstride + c;
        v = *tc;
        o = g.toff[rpar][(size_t)b * g.tstride + c];
        if (v) my_tc = tc;
      }
      if constexpr (kEarly) {  // (issued after the row: waiting for the row does not wait for these)
        const uint32_t w1off = P.W > 1 ? P.sw : 0u;
#pragma unroll
        for (int j = 0; j < kBAct; ++j) {
          const uint32_t la = j * kBThreads + tid, l = la < na ? a0 + la : 0u;
          ex0[j] = ldg64(P.state, l * P.sa);
          ex1[j] = ldg64(P.state, l * P.sa + w1off);
        }
      }
      if (tid == 0) {  // (the staged count is zeroed once the bucket is processed)
        s_g[0] = g.blc[rpar][b];
        s_g[1] = g.blo[rpar][b];
        s_g[2] = g.stg_cnt[b];
        s_g[3] = g.stg_off[b];
      }
      uint32_t tt, ns;
      const uint2 exix = block_excl_sum2<kBThreads>(v, v ? 1u : 0u, scratch, &tt, &ns);  // (syncs: s_g visible after)
      const uint32_t ex = exix.x, ix = exix.y;
      const uint32_t blc = s_g[0];
      if (v) {
        segp[ix] = blc + ex;
        sego[ix] = o;
      }
      if (tid == 0) {
        segp[ns] = blc + tt;  // staged segment
        s_g[4] = ns;
        const uint32_t cnt = blc + tt + s_g[2];
        s_g[5] = cnt > (uint32_t)kBucket;
        if (kDefer && s_g[5]) {
          a.skew_list[atomicAdd(skew_n, 1u)] = b;
          if (a.abort) a.abort[wpar] = a.slot + 1u;  // strict replay: the rest of it is void
        }
        // inbox slot: the bucket's own region (no shared counter), else the overflow region
        uint64_t lo = (uint64_t)b * g.region;
        if (kDefer && s_g[5]) {
          // deferred to the skew launch, which allocates
        } else if (cnt > g.region) {
          lo = (uint64_t)a.nb * g.region + atomicAdd(&g.ovf[wpar], cnt);
        }
        if (kDefer && s_g[5]) {
        } else if (lo + cnt > g.cap) {  // arena overflow: report, drop this bucket's mail
          atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
          s_lo = 0;
          s_hi = 0;
          g.cntb[(size_t)a.slot * a.nb + b] = 0u;
        } else {
          s_lo = (uint32_t)lo;
          s_hi = (uint32_t)lo + cnt;
          g.cntb[(size_t)a.slot * a.nb + b] = cnt;
        }
      }
    }
    // (kLateAlive: the flags reach LDS after the inbox loads are issued, so the bucket's first
    // barrier does not wait for their round trip; loads return in order, so the store's wait does
    // not wait for the inbox)
    if (!kLateAlive) reinterpret_cast<uint32_t*>(s_alive)[tid] = alive4;
    __syncthreads();
    AGX_STAMP(a, 1);
    const bool big = s_g[5] != 0;
    if (kDefer && big) {  // large inbox: left to the skew-list launch (row kept for it)
      __syncthreads();       // every thread has read s_g before the next bucket rewrites it
      continue;
    }
    if (kGather) {                   // fused: table row and staged tells consumed
      if (my_tc) *my_tc = 0u;
      if (tid == 0 && s_g[2]) g.stg_cnt[b] = 0u;
    }
    const uint32_t lo = s_lo, cnt = s_hi > s_lo ? s_hi - s_lo : 0u;
    // (a ring bucket's rings may hold mail; the plan's record, not ring_of: k_skew_scan may have
    // just returned the slot -- its drained ring messages are still in this superstep's scratch)
    const bool ringb = kBypass && !kWide && kSkew && a.ring_of && a.sk_rec[(size_t)it * kSkRec + 11] != 0u;
    if (cnt == 0 && !ringb) {  // no mail (most buckets of a sparse superstep at 10^7+ actors): write the empty
                     // backlog / tell-chunk entries bucket_finish would write, skip the pipeline
      if (tid == 0) {
        if constexpr (kGather) {
          g.blo[wpar][b] = lo;
          g.blc[wpar][b] = 0u;
        } else {
          a.chunk_off[b] = lo;
          a.chunk_cnt[b] = 0u;
          a.chunk_off[a.nb + b] = (uint32_t)((uint64_t)lo * a.kmax);
          a.chunk_cnt[a.nb + b] = 0u;
        }
        if constexpr (kGather || kOwner)
          if (g.emc[wpar]) g.emc[wpar][b] = 0u;
      }
      __syncthreads();
      continue;
    }
    // bypass: inbox item q < xblc is backlog item q (g.bl[rpar] at xblo + q), else sorted item xbst + q - xblc
    const uint32_t xblc = kBypass ? s_g[0] : 0u, xblo = kBypass ? s_g[1] : 0u, xbst = kBypass ? s_g[3] : lo;
    GatherView gv{};
    if (kGather) {
      gv.segp = s_pay;
      gv.sego = gv.segp + kRadix + 2;
      gv.nseg = s_g[4];
      gv.blc = s_g[0];
      gv.blo = s_g[1];
      gv.sto = s_g[3];
    }

    if constexpr (kDefer) {
      // ---- fast path: the whole bucket in one LDS tile
      uint32_t k[kBIpt], sv[kBIpt], pv[kBIpt], rk[kBIpt];
      const uint32_t wbase = w * (kBIpt * kWave);
      {  // locate every item first (LDS only), then issue all 3 x kBIpt loads back to back: selected
         // base pointers and no branches around the loads (per-item if/else made the compiler wait
         // for each item's loads before the next item's: 8 dependent round trips instead of 1)
        uint32_t sel[kBIpt], idx[kBIpt];
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          const uint32_t q = wbase + r * kWave + lane;
          sel[r] = 0;
          idx[r] = 0;
          if (q < cnt) {
            if (kGather) {
              idx[r] = gv.locate(q, sel[r]);
            } else if (kBypass && q < xblc) {
              idx[r] = xblo + q;
            } else {
              sel[r] = 1;
              idx[r] = iv.at(xbst + q - xblc);
            }
          }
        }
        // base pointers in SGPRs (uniform), so a per-item select is a register move, not a load
        // of the pointer from the kernel-argument block at a per-lane address
        const uint32_t *Bk = nullptr, *Bs = nullptr, *Bp = nullptr, *Ek = nullptr, *Es = nullptr, *Ep = nullptr;
        if (kGather || kBypass) {
          Bk = sgpr_ptr(g.bl[rpar].key);
          Bs = sgpr_ptr(g.bl[rpar].src);
          Bp = sgpr_ptr(g.bl[rpar].pay);
        }
        if (kGather) {
          Ek = sgpr_ptr(g.eg[rpar].key);
          Es = sgpr_ptr(g.eg[rpar].src);
          Ep = sgpr_ptr(g.eg[rpar].pay);
        }
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          const uint32_t *pk, *ps, *pp;
          if (kGather) {
            pk = sel[r] == 0 ? Bk : sel[r] == 1 ? Ek : g.stg.key;
            ps = sel[r] == 0 ? Bs : sel[r] == 1 ? Es : g.stg.src;
            pp = sel[r] == 0 ? Bp : sel[r] == 1 ? Ep : g.stg.pay;
          } else if (kBypass) {
            pk = sel[r] == 0 ? Bk : iv.m.key;
            ps = sel[r] == 0 ? Bs : iv.m.src;
            pp = sel[r] == 0 ? Bp : iv.m.pay;
          } else {
            pk = a.in.key;
            ps = a.in.src;
            pp = a.in.pay;
          }
          k[r] = ldg(pk, idx[r]);
          sv[r] = ldg(ps, idx[r]);
          pv[r] = ldg(pp, idx[r]);
        }
#pragma unroll
        for (int r = 0; r < kBIpt; ++r)
          if (wbase + r * kWave + lane >= cnt) k[r] = 0xFFFFFFFFu;
      }
      if (kLateAlive) reinterpret_cast<uint32_t*>(s_alive)[tid] = alive4;
      __syncthreads();  // (fused) the segment list in s_pay is read before the items overwrite it
      // in-order copy + sortedness check: local topologies (rings, stencils) arrive already in
      // actor order, and then the wave multisplit ranking is unnecessary (same result)
      for (uint32_t i = tid; i < kBucket + 4; i += kBThreads) s_seg[i] = 0;
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) {
        const uint32_t q = wbase + r * kWave + lane;
        if (q < cnt) {
          s_key[q] = k[r];
          s_src[q] = sv[r];
          s_pay[q] = pv[r];
        }
      }
      __syncthreads();
      // (and strictly increasing: at most one message per actor -- the dense path, dense_finish)
      uint32_t bad = 0;
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) {
        const uint32_t q = wbase + r * kWave + lane;
        if (q < cnt && q > 0) {
          const uint32_t p0 = s_key[q - 1] & amask, p1 = k[r] & amask;
          bad |= p0 > p1 ? 3u : p0 == p1 ? 2u : 0u;
        }
      }
      if (bad) atomicOr(&s_flags, bad);
      __syncthreads();
      const uint32_t flags = s_flags;
#ifdef AGX_PRESORT_WGRED  // diagnostic build knob: round 4's ockl workgroup reduction
      const bool presorted = __syncthreads_and(!(bad & 1u)) != 0;
#else
      const bool presorted = !(flags & 1u);
#endif
      if (kDense && !(flags & 2u) && a.kmax == 1) {
        dense_finish<KM, kGather, kOwner>(a, L, b, lo, cnt, a0, wpar, acc, kEarly ? ex0 : nullptr, kEarly ? ex1 : nullptr);
        continue;
      }
      uint32_t tl[kBAct];
      if (presorted) {
        // per-actor counts by LDS atomics (s_seg zeroed before the copy), then the block scan below
        // (same-box A/B, 10^8-actor ring: 1.07 ms vs 1.19 ms with run starts + a lower-bound search)
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          const uint32_t q = wbase + r * kWave + lane;
          if (q < cnt) atomicAdd(&s_seg[k[r] & amask], 1u);
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kBAct; ++j) tl[j] = s_seg[tid * kBAct + j];
      } else {
        for (uint32_t i = tid; i < kBWaves * kBucket / 2; i += kBThreads) reinterpret_cast<uint32_t*>(whist)[i] = 0;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          const uint32_t q = wbase + r * kWave + lane;
          rk[r] = wave_rank(q < cnt, k[r] & amask, a.bb, whist + w * kBucket, ltm);
        }
        __syncthreads();
        // per actor: wave prefixes in place, segment length
#pragma unroll
        for (int j = 0; j < kBAct; ++j) {
          const uint32_t la = tid * kBAct + j;  // blocked (for the scan below)
          uint32_t run = 0;
#pragma unroll
          for (int q = 0; q < kBWaves; ++q) {
            const uint32_t c2 = whist[q * kBucket + la];
            whist[q * kBucket + la] = (uint16_t)run;
            run += c2;
          }
          tl[j] = run;
        }
      }
      {  // segment starts: exclusive scan of per-actor counts (blocked)
        uint32_t run = 0;
#pragma unroll
        for (int j = 0; j < kBAct; ++j) run += tl[j];
        uint32_t t;
        uint32_t ex = block_excl_sum<kBThreads>(run, scratch, &t);
#pragma unroll
        for (int j = 0; j < kBAct; ++j) {
          s_seg[tid * kBAct + j] = ex;
          ex += tl[j];
        }
        if (tid == 0) s_seg[kBucket] = t;
        __syncthreads();
      }
      if (!presorted) {  // stable scatter into actor order (items come from registers)
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          const uint32_t q = wbase + r * kWave + lane;
          if (q < cnt) {
            const uint32_t la = k[r] & amask;
            const uint32_t pos = s_seg[la] + whist[w * kBucket + la] + rk[r];
            s_key[pos] = k[r];
            s_src[pos] = sv[r];
            s_pay[pos] = pv[r];
          }
        }
        __syncthreads();
      }
      AGX_STAMP(a, 2);
      bucket_finish<true, kWide, KM, kGather, kOwner>(a, L, b, lo, cnt, a0, na, wpar, 0u, acc, 0xFFFFFFFFu,
                                                      kEarly ? ex0 : nullptr, kEarly ? ex1 : nullptr);
    } else {
      // ---- general path (skewed bucket, > kBucket messages): admission first, then a stable
      // counting sort of the ADMITTED messages only into the global scratch copy.  Per actor
      // keep = alive ? min(len, C) : 0 (tail-drop: the first `keep` in canonical order are
      // admitted); messages of an actor already at `keep` are dead letters and skip the
      // ranking, so a hot actor of a bounded mailbox costs one key read per arrival.
      auto gkey = [&](uint32_t q) -> uint32_t {
        if (kGather) return gv.key(g, rpar, q);
        if (kBypass && q < xblc) return g.bl[rpar].key[xblo + q];
        return iv.m.key[iv.at(xbst + q - xblc)];
      };
      if constexpr (kBypass && !kWide) {
        // pre-partitioned by k_skew_* (above): the drained messages are in the scratch copy at
        // [lo, lo + ndrain) in actor order, the queued ones already in this superstep's backlog
        const uint32_t* r = a.sk_rec + (size_t)it * kSkRec;
        const uint32_t* act = a.sk_act + (size_t)it * kSkActPlanes * kBucket;
        for (uint32_t la = tid; la < kBucket; la += kBThreads) s_seg[la] = act[kBucket + la];
        if (tid == 0) s_seg[kBucket] = r[8];
        if (kLateAlive) reinterpret_cast<uint32_t*>(s_alive)[tid] = alive4;
        __syncthreads();
        // (r[1]: the bucket's inbox index space, or a ring bucket's drain scratch / tell slice)
        bucket_finish<false, kWide, KM, kGather, kOwner>(a, L, b, r[1], r[8], a0, na, wpar, 0u, acc, r[9]);
        continue;
      }
      uint32_t* s_run = s_key;   // LDS items are unused on this path
      uint32_t* s_tmp = s_src;
      uint32_t* s_keep = s_ecnt;  // (bucket_finish re-initialises ecnt)
      for (uint32_t i = tid; i < kBucket + 4; i += kBThreads) s_seg[i] = 0;
      for (uint32_t la = tid; la < kBucket; la += kBThreads) s_run[la] = 0;
      if (kLateAlive) reinterpret_cast<uint32_t*>(s_alive)[tid] = alive4;
      __syncthreads();
      for (uint32_t q0 = 0; q0 < cnt; q0 += 4 * kBThreads) {  // arrivals per actor (4 loads in flight)
        uint32_t kk[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) kk[j] = q0 + j * kBThreads + tid < cnt ? gkey(q0 + j * kBThreads + tid) : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (q0 + j * kBThreads + tid < cnt) atomicAdd(&s_seg[kk[j] & amask], 1u);
      }
      __syncthreads();
      uint32_t ndead0 = 0;
      {
        uint32_t v[kBAct], run = 0;
#pragma unroll
        for (int j = 0; j < kBAct; ++j) {
          const uint32_t la = tid * kBAct + j;
          const uint32_t len = s_seg[la];
          const uint32_t ab = s_alive[la];
          uint32_t Cc, Tc;
          mbox_limits(P, ab, Cc, Tc);
          const uint32_t keep = !(ab & 1u) ? 0u : ((Cc == 0 || len < Cc) ? len : Cc);
          ndead0 += len - keep;
          v[j] = keep;
          s_keep[la] = keep;
          run += keep;
        }
        uint32_t t;
        uint32_t ex = block_excl_sum<kBThreads>(run, scratch, &t);
#pragma unroll
        for (int j = 0; j < kBAct; ++j) {
          s_seg[tid * kBAct + j] = ex;
          ex += v[j];
        }
        if (tid == 0) s_seg[kBucket] = t;
      }
      __syncthreads();
      const uint32_t cnt2 = s_seg[kBucket];  // admitted messages
      uint32_t kn[kBIpt];  // keys of the next sub-tile, loaded one sub-tile ahead
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) {
        const uint32_t q = w * (kBIpt * kWave) + r * kWave + lane;
        kn[r] = q < cnt ? gkey(q) : 0xFFFFFFFFu;
      }
      for (uint32_t sub = 0; sub < cnt; sub += kBucket) {
        const uint32_t wbase = sub + w * (kBIpt * kWave);
        uint32_t k[kBIpt], sv[kBIpt], pv[kBIpt], rk[kBIpt];
        bool live[kBIpt];
        int any = 0;
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          k[r] = kn[r];
          const uint32_t q = wbase + r * kWave + lane;
          const uint32_t la = k[r] & amask;
          live[r] = q < cnt && s_run[la] < s_keep[la];  // actor not yet full: rank it
          any |= live[r];
        }
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          const uint32_t q = wbase + kBucket + r * kWave + lane;
          kn[r] = q < cnt ? gkey(q) : 0xFFFFFFFFu;
        }
        // every arrival of this sub-tile goes to an actor already at `keep`: all dead letters
        if (!__syncthreads_or(any)) continue;
        for (uint32_t i = tid; i < kBWaves * kBucket / 2; i += kBThreads) reinterpret_cast<uint32_t*>(whist)[i] = 0;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          const uint32_t q = wbase + r * kWave + lane;
          if (live[r]) {
            if (kGather) {
              uint32_t k2;
              gv.load(g, rpar, q, k2, sv[r], pv[r]);
            } else if (kBypass && q < xblc) {
              sv[r] = g.bl[rpar].src[xblo + q];
              pv[r] = g.bl[rpar].pay[xblo + q];
            } else {
              const uint32_t x = iv.at(xbst + q - xblc);
              sv[r] = iv.m.src[x];
              pv[r] = iv.m.pay[x];
            }
          }
        }
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) rk[r] = wave_rank(live[r], k[r] & amask, a.bb, whist + w * kBucket, ltm);
        __syncthreads();
        for (uint32_t la = tid; la < kBucket; la += kBThreads) {
          uint32_t run = 0;
#pragma unroll
          for (int q = 0; q < kBWaves; ++q) {
            const uint32_t c2 = whist[q * kBucket + la];
            whist[q * kBucket + la] = (uint16_t)run;
            run += c2;
          }
          s_tmp[la] = run;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          if (!live[r]) continue;
          const uint32_t la = k[r] & amask;
          const uint32_t rank = s_run[la] + whist[w * kBucket + la] + rk[r];  // among this actor's arrivals
          if (rank < s_keep[la]) {
            const uint32_t pos = lo + s_seg[la] + rank;
            a.scr.key[pos] = k[r];
            a.scr.src[pos] = sv[r];
            a.scr.pay[pos] = pv[r];
          }
        }
        __syncthreads();
        for (uint32_t la = tid; la < kBucket; la += kBThreads) s_run[la] += s_tmp[la];
        __syncthreads();
      }
      // the scratch copy holds the admitted messages in actor order; dead letters counted here
      __threadfence_block();
      bucket_finish<false, kWide, KM, kGather, kOwner>(a, L, b, lo, cnt2, a0, na, wpar, ndead0, acc);
    }
    }  // buckets of the batch (one unless listed)
  }
  if (!kOwner && !(kGather && kSkew) && blockIdx.x < nwork) flush_stats(a, acc);  // (block-uniform)
}

// Bucket starts after a multi-pass sort: bstart[x] = first index with bucket >= x
// (one thread per bucket, binary search over the sorted keys; the top levels of every
// search hit the same cached lines).
// Identity grouping (ident[0] != 0): the same search over the previous apply's tell arena in place,
// sorted item i at (i + ident[1]) mod ident[2].
static __global__ void __launch_bounds__(kThreads) k_bucket_bounds(const uint32_t* key, const uint32_t* d_n, uint32_t nb,
                                                            uint32_t bb, uint32_t* bstart, const uint32_t* ident,
                                                            const uint32_t* key_alt, const uint32_t* halt) {
  if (halt && halt[0]) return;  // (device-resident multi-rank replay stopped: k_mr_pack)
  const bool idn = ident && ident[0];
  const uint32_t n = idn ? ident[2] : *d_n, rot = idn ? ident[1] : 0u;
  const uint32_t* k = idn ? key_alt : key;
  // (one thread per bucket start: measured faster than 8- or 64-lane k-ary searches per start,
  // 21.6 vs 25.0 / 43.3 us at 10^8 -- the shared top levels of the binary searches stay cached)
  for (uint32_t x = blockIdx.x * kThreads + threadIdx.x; x <= nb; x += gridDim.x * kThreads) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint32_t j = mid + rot;
      if (((k[j >= n ? j - n : j] & kLocalMask) >> bb) < x) lo = mid + 1; else hi = mid;
    }
    bstart[x] = lo;
  }
}

// Sum the per-block counters of k_bucket_apply into out[0..kBStats).
static __global__ void __launch_bounds__(kScanThreads) k_stats_reduce(const unsigned long long* bstats, uint32_t nslots,
                                                               unsigned long long* out) {
  __shared__ unsigned long long s[kBStats];
  if (threadIdx.x < kBStats) s[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long v[kBStats] = {0, 0, 0, 0, 0};
  for (uint32_t i = threadIdx.x; i < nslots; i += blockDim.x)
#pragma unroll
    for (int k = 0; k < kBStats; ++k) v[k] += bstats[(size_t)i * kBStats + k];
#pragma unroll
  for (int k = 0; k < kBStats; ++k) atomicAdd(&s[k], v[k]);
  __syncthreads();
  if (threadIdx.x < kBStats) out[threadIdx.x] = s[threadIdx.x];
}

// Histogram columns of the host-staged chunks (one block per staged chunk).
static __global__ void __launch_bounds__(kThreads) k_chunk_hist(const uint32_t* key, uint32_t n, uint32_t* hist,
                                                         uint32_t stride, uint32_t col0, uint32_t shift, uint32_t bits,
                                                         uint32_t* chunk_off, uint32_t* chunk_cnt, uint32_t chunk0) {
  __shared__ uint32_t h[kRadix];
  const uint32_t mask = (1u << bits) - 1u;
  const uint32_t per = div_up(n, kStagedChunks);
  const uint32_t c = blockIdx.x;
  const uint32_t b0 = min(n, c * per), b1 = min(n, b0 + per);
  for (uint32_t d = threadIdx.x; d < kRadix; d += kThreads) h[d] = 0;
  __syncthreads();
  for (uint32_t i = b0 + threadIdx.x; i < b1; i += kThreads) atomicAdd(&h[((key[i] & kLocalMask) >> shift) & mask], 1u);
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < (1u << bits); d += kThreads)
    if (h[d]) hist[(size_t)d * stride + col0 + c] = h[d];
  if (threadIdx.x == 0) {
    chunk_off[chunk0 + c] = b0;
    chunk_cnt[chunk0 + c] = b1 - b0;
  }
}

// =========================================================================
// Multi-GPU helpers.  The apply left, per bucket b: its backlog chunk (bl arena) and its
// tells grouped by owner rank q in eg at toff[q][b] (tcnt[q][b] of them, sender order).
// Send buffer s2 = owner-major: for q, for b in order, bucket b's run for q — the stable
// owner partition of the tells in chunk order.  Backlog chunks go to the front of A.
// =========================================================================
struct McompactArgs {
  Chunks ch;
  CMsgs eg;           // owner-grouped tells
  uint32_t* tcnt;     // [R][tstride] run lengths (zeroed by the copy)
  const uint32_t* toff;
  Msgs out0, out1;
  uint32_t* off0;     // [nb] destination offsets of backlog chunks
  uint32_t* off1;     // [R][tstride] destination offsets of the owner runs in s2
  uint32_t* d_total;  // [0] backlog total, [1] tell total
  uint64_t* cvec;     // [R send counts..., backlog, staged]
  uint8_t* alive;
  const uint32_t* stopq;
  uint32_t* nstop;
  uint64_t* stats;
  uint32_t* step;
  uint32_t* heap_top;
  uint32_t* skew_n;
  uint64_t cap0, cap1;
  uint32_t R, tstride, n_staged;
  const uint32_t* halt;  // device-resident replays: [0] != 0 = stopped (k_mr_pack), every kernel returns
  uint32_t* dense_left;  // owner mode's one dense_left word (BucketArgs::dense_left[0]): cleared here, before
                         // this superstep's dense launch raises it for a bucket it leaves to the block launch
  // device-resident replays of plain behaviours: the runs for peer q go straight into q's send slab
  // ([slab][3] triples at the run's position within q's owner-major region); what does not fit the slab
  // goes to s2 at its owner-major offset (read only by the exact fallback, after k_slab_to_s2).  Null:
  // every run to s2 (host-planned exchange, CRDT rows beside the tells, loopback groups).
  uint32_t* sslab;
  uint32_t slab, rank;
};

static __global__ void __launch_bounds__(kScanThreads) k_mcompact_scan(McompactArgs a) {
  __shared__ uint32_t scratch[kScanThreads / kWave + 1];
  __shared__ uint32_t s_obase[AGX_MAX_RANKS + 1];
  if (a.halt && a.halt[0]) return;
  begin_step(a.step, a.heap_top);
  commit_stops(a.alive, a.stopq, a.nstop);
  if (threadIdx.x == 0) *a.skew_n = 0u;
  if (threadIdx.x == 0 && a.dense_left) a.dense_left[0] = 0u;
  const uint64_t nbl = block_scan_table<kScanThreads>(a.ch.cnt, a.off0, 1, a.ch.nb, a.ch.nb, scratch, nullptr);
  const uint64_t ntl = block_scan_table<kScanThreads>(a.tcnt, a.off1, a.R, a.ch.nb, a.tstride, scratch, s_obase);
  const uint32_t tid = threadIdx.x;
  const bool over = nbl > a.cap0 || ntl > a.cap1;
  if (tid == 0) {
    if (over) atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
    a.d_total[0] = over ? 0u : (uint32_t)nbl;
    a.d_total[1] = over ? 0u : (uint32_t)ntl;
    a.cvec[a.R] = over ? 0u : nbl;  // backlog kept locally
    a.cvec[a.R + 1] = a.n_staged;
  }
  if (tid < a.R) a.cvec[tid] = over ? 0u : (uint64_t)(s_obase[tid + 1] - s_obase[tid]);
}

// block-wide copy of n envelopes, four per thread in flight
__device__ __forceinline__ void copy_run(const CMsgs& s, uint32_t so, const Msgs& d, uint32_t dof, uint32_t n) {
  constexpr uint32_t U = 4;
  for (uint32_t i0 = 0; i0 < n; i0 += U * kThreads) {
    uint32_t k[U], sv[U], pv[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * kThreads + threadIdx.x;
      if (i < n) {
        k[u] = s.key[so + i];
        sv[u] = s.src[so + i];
        pv[u] = s.pay[so + i];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * kThreads + threadIdx.x;
      if (i < n) {
        d.key[dof + i] = k[u];
        d.src[dof + i] = sv[u];
        d.pay[dof + i] = pv[u];
      }
    }
  }
}

// block-wide copy of n envelopes into a peer's send slab (AoS triples from slot j0); slots past the slab
// go to `over` at dof + i instead (the exact fallback's source)
__device__ __forceinline__ void copy_run_slab(const CMsgs& s, uint32_t so, uint32_t* slabq, uint32_t j0, uint32_t slab,
                                              const Msgs& over, uint32_t dof, uint32_t n) {
  constexpr uint32_t U = 4;
  for (uint32_t i0 = 0; i0 < n; i0 += U * kThreads) {
    uint32_t k[U], sv[U], pv[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * kThreads + threadIdx.x;
      if (i < n) {
        k[u] = s.key[so + i];
        sv[u] = s.src[so + i];
        pv[u] = s.pay[so + i];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + u * kThreads + threadIdx.x;
      if (i >= n) continue;
      const uint32_t j = j0 + i;
      if (j < slab) {
        slabq[3 * (size_t)j] = k[u];
        slabq[3 * (size_t)j + 1] = sv[u];
        slabq[3 * (size_t)j + 2] = pv[u];
      } else {
        over.key[dof + i] = k[u];
        over.src[dof + i] = sv[u];
        over.pay[dof + i] = pv[u];
      }
    }
  }
}

static __global__ void __launch_bounds__(kThreads) k_mcompact_copy(McompactArgs a) {
  __shared__ uint32_t s_soff[AGX_MAX_RANKS];  // (direct slabs) start of each owner's region in s2
  if (a.halt && a.halt[0]) return;
  const bool go = a.d_total[0] != 0 || a.d_total[1] != 0;
  if (a.sslab && threadIdx.x == 0) {
    uint32_t o = 0;
    for (uint32_t q = 0; q < a.R; ++q) {
      s_soff[q] = o;
      o += (uint32_t)a.cvec[q];
    }
  }
  __syncthreads();
  for (uint32_t c = blockIdx.x; c < a.ch.nb; c += gridDim.x) {
    const uint32_t n = a.ch.cnt[c];
    if (go && n) {  // backlog chunk c -> front of the sort input
      copy_run(a.ch.bl, a.ch.off[c], a.out0, a.off0[c], n);
    }
    for (uint32_t q = 0; q < a.R; ++q) {  // bucket c's run for owner q -> s2
      const size_t x = (size_t)q * a.tstride + c;
      const uint32_t m = a.tcnt[x];
      if (!m) continue;
      const uint32_t so = a.toff[x], dof = a.off1[x];
      if (go) {
        if (a.sslab && q != a.rank)
          copy_run_slab(a.eg, so, a.sslab + (size_t)q * a.slab * 3, dof - s_soff[q], a.slab, a.out1, dof, m);
        else
          copy_run(a.eg, so, a.out1, dof, m);
      }
      __syncthreads();  // every thread has read the count before it is cleared
      if (threadIdx.x == 0) a.tcnt[x] = 0u;  // the apply writes non-zero entries only
    }
  }
}

// ---- Device-resident multi-rank supersteps (RCCL, plain behaviours).  The host-driven superstep
// copies the all-gathered count matrix to the host, plans the exchange and posts one exactly sized
// send / recv per peer.  Here the exchange moves fixed per-peer slabs of `slab` envelopes instead,
// so a replay of supersteps needs no host round trip: every rank reads the same all-gathered
// matrix cmat[R][R + 2] (send counts..., backlog, staged) on the device and takes the same decision
// -- halt[0] = 1 when some sender -> receiver count exceeds the slab (the host then redoes this
// superstep's exchange exactly and grows the slabs), 2 when nothing is in flight (quiescent), 3 when
// the inbox would exceed the capacity; halt[1] = the replay superstep that stopped.  Every later
// kernel of the replay returns at entry (the sends / receives still move their slabs, unread).
// Received runs land after the local backlog in sender-rank order -- the sharded canonical order
// of the host path.
struct MrArgs {
  const uint64_t* cmat;
  CMsgs s2;               // owner-major tells (k_mcompact_copy)
  uint32_t* sslab;        // [R][slab][3] (key, src, payload) per peer
  const uint32_t* rslab;  // [R][slab][3]
  Msgs A;                 // the sort input: [backlog][received runs, sender-rank order]
  uint32_t* d_n;
  uint32_t* halt;
  uint64_t* stats;
  uint64_t cap;
  uint32_t R, rank, slab, step;
  // CRDT rows (pw > 0): row i of s2rows belongs to tell i of s2 (k_pack_rows); a state gossip to
  // peer q travels as row i of srows[q] beside its envelope, and lands in rx[sender][i]
  const uint32_t* s2rows;
  uint32_t* srows;        // [R][slab][pw]
  uint32_t pw, heap_rows;
  uint32_t direct;        // k_mcompact_copy already wrote the peers' runs into their send slabs
};

// the plan every block derives from cmat: own send offsets, receive offsets, counts, the decision
// (code 0 = go, 1 = a count over the slab, 2 = quiescent, 3 = over capacity).  Host and device:
// the C ABI exports the same function (agx_mr_plan) so the decision is testable without a GPU.
struct MrPlan {
  uint32_t soff[AGX_MAX_RANKS + 1], scnt[AGX_MAX_RANKS], roff[AGX_MAX_RANKS + 1], rcnt[AGX_MAX_RANKS];
  uint32_t nbl, code;
};
__host__ __device__ inline void mr_decide(const uint64_t* cmat, uint32_t R, uint32_t rank, uint32_t slab, uint64_t cap,
                                          MrPlan& p) {
  const uint32_t S = R + 2;
  unsigned long long tot = 0;
  bool over = false;
  for (uint32_t r = 0; r < R; ++r)
    for (uint32_t c = 0; c < S; ++c) {
      const unsigned long long v = cmat[r * S + c];
      tot += v;
      if (c < R && c != r && v > slab) over = true;
    }
  p.nbl = (uint32_t)cmat[rank * S + R];
  uint32_t so = 0, ro = 0;
  for (uint32_t q = 0; q < R; ++q) {
    p.scnt[q] = (uint32_t)cmat[rank * S + q];
    p.soff[q] = so;
    so += p.scnt[q];
    p.rcnt[q] = (uint32_t)cmat[q * S + rank];
    p.roff[q] = ro;
    ro += p.rcnt[q];
  }
  p.soff[R] = so;
  p.roff[R] = ro;
  p.code = tot == 0 ? 2u : over ? 1u : (unsigned long long)p.nbl + ro > cap ? 3u : 0u;
}
__device__ __forceinline__ void mr_plan(const MrArgs& a, MrPlan& p) {
  if (threadIdx.x == 0) mr_decide(a.cmat, a.R, a.rank, a.slab, a.cap, p);
  __syncthreads();
}

// the decision, then this rank's owner-major runs -> the send slabs
static __global__ void __launch_bounds__(kThreads) k_mr_pack(MrArgs a) {
  __shared__ MrPlan p;
  if (a.halt[0]) return;
  mr_plan(a, p);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (p.code) {
      a.halt[0] = p.code;
      a.halt[1] = a.step;
      if (p.code == 3u) atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
    } else {
      *a.d_n = p.nbl + p.roff[a.R];
    }
  }
  if (p.code) return;
  {  // own run: straight from the send buffer to its place after the backlog (no slab, no wait
     // for the exchange)
    const uint32_t x0 = p.soff[a.rank], o0 = p.nbl + p.roff[a.rank];
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < p.scnt[a.rank]; i += gridDim.x * kThreads) {
      a.A.key[o0 + i] = a.s2.key[x0 + i];
      a.A.src[o0 + i] = a.s2.src[x0 + i];
      a.A.pay[o0 + i] = a.s2.pay[x0 + i];
    }
  }
  for (uint32_t q = 0; q < a.R && !a.direct; ++q) {
    if (q == a.rank) continue;
    uint32_t* d = a.sslab + (size_t)q * a.slab * 3;
    const uint32_t o = p.soff[q];
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < p.scnt[q]; i += gridDim.x * kThreads) {
      d[3 * i] = a.s2.key[o + i];
      d[3 * i + 1] = a.s2.src[o + i];
      d[3 * i + 2] = a.s2.pay[o + i];
    }
  }
  if (!a.pw) return;
  // state gossips' rows -> the row slabs (a wave copies its lanes' rows one after the other)
  const uint32_t lane = lane_id();
  for (uint32_t q = 0; q < a.R; ++q) {
    if (q == a.rank) continue;
    const uint32_t o = p.soff[q], n = p.scnt[q];
    for (uint32_t ib = blockIdx.x * kThreads + threadIdx.x - lane; ib < n; ib += gridDim.x * kThreads) {
      const uint32_t i = ib + lane;
      for (uint64_t mm = __ballot(i < n && is_wide(a.s2.src[o + i])); mm; mm &= mm - 1) {
        const uint32_t j = ib + (uint32_t)__builtin_ctzll(mm);
        const uint4* sr = reinterpret_cast<const uint4*>(a.s2rows + (size_t)(o + j) * a.pw);
        uint4* dr = reinterpret_cast<uint4*>(a.srows + ((size_t)q * a.slab + j) * a.pw);
        for (uint32_t k2 = lane; k2 < a.pw / 4; k2 += kWave) dr[k2] = sr[k2];
      }
    }
  }
}

// exact fallback of a superstep whose peer runs went straight into the send slabs (a count over the
// slab): the slab parts back into s2's owner-major regions, so the host-planned exchange sends s2 whole
// (the parts past the slab are there already)
static __global__ void __launch_bounds__(kThreads) k_slab_to_s2(const uint64_t* cmat, const uint32_t* sslab, Msgs s2,
                                                               uint32_t R, uint32_t rank, uint32_t slab) {
  const uint32_t S = R + 2;
  uint32_t o = 0;
  for (uint32_t q = 0; q < R; ++q) {
    const uint32_t n = (uint32_t)cmat[rank * S + q];
    if (q != rank) {
      const uint32_t* d = sslab + (size_t)q * slab * 3;
      for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < min(n, slab); i += gridDim.x * kThreads) {
        s2.key[o + i] = d[3 * (size_t)i];
        s2.src[o + i] = d[3 * (size_t)i + 1];
        s2.pay[o + i] = d[3 * (size_t)i + 2];
      }
    }
    o += n;
  }
}

// received slabs (and the own run) -> A after the backlog, sender-rank order
static __global__ void __launch_bounds__(kThreads) k_mr_unpack(MrArgs a) {
  __shared__ MrPlan p;
  if (a.halt[0]) return;
  mr_plan(a, p);
  if (p.code) return;
  const uint32_t n = p.roff[a.R];
  for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
    uint32_t r = 0;
    while (i >= p.roff[r + 1]) ++r;
    if (r == a.rank) continue;  // (own run: placed by k_mr_pack)
    const uint32_t j = i - p.roff[r], o = p.nbl + i;
    const uint32_t* s = a.rslab + ((size_t)r * a.slab + j) * 3;
    a.A.key[o] = s[0];
    a.A.src[o] = s[1];
    // a state gossip's row arrived in rx[r][j]: its handle points there
    a.A.pay[o] = a.pw && is_wide(s[1]) ? (s[2] & ~kHandleMask) | (a.heap_rows + r * a.slab + j) : s[2];
  }
}

// ORSet-only full-state populations: the state effects of every replica run the apply listed
// (orset_protocol did its tells and snapshot-row allocation): one wave per replica, lane = element
// (orset_merge_wave).  A separate, lean kernel: far more waves in flight than the apply's 4 per
// SIMD to cover the replica's state / row round trips.
static __global__ void __launch_bounds__(kThreads) k_orset_merge(DevParams P, const uint4* orw, const uint2* orm,
                                                             const uint32_t* orw_n) {
  const uint32_t n = orw_n[0];
  const CrdtHeap H = crdt_heap(P);
  const uint32_t nw = gridDim.x * (kThreads / kWave);
  for (uint32_t it = blockIdx.x * (kThreads / kWave) + threadIdx.x / kWave; it < n; it += nw) {
    const uint4 w = orw[it];
    const uint2* msg = orm + w.z;
    orset_merge_wave(P, H, w.x, w.y & 0xFFu, 0u, w.y >> 8, w.w, [&](uint32_t q) { return msg[q].x; },
                     [&](uint32_t q) { return msg[q].y; });
  }
}

// messages in flight after the last apply = all chunk counts (+ the bounded-mailbox rings)
static __global__ void __launch_bounds__(kScanThreads) k_inflight(const uint32_t* chunk_cnt, uint32_t nchunks,
                                                           unsigned long long* out,
                                                           const unsigned long long* ring_total) {
  __shared__ unsigned long long s;
  if (threadIdx.x == 0) s = ring_total ? *ring_total : 0ull;  // (+ messages queued in rings)
  __syncthreads();
  unsigned long long v = 0;
  for (uint32_t i = threadIdx.x; i < nchunks; i += blockDim.x) v += chunk_cnt[i];
  atomicAdd(&s, v);
  __syncthreads();
  if (threadIdx.x == 0) *out = s;
}

// Workload setup: R-MAT destinations of the local rows' out-edges (workloads.rmat_cols).
__device__ __forceinline__ uint32_t rmat_dst(uint64_t e, uint32_t bits, uint32_t ta, uint32_t tb, uint32_t tc,
                                             uint64_t seed, uint32_t n) {
  uint64_t col = 0;
  for (uint32_t bit = 0; bit < bits; ++bit) {
    const uint32_t q = (uint32_t)(splitmix64(e * 64ull + bit + seed) & 0xFFFFull);
    const uint64_t db = ((q >= ta && q < tb) || q >= tc) ? 1ull : 0ull;
    col |= db << (bits - 1 - bit);
  }
  return (uint32_t)(col % n);
}

static __global__ void __launch_bounds__(kThreads) k_gen_rmat(const uint64_t* lrow, const uint64_t* gstart, uint32_t* col,
                                                       uint32_t n_local, uint32_t bits, uint32_t ta, uint32_t tb,
                                                       uint32_t tc, uint64_t seed, uint32_t n_global) {
  for (uint32_t l = blockIdx.x * kThreads + threadIdx.x; l < n_local; l += gridDim.x * kThreads) {
    const uint64_t b = lrow[l], deg = lrow[l + 1] - b, g0 = gstart[l];
    for (uint64_t j = 0; j < deg; ++j) col[b + j] = rmat_dst(g0 + j, bits, ta, tb, tc, seed, n_global);
  }
}

// End of a fused superstep graph: the replay's per-superstep inbox sizes (and strict abort marks)
// into ring slot (*ctr % 4) of the device-mapped pinned host ring -- one block, so the counter it
// reads and bumps is never raced.  The host knows the slot of every replay (same counter).
// Row layout: [inbox sizes][abort marks x2][the error word, lo / hi] (kRingTail words after the rows):
// the host reads the run's error word from the last replay's row instead of copying it back.
constexpr uint32_t kRingTail = 4;
static __global__ void __launch_bounds__(kScanThreads) k_replay_out(const uint32_t* cntb, uint32_t n, const uint32_t* abort,
                                                            const unsigned long long* err, uint32_t* ring, uint32_t* ctr,
                                                            uint32_t stride) {
  const uint32_t c = *ctr;
  uint32_t* dst = ring + (size_t)(c % 4u) * stride;
  for (uint32_t i = threadIdx.x; i < n; i += kScanThreads) dst[i] = cntb[i];
  if (threadIdx.x < 2) dst[stride - kRingTail + threadIdx.x] = abort ? abort[threadIdx.x] : 0u;
  if (threadIdx.x == 2) {
    const unsigned long long v = *err;
    dst[stride - 2] = (uint32_t)v;
    dst[stride - 1] = (uint32_t)(v >> 32);
  }
  __syncthreads();
  if (threadIdx.x == 0) *ctr = c + 1u;
}

// Multi-rank exchange: the owner-major tells (SoA) interleaved as (key, src, payload) triples, so
// each peer's run is ONE contiguous ncclSend instead of three; and back to SoA after the receive.
static __global__ void __launch_bounds__(kThreads) k_pack_aos(CMsgs s, const uint32_t* d_total, uint32_t* out) {
  const uint32_t n = d_total[1];
  for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
    const uint32_t k = s.key[i], sv = s.src[i], pv = s.pay[i];
    out[3 * (size_t)i] = k;
    out[3 * (size_t)i + 1] = sv;
    out[3 * (size_t)i + 2] = pv;
  }
}
static __global__ void __launch_bounds__(kThreads) k_unpack_aos(const uint32_t* in, uint32_t n, Msgs d, uint32_t dof) {
  for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
    const uint32_t k = in[3 * (size_t)i], sv = in[3 * (size_t)i + 1], pv = in[3 * (size_t)i + 2];
    d.key[dof + i] = k;
    d.src[dof + i] = sv;
    d.pay[dof + i] = pv;
  }
}

static __global__ void k_set_u32(uint32_t* p, uint32_t v) {
  if (threadIdx.x == 0) *p = v;
}

// fused mode: messages in flight after the last superstep = its backlog + tells + staged
static __global__ void __launch_bounds__(kScanThreads) k_inflight_fused(const uint32_t* blc0, const uint32_t* blc1,
                                                                 const uint32_t* emc0, const uint32_t* emc1,
                                                                 const uint32_t* stg_cnt, uint32_t last_par,
                                                                 uint32_t nb, unsigned long long* out) {
  __shared__ unsigned long long s;
  const bool p1 = last_par != 0;  // parity written by the last superstep
  const uint32_t* blc = p1 ? blc1 : blc0;
  const uint32_t* emc = p1 ? emc1 : emc0;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  unsigned long long v = 0;
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) v += (unsigned long long)blc[i] + emc[i] + stg_cnt[i];
  atomicAdd(&s, v);
  __syncthreads();
  if (threadIdx.x == 0) *out = s;
}

}  // namespace agx

namespace agx {

// Multi-rank CRDT rows.  After the owner partition, the rows of state gossips that
// leave this rank are packed in the order of the partitioned tells (row i <-> tell i);
// they travel beside the envelopes and land in `rx` at the receiver's sort-input index.
static __global__ void __launch_bounds__(kThreads) k_pack_rows(CMsgs s2, const uint32_t* d_total, DevParams P,
                                                        uint32_t* out) {
  const uint32_t n = d_total[1];
  const CrdtHeap H = crdt_heap(P);
  const uint32_t lane = lane_id();
  // (wave-uniform trips: each wave copies its lanes' rows one after the other, 16 B per lane)
  for (uint32_t ib = blockIdx.x * kThreads + threadIdx.x - lane; ib < n; ib += gridDim.x * kThreads) {
    const uint32_t i = ib + lane;
    const bool need = i < n && is_wide(s2.src[i]) && (s2.key[i] >> kOwnerShift) != P.rank;
    const uint32_t src = need ? s2.pay[i] & kHandleMask : 0u;
    if (H.pw < kWaveRowU32) {  // short rows: one per lane
      if (need) {
        const uint4* s = reinterpret_cast<const uint4*>(H.row(src));
        uint4* d = reinterpret_cast<uint4*>(out + (size_t)i * H.pw);
        for (uint32_t k2 = 0; k2 < H.pw / 4; ++k2) d[k2] = s[k2];
      }
      continue;
    }
    for (uint64_t mm = __ballot(need); mm; mm &= mm - 1) {
      const int j = __builtin_ctzll(mm);
      const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)src, j);
      const uint4* s = reinterpret_cast<const uint4*>(H.row(sj));
      uint4* d = reinterpret_cast<uint4*>(out + (size_t)(ib + (uint32_t)j) * H.pw);
      for (uint32_t k2 = lane; k2 < H.pw / 4; k2 += kWave) d[k2] = s[k2];
    }
  }
}

// Received gossips from other ranks [lo, hi) minus this rank's own segment: point
// their handles at the rx rows (handle = heap_rows + sort-input index).
static __global__ void __launch_bounds__(kThreads) k_fix_rx(Msgs a, uint32_t lo, uint32_t hi, uint32_t self_lo,
                                                     uint32_t self_hi, uint32_t heap_rows) {
  for (uint32_t i = lo + blockIdx.x * kThreads + threadIdx.x; i < hi; i += gridDim.x * kThreads)
    if ((i < self_lo || i >= self_hi) && is_wide(a.src[i])) a.pay[i] = (a.pay[i] & ~kHandleMask) | (heap_rows + i);
}

}  // namespace agx

#include "agx_ring.h"
