// agx_kernels.h — the superstep kernels (gfx950, wave64, integer only).
//
// One BSP superstep replaces one round of Mailbox.run/processMailbox over
// every scheduled mailbox (akka-actor/src/main/scala/akka/dispatch/Mailbox.scala:227-277):
//
//   k_compact_scan / k_compact_copy   scan-compacted emission: per-tile backlog
//                                     and emission chunks -> one dense array
//                                     (backlog first, then tells in sender order)
//   k_sort_upsweep / k_sort_rowscan / k_sort_downsweep
//                                     LDS-staged stable LSD radix sort of the
//                                     envelopes by destination ActorRef
//                                     (Mailbox.enqueue into per-actor FIFOs)
//   k_apply                           segmented mailbox drain (throughput cap,
//                                     bounded tail-drop, dead letters) +
//                                     behaviour-apply + tell emission
//
// Envelopes are SoA u32 {key, src, payload} = 12 B.
#pragma once
#include "agx_device.h"

namespace agx {

// ---------------------------------------------------------------- geometry
constexpr int kApplyThreads = 256;
constexpr int kApplyIpt = 8;
constexpr int kApplyTile = kApplyThreads * kApplyIpt;  // 2048 envelopes

constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / kWave;
constexpr int kSortIpt = 16;
constexpr int kSortTile = kSortThreads * kSortIpt;  // 4096 envelopes
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;

constexpr int kScanThreads = 1024;

// stats slots (u64) on device
enum { ST_DELIVERED = 0, ST_DEAD = 1, ST_UNHANDLED = 2, ST_EMITTED = 3, ST_STEPS = 4, ST_ERROR = 5, ST_ACTIVE = 6, ST_N = 8 };
constexpr uint64_t kErrCapacity = 1;

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

// =========================================================================
// Compaction: chunk list = [bl chunk 0..nt) [em chunk 0..nt) [staged]
//   mode 0 (single rank): all chunks -> stream 0 (sort input), in that order
//   mode 1 (multi rank):  bl -> stream 0 (sort input), em -> stream 1 (send buffer),
//                         staged handled by the host after the exchange
// =========================================================================
// Commit Behaviors.stopped results of the previous apply: alive[l] = 0.
// (k_apply never writes `alive`, so every tile classifies against the
// alive-at-step-start value — deterministic across tile schedules.)
__device__ __forceinline__ void commit_stops(uint8_t* alive, const uint32_t* stopq, uint32_t* nstop) {
  const uint32_t ns = *nstop;
  for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) alive[stopq[i]] = 0;
  __syncthreads();
  if (threadIdx.x == 0) *nstop = 0;
}
__global__ void __launch_bounds__(kScanThreads) k_commit_stops(uint8_t* alive, const uint32_t* stopq, uint32_t* nstop) {
  commit_stops(alive, stopq, nstop);
}

struct CompactArgs {
  uint8_t* alive;
  const uint32_t* stopq;
  uint32_t* nstop;
  uint32_t* d_bump;    // emission bump allocator, reset here for the next apply
  const uint32_t* cnt_bl;
  const uint32_t* cnt_em;
  uint32_t* off_bl;
  uint32_t* off_em;
  uint32_t* d_n;       // in: sorted count of the step that produced the chunks; out: stream-0 total (mode 0)
  uint32_t* d_total;   // [0] stream-0 total, [1] stream-1 total, [2] nt used
  uint64_t* stats;
  uint32_t n_staged;
  uint32_t mode;
  uint64_t cap0, cap1;
};

__global__ void __launch_bounds__(kScanThreads) k_compact_scan(CompactArgs a) {
  __shared__ uint32_t scratch[kScanThreads / kWave + 1];
  __shared__ uint32_t s_nt;
  __shared__ uint64_t s_run0, s_run1;
  const int tid = threadIdx.x;
  commit_stops(a.alive, a.stopq, a.nstop);
  if (tid == 0) {
    s_nt = div_up(*a.d_n, kApplyTile);
    s_run0 = 0;
    s_run1 = 0;
  }
  __syncthreads();
  const uint32_t nt = s_nt;
  // backlog chunks: stream 0
  for (uint32_t base = 0; base < nt; base += kScanThreads) {
    uint32_t i = base + tid;
    uint32_t v = i < nt ? a.cnt_bl[i] : 0u, tot;
    uint32_t ex = block_excl_sum<kScanThreads>(v, scratch, &tot);
    if (i < nt) a.off_bl[i] = (uint32_t)(s_run0 + ex);
    __syncthreads();
    if (tid == 0) s_run0 += tot;
    __syncthreads();
  }
  // emission chunks: stream 0 (mode 0) or stream 1 (mode 1)
  for (uint32_t base = 0; base < nt; base += kScanThreads) {
    uint32_t i = base + tid;
    uint32_t v = i < nt ? a.cnt_em[i] : 0u, tot;
    uint32_t ex = block_excl_sum<kScanThreads>(v, scratch, &tot);
    uint64_t run = a.mode == 0 ? s_run0 : s_run1;
    if (i < nt) a.off_em[i] = (uint32_t)(run + ex);
    __syncthreads();
    if (tid == 0) {
      if (a.mode == 0) s_run0 += tot; else s_run1 += tot;
    }
    __syncthreads();
  }
  if (tid == 0) {
    uint64_t t0 = s_run0, t1 = s_run1;
    if (a.mode == 0) t0 += a.n_staged;
    bool over = t0 > a.cap0 || t1 > a.cap1;
    if (over) atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
    a.d_total[0] = over ? 0u : (uint32_t)t0;
    a.d_total[1] = over ? 0u : (uint32_t)t1;
    a.d_total[2] = nt;
    if (a.mode == 0) *a.d_n = over ? 0u : (uint32_t)t0;
    *a.d_bump = 0;
  }
}

struct CopyArgs {
  CMsgs bl, em, st;         // chunk storage (bl: tile * kApplyTile, em: base_em[tile])
  Msgs out0, out1;          // stream 0 / stream 1
  const uint32_t* cnt_bl;
  const uint32_t* cnt_em;
  const uint32_t* off_bl;
  const uint32_t* off_em;
  const uint32_t* base_em;
  const uint32_t* d_total;  // [0] t0, [1] t1, [2] nt
  uint32_t n_staged;
  uint32_t mode;
};

__device__ __forceinline__ void copy_run(const CMsgs& s, uint64_t s0, const Msgs& d, uint64_t d0, uint32_t n) {
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    d.key[d0 + i] = s.key[s0 + i];
    d.src[d0 + i] = s.src[s0 + i];
    d.pay[d0 + i] = s.pay[s0 + i];
  }
}

__global__ void __launch_bounds__(256) k_compact_copy(CopyArgs a) {
  const uint32_t nt = a.d_total[2];
  if (a.d_total[0] == 0 && a.d_total[1] == 0) return;  // empty or capacity overflow
  const uint32_t nchunks = 2 * nt + (a.mode == 0 ? 1u : 0u);
  for (uint32_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    if (c < nt) {
      copy_run(a.bl, (uint64_t)c * kApplyTile, a.out0, a.off_bl[c], a.cnt_bl[c]);
    } else if (c < 2 * nt) {
      uint32_t t = c - nt;
      copy_run(a.em, a.base_em[t], a.mode == 0 ? a.out0 : a.out1, a.off_em[t], a.cnt_em[t]);
    } else {
      copy_run(a.st, 0, a.out0, (uint64_t)a.d_total[0] - a.n_staged, a.n_staged);
    }
  }
}

// =========================================================================
// Stable LSD radix sort pass over `bits` bits at `shift` (bits <= 8).
//   upsweep:   per-tile digit histogram -> hist[d * stride + t]
//   rowscan:   per digit, exclusive scan over tiles; tot[d] = digit total
//   downsweep: wave-level multisplit (ballot match) ranks, LDS staging,
//              coalesced scatter to the output
// =========================================================================
struct SortArgs {
  CMsgs in;
  Msgs out;
  const uint32_t* d_n;
  uint32_t* hist;
  uint32_t* tot;
  uint32_t stride;  // >= max tiles
  uint32_t shift, bits;
};

__global__ void __launch_bounds__(kSortThreads) k_sort_upsweep(SortArgs a) {
  __shared__ uint32_t h[kSortWaves][kRadix];
  const uint32_t n = *a.d_n, nt = div_up(n, kSortTile);
  const int tid = threadIdx.x, w = tid / kWave;
  const uint32_t mask = (1u << a.bits) - 1u, nd = 1u << a.bits;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    for (int i = tid; i < kSortWaves * kRadix; i += kSortThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint32_t base = t * kSortTile;
    if (base + kSortTile <= n) {
      const uint4* k4 = reinterpret_cast<const uint4*>(a.in.key + base);
#pragma unroll
      for (int j = 0; j < kSortIpt / 4; ++j) {
        uint4 v = k4[j * kSortThreads + tid];
        atomicAdd(&h[w][(v.x >> a.shift) & mask], 1u);
        atomicAdd(&h[w][(v.y >> a.shift) & mask], 1u);
        atomicAdd(&h[w][(v.z >> a.shift) & mask], 1u);
        atomicAdd(&h[w][(v.w >> a.shift) & mask], 1u);
      }
    } else {
      for (uint32_t i = base + tid; i < n; i += kSortThreads) atomicAdd(&h[w][(a.in.key[i] >> a.shift) & mask], 1u);
    }
    __syncthreads();
    for (uint32_t d = tid; d < nd; d += kSortThreads) {
      uint32_t s = 0;
#pragma unroll
      for (int q = 0; q < kSortWaves; ++q) s += h[q][d];
      a.hist[d * a.stride + t] = s;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) k_sort_rowscan(SortArgs a) {
  __shared__ uint32_t scratch[256 / kWave + 1];
  __shared__ uint32_t s_run;
  const uint32_t n = *a.d_n, nt = div_up(n, kSortTile);
  const uint32_t d = blockIdx.x;  // one block per digit
  if (d >= (1u << a.bits)) return;
  uint32_t* row = a.hist + (size_t)d * a.stride;
  if (threadIdx.x == 0) s_run = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nt; base += 256) {
    uint32_t i = base + threadIdx.x;
    uint32_t v = i < nt ? row[i] : 0u, tot;
    uint32_t ex = block_excl_sum<256>(v, scratch, &tot);
    if (i < nt) row[i] = s_run + ex;
    __syncthreads();
    if (threadIdx.x == 0) s_run += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) a.tot[d] = s_run;
}

__global__ void __launch_bounds__(kSortThreads) k_sort_downsweep(SortArgs a) {
  __shared__ uint32_t whist[kSortWaves][kRadix];
  __shared__ uint32_t s_dbase[kRadix];  // exclusive scan of digit totals
  __shared__ uint32_t s_ldig[kRadix];   // tile-local digit base
  __shared__ uint32_t s_gadj[kRadix];   // global pos = s_gadj[d] + local pos
  __shared__ uint32_t scratch[kSortThreads / kWave + 1];
  __shared__ uint32_t s_key[kSortTile], s_src[kSortTile], s_pay[kSortTile];

  const uint32_t n = *a.d_n, nt = div_up(n, kSortTile);
  const int tid = threadIdx.x, w = tid / kWave;
  const uint32_t lane = lane_id();
  const uint32_t mask = (1u << a.bits) - 1u, nd = 1u << a.bits;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  if (nt == 0) return;
  {  // digit bases (same for all tiles)
    uint32_t v = (uint32_t)tid < nd ? a.tot[tid] : 0u, tot;
    uint32_t ex = block_excl_sum<kSortThreads>(v, scratch, &tot);
    if ((uint32_t)tid < nd) s_dbase[tid] = ex;
  }
  __syncthreads();

  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    for (int i = tid; i < kSortWaves * kRadix; i += kSortThreads) (&whist[0][0])[i] = 0;
    __syncthreads();
    const uint32_t base = t * kSortTile;
    const uint32_t wbase = base + w * (kSortIpt * kWave);
    uint32_t k[kSortIpt], s[kSortIpt], p[kSortIpt], rk[kSortIpt];
#pragma unroll
    for (int r = 0; r < kSortIpt; ++r) {
      uint32_t i = wbase + r * kWave + lane;
      if (i < n) {
        k[r] = a.in.key[i];
        s[r] = a.in.src[i];
        p[r] = a.in.pay[i];
      } else {
        k[r] = 0xFFFFFFFFu;
      }
    }
    // wave-level multisplit: rank of each item among equal digits, in item order
#pragma unroll
    for (int r = 0; r < kSortIpt; ++r) {
      uint32_t i = wbase + r * kWave + lane;
      bool valid = i < n;
      uint32_t d = (k[r] >> a.shift) & mask;
      uint64_t m = __ballot(valid);
      for (uint32_t b = 0; b < a.bits; ++b) {
        uint32_t bit = (d >> b) & 1u;
        uint64_t bal = __ballot(bit);
        m &= bit ? bal : ~bal;
      }
      uint32_t before = (uint32_t)__popcll(m & lt_mask);
      uint32_t cnt = (uint32_t)__popcll(m);
      uint32_t old = 0;
      if (valid) old = whist[w][d];
      __builtin_amdgcn_wave_barrier();
      if (valid && before == 0) whist[w][d] = old + cnt;
      __builtin_amdgcn_wave_barrier();
      rk[r] = old + before;
    }
    __syncthreads();
    // per digit: wave prefixes, tile count; tile-local digit base
    uint32_t cnt_d = 0;
    if ((uint32_t)tid < nd) {
      uint32_t run = 0;
#pragma unroll
      for (int q = 0; q < kSortWaves; ++q) {
        uint32_t c = whist[q][tid];
        whist[q][tid] = run;
        run += c;
      }
      cnt_d = run;
    }
    uint32_t tot;
    uint32_t lex = block_excl_sum<kSortThreads>(cnt_d, scratch, &tot);
    if ((uint32_t)tid < nd) {
      s_ldig[tid] = lex;
      s_gadj[tid] = s_dbase[tid] + a.hist[tid * a.stride + t] - lex;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortIpt; ++r) {
      uint32_t i = wbase + r * kWave + lane;
      if (i < n) {
        uint32_t d = (k[r] >> a.shift) & mask;
        uint32_t lp = s_ldig[d] + whist[w][d] + rk[r];
        s_key[lp] = k[r];
        s_src[lp] = s[r];
        s_pay[lp] = p[r];
      }
    }
    __syncthreads();
    const uint32_t cnt_tile = min((uint32_t)kSortTile, n - base);
    for (uint32_t lp = tid; lp < cnt_tile; lp += kSortThreads) {
      uint32_t kk = s_key[lp];
      uint32_t g = s_gadj[(kk >> a.shift) & mask] + lp;
      a.out.key[g] = kk;
      a.out.src[g] = s_src[lp];
      a.out.pay[g] = s_pay[lp];
    }
    __syncthreads();
  }
}

// =========================================================================
// Segmented drain + behaviour-apply.
// Input: envelopes sorted by key (stable).  For item i of actor a's segment,
// p = position in the segment (backlog first, then arrivals in canonical
// order).  Classification (Mailbox.scala:260-277, 551-565):
//   !alive               -> dead letter
//   p <  T               -> drained: invoked in order by the segment head thread
//   T <= p < C (or C=0)  -> stays queued (backlog chunk)
//   p >= C               -> dead letter (bounded tail-drop)
// =========================================================================
struct ApplyArgs {
  DevParams P;
  CMsgs in;
  const uint32_t* d_n;
  Msgs bl;    // backlog chunks (tile * kApplyTile)
  Msgs em;    // emission chunks, bump-allocated: chunk t at base_em[t]
  uint32_t* cnt_bl;
  uint32_t* cnt_em;
  uint32_t* base_em;
  uint32_t* d_bump;
  uint64_t cap_em;   // capacity of the emission buffer
  uint64_t* stats;
};

// first index of the run of `kb` that ends at `hi` (keys sorted; keys[hi] == kb)
__device__ __forceinline__ uint32_t run_start(const uint32_t* keys, uint32_t hi, uint32_t kb) {
  uint32_t step = 1;
  while (hi >= step && keys[hi - step] == kb) {
    hi -= step;
    step <<= 1;
  }
  uint32_t lo = hi >= step ? hi - step + 1 : 0;  // keys[lo-1] != kb (or lo == 0)
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (keys[mid] == kb) hi = mid; else lo = mid + 1;
  }
  return hi;
}

template <bool kWrite>
struct Emitter {
  const DevParams* P;
  Msgs out;
  uint64_t pos;       // next write position (kWrite)
  uint32_t self;      // sender id (global)
  uint32_t n_valid;   // tells to a known actor
  uint32_t n_all;     // all tells
  __device__ __forceinline__ void operator()(uint32_t dst, uint32_t pay) {
    ++n_all;
    if (dst >= P->n_global) return;  // unknown ref -> deadLetters
    ++n_valid;
    if (kWrite) {
      uint32_t key = (P->R > 1) ? P->route[dst] : dst;
      out.key[pos] = key;
      out.src[pos] = self;
      out.pay[pos] = pay;
      ++pos;
    }
  }
};

__global__ void __launch_bounds__(kApplyThreads) k_apply(ApplyArgs a) {
  __shared__ uint32_t s_lastkey[kApplyThreads];
  __shared__ int s_maxscratch[kApplyThreads / kWave + 1];
  __shared__ uint32_t s_scratch[kApplyThreads / kWave + 1];
  __shared__ uint32_t s_carry;
  __shared__ uint32_t s_ebase;
  __shared__ unsigned long long s_stat[5];

  const DevParams& P = a.P;
  const uint32_t n = *a.d_n, nt = div_up(n, kApplyTile);
  const int tid = threadIdx.x;
  const uint32_t T = P.T, C = P.C;
  if (blockIdx.x == 0 && tid == 0 && n > 0) atomicAdd((unsigned long long*)&a.stats[ST_STEPS], 1ull);

  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const uint32_t base = t * kApplyTile;
    const uint32_t i0 = base + tid * kApplyIpt;
    if (tid < 5) s_stat[tid] = 0;
    uint32_t k[kApplyIpt];
    if (i0 + kApplyIpt <= n) {
      const uint4* k4 = reinterpret_cast<const uint4*>(a.in.key + i0);
      uint4 v0 = k4[0], v1 = k4[1];
      k[0] = v0.x; k[1] = v0.y; k[2] = v0.z; k[3] = v0.w;
      k[4] = v1.x; k[5] = v1.y; k[6] = v1.z; k[7] = v1.w;
    } else {
#pragma unroll
      for (int j = 0; j < kApplyIpt; ++j) k[j] = (i0 + j < n) ? a.in.key[i0 + j] : 0xFFFFFFFFu;
    }
    s_lastkey[tid] = k[kApplyIpt - 1];
    if (tid == 0) {
      // segment start carried into this tile (galloping search backwards)
      uint32_t kb = a.in.key[base];
      s_carry = (base > 0 && a.in.key[base - 1] == kb) ? run_start(a.in.key, base, kb) : base;
    }
    __syncthreads();
    uint32_t prevk = tid > 0 ? s_lastkey[tid - 1] : (base > 0 ? a.in.key[base - 1] : 0xFFFFFFFEu);
    // head flags + running last-head index inside the thread
    int hs[kApplyIpt];
    int lh = -1;
    uint32_t headmask = 0;
#pragma unroll
    for (int j = 0; j < kApplyIpt; ++j) {
      uint32_t i = i0 + j;
      bool head = i < n && (i == 0 || k[j] != (j == 0 ? prevk : k[j - 1]));
      if (head) { lh = (int)i; headmask |= 1u << j; }
      hs[j] = lh;
    }
    int carry = block_excl_max<kApplyThreads>(lh, s_maxscratch);
    if (carry < 0) carry = (int)s_carry;

    // classify items; backlog compaction
    uint32_t nbl = 0, ndead = 0;
    uint32_t blmask = 0;
    uint8_t al[kApplyIpt];
#pragma unroll
    for (int j = 0; j < kApplyIpt; ++j) {
      uint32_t i = i0 + j;
      al[j] = 0;
      if (i >= n) continue;
      uint32_t ss = hs[j] >= 0 ? (uint32_t)hs[j] : (uint32_t)carry;
      uint32_t p = i - ss;
      uint32_t l = k[j] & kLocalMask;
      al[j] = P.alive[l];
      if (!al[j]) { ++ndead; continue; }
      if (p < T) continue;  // drained by the head thread
      if (C == 0 || p < C) { blmask |= 1u << j; ++nbl; } else ++ndead;
    }
    uint32_t bltot;
    uint32_t bloff = block_excl_sum<kApplyThreads>(nbl, s_scratch, &bltot);
    if (blmask) {
      const size_t ob = (size_t)t * kApplyTile + bloff;
      uint32_t q = 0;
#pragma unroll
      for (int j = 0; j < kApplyIpt; ++j)
        if (blmask & (1u << j)) {
          uint32_t i = i0 + j;
          a.bl.key[ob + q] = k[j];
          a.bl.src[ob + q] = a.in.src[i];
          a.bl.pay[ob + q] = a.in.pay[i];
          ++q;
        }
    }
    if (tid == 0) a.cnt_bl[t] = bltot;

    // ---- phase A: count emissions of the segments headed in this thread
    uint32_t nem = 0;
    uint64_t wv[AGX_MAX_WORDS];
    if (headmask) {
#pragma unroll
      for (int j = 0; j < kApplyIpt; ++j) {
        if (!(headmask & (1u << j)) || !al[j]) continue;
        const uint32_t i = i0 + j, kb = k[j], l = kb & kLocalMask;
        const uint32_t self = P.R > 1 ? P.gid[l] : l;
        const uint32_t kind = P.kind[l];
#pragma unroll
        for (int q = 0; q < (int)AGX_MAX_WORDS; ++q) wv[q] = (q < (int)P.W) ? P.state[(size_t)q * P.n_local + l] : 0ull;
        Emitter<false> em{&P, {}, 0, self, 0, 0};
        for (uint32_t q = 0; q < T; ++q) {
          uint32_t ii = i + q;
          if (ii >= n || (q > 0 && a.in.key[ii] != kb)) break;
          uint32_t r = apply_msg(P, kind, self, l, wv, a.in.src[ii], a.in.pay[ii], em);
          if (r == AGX_RES_STOPPED) break;
        }
        nem += em.n_valid;
      }
    }
    uint32_t emtot;
    uint32_t emoff = block_excl_sum<kApplyThreads>(nem, s_scratch, &emtot);
    if (tid == 0) {
      uint32_t b = emtot ? atomicAdd(a.d_bump, emtot) : 0u;
      if ((uint64_t)b + emtot > a.cap_em) {  // out of emission capacity: abort the run
        atomicOr((unsigned long long*)&a.stats[ST_ERROR], (unsigned long long)kErrCapacity);
        emtot = 0;
        b = 0xFFFFFFFFu;
      }
      a.cnt_em[t] = emtot;
      a.base_em[t] = b;
      s_ebase = b;
    }
    __syncthreads();
    const uint32_t ebase = s_ebase;

    // ---- phase B: apply for real, write emissions and state
    uint32_t ndel = 0, nunh = 0, nall = 0, nact = 0;
    if (headmask && ebase != 0xFFFFFFFFu) {
      Emitter<true> em{&P, a.em, (uint64_t)ebase + emoff, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < kApplyIpt; ++j) {
        if (!(headmask & (1u << j)) || !al[j]) continue;
        const uint32_t i = i0 + j, kb = k[j], l = kb & kLocalMask;
        const uint32_t self = P.R > 1 ? P.gid[l] : l;
        const uint32_t kind = P.kind[l];
        em.self = self;
        ++nact;
#pragma unroll
        for (int q = 0; q < (int)AGX_MAX_WORDS; ++q) wv[q] = (q < (int)P.W) ? P.state[(size_t)q * P.n_local + l] : 0ull;
        uint32_t nd = 0;
        for (uint32_t q = 0; q < T; ++q) {
          uint32_t ii = i + q;
          if (ii >= n || (q > 0 && a.in.key[ii] != kb)) break;
          ++nd;
        }
        for (uint32_t q = 0; q < nd; ++q) {
          uint32_t ii = i + q;
          uint32_t r = apply_msg(P, kind, self, l, wv, a.in.src[ii], a.in.pay[ii], em);
          ++ndel;
          if (r == AGX_RES_UNHANDLED) ++nunh;
          if (r == AGX_RES_STOPPED) {
            P.stopq[atomicAdd(P.nstop, 1u)] = l;
            ndead += nd - q - 1;
            break;
          }
        }
#pragma unroll
        for (int q = 0; q < (int)AGX_MAX_WORDS; ++q)
          if (q < (int)P.W) P.state[(size_t)q * P.n_local + l] = wv[q];
      }
      nall = em.n_all;
      ndead += em.n_all - em.n_valid;
    }
    // tile stats -> global
    uint32_t v0 = ndel, v1 = ndead, v2 = nunh, v3 = nall, v4 = nact;
    v0 = wave_incl_sum(v0); v1 = wave_incl_sum(v1); v2 = wave_incl_sum(v2); v3 = wave_incl_sum(v3);
    v4 = wave_incl_sum(v4);
    if (lane_id() == kWave - 1) {
      atomicAdd(&s_stat[0], (unsigned long long)v0);
      atomicAdd(&s_stat[1], (unsigned long long)v1);
      atomicAdd(&s_stat[2], (unsigned long long)v2);
      atomicAdd(&s_stat[3], (unsigned long long)v3);
      atomicAdd(&s_stat[4], (unsigned long long)v4);
    }
    __syncthreads();
    if (tid == 0) {
      if (s_stat[0]) atomicAdd((unsigned long long*)&a.stats[ST_DELIVERED], s_stat[0]);
      if (s_stat[1]) atomicAdd((unsigned long long*)&a.stats[ST_DEAD], s_stat[1]);
      if (s_stat[2]) atomicAdd((unsigned long long*)&a.stats[ST_UNHANDLED], s_stat[2]);
      if (s_stat[3]) atomicAdd((unsigned long long*)&a.stats[ST_EMITTED], s_stat[3]);
      if (s_stat[4]) atomicAdd((unsigned long long*)&a.stats[ST_ACTIVE], s_stat[4]);
    }
    __syncthreads();
  }
}

// messages still in flight after the last apply (backlog + emitted chunks)
__global__ void __launch_bounds__(kScanThreads) k_inflight(const uint32_t* d_n, const uint32_t* cnt_bl,
                                                           const uint32_t* cnt_em, unsigned long long* out) {
  __shared__ unsigned long long s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  const uint32_t nt = div_up(*d_n, kApplyTile);
  unsigned long long v = 0;
  for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) v += (unsigned long long)cnt_bl[i] + cnt_em[i];
  atomicAdd(&s, v);
  __syncthreads();
  if (threadIdx.x == 0) *out = s;
}

// partition helper: per-owner send counts (digit totals of the owner pass) -> u64 vector
__global__ void k_pack_counts(const uint32_t* tot, const uint32_t* d_total, uint64_t* vec, uint32_t R,
                              uint32_t n_staged) {
  uint32_t i = threadIdx.x;
  if (i < R) vec[i] = tot[i];
  if (i == 0) {
    vec[R] = d_total[0];  // backlog kept locally
    vec[R + 1] = n_staged;
  }
}

}  // namespace agx
