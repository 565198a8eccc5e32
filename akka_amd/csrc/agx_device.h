// agx_device.h — device-side building blocks for the gfx950 dispatch engine:
// wave64 / block scans, the behaviour table (typed Behaviors.receive subset)
// and the counter RNG.  Integer only; no MFMA (the path is HBM/scatter-bound).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/akka_gpu.h"

namespace agx {

constexpr int kWave = 64;               // CDNA wavefront
constexpr uint32_t kLocalMask = 0x0FFFFFFFu;  // key = (owner << 28) | local
constexpr int kOwnerShift = 28;

// ------------------------------------------------------------------ params
struct DevParams {
  uint32_t n_global, n_local, W, T, C, R, rank, kmax;
  uint32_t ring_stride, fan_k;  // ring_stride pre-reduced mod n_global
  uint64_t fan_seed, zipf_n;
  const uint32_t* zipf_cdf;
  const uint2* zipf_ent;      // [2^kZipfBits] direct answers / search ranges (see zipf_dest)
  const uint32_t* zipf_perm;
  const uint64_t* row_ptr;  // local rows
  const uint32_t* col;      // global dst ids
  const uint32_t* route;    // global id -> (owner<<28)|local   (R > 1 only)
  const uint32_t* gid;      // local -> global id              (R > 1 only)
  uint8_t* kind;
  uint8_t* alive;           // read-only inside k_apply; stops are committed after it
  uint32_t* stopq;          // actors that returned Behaviors.stopped this step
  uint32_t* nstop;
  uint64_t* state;          // word-major SoA: state[w * n_local + l]; CRDT engines (pw > 0): actor-major,
                            // state[l * pitch + w] (wide_state)
  uint32_t pitch;           // u64 words per actor row of an actor-major engine (0: word-major)
  // words 0 / 1 of a plain behaviour: state[l * sa + w * sw] -- word-major (sa 1, sw n_local), or
  // actor-major pairs of a two-word engine (sa 2, sw 1: one line holds both words of 8 actors, so
  // a sparse superstep touches one state line per activation instead of two)
  uint32_t sa, sw;
  // CRDT state gossips (agx_crdt.h): snapshot rows, row-major, `pw` u32 each.
  // heap = 2 x heap_rows rows (ping-pong by superstep parity); rx = rows
  // received from other ranks this superstep (handle - heap_rows).
  uint32_t* heap;
  const uint32_t* rx;
  uint32_t* heap_top;       // [2] rows allocated in heap[parity]
  const uint32_t* step;     // superstep counter (bumped by the first kernel of a step)
  uint32_t heap_rows, pw, gossip_f;
  uint64_t gossip_seed;
  uint32_t delta_max;             // delta-CRDT mode (Replicator max-delta-size), 0 = off
  unsigned long long* err;        // stats[ST_ERROR]: capacity errors raised inside a behaviour
  // compiled behaviours (agx_set_behaviors): case / action tables, behaviour b = cases [bfirst[b], bfirst[b+1])
  const agx_case* bcase;
  const agx_act* bact;
  const uint32_t* bfirst;
  uint32_t n_beh;
  // the reply path (agx_set_outbound): tells to ids [host_lo, host_lo + host_n) go to the outbox
  uint32_t host_lo, host_n, outbox_cap;
  uint32_t* outbox;     // [outbox_cap][3] dst, src, payload
  uint32_t* outbox_n;   // envelopes appended (may pass outbox_cap: reported as a capacity error)
  // mailbox classes (agx_set_mailbox_class): the class of an actor is bits 1..3 of its alive byte;
  // nmc == 0 -> every actor uses class 0 (C, T above); else capacity mcap[class], drain
  // min(Tr, capacity) (Tr = the dispatcher throughput, >= 1)
  uint32_t nmc, Tr;
  uint32_t mcap[AGX_MAX_MAILBOX_CLASSES];
};

// An actor's bounded capacity (0 = unbounded) and drain limit from its alive byte (bit 0 = alive,
// bits 1..3 = mailbox class): Mailboxes.lookupConfigurator per actor (Mailboxes.scala:204-260).
// actor l's state row in a CRDT engine (actor-major, P.pitch u64 words per row)
__device__ __forceinline__ uint64_t* wide_state(const DevParams& P, uint32_t l) {
  return P.pitch ? P.state + (size_t)l * P.pitch : P.state + l;
}
// the stride between consecutive words of one actor's state (1 actor-major, n_local word-major)
__device__ __forceinline__ size_t wide_nl(const DevParams& P) { return P.pitch ? 1u : P.n_local; }

// word w (0 or 1) of a plain behaviour's state (P.sa / P.sw above; 32-bit offsets)
__device__ __forceinline__ uint32_t sidx(const DevParams& P, uint32_t l, uint32_t w) { return l * P.sa + w * P.sw; }

__device__ __forceinline__ void mbox_limits(const DevParams& P, uint32_t abyte, uint32_t& C, uint32_t& T) {
  if (P.nmc == 0) {  // (uniform: one mailbox type for the whole dispatcher)
    C = P.C;
    T = P.T;
    return;
  }
  C = P.mcap[(abyte >> 1) & (AGX_MAX_MAILBOX_CLASSES - 1)];
  T = C && P.Tr > C ? C : P.Tr;
}

// A tell to a host-side actor (agx_set_outbound): appended to the outbox (when `write`); returns
// false for any other id.  One thread's appends are ordered (same counter, program order), so each
// sender's outbound tells keep their emission order.
__device__ __forceinline__ bool outbound_tell(const DevParams& P, uint32_t dst, uint32_t src, uint32_t pay,
                                              bool write) {
  if (dst - P.host_lo >= P.host_n) return false;
  if (write) {
    // an append past outbox_cap is dropped and reported (then cleared) by agx_take_outbound from the
    // count itself -- not through the sticky error word, so the engine stays usable
    const uint32_t i = atomicAdd(P.outbox_n, 1u);
    if (i < P.outbox_cap) {
      P.outbox[3 * (size_t)i] = dst;
      P.outbox[3 * (size_t)i + 1] = src;
      P.outbox[3 * (size_t)i + 2] = pay;
    }
  }
  return true;
}

// ------------------------------------------------------------------ RNG
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t fanout_rand(uint64_t seed, uint32_t self, uint32_t h, uint32_t j) {
  return splitmix64(seed ^ splitmix64(((uint64_t)self << 32) ^ ((uint64_t)h << 4) ^ (uint64_t)j));
}
// First index i with cdf[i] >= u (clamped to n - 1), as a destination perm[i].  The top kZipfBits
// of u select an entry of the `zent` index built at agx_set_fanout: when every u of that range has
// the same answer i (the Zipf head: a hot destination spans many ranges) the entry holds perm[i]
// itself, {perm[i], kZipfDirect} -- one load in all; otherwise the search range {lo, hi} (lo = the
// answer for u = t << (32 - kZipfBits), hi = that of the next range, n - 1 after the last), a binary
// search over the CDF thresholds in it, then perm.  Same answer as the search over [0, n - 1].
constexpr uint32_t kZipfBits = 20;
constexpr uint32_t kZipfDirect = 0xFFFFFFFFu;  // (a range's hi is <= n - 1 < 2^32 - 1)
__device__ __forceinline__ uint32_t zipf_dest(const uint32_t* cdf, const uint32_t* perm, const uint2* zent, uint64_t r) {
  const uint32_t u = (uint32_t)(r >> 32);
  const uint2 z = zent[u >> (32 - kZipfBits)];
  if (z.y == kZipfDirect) return z.x;
  uint32_t lo = z.x, hi = z.y;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (cdf[mid] >= u) hi = mid; else lo = mid + 1;
  }
  return perm[lo];
}

// ------------------------------------------------------------------ scans
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// inclusive wave64 sum scan over the whole (fully active) wave, in DPP: row_shr 1/2/4/8 scans each
// 16-lane row, row_bcast 15 / 31 carry the row totals into the rows above.  Six VALU ops with DPP
// operands instead of six ds_bpermute round trips through the LDS crossbar (__shfl_up): every
// block scan of the apply chain uses it.  (Lanes with no DPP source keep `old` = 0.)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return v;
}
__device__ __forceinline__ int wave_incl_max(int v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    int t = __shfl_up(v, d, kWave);
    if (lane >= (uint32_t)d) v = max(v, t);
  }
  return v;
}

// Block exclusive sum over NT threads (NT multiple of 64, <= 1024).
// `scratch` needs NT/64 + 1 u32.  Returns exclusive prefix; *total = block sum.
// Two barriers: every thread sums the NT/64 wave totals itself (LDS broadcast reads) instead of
// one thread scanning them between two barriers.
template <int NT>
__device__ __forceinline__ uint32_t block_excl_sum(uint32_t v, uint32_t* scratch, uint32_t* total) {
  constexpr int NW = NT / kWave;
  const int tid = threadIdx.x, w = tid / kWave, lane = tid % kWave;
  const uint32_t inc = wave_incl_sum(v);
  if (lane == kWave - 1) scratch[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t t = scratch[i];
    pre += i < w ? t : 0u;
    tot += t;
  }
  *total = tot;
  __syncthreads();  // (scratch is reused by the caller's next scan)
  return pre + inc - v;
}

// Two block exclusive sums at once (one set of barriers).  `scratch` needs 2 * (NT/64 + 1) u32.
template <int NT>
__device__ __forceinline__ uint2 block_excl_sum2(uint32_t v0, uint32_t v1, uint32_t* scratch, uint32_t* t0,
                                                 uint32_t* t1) {
  constexpr int NW = NT / kWave;
  const int tid = threadIdx.x, w = tid / kWave, lane = tid % kWave;
  const uint32_t i0 = wave_incl_sum(v0), i1 = wave_incl_sum(v1);
  if (lane == kWave - 1) {
    scratch[w] = i0;
    scratch[NW + 1 + w] = i1;
  }
  __syncthreads();
  uint32_t p0 = 0, p1 = 0, s0 = 0, s1 = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t a = scratch[i], b = scratch[NW + 1 + i];
    p0 += i < w ? a : 0u;
    p1 += i < w ? b : 0u;
    s0 += a;
    s1 += b;
  }
  *t0 = s0;
  *t1 = s1;
  __syncthreads();
  return make_uint2(p0 + i0 - v0, p1 + i1 - v1);
}

// Block exclusive max over NT threads; identity -1.
template <int NT>
__device__ __forceinline__ int block_excl_max(int v, int* scratch) {
  constexpr int NW = NT / kWave;
  const int tid = threadIdx.x, w = tid / kWave, lane = tid % kWave;
  int inc = wave_incl_max(v);
  int exc = __shfl_up(inc, 1, kWave);
  if (lane == 0) exc = -1;
  if (lane == kWave - 1) scratch[w] = inc;
  __syncthreads();
  if (tid == 0) {
    int run = -1;
    for (int i = 0; i < NW; ++i) { int t = scratch[i]; scratch[i] = run; run = max(run, t); }
  }
  __syncthreads();
  int r = max(scratch[w], exc);
  __syncthreads();
  return r;
}

// ------------------------------------------------------------------ behaviours
// One ActorCell.invoke of one message (akka-actor/.../ActorCell.scala:539-555)
// through the typed ActorAdapter (TY/internal/adapter/ActorAdapter.scala:77-168).
// `Emit` is called for each tell: emit(dst_global, payload).
//
// KM is the set of behaviour kinds compiled in (bit k = kind k).  The engine
// launches the narrowest specialisation that covers every registered kind, so a
// population of one behaviour runs a small, branch-free apply kernel.
constexpr uint32_t kb(uint32_t k) { return 1u << (k < AGX_KIND_COMPILED ? k : AGX_KIND_COMPILED); }
// KM flag (not a kind): the variant runs delta-CRDT replication (agx_set_delta_crdt).  Variants
// without it compile the delta code out (its registers would spill the full-state merges).
constexpr uint32_t kDeltaKM = 1u << 31;
constexpr uint32_t KM_ALL = kb(AGX_KIND_COUNTER) | kb(AGX_KIND_RING) | kb(AGX_KIND_FANOUT) | kb(AGX_KIND_FORWARD_RR) |
                            kb(AGX_KIND_STOP_AFTER) | kb(AGX_KIND_PINGPONG) | kb(AGX_KIND_EVEN);

// ---- compiled behaviours (include/akka_gpu.h "compiled behaviours"; akka_amd/typed.py lowers them)
__device__ __forceinline__ uint64_t cb_operand(uint32_t src, uint32_t word, int64_t k, uint32_t pay, const uint64_t* w,
                                               uint32_t sender, uint32_t self) {
  uint64_t b = 0;
  switch (src) {
    case AGX_V_PAYLOAD: b = pay; break;
    case AGX_V_TAG: b = pay >> 24; break;
    case AGX_V_ARG: b = pay & 0xFFFFFFu; break;
    case AGX_V_WORD: b = w[word & 1u]; break;
    case AGX_V_SENDER: b = sender; break;
    case AGX_V_SELF: b = self; break;
    default: break;
  }
  return b + (uint64_t)k;
}
__device__ __forceinline__ bool cb_cmp(uint32_t op, uint64_t a, uint64_t b) {
  switch (op) {
    case AGX_CMP_EQ: return a == b;
    case AGX_CMP_NE: return a != b;
    case AGX_CMP_LT: return a < b;
    case AGX_CMP_LE: return a <= b;
    case AGX_CMP_GT: return a > b;
    case AGX_CMP_GE: return a >= b;
    default: return true;
  }
}
// ReceiveBuilder.receive (TY/javadsl/ReceiveBuilder.scala:209-218): the first case whose tests hold
template <typename Emit>
__device__ __forceinline__ uint32_t compiled_apply(const DevParams& P, uint32_t& kind, uint32_t self, uint64_t* w,
                                                uint32_t src, uint32_t pay, Emit& emit) {
  const uint32_t b = kind - AGX_KIND_COMPILED;
  if (b >= P.n_beh) return AGX_RES_UNHANDLED;
  const uint32_t c1 = P.bfirst[b + 1];
  for (uint32_t c = P.bfirst[b]; c < c1; ++c) {
    const agx_case C = P.bcase[c];
    if (!cb_cmp(C.cmp1, cb_operand(C.src1, C.word1, C.k1, pay, w, src, self),
                cb_operand(C.src2, C.word2, C.k2, pay, w, src, self)))
      continue;
    if (!cb_cmp(C.cmp2, cb_operand(C.src3, C.word3, C.k3, pay, w, src, self),
                cb_operand(C.src4, C.word4, C.k4, pay, w, src, self)))
      continue;
    for (uint32_t i = C.act_first; i < (uint32_t)C.act_first + C.act_count; ++i) {
      const agx_act A = P.bact[i];
      const uint64_t v = cb_operand(A.src, A.sword, A.k, pay, w, src, self);
      switch (A.op) {
        case AGX_A_SET: w[A.word & 1u] = v; break;
        case AGX_A_ADD: w[A.word & 1u] += v; break;
        case AGX_A_MAX: w[A.word & 1u] = v > w[A.word & 1u] ? v : w[A.word & 1u]; break;
        case AGX_A_MIN: w[A.word & 1u] = v < w[A.word & 1u] ? v : w[A.word & 1u]; break;
        case AGX_A_TELL: {
          uint64_t d;
          if (A.dsrc == AGX_V_SELF) {  // (self + dk) mod n: ring neighbours
            int64_t x = ((int64_t)self + A.dk) % (int64_t)P.n_global;
            d = (uint64_t)(x < 0 ? x + (int64_t)P.n_global : x);
          } else {
            d = cb_operand(A.dsrc, A.dword, A.dk, pay, w, src, self);
          }
          emit(d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d, A.or_mask ? ((uint32_t)v & 0xFFFFFFu) | A.or_mask : (uint32_t)v);
          break;
        }
        default: break;
      }
    }
    if (C.result == AGX_RES_BECOME) {
      kind = AGX_KIND_COMPILED + C.next;
      return AGX_RES_SAME;
    }
    return C.result;
  }
  return AGX_RES_UNHANDLED;
}

// `kind` is the actor's current behaviour: a compiled behaviour's become updates it (the caller
// keeps it for the rest of the drain and stores it back).
template <uint32_t KM, typename Emit>
__device__ __forceinline__ uint32_t apply_msg(const DevParams& P, uint32_t& kind_io, uint32_t self, uint32_t local,
                                              uint64_t* w, uint32_t src, uint32_t pay, Emit&& emit) {
  uint32_t kind = kind_io;
  if constexpr (KM == kb(AGX_KIND_RING)) kind = AGX_KIND_RING;  // single-kind specialisations: no dispatch
  if constexpr (KM == kb(AGX_KIND_FORWARD_RR)) kind = AGX_KIND_FORWARD_RR;
  if constexpr (KM == kb(AGX_KIND_FANOUT)) kind = AGX_KIND_FANOUT;
  if constexpr (KM == kb(AGX_KIND_COUNTER)) kind = AGX_KIND_COUNTER;
  if constexpr ((KM & kb(AGX_KIND_COMPILED)) != 0)
    if (kind >= AGX_KIND_COMPILED) return compiled_apply(P, kind_io, self, w, src, pay, emit);
  switch (kind) {
    case AGX_KIND_COUNTER:
      if constexpr ((KM & kb(AGX_KIND_COUNTER)) != 0) {
        w[0] += 1;
        w[1] += pay;  // w[1] exists (array of AGX_MAX_WORDS); only stored back if W > 1
      }
      return AGX_RES_SAME;
    case AGX_KIND_RING:
      if constexpr ((KM & kb(AGX_KIND_RING)) != 0) {
        w[0] += 1;
        if (pay > 0) {
          uint32_t d = self + P.ring_stride;  // both < n_global < 2^31: no overflow, one conditional subtract
          emit(d >= P.n_global ? d - P.n_global : d, pay - 1);
        }
      }
      return AGX_RES_SAME;
    case AGX_KIND_FANOUT:
      if constexpr ((KM & kb(AGX_KIND_FANOUT)) != 0) {
        w[0] += 1;
        w[1] += pay;
        const uint32_t ttl = pay >> 24, h = pay & 0x00FFFFFFu;  // ttl 8 bits, hash 24 bits
        if (ttl > 0)
          for (uint32_t j = 0; j < P.fan_k; ++j) {
            uint64_t r = fanout_rand(P.fan_seed, self, h, j);
            uint32_t d = zipf_dest(P.zipf_cdf, P.zipf_perm, P.zipf_ent, r);
            emit(d, ((ttl - 1) << 24) | ((uint32_t)r & 0x00FFFFFFu));
          }
      }
      return AGX_RES_SAME;
    case AGX_KIND_FORWARD_RR:
      if constexpr ((KM & kb(AGX_KIND_FORWARD_RR)) != 0) {
        w[0] += 1;
        if (pay > 0) {
          uint64_t b = P.row_ptr[local], deg = P.row_ptr[local + 1] - b;
          if (deg) {
            // cursor mod degree; 32-bit remainder when both fit (the common case)
            uint64_t r = (w[1] <= 0xFFFFFFFFull && deg <= 0xFFFFFFFFull) ? (uint64_t)((uint32_t)w[1] % (uint32_t)deg)
                                                                         : w[1] % deg;
            uint64_t e = b + r;
            w[1] += 1;
            emit(P.col[e], pay - 1);
          }
        }
      }
      return AGX_RES_SAME;
    case AGX_KIND_STOP_AFTER:
      if constexpr ((KM & kb(AGX_KIND_STOP_AFTER)) != 0) {
        w[0] += 1;
        return (w[0] >= w[1]) ? AGX_RES_STOPPED : AGX_RES_SAME;
      }
      return AGX_RES_SAME;
    case AGX_KIND_PINGPONG:
      if constexpr ((KM & kb(AGX_KIND_PINGPONG)) != 0) {
        // BenchmarkActors.PingPong (akka-bench-jmh/.../actor/BenchmarkActors.scala:20-32)
        uint32_t res = (w[0] == 0) ? AGX_RES_STOPPED : AGX_RES_SAME;
        w[1] += 1;
        emit(src, pay);
        w[0] -= 1;
        return res;
      }
      return AGX_RES_SAME;
    case AGX_KIND_EVEN:
      if constexpr ((KM & kb(AGX_KIND_EVEN)) != 0) {
        if (pay & 1u) return AGX_RES_UNHANDLED;
        w[0] += 1;
      }
      return AGX_RES_SAME;
    default:
      return AGX_RES_SAME;
  }
}

}  // namespace agx
