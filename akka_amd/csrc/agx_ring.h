// agx_ring.h — bounded mailboxes whose queued messages stay put (single-rank multi-pass engines).
//
// A BoundedMailbox's queue is a linked list of nodes: an enqueued message is written once, stays
// where it is while it waits, and is read once when it is dequeued
// (akka-actor/src/main/java/akka/dispatch/AbstractBoundedNodeQueue.java:92-113, 155-173).  The BSP
// backlog arena re-copies every queued message every superstep instead (the backlog
// is rewritten into the other parity's arena), which at 10^8 actors under BoundedMailbox(64) is the
// bulk of the superstep's HBM traffic (round 3: 13x the algorithmic bytes, most of it re-streamed
// backlog).  In ring mode every actor owns a ring of `rc` (the largest mailbox capacity) message
// slots plus one word head | length << 16, and one kernel per superstep (k_ring_apply, a block per
// bucket of 2048 actors) does what the four-kernel skew path and the block apply did:
//
//   arrivals  = the bucket's sorted new mail (radix passes, canonical order inside every actor);
//   per actor (Mailbox.scala:260-277 processMailbox, :551-565 bounded enqueue), with L queued,
//     rr  = alive ? min(L, T) : 0                 ring messages drained (the oldest first),
//     adm = alive ? min(arrivals, C - L) : 0      arrivals admitted (tail-drop beyond C),
//     da  = min(adm, T - rr)                      admitted arrivals drained after them,
//     the other adm - da admitted arrivals are appended to the ring (written once);
//   a stopped actor's ring and arrivals are dead letters (AbstractDispatcher.scala:221-227).
// This is bucket_finish's rule over the inbox [queued ++ arrivals] -- keep = min(len, C), drained =
// min(keep, T), the rest queued -- with the queued part never moved.
//
// Drained messages (ring heads, then the arrivals of rank < da) are gathered actor by actor into a
// drain buffer (LDS when the bucket drains <= kBucket messages, else the bucket's slice of a global
// scratch), applied in order (apply_msg), and each drained message's tell (max_emit 1) is staged over
// its own consumed slot, then compacted in sender order into the bucket's slice of the tell arena --
// the chunk the next superstep's radix passes read.  Per superstep a queued message costs one append
// and one read, never a copy per superstep it waits; an arrival to a full mailbox costs one key read.
#pragma once

namespace agx {

constexpr uint32_t kRingApplyMaxC = 0xFFFFu;  // head / length are 16-bit fields
constexpr uint32_t kRingListBatch = 32;      // marked buckets found per ballot (after k_ring_tiny)

struct RingArgs {
  uint32_t* state;   // [n_local] head | len << 16
  uint32_t* src;     // [n_local][rc]
  uint32_t* pay;
  uint32_t* dk;      // drain scratch / tell staging, [nb][kBucket * dstride] (buckets draining > kBucket)
  uint32_t* ds;
  uint32_t* dp;
  unsigned long long* total;  // messages held in rings (in flight)
  uint32_t* nz;      // [nb][kBucket / 32] one bit per actor: its ring holds mail (the wave path's scan)
  uint32_t rc;       // ring slots per actor (>= every mailbox class's capacity)
  uint32_t dstride;  // drain slots per actor of a bucket's slice (the largest throughput)
};

struct RingLds {
  uint32_t whist32[kBWaves * kBucket / 2];  // 32 KB: u16 per-wave actor counts (ranking), then the staged tell keys
  uint32_t cnt[kBucket];                    // arrivals per actor, then the running count over tiles
  uint32_t dpos[kBucket];                   // drain slot of the actor's first admitted arrival
  uint32_t dadm[kBucket];                   // da | adm << 16
  uint16_t tail[kBucket];                   // ring slot of the actor's first appended arrival
  uint32_t bsrc[kBucket], bpay[kBucket];    // LDS drain buffer (a bucket that drains <= kBucket)
  uint32_t nh[kRadix];                      // next first-pass digit histogram of the bucket's tells
  uint32_t scratch[2 * (kBWaves + 1)];
};

template <uint32_t KM>
static __global__ void __launch_bounds__(kBThreads, 4) k_ring_apply(BucketArgs a, RingArgs g) {
  __shared__ RingLds S;
  uint16_t* const whist = reinterpret_cast<uint16_t*>(S.whist32);
  const DevParams& P = a.P;
  const uint32_t tid = threadIdx.x, w = tid / kWave, lane = lane_id();
  const uint64_t ltm = lanemask_lt();
  const uint32_t amask = (1u << a.bb) - 1u, nhmask = (1u << a.nx_bits) - 1u;
  const InView iv = in_view(a);
  const uint32_t rc = g.rc;
  if (blockIdx.x == 0) {
    if (tid == 0 && *a.d_ninbox > 0) atomicAdd((unsigned long long*)&a.stats[ST_STEPS], 1ull);
    for (uint32_t i = tid; i < kStagedChunks; i += kBThreads) a.chunk_cnt[2 * a.nb + i] = 0;  // staged consumed
  }
  const uint32_t *Mk = sgpr_ptr(iv.m.key), *Ms = sgpr_ptr(iv.m.src), *Mp = sgpr_ptr(iv.m.pay);
  uint32_t acc[kBStats] = {0u, 0u, 0u, 0u, 0u};  // delivered, dead letters, unhandled, tells, active actors
  long long dring = 0;                           // this thread's change of the messages held in rings
  // after k_ring_tiny (a.blist set): only the buckets it marked, found kListBatch at a time by one
  // ballot (k_bucket_apply's listed mode)
  const bool listed = a.blist != nullptr;
  __shared__ uint32_t s_todo;
  for (uint32_t it = blockIdx.x; it < a.nb; it += (listed ? kRingListBatch : 1u) * gridDim.x) {
  uint32_t todo = 1u;
  if (listed) {
    if (w == 0) {
      const uint32_t bw = it + lane * gridDim.x;
      const uint64_t mk = __ballot(lane < kRingListBatch && bw < a.nb && a.blist[bw] != 0u);
      if (lane == 0) s_todo = (uint32_t)mk;
    }
    __syncthreads();
    todo = s_todo;
    __syncthreads();
  }
  for (; todo; todo &= todo - 1u) {
    const uint32_t b = it + (uint32_t)__builtin_ctz(todo) * gridDim.x;
    const uint32_t a0 = b << a.bb;
    const uint32_t na = min(1u << a.bb, P.n_local - a0);
    AGX_STAMP(a, 0);
    const uint32_t bs = a.bstart[b], n = a.bstart[b + 1] - bs;
    // ---- this thread's four actors (blocked: la = 4 tid + j): flags, limits, ring words
    const uint32_t la0 = tid * kBAct;
    uint32_t alive4 = *reinterpret_cast<const uint32_t*>(P.alive + a0 + la0);  // (padded to whole buckets)
    if (la0 + kBAct > na) alive4 &= la0 >= na ? 0u : 0xFFFFFFFFu >> (8 * (kBAct - (na - la0)));
    uint32_t rsv[kBAct] = {0u, 0u, 0u, 0u};
    if (la0 + kBAct <= na) {
      const uint4 v = *reinterpret_cast<const uint4*>(g.state + a0 + la0);
      rsv[0] = v.x; rsv[1] = v.y; rsv[2] = v.z; rsv[3] = v.w;
    } else {
#pragma unroll
      for (int j = 0; j < kBAct; ++j) rsv[j] = la0 + j < na ? g.state[a0 + la0 + j] : 0u;
    }
    for (uint32_t i = tid; i < kBucket; i += kBThreads) S.cnt[i] = 0;
    for (uint32_t d = tid; d < kRadix; d += kBThreads) S.nh[d] = 0;
    __syncthreads();
    // ---- arrivals per actor (keys only: an arrival to a full mailbox costs this one read)
    const uint32_t wbase = w * (kBIpt * kWave);
    uint32_t k[kBIpt];
    for (uint32_t t0 = 0; t0 < n; t0 += 2 * kBucket) {  // (two tiles' key loads in flight: hub buckets)
      uint32_t ix[2 * kBIpt], k2[2 * kBIpt];
#pragma unroll
      for (int r = 0; r < 2 * kBIpt; ++r) {
        const uint32_t q = t0 + (r / kBIpt) * kBucket + wbase + (r % kBIpt) * kWave + lane;
        ix[r] = q < n ? iv.at(bs + q) : 0u;
      }
#pragma unroll
      for (int r = 0; r < 2 * kBIpt; ++r) k2[r] = ldg(Mk, ix[r]);
#pragma unroll
      for (int r = 0; r < 2 * kBIpt; ++r)  // (a hot actor's wave of arrivals: one aggregated LDS atomic)
        if (t0 + (r / kBIpt) * kBucket + wbase + (r % kBIpt) * kWave + lane < n) lds_hist_inc(S.cnt, k2[r] & amask);
    }
    __syncthreads();
    AGX_STAMP(a, 1);
    // ---- per actor: admission, drain and ring bookkeeping (kept in LDS: rr = dpos - ds, da | adm)
    uint32_t ds[kBAct];
    uint32_t dsum = 0, ndead = 0;
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      const uint32_t la = la0 + j, ab = (alive4 >> (8 * j)) & 0xFFu, arr = S.cnt[la];
      uint32_t C, T;
      mbox_limits(P, ab, C, T);
      const uint32_t H = rsv[j] & 0xFFFFu, L = rsv[j] >> 16;
      const bool al = (ab & 1u) != 0;
      const uint32_t Lk = al ? min(L, C) : 0u;  // (L > C only after a class change: keep = min(len, C))
      const uint32_t rr = min(Lk, T);
      const uint32_t adm = al ? min(arr, C - Lk) : 0u;
      const uint32_t da = min(adm, T - rr);
      ndead += arr - adm + (L - Lk);  // tail-dropped arrivals and queued ones; a stopped actor's queue
      dsum += rr + da;
      S.dadm[la] = da | adm << 16;
      const uint32_t t = H + Lk;
      S.tail[la] = (uint16_t)(t < rc ? t : t - rc);
      S.dpos[la] = rr;  // (+ the segment start below)
    }
    uint32_t D;
    uint32_t dseg = block_excl_sum<kBThreads>(dsum, S.scratch, &D);  // (syncs: S.cnt reads done)
    const bool lds_drain = D <= (uint32_t)kBucket;
    const size_t sbase = (size_t)b * kBucket * g.dstride;  // the bucket's slice of the global scratch
    uint32_t* const bsrc = lds_drain ? S.bsrc : g.ds + sbase;
    uint32_t* const bpay = lds_drain ? S.bpay : g.dp + sbase;
    uint32_t rmax = 0;
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      const uint32_t la = la0 + j, rr = S.dpos[la], dd = S.dadm[la];
      ds[j] = dseg;
      S.dpos[la] = dseg + rr;
      S.cnt[la] = 0;  // (from here: admitted arrivals placed by earlier tiles)
      dseg += rr + (dd & 0xFFFFu);
      rmax = max(rmax, rr);
    }
    AGX_STAMP(a, 2);
    // ring heads -> the front of each actor's drain segment (a thread's loads of one position together)
    for (uint32_t q = 0; q < rmax; ++q) {
      uint32_t hs[kBAct], hp[kBAct], rr[kBAct];
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        rr[j] = S.dpos[la0 + j] - ds[j];
        uint32_t x = (rsv[j] & 0xFFFFu) + q;
        x = x < rc ? x : x - rc;
        // (an actor with no ring head to drain -- past n_local in the last bucket too -- reads slot 0
        // of the bucket's first actor: the rings are allocated for exactly n_local actors)
        const size_t o = q < rr[j] ? (size_t)(a0 + la0 + j) * rc + x : (size_t)a0 * rc;
        hs[j] = g.src[o];
        hp[j] = g.pay[o];
      }
#pragma unroll
      for (int j = 0; j < kBAct; ++j)
        if (q < rr[j]) {
          bsrc[ds[j] + q] = hs[j];
          bpay[ds[j] + q] = hp[j];
        }
    }
    __syncthreads();
    AGX_STAMP(a, 3);
    // ---- placement: stable rank of every admitted arrival among its actor's arrivals; ranks < da to
    // the drain buffer, the rest of the admitted ones appended to the ring
    for (uint32_t t0 = 0; t0 < n; t0 += kBucket) {
      {  // (a single-tile bucket's keys come back from the L2: its count pass just read them)
        uint32_t ix[kBIpt];
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          const uint32_t q = t0 + wbase + r * kWave + lane;
          ix[r] = q < n ? iv.at(bs + q) : 0u;
        }
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) k[r] = ldg(Mk, ix[r]);
      }
      bool live[kBIpt];
      int any = 0;
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) {
        const uint32_t q = t0 + wbase + r * kWave + lane, la = k[r] & amask;
        // an actor whose admitted arrivals were all placed by earlier tiles: a dead letter, not ranked
        live[r] = q < n && S.cnt[la] < (S.dadm[la] >> 16);
        any |= live[r];
      }
      if (!__syncthreads_or(any)) continue;  // (uniform) every arrival of this tile is a dead letter
      uint32_t sv[kBIpt], pv[kBIpt];
      {
        uint32_t ix[kBIpt];
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          const uint32_t q = t0 + wbase + r * kWave + lane;
          ix[r] = live[r] ? iv.at(bs + q) : 0u;
        }
#pragma unroll
        for (int r = 0; r < kBIpt; ++r) {
          sv[r] = ldg(Ms, ix[r]);
          pv[r] = ldg(Mp, ix[r]);
        }
      }
      for (uint32_t x = tid; x < kBWaves * kBucket / 2; x += kBThreads) S.whist32[x] = 0;
      __syncthreads();
      uint32_t rk[kBIpt];
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) rk[r] = wave_rank(live[r], k[r] & amask, a.bb, whist + w * kBucket, ltm);
      __syncthreads();
      uint32_t tt[kBAct];  // this tile's live arrivals of the thread's actors
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {  // earlier waves' counts: exclusive prefix over the waves, in place
        const uint32_t la = la0 + j;
        uint32_t run = 0;
#pragma unroll
        for (int x = 0; x < kBWaves; ++x) {
          const uint32_t c2 = whist[x * kBucket + la];
          whist[x * kBucket + la] = (uint16_t)run;
          run += c2;
        }
        tt[j] = run;
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) {
        if (!live[r]) continue;
        const uint32_t la = k[r] & amask;
        const uint32_t rank = S.cnt[la] + whist[w * kBucket + la] + rk[r];
        const uint32_t dd = S.dadm[la], da = dd & 0xFFFFu, adm = dd >> 16;
        if (rank < da) {
          bsrc[S.dpos[la] + rank] = sv[r];
          bpay[S.dpos[la] + rank] = pv[r];
        } else if (rank < adm) {
          uint32_t x = S.tail[la] + (rank - da);
          x = x < rc ? x : x - rc;
          const size_t o = (size_t)(a0 + la) * rc + x;
          g.src[o] = sv[r];
          g.pay[o] = pv[r];
        }
      }
      __syncthreads();  // (every rank of this tile formed before the running counts advance)
#pragma unroll
      for (int j = 0; j < kBAct; ++j) S.cnt[la0 + j] += tt[j];
      __syncthreads();
    }
    AGX_STAMP(a, 4);
    // ---- state of the actors that drain (issued here, used by the drain).  FORWARD_RR (C5): each
    // actor's out-edge row and the destination of its next round-robin edge, all four actors' loads
    // together (bucket_finish's hint: no dependent row_ptr -> col loads inside the serial drain)
    uint64_t w0[kBAct], w1[kBAct];
    uint32_t kd[kBAct], drn[kBAct];
    constexpr bool kKindNeeded = (KM & (KM - 1)) != 0 || (KM & kb(AGX_KIND_COMPILED)) != 0;
    constexpr bool kFwd = KM == kb(AGX_KIND_FORWARD_RR);
    constexpr bool kFan = KM == kb(AGX_KIND_FANOUT);
    constexpr uint32_t kNoHint = 0xFFFFFFFFu;
    uint64_t frb[kBAct], fre[kBAct];
#pragma unroll
    for (int j = 0; j < kBAct; ++j) drn[j] = S.dpos[la0 + j] - ds[j] + (S.dadm[la0 + j] & 0xFFFFu);
    // (before the state loads: their registers are not live across the lookups)
    // FANOUT with one tell per message (C3 steady): every drained message's Zipf destination (index
    // range, binary search, permutation), written over the message's sender (FANOUT does not read it)
    const bool fan_pre = kFan && P.fan_k == 1;
    uint32_t* const skey = lds_drain ? S.whist32 : g.dk + sbase;  // (tell staging; free until the drain)
    if (kFan && fan_pre) {
      // every drain slot's actor into the staging area, then the whole block looks up the slots'
      // Zipf destinations, four per thread in lockstep (independent chains, not one per actor)
#pragma unroll
      for (int j = 0; j < kBAct; ++j)
        for (uint32_t q = 0; q < drn[j]; ++q) skey[ds[j] + q] = a0 + la0 + j;
      __syncthreads();
      for (uint32_t j0 = tid; j0 < D; j0 += 4 * kBThreads) {
        uint32_t uu[4], lo[4], hi[4];
        bool need[4];
        bool dir[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t j = j0 + c * kBThreads, pv = j < D ? bpay[j] : 0u;
          need[c] = j < D && (pv >> 24) > 0;
          uu[c] = need[c] ? (uint32_t)(fanout_rand(P.fan_seed, skey[j], pv & 0x00FFFFFFu, 0) >> 32) : 0u;
          const uint32_t t = uu[c] >> (32 - kZipfBits);
          const uint2 z = need[c] ? P.zipf_ent[t] : make_uint2(0u, 0u);
          dir[c] = z.y == kZipfDirect;  // (the Zipf head: the destination itself, no search)
          lo[c] = z.x;
          hi[c] = dir[c] ? z.x : z.y;
        }
        for (;;) {
          bool more = false;
          uint32_t cv[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) cv[c] = lo[c] < hi[c] ? P.zipf_cdf[(lo[c] + hi[c]) >> 1] : 0u;
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (lo[c] < hi[c]) {
              const uint32_t mid = (lo[c] + hi[c]) >> 1;
              if (cv[c] >= uu[c]) hi[c] = mid; else lo[c] = mid + 1;
              more |= lo[c] < hi[c];
            }
          if (!more) break;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (need[c]) bsrc[j0 + c * kBThreads] = dir[c] ? lo[c] : P.zipf_perm[lo[c]];
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < kBAct; ++j) {
      const uint32_t l = drn[j] ? a0 + la0 + j : a0;  // (no drain: a harmless cached load, masked below)
      w0[j] = ldg64(P.state, sidx(P, l, 0));
      w1[j] = P.W > 1 ? ldg64(P.state, sidx(P, l, 1)) : 0ull;
      kd[j] = kKindNeeded ? P.kind[l] : 0u;
      if constexpr (kFwd) {
        frb[j] = P.row_ptr[l];
        fre[j] = P.row_ptr[l + 1];
      }
    }
    if constexpr (kFwd) {  // the hint (degree, first destination) -> LDS (S.cnt / S.dpos are free now)
      uint32_t fdst[kBAct];
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        const uint64_t deg = fre[j] - frb[j];
        const bool ok = drn[j] && deg < kNoHint && w1[j] <= 0xFFFFFFFFull;
        S.cnt[la0 + j] = ok ? (uint32_t)deg : kNoHint;
        fdst[j] = ok && deg ? P.col[frb[j] + (uint32_t)w1[j] % (uint32_t)deg] : 0u;
      }
#pragma unroll
      for (int j = 0; j < kBAct; ++j) S.dpos[la0 + j] = fdst[j];
    }
    AGX_STAMP(a, 5);
    // ---- drain + apply, actor after actor; tell e of an actor is staged at its drain slot e (already
    // consumed: tell e comes from a message at slot >= e)
    uint32_t ecl[kBAct];
    uint32_t esum = 0;
#pragma unroll 1
    for (int j = 0; j < kBAct; ++j) {
      ecl[j] = 0;
      if (!drn[j]) continue;
      const uint32_t la = la0 + j, l = a0 + la;
      const uint32_t self = l;  // (single rank: local id = global id)
      EmitterLds em{&P, skey + ds[j], bsrc + ds[j], bpay + ds[j], 0, self, 0, 0, S.nh, a.nx_shift, nhmask};
      uint64_t wv[2] = {w0[j], w1[j]};
      uint32_t kcur = kd[j];
      ++acc[4];
      uint32_t hdeg = kNoHint, hdst = 0;
      bool fresh = true;  // no forward yet: the next edge is hdst
      if constexpr (kFwd) {
        hdeg = S.cnt[la];
        hdst = S.dpos[la];
      }
      for (uint32_t q = 0; q < drn[j]; ++q) {
        const uint32_t s = bsrc[ds[j] + q], p = bpay[ds[j] + q];
        uint32_t r;
        if (kFan && fan_pre) {  // apply_msg's FANOUT with the destination looked up above (in s)
          wv[0] += 1;
          wv[1] += p;
          const uint32_t ttl = p >> 24;
          if (ttl > 0) {
            const uint64_t rr = fanout_rand(P.fan_seed, self, p & 0x00FFFFFFu, 0);
            em(s, ((ttl - 1) << 24) | ((uint32_t)rr & 0x00FFFFFFu));
          }
          r = AGX_RES_SAME;
        } else if (kFwd && hdeg != kNoHint && wv[1] <= 0xFFFFFFFFull) {
          // apply_msg's FORWARD_RR with the prefetched row (same cursor arithmetic)
          wv[0] += 1;
          if (p > 0 && hdeg) {
            const uint32_t d = fresh ? hdst : P.col[P.row_ptr[l] + (uint32_t)wv[1] % hdeg];
            fresh = false;
            wv[1] += 1;
            em(d, p - 1);
          }
          r = AGX_RES_SAME;
        } else {
          r = apply_msg<KM>(P, kcur, self, l, wv, s, p, em);
        }
        ++acc[0];
        if (r == AGX_RES_UNHANDLED) ++acc[2];
        if (r == AGX_RES_STOPPED) {
          P.stopq[atomicAdd(P.nstop, 1u)] = l;
          ndead += drn[j] - q - 1;  // drained-but-unprocessed after the stop
          break;
        }
      }
      stg64(P.state, sidx(P, l, 0), wv[0]);
      if (P.W > 1) stg64(P.state, sidx(P, l, 1), wv[1]);
      if constexpr ((KM & kb(AGX_KIND_COMPILED)) != 0)
        if (kcur != kd[j]) P.kind[l] = (uint8_t)kcur;
      acc[3] += em.n_all;
      ndead += em.n_all - em.n_valid;
      ecl[j] = em.n_valid;
      esum += em.n_valid;
    }
    AGX_STAMP(a, 6);
    // ---- tells in sender order into the bucket's slice of the tell arena
    uint32_t emtot;
    uint32_t eo = block_excl_sum<kBThreads>(esum, S.scratch, &emtot);  // (syncs: staging complete)
    const uint64_t embase = (uint64_t)b * kBucket * g.dstride;
    if (lds_drain) {
#pragma unroll 1
      for (int j = 0; j < kBAct; ++j) {
        for (uint32_t e = 0; e < ecl[j]; ++e) {
          a.em.key[embase + eo + e] = skey[ds[j] + e];
          a.em.src[embase + eo + e] = bsrc[ds[j] + e];
          a.em.pay[embase + eo + e] = bpay[ds[j] + e];
        }
        eo += ecl[j];
      }
    } else {  // staged in the bucket's global slice (hub buckets draining > kBucket): one LDS index of
              // source slots (S.whist32 is free here), then a block-wide copy with independent loads
      constexpr uint32_t kMap = kBWaves * kBucket / 2;
      for (uint32_t base = 0; base < emtot; base += kMap) {
        uint32_t o = eo;
#pragma unroll 1
        for (int j = 0; j < kBAct; ++j)
          for (uint32_t e = 0; e < ecl[j]; ++e, ++o)
            if (o >= base && o < base + kMap) S.whist32[o - base] = ds[j] + e;
        __syncthreads();
        const uint32_t m = min(kMap, emtot - base);
#pragma unroll 4
        for (uint32_t i = tid; i < m; i += kBThreads) {
          const uint32_t x = S.whist32[i];
          a.em.key[embase + base + i] = skey[x];
          a.em.src[embase + base + i] = bsrc[x];
          a.em.pay[embase + base + i] = bpay[x];
        }
        __syncthreads();
      }
    }
    AGX_STAMP(a, 7);
    // ---- ring words, chunk entries, next first-pass histogram column
    {
      uint32_t nv[kBAct];
#pragma unroll
      for (int j = 0; j < kBAct; ++j) {
        const uint32_t ab = (alive4 >> (8 * j)) & 0xFFu;
        uint32_t C, T;
        mbox_limits(P, ab, C, T);
        const uint32_t H = rsv[j] & 0xFFFFu, L = rsv[j] >> 16, dd = S.dadm[la0 + j];
        const uint32_t Lk = (ab & 1u) ? min(L, C) : 0u;
        const uint32_t da = dd & 0xFFFFu, rr = drn[j] - da, qa = (dd >> 16) - da;
        const uint32_t nl = Lk - rr + qa;
        uint32_t h = H + rr;
        h = h < rc ? h : h - rc;
        nv[j] = nl ? (h | nl << 16) : 0u;
        dring += (long long)nl - (long long)L;
      }
      if (la0 + kBAct <= na) {
        *reinterpret_cast<uint4*>(g.state + a0 + la0) = make_uint4(nv[0], nv[1], nv[2], nv[3]);
      } else {
#pragma unroll
        for (int j = 0; j < kBAct; ++j)
          if (la0 + j < na) g.state[a0 + la0 + j] = nv[j];
      }
      // the bucket's non-empty-ring bits (S.cnt is free here): thread t's four actors are bits
      // 4 t .. 4 t + 3 of the bucket
      uint32_t nib = 0;
#pragma unroll
      for (int j = 0; j < kBAct; ++j) nib |= (nv[j] != 0u ? 1u : 0u) << j;
      if (tid < kBucket / 32) S.cnt[tid] = 0u;
      __syncthreads();
      if (nib) atomicOr(&S.cnt[la0 >> 5], nib << (la0 & 31u));
      __syncthreads();
      if (tid < kBucket / 32) g.nz[(size_t)b * (kBucket / 32) + tid] = S.cnt[tid];
    }
    acc[1] += ndead;
    if (tid == 0) {
      a.chunk_off[b] = bs;
      a.chunk_cnt[b] = 0u;  // (no backlog: queued messages are in the rings)
      a.chunk_off[a.nb + b] = (uint32_t)embase;
      a.chunk_cnt[a.nb + b] = emtot;
      if (a.emmeta) a.emmeta[b] = make_uint4(0u, 0u, 2u, 0u);  // (not summarised: forces the radix passes)
    }
    __syncthreads();  // (S.nh complete)
    for (uint32_t d = tid; d < (1u << a.nx_bits); d += kBThreads)
      if (S.nh[d]) atomicAdd(&a.nhist[(size_t)d * a.nhist_stride + a.ng + b / a.G], S.nh[d]);
    __syncthreads();  // (LDS reused by the next bucket)
    AGX_STAMP(a, 8);
  }
  }
  if (blockIdx.x < a.nb) flush_stats(a, acc);
  // messages held in rings: the block's change, two's complement into the u64 total
  const uint32_t gp = wave_incl_sum(dring > 0 ? (uint32_t)dring : 0u), gn = wave_incl_sum(dring < 0 ? (uint32_t)-dring : 0u);
  if (lane == kWave - 1 && gp != gn) atomicAdd(g.total, (unsigned long long)((long long)gp - (long long)gn));
}


// ---- Wave-per-bucket ring apply.  A sparse superstep (C3: 4883 buckets of a few dozen arrivals
// and a handful of actors with queued mail each) is dominated by the block kernel's per-bucket
// chain of phases, so -- as k_tiny_apply does for the backlog arena -- every bucket whose arrivals
// fit kRingTinyN, whose actors with work (arrivals or a non-empty ring) fit kTinyMax and whose drains
// fit kRingTinyD is done by one wave; k_ring_apply then takes only the buckets marked in a.blist.
// Same per-actor rule as k_ring_apply (admission, ring heads first, appends, dead letters), same
// tell order (actor order), same ring words.
#ifndef AGX_RING_IPL
#define AGX_RING_IPL 2  // arrivals per lane of the wave path (A/B build knob)
#endif
#ifndef AGX_RING_DPL
#define AGX_RING_DPL 4  // drained messages per lane of the wave path (A/B build knob)
#endif
constexpr uint32_t kRingIpl = AGX_RING_IPL;
constexpr uint32_t kRingTinyN = kRingIpl * kWave;         // arrivals of a wave-path bucket
constexpr uint32_t kRingTinyD = AGX_RING_DPL * kWave;     // drained messages of a wave-path bucket
static_assert(AGX_RING_DPL % 4 == 0, "lockstep passes of four drain slots per lane");
static_assert(kBucket == 32 * kWave, "lane l owns the ring words of actors [32 l, 32 l + 32)");

struct RingTinyLds {                              // one per wave (5.6 KB at 2 arrivals / 4 drains per lane)
  uint32_t src[kRingTinyN], pay[kRingTinyN];      // arrivals by (actor, inbox position)
  uint32_t dk[kRingTinyD], ds[kRingTinyD], dp[kRingTinyD];  // drained messages, then the staged tells
  uint32_t am[kWave], mw[kWave], pw[kWave];       // arrival bits, active bits, active prefix per 32 actors
  uint16_t act[kTinyMax], ast[kTinyMax], alen[kTinyMax];  // active actors in order; their arrival runs
};

struct RingStageEmitter {  // max_emit 1: tell e of a message staged at its drain slot's run (e <= slot)
  const DevParams* P;
  uint32_t *key, *src, *pay;
  uint32_t slot, self;
  uint32_t n_valid, n_all;
  __device__ __forceinline__ void operator()(uint32_t dst, uint32_t p) {
    if (dst >= P->n_global) {  // the reply path (outbox) or an unknown ref -> deadLetters
      if (!outbound_tell(*P, dst, self, p, true)) ++n_all;
      return;
    }
    ++n_all;
    ++n_valid;
    key[slot] = dst;
    src[slot] = self;
    pay[slot] = p;
    ++slot;
  }
  __device__ __forceinline__ void wide(uint32_t, uint32_t) {}
};

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// returns false (nothing written) when the bucket exceeds the wave path's bounds
template <uint32_t KM>
__device__ __forceinline__ bool ring_tiny_bucket(const BucketArgs& a, const RingArgs& g, const InView& iv,
                                                 RingTinyLds& T, uint32_t b, uint32_t bs, uint32_t n) {
  const DevParams& P = a.P;
  const uint32_t lane = lane_id(), rc = g.rc;
  const uint32_t amask = (1u << a.bb) - 1u, a0 = b << a.bb;
  const uint32_t na = min(1u << a.bb, P.n_local - a0);
  // ---- actors with queued mail: one bit each, lane l holding actors [32 l, 32 l + 32)
  const uint32_t rm = g.nz[(size_t)b * kWave + lane];
  // ---- arrivals: stable rank by (actor, position), run starts / lengths (tiny_bucket's rank loop)
  uint32_t k[kRingIpl], sv[kRingIpl], pv[kRingIpl], la[kRingIpl];
#pragma unroll
  for (uint32_t r = 0; r < kRingIpl; ++r) {
    const uint32_t q = r * kWave + lane;
    const uint32_t i = q < n ? iv.at(bs + q) : 0u;
    k[r] = q < n ? ldg(iv.m.key, i) : 0u;
    sv[r] = q < n ? ldg(iv.m.src, i) : 0u;
    pv[r] = q < n ? ldg(iv.m.pay, i) : 0u;
  }
#pragma unroll
  for (uint32_t r = 0; r < kRingIpl; ++r) la[r] = r * kWave + lane < n ? k[r] & amask : 0xFFFFFFFFu;
  T.am[lane] = 0u;
  wave_sync_lds();
  uint32_t rank[kRingIpl] = {}, st[kRingIpl] = {}, len[kRingIpl] = {};
#pragma unroll
  for (uint32_t r2 = 0; r2 < kRingIpl; ++r2) {
    const uint32_t jn = n > r2 * kWave ? min(n - r2 * kWave, (uint32_t)kWave) : 0u;
    for (uint32_t jj = 0; jj < jn; ++jj) {
      const uint32_t lj = (uint32_t)__builtin_amdgcn_readlane((int)la[r2], (int)jj), j = r2 * kWave + jj;
#pragma unroll
      for (uint32_t r = 0; r < kRingIpl; ++r) {
        const bool lt = lj < la[r], eq = lj == la[r];
        st[r] += lt;
        len[r] += eq;
        rank[r] += lt || (eq && j < r * kWave + lane);
      }
    }
  }
#pragma unroll
  for (uint32_t r = 0; r < kRingIpl; ++r)
    if (r * kWave + lane < n) {
      T.src[rank[r]] = sv[r];
      T.pay[rank[r]] = pv[r];
      if (rank[r] == st[r]) atomicOr(&T.am[la[r] >> 5], 1u << (la[r] & 31u));
    }
  wave_sync_lds();
  // ---- the active actors (arrivals or queued mail) in actor order
  const uint32_t m = rm | T.am[lane], c = __builtin_popcount(m);
  const uint32_t cinc = wave_incl_sum(c), A = (uint32_t)__builtin_amdgcn_readlane((int)cinc, kWave - 1);
  if (A > kTinyMax) return false;
  uint32_t pe = cinc - c;
  T.mw[lane] = m;
  T.pw[lane] = pe;
  for (uint32_t mm = m; mm; mm &= mm - 1u, ++pe) {
    T.act[pe] = (uint16_t)(lane * 32u + (uint32_t)__builtin_ctz(mm));
    T.alen[pe] = 0;
  }
  wave_sync_lds();
#pragma unroll
  for (uint32_t r = 0; r < kRingIpl; ++r)
    if (r * kWave + lane < n && rank[r] == st[r]) {  // run head: its actor's active index
      const uint32_t wd = la[r] >> 5, idx = T.pw[wd] + __builtin_popcount(T.mw[wd] & ((1u << (la[r] & 31u)) - 1u));
      T.ast[idx] = (uint16_t)st[r];
      T.alen[idx] = (uint16_t)len[r];
    }
  wave_sync_lds();
  // ---- per active actor (lane j: active actors kTinyIpl j + i, so lane order is actor order)
  uint32_t hl[kTinyIpl], sw[kTinyIpl], ab[kTinyIpl], hk[kTinyIpl], rr[kTinyIpl], da[kTinyIpl], adm[kTinyIpl],
      Lk[kTinyIpl], arr[kTinyIpl], as0[kTinyIpl];
  uint64_t w0[kTinyIpl], w1[kTinyIpl];
  bool on[kTinyIpl];
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i) {
    const uint32_t x = lane * kTinyIpl + i;
    on[i] = x < A;
    hl[i] = on[i] ? a0 + T.act[x] : a0;
    arr[i] = on[i] ? T.alen[x] : 0u;
    as0[i] = on[i] ? T.ast[x] : 0u;
  }
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i) {  // (all loads in flight together)
    sw[i] = on[i] ? g.state[hl[i]] : 0u;
    ab[i] = on[i] ? P.alive[hl[i]] : 0u;
    hk[i] = on[i] ? P.kind[hl[i]] : 0u;
    w0[i] = on[i] ? ldg64(P.state, sidx(P, hl[i], 0)) : 0ull;
    w1[i] = on[i] && P.W > 1 ? ldg64(P.state, sidx(P, hl[i], 1)) : 0ull;
  }
  uint32_t ndead = 0, dl = 0;
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i) {
    uint32_t C, Tt;
    mbox_limits(P, ab[i], C, Tt);
    const uint32_t L = sw[i] >> 16;
    const bool al = on[i] && (ab[i] & 1u) != 0;
    Lk[i] = al ? min(L, C) : 0u;
    rr[i] = min(Lk[i], Tt);
    adm[i] = al ? min(arr[i], C - Lk[i]) : 0u;
    da[i] = min(adm[i], Tt - rr[i]);
    ndead += arr[i] - adm[i] + (L - Lk[i]);
    dl += rr[i] + da[i];
  }
  const uint32_t dinc = wave_incl_sum(dl), D = (uint32_t)__builtin_amdgcn_readlane((int)dinc, kWave - 1);
  if (D > kRingTinyD) return false;
  // ---- drain buffer: ring heads, then the drained arrivals; admitted arrivals beyond them -> ring
  uint32_t d0[kTinyIpl];
  {
    uint32_t o = dinc - dl;
#pragma unroll
    for (uint32_t i = 0; i < kTinyIpl; ++i) {
      d0[i] = o;
      o += rr[i] + da[i];
    }
  }
  // slot metadata: the actor (bit 31: a ring head, whose ring slot is in ds) or the arrival itself
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i) {
    const uint32_t h0 = sw[i] & 0xFFFFu;
    for (uint32_t q = 0; q < rr[i]; ++q) {
      const uint32_t x = h0 + q;
      T.dk[d0[i] + q] = hl[i] | 0x80000000u;
      T.ds[d0[i] + q] = x < rc ? x : x - rc;
    }
    for (uint32_t q = 0; q < da[i]; ++q) {
      T.dk[d0[i] + rr[i] + q] = hl[i];
      T.ds[d0[i] + rr[i] + q] = T.src[as0[i] + q];
      T.dp[d0[i] + rr[i] + q] = T.pay[as0[i] + q];
    }
    const uint32_t t0 = h0 + Lk[i];
    for (uint32_t q = da[i]; q < adm[i]; ++q) {  // appended: ring slot head + Lk + (rank - da)  (< 2 rc)
      const uint32_t x = t0 + (q - da[i]);
      const size_t o = (size_t)hl[i] * rc + (x < rc ? x : x - rc);
      g.src[o] = T.src[as0[i] + q];
      g.pay[o] = T.pay[as0[i] + q];
    }
  }
  wave_sync_lds();
  // ring heads: every drained ring message of the bucket, four slots per lane in lockstep per pass
  constexpr uint32_t kF = 4;
#pragma unroll 1
  for (uint32_t f0 = 0; f0 < kRingTinyD / kWave; f0 += kF) {
    uint32_t hs[kF], hp[kF];
    bool rg[kF];
#pragma unroll
    for (uint32_t f = 0; f < kF; ++f) {
      const uint32_t j = (f0 + f) * kWave + lane;
      const uint32_t dk = j < D ? T.dk[j] : 0u;
      rg[f] = (dk >> 31) != 0u;
      const size_t o = rg[f] ? (size_t)(dk & 0x7FFFFFFFu) * rc + T.ds[j] : 0u;
      hs[f] = rg[f] ? g.src[o] : 0u;
      hp[f] = rg[f] ? g.pay[o] : 0u;
    }
#pragma unroll
    for (uint32_t f = 0; f < kF; ++f)
      if (rg[f]) {
        T.ds[(f0 + f) * kWave + lane] = hs[f];
        T.dp[(f0 + f) * kWave + lane] = hp[f];
      }
  }
  wave_sync_lds();
  // FANOUT with one tell per message (C3 steady): every drained message's Zipf destination, the
  // wave's slots in lockstep (index range, each binary-search step's loads together, then the
  // permutation), written over the message's sender (FANOUT does not read it)
  constexpr bool kFan = KM == kb(AGX_KIND_FANOUT);
  const bool fan_pre = kFan && P.fan_k == 1;
  if (kFan && fan_pre) {
#pragma unroll 1
    for (uint32_t f0 = 0; f0 < kRingTinyD / kWave; f0 += kF) {
      uint32_t uu[kF], lo2[kF], hi2[kF];
      bool need[kF];
      bool dir[kF];
#pragma unroll
      for (uint32_t f = 0; f < kF; ++f) {
        const uint32_t j = (f0 + f) * kWave + lane, pv = j < D ? T.dp[j] : 0u;
        need[f] = j < D && (pv >> 24) > 0;
        uu[f] = need[f] ? (uint32_t)(fanout_rand(P.fan_seed, T.dk[j] & 0x7FFFFFFFu, pv & 0x00FFFFFFu, 0) >> 32) : 0u;
        const uint32_t t = uu[f] >> (32 - kZipfBits);
        const uint2 z = need[f] ? P.zipf_ent[t] : make_uint2(0u, 0u);
        dir[f] = z.y == kZipfDirect;  // (the Zipf head: the destination itself, no search)
        lo2[f] = z.x;
        hi2[f] = dir[f] ? z.x : z.y;
      }
      for (;;) {
        bool more = false;
        uint32_t cv[kF];
#pragma unroll
        for (uint32_t f = 0; f < kF; ++f) cv[f] = lo2[f] < hi2[f] ? P.zipf_cdf[(lo2[f] + hi2[f]) >> 1] : 0u;
#pragma unroll
        for (uint32_t f = 0; f < kF; ++f)
          if (lo2[f] < hi2[f]) {
            const uint32_t mid = (lo2[f] + hi2[f]) >> 1;
            if (cv[f] >= uu[f]) hi2[f] = mid; else lo2[f] = mid + 1;
            more |= lo2[f] < hi2[f];
          }
        if (!more) break;
      }
      uint32_t dd[kF];
#pragma unroll
      for (uint32_t f = 0; f < kF; ++f) dd[f] = need[f] ? (dir[f] ? lo2[f] : P.zipf_perm[lo2[f]]) : 0u;
#pragma unroll
      for (uint32_t f = 0; f < kF; ++f)
        if (need[f]) T.ds[(f0 + f) * kWave + lane] = dd[f];
    }
    wave_sync_lds();
  }
  // ---- drain + apply, actor after actor (tell e staged at drain slot d0 + e)
  uint32_t ndel = 0, nunh = 0, nall = 0, nact = 0, ncount = 0;
  uint32_t ecl[kTinyIpl];
  long long dring = 0;
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i) {
    ecl[i] = 0;
    const uint32_t drn = rr[i] + da[i], l = hl[i];
    if (drn) {
      ++nact;
      RingStageEmitter em{&P, T.dk + d0[i], T.ds + d0[i], T.dp + d0[i], 0, l, 0, 0};
      uint64_t wv[2] = {w0[i], w1[i]};
      uint32_t kcur = hk[i];
      for (uint32_t q = 0; q < drn; ++q) {
        const uint32_t s = T.ds[d0[i] + q], p = T.dp[d0[i] + q];
        uint32_t r;
        if (kFan && fan_pre) {  // apply_msg's FANOUT with the destination looked up above (in s)
          wv[0] += 1;
          wv[1] += p;
          const uint32_t ttl = p >> 24;
          if (ttl > 0) em(s, ((ttl - 1) << 24) | ((uint32_t)fanout_rand(P.fan_seed, l, p & 0x00FFFFFFu, 0) & 0x00FFFFFFu));
          r = AGX_RES_SAME;
        } else {
          r = apply_msg<KM>(P, kcur, l, l, wv, s, p, em);
        }
        ++ndel;
        if (r == AGX_RES_UNHANDLED) ++nunh;
        if (r == AGX_RES_STOPPED) {
          P.stopq[atomicAdd(P.nstop, 1u)] = l;
          ndead += drn - q - 1;  // drained-but-unprocessed after the stop
          break;
        }
      }
      P.state[sidx(P, l, 0)] = wv[0];
      if (P.W > 1) P.state[sidx(P, l, 1)] = wv[1];
      if constexpr ((KM & kb(AGX_KIND_COMPILED)) != 0)
        if (kcur != hk[i]) P.kind[l] = (uint8_t)kcur;
      nall += em.n_all;
      ndead += em.n_all - em.n_valid;
      ecl[i] = em.n_valid;
      ncount += em.n_valid;
    }
    if (on[i]) {  // the ring word: head past the drained ring messages, length after drains / appends
      const uint32_t L = sw[i] >> 16, nl = Lk[i] - rr[i] + (adm[i] - da[i]);
      uint32_t h = (sw[i] & 0xFFFFu) + rr[i];
      h = h < rc ? h : h - rc;
      const uint32_t nv = nl ? (h | nl << 16) : 0u;
      if (nv != sw[i]) g.state[l] = nv;
      dring += (long long)nl - (long long)L;
    }
  }
  // ---- the bucket's non-empty-ring bits after this superstep (T.am is free again)
  T.am[lane] = 0u;
  wave_sync_lds();
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i)
    if (on[i] && Lk[i] - rr[i] + (adm[i] - da[i]) != 0u) {
      const uint32_t x = hl[i] - a0;
      atomicOr(&T.am[x >> 5], 1u << (x & 31u));
    }
  wave_sync_lds();
  g.nz[(size_t)b * kWave + lane] = T.am[lane];
  // ---- tells in actor order into the bucket's slice of the tell arena
  const uint32_t tinc = wave_incl_sum(ncount), emtot = (uint32_t)__builtin_amdgcn_readlane((int)tinc, kWave - 1);
  const uint64_t embase = (uint64_t)b * kBucket * g.dstride;
  const uint32_t col = a.ng + b / a.G, nhmask = (1u << a.nx_bits) - 1u;
  uint32_t toff = tinc - ncount;
#pragma unroll
  for (uint32_t i = 0; i < kTinyIpl; ++i)
    for (uint32_t e = 0; e < ecl[i]; ++e, ++toff) {
      const uint32_t d = T.dk[d0[i] + e];
      a.em.key[embase + toff] = d;
      a.em.src[embase + toff] = T.ds[d0[i] + e];
      a.em.pay[embase + toff] = T.dp[d0[i] + e];
      atomicAdd(&a.nhist[(size_t)((d >> a.nx_shift) & nhmask) * a.nhist_stride + col], 1u);
    }
  if (lane == 0) {
    a.chunk_off[b] = bs;
    a.chunk_cnt[b] = 0u;  // (no backlog: queued messages are in the rings)
    a.chunk_off[a.nb + b] = (uint32_t)embase;
    a.chunk_cnt[a.nb + b] = emtot;
    if (a.emmeta) a.emmeta[b] = make_uint4(0u, 0u, 2u, 0u);
  }
  const uint32_t v0 = wave_incl_sum(ndel), v1 = wave_incl_sum(ndead), v2 = wave_incl_sum(nunh),
                 v3 = wave_incl_sum(nall), v4 = wave_incl_sum(nact);
  const uint32_t gp = wave_incl_sum(dring > 0 ? (uint32_t)dring : 0u),
                 gn = wave_incl_sum(dring < 0 ? (uint32_t)-dring : 0u);
  if (lane == kWave - 1) {
    unsigned long long* bst = a.bstats + (size_t)blockIdx.x * kBStats;
    if (v0) atomicAdd(&bst[0], (unsigned long long)v0);
    if (v1) atomicAdd(&bst[1], (unsigned long long)v1);
    if (v2) atomicAdd(&bst[2], (unsigned long long)v2);
    if (v3) atomicAdd(&bst[3], (unsigned long long)v3);
    if (v4) atomicAdd(&bst[4], (unsigned long long)v4);
    if (gp != gn) atomicAdd(g.total, (unsigned long long)((long long)gp - (long long)gn));
  }
  return true;
}

template <uint32_t KM>
static __global__ void __launch_bounds__(kTinyThreads, 4) k_ring_tiny(BucketArgs a, RingArgs g) {
  __shared__ RingTinyLds T[kTinyWaves];
  const uint32_t w = threadIdx.x / kWave, lane = lane_id();
  const InView iv = in_view(a);
  const uint32_t nw = gridDim.x * kTinyWaves;
  for (uint32_t bw = blockIdx.x * kTinyWaves + w; bw < a.nb; bw += nw) {
    uint32_t bs = 0, be = 0;
    if (lane == 0) {
      bs = a.bstart[bw];
      be = a.bstart[bw + 1];
    }
    bs = (uint32_t)__builtin_amdgcn_readlane((int)bs, 0);
    be = (uint32_t)__builtin_amdgcn_readlane((int)be, 0);
    const bool tiny = be - bs <= kRingTinyN && ring_tiny_bucket<KM>(a, g, iv, T[w], bw, bs, be - bs);
    if (lane == 0) a.blist[bw] = tiny ? 0u : 1u;  // (the block launch's work marks)
  }
}

}  // namespace agx
