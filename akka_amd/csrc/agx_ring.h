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

struct RingArgs {
  uint32_t* state;   // [n_local] head | len << 16
  uint32_t* src;     // [n_local][rc]
  uint32_t* pay;
  uint32_t* dk;      // drain scratch / tell staging, [nb][kBucket * dstride] (buckets draining > kBucket)
  uint32_t* ds;
  uint32_t* dp;
  unsigned long long* total;  // messages held in rings (in flight)
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
  for (uint32_t b = blockIdx.x; b < a.nb; b += gridDim.x) {
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
    for (uint32_t t0 = 0; t0 < n; t0 += kBucket) {
      uint32_t ix[kBIpt];
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) {
        const uint32_t q = t0 + wbase + r * kWave + lane;
        ix[r] = q < n ? iv.at(bs + q) : 0u;
      }
#pragma unroll
      for (int r = 0; r < kBIpt; ++r) k[r] = ldg(Mk, ix[r]);
#pragma unroll
      for (int r = 0; r < kBIpt; ++r)  // (a hot actor's wave of arrivals: one aggregated LDS atomic)
        if (t0 + wbase + r * kWave + lane < n) lds_hist_inc(S.cnt, k[r] & amask);
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
        const size_t o = (size_t)(a0 + la0 + j) * rc + (q < rr[j] ? x : 0u);
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
    // FANOUT with one tell per message (C3 steady): every drained message's Zipf destination, the
    // four actors' q-th messages in lockstep (index range, each binary-search step's loads together,
    // then the permutation), written over the message's sender (FANOUT does not read it)
    const bool fan_pre = kFan && P.fan_k == 1;
    if (kFan && fan_pre) {
      uint32_t dmax = 0;
#pragma unroll
      for (int j = 0; j < kBAct; ++j) dmax = max(dmax, drn[j]);
      for (uint32_t q = 0; q < dmax; ++q) {
        uint32_t lo[kBAct], hi[kBAct], uu[kBAct];
        bool need[kBAct];
#pragma unroll
        for (int j = 0; j < kBAct; ++j) {
          const uint32_t pv = q < drn[j] ? bpay[ds[j] + q] : 0u;
          need[j] = (pv >> 24) > 0;
          uu[j] = need[j] ? (uint32_t)(fanout_rand(P.fan_seed, a0 + la0 + j, pv & 0x00FFFFFFu, 0) >> 32) : 0u;
          const uint32_t t = uu[j] >> (32 - kZipfBits);
          lo[j] = need[j] ? P.zipf_idx[t] : 0u;
          hi[j] = need[j] ? P.zipf_idx[t + 1] : 0u;
        }
        for (;;) {
          bool more = false;
          uint32_t c[kBAct];
#pragma unroll
          for (int j = 0; j < kBAct; ++j) c[j] = lo[j] < hi[j] ? P.zipf_cdf[(lo[j] + hi[j]) >> 1] : 0u;
#pragma unroll
          for (int j = 0; j < kBAct; ++j)
            if (lo[j] < hi[j]) {
              const uint32_t mid = (lo[j] + hi[j]) >> 1;
              if (c[j] >= uu[j]) hi[j] = mid; else lo[j] = mid + 1;
              more |= lo[j] < hi[j];
            }
          if (!more) break;
        }
#pragma unroll
        for (int j = 0; j < kBAct; ++j)
          if (need[j]) bsrc[ds[j] + q] = P.zipf_perm[lo[j]];
      }
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
    uint32_t* const skey = lds_drain ? S.whist32 : g.dk + sbase;
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
#pragma unroll 1
    for (int j = 0; j < kBAct; ++j) {
      for (uint32_t e = 0; e < ecl[j]; ++e) {
        a.em.key[embase + eo + e] = skey[ds[j] + e];
        a.em.src[embase + eo + e] = bsrc[ds[j] + e];
        a.em.pay[embase + eo + e] = bpay[ds[j] + e];
      }
      eo += ecl[j];
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
  if (blockIdx.x < a.nb) flush_stats(a, acc);
  // messages held in rings: the block's change, two's complement into the u64 total
  const uint32_t gp = wave_incl_sum(dring > 0 ? (uint32_t)dring : 0u), gn = wave_incl_sum(dring < 0 ? (uint32_t)-dring : 0u);
  if (lane == kWave - 1 && gp != gn) atomicAdd(g.total, (unsigned long long)((long long)gp - (long long)gn));
}

}  // namespace agx
