// agx_engine.hip — host runtime of the MI355X batched actor-dispatch engine
// and the C ABI declared in include/akka_gpu.h.
//
// One engine = one rank = one GPU (or one virtual rank of a loopback group).
// Actor state and envelopes live structure-of-arrays in HBM; a superstep is
//   [exchange (R > 1)] -> compaction -> stable radix sort by destination ->
//   segmented drain + behaviour-apply (emits the next step's tells).
// No host round trip per superstep on one GPU; with R > 1 the host reads the
// per-peer counts once per superstep to size the RCCL send/recv group.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "agx_kernels.h"
#include "agx_tellq.h"
#include "agx_variants.h"

using namespace agx;

namespace {

thread_local std::string g_err;

agx_status set_err(agx_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return st;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return set_err(AGX_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                     __LINE__);                                                                \
  } while (0)

#define NCCL_TRY(expr)                                                                            \
  do {                                                                                            \
    ncclResult_t _r = (expr);                                                                     \
    if (_r != ncclSuccess)                                                                        \
      return set_err(AGX_ECOMM, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r), __FILE__, \
                     __LINE__);                                                                   \
  } while (0)

#define AGX_TRY(expr)              \
  do {                             \
    agx_status _s = (expr);        \
    if (_s != AGX_OK) return _s;   \
  } while (0)

uint32_t ceil_log2(uint64_t x) {
  uint32_t b = 0;
  while ((1ull << b) < x) ++b;
  return b;
}

int32_t java_hash_decimal(uint32_t id) {
  char buf[16];
  int n = 0;
  do {
    buf[n++] = (char)('0' + id % 10u);
    id /= 10u;
  } while (id);
  uint32_t h = 0;
  for (int i = n - 1; i >= 0; --i) h = h * 31u + (uint32_t)buf[i];
  return (int32_t)h;
}

struct DevMsgs {
  uint32_t* key = nullptr;
  uint32_t* src = nullptr;
  uint32_t* pay = nullptr;
  Msgs m() const { return {key, src, pay}; }
  CMsgs c() const { return {key, src, pay}; }
};

enum KClass { K_CROWSCAN, K_CDOWN, K_UPSWEEP, K_ROWSCAN, K_DOWNSWEEP, K_APPLY, K_EXCHANGE, K_MCOMPACT, K_SKEW, K_TICK,
              K_BOUNDS, K_SKEWPRE, K_TINY, K_RINGAPPLY, K_DENSE, K_NCLASS };
const char* kClassNames[K_NCLASS] = {"chunk_rowscan", "chunk_downsweep", "sort_upsweep", "sort_rowscan",
                                     "sort_downsweep", "bucket_apply", "exchange", "mcompact", "bucket_apply_skew",
                                     "fused_tick", "bucket_bounds", "skew_prepass", "bucket_apply_tiny",
                                     "ring_apply", "bucket_apply_dense"};

constexpr uint32_t kGraphSizes[5] = {1, 2, 4, 8, 16};  // superstep replays (agx_engine::gx)
constexpr uint32_t kRowAlign = 32;  // CRDT row pitch (u32) of rows wider than one 128-B line
constexpr uint32_t kStatBlk = 16;                    // d_stats block (see agx_engine::d_stats)
constexpr uint32_t kStatSred = ST_N, kStatInfl = ST_N + kBStats;
static_assert(kStatInfl < kStatBlk, "stats block layout");

struct SortPlan {  // LSD passes over key bits [bb, key_bits)
  uint32_t npass = 1;
  uint32_t shift[4] = {0}, bits[4] = {0};
};

}  // namespace

struct agx_engine {
  agx_cfg cfg{};
  TellQueue tq;  // agx_tell: the lock-free tell path (agx_tellq.h), taken by agx_run
  hipStream_t stream = nullptr;
  uint64_t n_global = 0, n_local = 0, cap = 0, cap_emit = 0;
  uint32_t max_supers = 1, dstride = 4, dsub = kSub;  // dense passes: super-tiles (at most), table row stride, max tiles
                                                      // per super-tile (the size itself is chosen per pass: pass_super)
  uint32_t T = 1, C = 0, W = 1, kmax = 1, R = 1, rank = 0, num_shards = 1000, key_bits = 1;
  uint32_t Traw = 1;  // dispatcher throughput (>= 1); T = min(Traw, C) for the default mailbox class
  // mailbox classes (agx_set_mailbox_class): capacity per class, class 0 = cfg.capacity
  uint32_t mcap[AGX_MAX_MAILBOX_CLASSES] = {0};
  uint32_t mclass_set = 1u;  // bit c: class c configured (class 0 always)
  bool mclasses = false;     // some class other than 0 configured: kernels look up per-actor limits
  // the reply path (agx_set_outbound): host-side actor ids and the outbox
  uint32_t host_lo = 0, host_n = 0;
  uint64_t outbox_cap = 0;
  uint32_t *d_outbox = nullptr, *d_outbox_n = nullptr;
  std::vector<uint32_t> outq;  // taken from the device, not yet handed to the host (dst, src, payload)
  uint64_t outbox_lost = 0;    // outbound tells dropped at a full outbox, not reported yet (agx_take_outbound)
  uint32_t bb = kBucketBits;  // bucket bits (agx_cfg.bucket_actors)

  // sharding tables (R > 1)
  std::vector<uint32_t> h_gid, h_route;
  // host mirrors of the actor SoA (uploaded before the first run after a change)
  std::vector<uint8_t> h_kind, h_alive;
  std::vector<uint64_t> h_state;  // word-major
  bool actors_dirty = true;
  uint32_t kinds_mask = 0;  // bit k set when some local actor has behaviour kind k (selects the apply variant)
  std::vector<uint64_t> h_row;  // local CSR rows (graph)
  std::vector<uint32_t> h_col;
  bool graph_set = false;

  uint8_t *d_kind = nullptr, *d_alive = nullptr;
  uint32_t *d_stopq = nullptr, *d_nstop = nullptr;
  uint64_t* d_state = nullptr;
  // CRDT engines (pw > 0 at the first upload) keep the device state actor-major, `pitch` u64 per
  // actor (a replica's words are one contiguous, 128-B aligned row); the host mirror stays word-major
  uint32_t pitch = 0;
  uint32_t *d_gid = nullptr, *d_route = nullptr;
  uint32_t ring_stride = 1, fan_k = 0;
  uint64_t fan_seed = 0, zipf_n = 0;
  uint32_t *d_zcdf = nullptr, *d_zperm = nullptr;
  uint2* d_zent = nullptr;
  uint64_t* d_row = nullptr;
  uint32_t* d_col = nullptr;
  // CRDT state gossips (agx_crdt.h): snapshot heap, 2 x cap rows of pw u32
  uint32_t pw = 0, gossip_f = 0;
  uint32_t delta_max = 0;  // delta-CRDT mode (agx_set_delta_crdt): Replicator max-delta-size, 0 = off
  bool layout_checked = false;  // RCCL: rows / tells sized alike on every rank (run_multi_rccl)
  uint32_t tiny_max = kTinyMax;  // multi-pass: inboxes up to this size take the wave path (AGX_TINY, 0 = off)
  // compiled behaviours (agx_set_behaviors)
  agx_case* d_bcase = nullptr;
  agx_act* d_bact = nullptr;
  uint32_t* d_bfirst = nullptr;
  uint32_t n_beh = 0;
  uint64_t heap_rows = 0;  // per parity: one region of 2^bb rows per bucket, then an overflow area of `cap` rows
  uint64_t gossip_seed = 0;
  uint32_t *d_heap = nullptr, *d_heap_top = nullptr, *d_step = nullptr;
  uint32_t *d_rx = nullptr, *d_s2rows = nullptr;  // multi-rank: received rows / rows packed for sending
  uint64_t rx_rows = 0;                            // rows of d_rx (>= cap; >= R x slab on the device path)
  uint32_t* d_srows = nullptr;                     // device-resident exchange: [R][slab][pw] row send slabs
  uint32_t *d_s2p = nullptr, *d_rcvp = nullptr;    // multi-rank: tells as (key, src, payload) triples, sent / received
  // device-resident multi-rank replays (run_multi_rccl, plain behaviours): fixed per-peer slabs of
  // `slab` envelopes, the replay's stop word halt[2] (k_mr_pack); h_halt = its pinned copy
  uint32_t *d_sslab = nullptr, *d_rslab = nullptr, *d_halt = nullptr, *h_halt = nullptr;
  uint32_t slab = 0;
  uint64_t mr_exact = 0;  // supersteps whose exchange the host redid exactly (a count over the slab)
  uint64_t mr_replays = 0;  // multi-rank replays launched as a captured graph
  // exchange accounting (agx_exchange_info): supersteps on the device-resident / host-planned
  // exchange, bytes this rank sent to its peers (envelopes + CRDT rows), and mr_host = 1 once every
  // rank agreed that the CRDT row slabs do not fit (mr_slabs) -- the host-planned path from then on
  uint64_t mr_dev_steps = 0, mr_host_steps = 0, mr_sent_env = 0, mr_sent_rows = 0;
  bool mr_host = false;
  bool mr_direct = false;  // the last device-resident superstep wrote its peer runs straight into the send slabs

  DevMsgs A, B, scr, bl, em, stg, s2;
  // single-rank multi-pass: the tell arena by superstep parity (em = even, em2 = odd superstep
  // counter): the apply writes one while identity grouping reads the other in place
  DevMsgs em2;
  bool ident_on = false;        // identity grouping enabled (multi-pass, > 1 radix pass; AGX_NO_IDENT=1 disables)
  uint4* d_emmeta = nullptr;    // [nb] per tell chunk: first key, last key, descents, descent position
  uint32_t *d_slsum = nullptr, *d_ident = nullptr;  // slice summaries; {on, rotation, total}
  uint64_t stg_cap = 0;
  uint32_t nb = 1, nchunks = 3;                // buckets; chunks = 2 nb + kStagedChunks
  uint32_t G = 1, ng = 1, nunits = 3, cstride = 4;  // first-pass histogram units (G buckets each)
  SortPlan plan;
  uint32_t *d_chunk_off = nullptr, *d_chunk_cnt = nullptr;
  uint32_t* d_hist_c = nullptr;  // [kRadix][cstride] first-pass histograms per unit
  uint32_t* d_hist_d = nullptr;  // [kRadix][dstride] dense-pass histograms per super-tile
  uint32_t *d_tot = nullptr, *d_bstart = nullptr, *d_n = nullptr, *d_total = nullptr, *d_moff0 = nullptr, *d_moff1 = nullptr;
  unsigned long long *d_bstats = nullptr, *d_sred = nullptr;  // per-block apply counters, their sum
  // d_stats = one block of kStatBlk u64: [0, ST_N) counters, [ST_N, +kBStats) = d_sred (sum of the
  // per-block apply counters), [kStatInfl] = d_inflight -- read back with ONE copy + ONE sync
  uint64_t *d_stats = nullptr, *d_cvec = nullptr, *d_cmat = nullptr, *d_inflight = nullptr;
  uint64_t* h_stat = nullptr;    // pinned copy of the d_stats block
  uint32_t* h_pin = nullptr;     // pinned ring of per-step totals
  uint64_t* h_pin64 = nullptr;   // pinned scratch (count matrix, stats)

  // fused superstep (single rank, one radix pass): gather-apply, parity-double-buffered arenas
  bool fused = false;
  DevMsgs bl2, eg0, eg1;
  uint32_t *d_tcnt[2] = {nullptr, nullptr}, *d_toff[2] = {nullptr, nullptr};
  uint32_t *d_blpre = nullptr, *d_ninbox = nullptr;  // multi-pass: backlog prefix, inbox total
  uint32_t *d_blo[2] = {nullptr, nullptr}, *d_blc[2] = {nullptr, nullptr}, *d_emc[2] = {nullptr, nullptr};
  uint32_t *d_stg_off = nullptr, *d_stg_cnt = nullptr, *d_ovf = nullptr, *d_cntb = nullptr, *d_parv = nullptr;
  uint32_t* h_cntb = nullptr;  // pinned [kLag][kGraphSteps][nb]: per-superstep inbox sizes of the replays in flight
  uint32_t cur_slot = 0;       // superstep index within the replay being captured / launched
  uint64_t host_steps = 0;     // fused: supersteps with mail, counted on the host from h_cntb
  uint32_t par = 0;  // fused: parity of the next superstep (host-tracked; graphs are captured per parity)
  uint32_t *d_skew_list = nullptr, *d_skew_n = nullptr;  // buckets for the general-path launch
  // single-rank multi-pass, plain behaviours: k_tiny_apply drains the buckets of <= tiny_max messages
  // one wave each and marks the others here ([nb]) for the block launch (AGX_TINY_LAUNCH=0: no wave
  // path, the block launch takes every bucket)
  uint32_t* d_blist = nullptr;
  uint32_t* d_dense_left = nullptr;  // [2] BucketArgs::dense_left
  bool tiny_launch = true;
  hipEvent_t tev[2] = {nullptr, nullptr};  // agx_run_timed: device time of a run (engine stream)
  bool timing = false;
  bool dense_fused = true;  // the dense launch also in the fused superstep (AGX_DENSE_FUSED=0: not)
  // the dense launch in the multi-rank (owner-grouping) superstep (AGX_DENSE_OWNER=0: not).  Round 6:
  // owner classes placed straight from registers (no staged multisplit) and the dense_left shortcut
  // (the block launch returns at entry when it took every bucket): R = 8 x 1M loopback, one hardware
  // queue, apply 32.7 us (block launch) -> 19.9 + 5.6 us (dense + returning block launch) per rank-step
  bool dense_owner = true;
  bool dense_alone = true;  // fused strict replays: the dense launch alone (cleared at its first recovery)
  bool recover_dense = false;  // run_single's recovery of a dense-alone superstep: the block + skew launches
  int dense_launch = -1;  // k_dense_apply before the block launch: 1 on, 0 off, -1 (default) ring populations
  // ring apply (agx_ring.h): bounded mailboxes whose queued messages stay in per-actor rings; decided
  // at the first run (setup_ring_apply), then k_ring_tiny + k_ring_apply per superstep replace the tiny /
  // block / skew launches.  On by default for deep bounded mailboxes (capacity >= kRingAutoC);
  // AGX_RING_APPLY=1 / 0 forces it.
  bool rg_on = false;
  uint32_t rg_c = 0, rg_dstride = 0;
  uint32_t *d_rg_state = nullptr, *d_rg_src = nullptr, *d_rg_pay = nullptr;
  uint32_t *d_rg_dk = nullptr, *d_rg_ds = nullptr, *d_rg_dp = nullptr;
  uint32_t* d_rg_nz = nullptr;  // [nb][64] non-empty-ring bits
  uint64_t em_cap = 0;  // entries of the tell arenas em / em2
  // multi-pass, plain behaviours: skewed buckets split over workgroups (k_skew_*, agx_kernels.h)
  uint32_t *d_sk_rec = nullptr, *d_sk_act = nullptr, *d_sk_pc = nullptr, *d_sk_meta = nullptr;
  uint32_t sk_budget = 0, sk_rows = 0;
  // bounded-mailbox rings (multi-pass, plain behaviours, every mailbox class bounded by <= kRingMaxC):
  // a skewed bucket's queued messages stay in per-actor rings instead of the backlog arena.
  // ring_res: pool slots whose drain scratch / tell slices were reserved after the arenas at
  // create (ring_lo0 = acap); the pool itself is allocated at the first run whose mailbox classes
  // allow it, with ring_c = the largest capacity, and fixes the classes from then on.
  uint32_t ring_res = 0, ring_slots = 0, ring_c = 0;
  bool ring_live = false;
  uint32_t *d_ring_of = nullptr, *d_ring_state = nullptr, *d_ring_src = nullptr, *d_ring_pay = nullptr;
  uint32_t* d_ring_next = nullptr;  // [0] slots handed out, [1] free-stack depth
  uint32_t* d_ring_free = nullptr;
  // ORSet-only full-state populations: the apply's work list for k_orset_merge
  uint4* d_orw = nullptr;
  uint2* d_orm = nullptr;
  uint32_t* d_orw_n = nullptr;
  unsigned long long* d_ring_total = nullptr;
  uint32_t tstride = 4, region = 0;
  uint64_t acap = 0;  // arena capacity (fused: regions + overflow area)
  uint32_t apply_grid = kMaxApplyGrid;  // AGX_APPLY_GRID test knob: fewer blocks, each looping over buckets
  // blocks of the skew-list launch (grid-stride over the list; AGX_SKEW_GRID diagnostic knob): one
  // round of workgroups (2 per CU) -- an empty list at 10^8 actors cost 18 us with 4096 blocks
  uint32_t skew_grid = 512;
  bool stamps_skew = false;  // AGX_STAMPS_SKEW (diagnostic): phase stamps of the skew launch only
  std::vector<uint32_t> hd_key, hd_src, hd_pay;  // staged tells on the device, not yet consumed (fused)
  bool stg_pending = false;

  // host-staged tells (consumed by the next superstep)
  std::vector<uint32_t> hs_key, hs_src, hs_pay;
  uint32_t n_staged_dev = 0;  // staged tells uploaded for the next step
  uint64_t staged_total = 0, staged_dead = 0;
  uint64_t inflight_dev = 0;    // the device's in-flight count when inflight_known (agx_stage_tells' check)
  bool inflight_known = false;  // inflight_dev is current (cleared by every agx_run)
  bool last_run_ok = false;     // the last agx_run returned AGX_OK (agx_pump_idle's in-flight reschedule)
  bool tev1_recorded = false;   // agx_run_timed: run_single recorded the end event

  ncclComm_t comm = nullptr;
  bool started = false;
  // superstep graphs (single rank)
  static constexpr uint32_t kGraphSteps = 16;  // largest replay (kGraphSizes = 1, 2, 4, 8, 16); a replay boundary costs
                                              // ~18 us (graph launch + k_replay_out); with D2H copies per replay,
                                              // 16-superstep replays had measured slower (67 vs 24.7 us/superstep)
  bool graphs_enabled = true;
  // gx[strict][parity][size]: replays of kGraphSizes[size] supersteps; fused graphs exist per
  // starting parity (the parity is a kernel argument), multi-pass ones use gx[0][0][*].  A budget
  // of K supersteps replays its binary decomposition (20 = 8 + 8 + 4), never a run of singles.
  static constexpr uint32_t kNSizes = 5;
  hipGraphExec_t gx[2][2][kNSizes] = {};
  bool gx_persist[2][2][kNSizes] = {};  // that replay is one persistent launch (capture_steps)
  uint64_t persist_launches = 0, persist_supersteps = 0;  // replays launched as persistent launches (agx_persist_info)
  // multi-rank device-resident replays (run_multi_rccl): kMrReplay supersteps -- phase 1, the count
  // all-gather, k_mr_pack, the slab sends / receives, unpack, bucket passes, apply -- captured once as
  // one graph (RCCL collectives are captured with the kernels); mr_graph_ok cleared when a capture
  // fails (the replays then stay eager).  Opt-in: AGX_MR_GRAPH=1 (see run_multi_rccl).
  hipGraphExec_t mr_gx = nullptr;
  bool mr_graph_ok = true;
  // fused "strict" replays: graphs without the (usually empty) skew-list launches.  A superstep that
  // defers a skewed bucket marks d_abort; the rest of the replay is void and run_single runs the
  // deferred skew launch, then continues with the full graphs (strict_ok cleared for this engine).
  uint32_t* d_abort = nullptr;  // [2] (BucketArgs::abort)
  // persistent fused supersteps (k_dense_fused<.., true>): a captured replay of K dense-alone strict
  // supersteps is ONE launch with a grid barrier between supersteps (opt-in, AGX_PERSIST=1; default: K launches)
  int persist = -1;              // -1 not decided yet, 0 off (knob, too many buckets, a barrier timeout), 1 on
  uint32_t persist_steps = 0;    // capture_steps -> launch_apply: supersteps of the persistent launch
  uint32_t persist_vid = ~0u;    // the apply variant `persist` was decided for
  bool captured_persist = false; // the last capture_steps was one persistent launch
  uint32_t* d_pbar = nullptr;    // [4] grid barrier: arrivals, generation, timed out
  uint32_t* h_abort = nullptr;  // pinned [kLag][2]: the marks after each replay (eager path)
  // fused graphs end with k_replay_out, which writes the replay's inbox-size rows and abort marks
  // straight into the pinned host ring (device-mapped) at ring slot (replay counter % kLag): no
  // D2H copy between replays (those cost ~26 us per replay boundary, rocprofv3 kernel trace)
  uint32_t* d_ring = nullptr;   // device pointer of h_cntb
  uint32_t* d_rctr = nullptr;   // device replay counter (k_replay_out)
  uint64_t replay_ctr = 0;      // host mirror: fused graph replays launched
  bool strict_ok = true;        // AGX_NO_STRICT=1 disables
  bool strict_env = true;       // (the AGX_NO_STRICT knob; strict_ok is re-armed after clean replays)
  uint32_t clean_steps = 0;     // fused supersteps since the last skewed bucket (full graphs)
  uint32_t max_replay_si = 4;   // largest replay used: kGraphSizes[max_replay_si] (AGX_MAX_REPLAY knob)
  hipEvent_t lag_ev[4] = {};    // run_single's replay events (created once)
  bool strict_cap = false;      // the superstep being launched / captured is strict
  bool skew_only = false;       // recovery: the deferred skew launch alone
  unsigned long long* d_dbg = nullptr;  // AGX_STAMPS diagnostic build only

  // profiling
  bool prof = false;
  struct Rec { int cls; hipEvent_t a, b; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  double prof_ms[K_NCLASS] = {0};
  uint64_t prof_n[K_NCLASS] = {0};
  // profiled dense launches (K_DENSE) that took every bucket, read from the device's dense_left words
  // after the launch: the wave / block launches after them returned at entry (agx_profile_read items)
  uint64_t prof_items[K_NCLASS] = {0};
};

namespace {

agx_status ensure_dev(agx_engine* e) {
  HIP_TRY(hipSetDevice((int)e->cfg.device));
  return AGX_OK;
}

template <typename T>
agx_status dalloc(T** p, uint64_t n) {
  if (n == 0) n = 1;
  HIP_TRY(hipMalloc((void**)p, n * sizeof(T)));
  return AGX_OK;
}

agx_status alloc_msgs(DevMsgs& m, uint64_t n) {
  AGX_TRY(dalloc(&m.key, n));
  AGX_TRY(dalloc(&m.src, n));
  AGX_TRY(dalloc(&m.pay, n));
  return AGX_OK;
}

void free_msgs(DevMsgs& m) {
  hipFree(m.key);
  hipFree(m.src);
  hipFree(m.pay);
  m = DevMsgs{};
}

// --------------------------------------------------------------- profiling
void prof_begin(agx_engine* e, int cls, hipEvent_t* out_b) {
  *out_b = nullptr;
  if (!e->prof) return;
  if (e->ev_used + 2 > e->ev_pool.size()) {
    if (e->ev_pool.size() >= 200000) return;
    for (int i = 0; i < 1024; ++i) {
      hipEvent_t ev;
      if (hipEventCreate(&ev) != hipSuccess) return;
      e->ev_pool.push_back(ev);
    }
  }
  hipEvent_t a = e->ev_pool[e->ev_used++], b = e->ev_pool[e->ev_used++];
  hipEventRecord(a, e->stream);
  e->recs.push_back({cls, a, b});
  *out_b = b;
}
void prof_end(agx_engine* e, hipEvent_t b) {
  if (b) hipEventRecord(b, e->stream);
}
void prof_collect(agx_engine* e) {
  if (e->recs.empty()) return;
  hipStreamSynchronize(e->stream);
  for (auto& r : e->recs) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      e->prof_ms[r.cls] += ms;
      e->prof_n[r.cls] += 1;
    }
  }
  e->recs.clear();
  e->ev_used = 0;
}

struct Scope {
  agx_engine* e;
  hipEvent_t b;
  Scope(agx_engine* e_, int cls) : e(e_) { prof_begin(e, cls, &b); }
  ~Scope() { prof_end(e, b); }
};

void drop_graphs(agx_engine* e);

DevParams make_params(agx_engine* e) {
  DevParams P{};
  P.n_global = (uint32_t)e->n_global;
  P.n_local = (uint32_t)e->n_local;
  P.W = e->W;
  P.T = e->T;
  P.C = e->C;
  P.Tr = e->Traw;
  P.nmc = e->mclasses ? 1u : 0u;
  for (uint32_t c = 0; c < AGX_MAX_MAILBOX_CLASSES; ++c) P.mcap[c] = e->mcap[c];
  P.host_lo = e->host_lo;
  P.host_n = e->host_n;
  P.outbox = e->d_outbox;
  P.outbox_n = e->d_outbox_n;
  P.outbox_cap = (uint32_t)e->outbox_cap;
  P.R = e->R;
  P.rank = e->rank;
  P.kmax = e->kmax;
  P.ring_stride = (uint32_t)(e->ring_stride % e->n_global);
  P.fan_k = e->fan_k;
  P.fan_seed = e->fan_seed;
  P.zipf_n = e->zipf_n;
  P.zipf_cdf = e->d_zcdf;
  P.zipf_ent = e->d_zent;
  P.zipf_perm = e->d_zperm;
  P.row_ptr = e->d_row;
  P.col = e->d_col;
  P.route = e->d_route;
  P.gid = e->d_gid;
  P.kind = e->d_kind;
  P.alive = e->d_alive;
  P.state = e->d_state;
  P.pitch = e->pitch;
  P.sa = e->pitch ? e->pitch : 1u;
  P.sw = e->pitch ? 1u : (uint32_t)e->n_local;
  P.stopq = e->d_stopq;
  P.nstop = e->d_nstop;
  P.heap = e->d_heap;
  P.rx = e->d_rx;
  P.heap_top = e->d_heap_top;
  P.step = e->d_step;
  P.heap_rows = (uint32_t)e->heap_rows;
  P.pw = e->pw;
  P.gossip_f = e->gossip_f;
  P.gossip_seed = e->gossip_seed;
  P.delta_max = e->delta_max;
  P.bcase = e->d_bcase;
  P.bact = e->d_bact;
  P.bfirst = e->d_bfirst;
  P.n_beh = e->n_beh;
  P.err = reinterpret_cast<unsigned long long*>(e->d_stats + ST_ERROR);
  return P;
}

uint32_t grid_for(uint64_t tiles, uint32_t cap) { return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(tiles, cap)); }

// ------------------------------------------------------------ kernel steps
bool bypass_mode(const agx_engine* e) { return !e->fused && e->R == 1; }
// single-rank multi-pass: the tell arena the superstep of parity `par` writes
const DevMsgs& em_arena(const agx_engine* e, uint32_t par) { return par ? e->em2 : e->em; }

Chunks make_chunks(agx_engine* e) {
  Chunks c{};
  c.bl = e->bl.c();
  c.em = bypass_mode(e) ? em_arena(e, e->par ^ 1u).c() : e->em.c();  // (the previous apply's tells)
  c.st = e->stg.c();
  c.off = e->d_chunk_off;
  c.cnt = e->d_chunk_cnt;
  c.nb = e->nb;
  return c;
}

// one dense LSD pass (reduce-then-scan) over `bits` bits at `shift`
agx_status launch_dense_pass(agx_engine* e, const DevMsgs& in, const DevMsgs& out, const uint32_t* d_n, uint32_t shift,
                             uint32_t bits) {
  SortArgs sa{};
  sa.in = in.c();
  sa.out = out.m();
  sa.d_n = d_n;
  sa.hist = e->d_hist_d;
  sa.tot = e->d_tot;
  sa.bstart = e->d_bstart;
  sa.stride = e->dstride;
  sa.maxsub = e->dsub;
  sa.shift = shift;
  sa.bits = bits;
  // (multi-rank: the device-resident replays' stop word -- [0] != 0 makes the pass return, like identity)
  sa.ident = e->ident_on ? e->d_ident : e->R > 1 ? e->d_halt : nullptr;
  const uint32_t g = grid_for(e->max_supers, 4096);
  {
    Scope s(e, K_UPSWEEP);
    hipLaunchKernelGGL(k_sort_upsweep, dim3(g), dim3(kThreads), 0, e->stream, sa);
  }
  {
    Scope s(e, K_ROWSCAN);
    hipLaunchKernelGGL(k_sort_rowscan, dim3(1u << bits), dim3(kThreads), 0, e->stream, sa);
  }
  {
    Scope s(e, K_DOWNSWEEP);
    hipLaunchKernelGGL(k_sort_downsweep, dim3(g), dim3(kThreads), 0, e->stream, sa);
  }
  HIP_TRY(hipGetLastError());
  return AGX_OK;
}

// Group the mail by bucket.  first_from_chunks: pass 0 reads the chunk list written
// by the previous k_bucket_apply (single rank); otherwise every pass reads the dense A.
// Returns the buffer holding the result.
agx_status launch_bucket_sort(agx_engine* e, bool first_from_chunks, DevMsgs** result) {
  DevMsgs* src = &e->A;
  DevMsgs* dst = &e->B;
  uint32_t p0 = 0;
  if (first_from_chunks) {
    ChunkSortArgs ca{};
    ca.ch = make_chunks(e);
    ca.out = e->A.m();
    ca.hist = e->d_hist_c;
    ca.tot = e->d_tot;
    ca.d_n = e->d_n;
    ca.bstart = e->d_bstart;
    ca.stats = e->d_stats;
    ca.alive = e->d_alive;
    ca.stopq = e->d_stopq;
    ca.nstop = e->d_nstop;
    ca.step = e->d_step;  // superstep counter: CRDT heap parity and the backlog arena parity
    ca.blpre = e->d_blpre;
    ca.bl_stot = e->d_blpre + e->nb;
    ca.bl_sbase = e->d_blpre + e->nb + kMaxBlSlices;
    ca.d_ninbox = e->d_ninbox;
    ca.ring_total = e->ring_live || e->rg_on ? e->d_ring_total : nullptr;
    ca.bypass = 1;
    ca.heap_top = e->d_heap_top;
    ca.skew_n = e->d_skew_n;
    ca.cap = e->cap;
    ca.stride = e->cstride;
    ca.nunits = e->nunits;
    ca.ng = e->ng;
    ca.G = e->G;
    ca.shift = e->plan.shift[0];
    ca.bits = e->plan.bits[0];
    const uint32_t nsl = (e->nb + kBlSlice - 1) / kBlSlice;
    if (e->ident_on) {
      ca.emmeta = e->d_emmeta;
      ca.slsum = e->d_slsum;
      ca.ident = e->d_ident;
    }
    {
      Scope s(e, K_CROWSCAN);
      if (e->ident_on && e->plan.npass > 1) {
        // the decision first (slice summaries, k_ident_combine), then the rowscan proper, whose digit
        // rows are skipped under identity (k_bucket_bounds finds the bucket starts in place)
        ca.part = 1;
        hipLaunchKernelGGL(k_chunk_rowscan, dim3(nsl + 1), dim3(kThreads), 0, e->stream, ca);
        hipLaunchKernelGGL(k_ident_combine, dim3(1), dim3(kWave), 0, e->stream, e->d_slsum, nsl, e->d_ident,
                           reinterpret_cast<unsigned long long*>(e->d_stats + ST_IDENT));
        ca.part = 2;
        hipLaunchKernelGGL(k_chunk_rowscan, dim3((1u << ca.bits) + nsl), dim3(kThreads), 0, e->stream, ca);
      } else {
        hipLaunchKernelGGL(k_chunk_rowscan, dim3((1u << ca.bits) + nsl + (e->ident_on ? nsl + 1 : 0)), dim3(kThreads), 0,
                           e->stream, ca);
        if (e->ident_on)  // this superstep's grouping: identity (no pass) or the radix passes
          hipLaunchKernelGGL(k_ident_combine, dim3(1), dim3(kWave), 0, e->stream, e->d_slsum, nsl, e->d_ident,
                             reinterpret_cast<unsigned long long*>(e->d_stats + ST_IDENT));
      }
    }
    {
      Scope s(e, K_CDOWN);
      hipLaunchKernelGGL(k_chunk_downsweep, dim3(grid_for(e->nunits, 4096)), dim3(kThreads), 0, e->stream, ca);
    }
    HIP_TRY(hipGetLastError());
    p0 = 1;
  }
  for (uint32_t p = p0; p < e->plan.npass; ++p) {
    AGX_TRY(launch_dense_pass(e, *src, *dst, e->d_n, e->plan.shift[p], e->plan.bits[p]));
    std::swap(src, dst);
  }
  if (e->plan.npass > 1) {  // digits of the last pass are not buckets: find the bucket starts
    Scope s(e, K_BOUNDS);
    const bool idn = e->ident_on && first_from_chunks;
    hipLaunchKernelGGL(k_bucket_bounds, dim3(grid_for((e->nb + kThreads) / kThreads, 4096)), dim3(kThreads), 0,
                       e->stream, src->key, e->d_n, e->nb, e->bb, e->d_bstart, idn ? e->d_ident : nullptr,
                       idn ? em_arena(e, e->par ^ 1u).key : nullptr, e->R > 1 ? e->d_halt : nullptr);
    HIP_TRY(hipGetLastError());
  }
  *result = src;
  return AGX_OK;
}

// multi-pass, plain behaviours: partition the skewed buckets over workgroups before the skew
// launch (k_skew_plan / count / scan / scatter, agx_kernels.h); grids are fixed (graph capture),
// the kernels stride over the device-side part and bucket counts
void skew_prepass(agx_engine* e, const BucketArgs& ba, const SkewArgs& ska) {
  const uint32_t gp = std::min<uint32_t>(e->sk_rows, 1024), gb = grid_for(e->nb, kMaxApplyGrid);
  hipLaunchKernelGGL(k_skew_plan, dim3(1), dim3(kScanThreads), 0, e->stream, ba, ska);
  hipLaunchKernelGGL(k_skew_count, dim3(gp), dim3(kBThreads), 0, e->stream, ba, ska);
  hipLaunchKernelGGL(k_skew_scan, dim3(gb), dim3(kBThreads), 0, e->stream, ba, ska);
  hipLaunchKernelGGL(k_skew_scatter, dim3(gp), dim3(kBThreads), 0, e->stream, ba, ska);
}

// the k_bucket_apply variant for the registered behaviour kinds (agx_variants.h)
uint32_t apply_variant(const agx_engine* e) {
  const uint32_t km = e->kinds_mask & ~kb(AGX_KIND_NONE);
  if (e->pw && e->delta_max) {  // delta-CRDT replication: the variants that carry the delta code
    if (km == kb(AGX_KIND_GCOUNTER)) return V_GC_DELTA;
    if (km == kb(AGX_KIND_PNCOUNTER)) return V_PN_DELTA;
    if (km == kb(AGX_KIND_ORSET)) return V_OR_DELTA;
    return V_ALL_DELTA;
  }
  if (e->pw) {  // CRDT kinds registered: single-kind populations get specialised merges
    if (km == kb(AGX_KIND_GCOUNTER)) return V_GC;
    if (km == kb(AGX_KIND_PNCOUNTER)) return V_PN;
    if (km == kb(AGX_KIND_ORSET)) return V_OR;
    if ((km & ~kCrdtKM) == 0) return V_CRDT;  // CRDT kinds only: no plain-behaviour code
    return V_ALL_WIDE;
  }
  if (km == kb(AGX_KIND_RING)) return V_RING;  // behaviour-specialised variants (see apply_msg)
  if (km == kb(AGX_KIND_FORWARD_RR)) return V_FWD;
  if (km == kb(AGX_KIND_FANOUT)) return V_FANOUT;
  if (km == kb(AGX_KIND_COUNTER)) return V_COUNTER;
  if (km == kb(AGX_KIND_COMPILED)) return V_COMPILED;  // compiled behaviours only (agx_set_behaviors)
  if (km & kb(AGX_KIND_COMPILED)) return V_ALL_COMPILED;
  return V_ALL;
}

// the lean dense-bucket launch before the block launch (k_dense_apply / k_dense_fused): plain
// behaviours, one tell per message, no bounded-mailbox rings; by default for ring populations
bool dense_on(const agx_engine* e, uint32_t vid) {
  const bool mode_ok = e->fused ? e->dense_fused : e->R == 1 || e->dense_owner;
  // (k_dense_fused reads a fused bucket's table row one sender bucket per thread: nb <= 512, which
  // the fused superstep's <= 2^20 actors guarantee)
  if (e->fused && e->nb > (uint32_t)kDenseThreads) return false;
  return mode_ok && !kVariants[vid].wide && e->kmax == 1 && !e->ring_live &&
         (e->dense_launch == 1 || (e->dense_launch < 0 && vid == V_RING));
}

agx_status launch_apply(agx_engine* e, const DevMsgs& sorted) {
  // the chunk histograms consumed by this step's first pass were zeroed by k_chunk_downsweep;
  // on the multi-rank path (no chunk pass) they are never read, so stale columns are harmless
  BucketArgs ba{};
  ba.P = make_params(e);
  ba.in = sorted.c();
  ba.d_n = e->d_n;
  ba.bstart = e->d_bstart;
  ba.scr = e->scr.m();
  ba.bl = e->bl.m();
  ba.em = e->em.m();
  ba.chunk_off = e->d_chunk_off;
  ba.chunk_cnt = e->d_chunk_cnt;
  ba.nhist = e->d_hist_c;
  ba.nhist_stride = e->cstride;
  ba.G = e->G;
  ba.ng = e->ng;
  ba.nx_shift = e->plan.shift[0];
  ba.nx_bits = e->plan.bits[0];
  ba.nb = e->nb;
  ba.bb = e->bb;
  ba.kmax = e->kmax;
  ba.stats = e->d_stats;
  ba.bstats = e->d_bstats;
  ba.skew_list = e->d_skew_list;
  ba.skew_n = e->d_skew_n;
  if (e->fused) {
    ba.par = e->par;
    ba.slot = e->cur_slot;
    if (e->strict_cap) ba.abort = e->d_abort;
    ba.P.step = e->d_parv + e->par;  // CRDT heap parity = superstep parity
  }
  if (e->fused) {
    GatherArgs& g = ba.g;
    g.bl[0] = e->bl.m();
    g.bl[1] = e->bl2.m();
    g.eg[0] = e->eg0.m();
    g.eg[1] = e->eg1.m();
    g.stg = e->stg.c();
    for (int q = 0; q < 2; ++q) {
      g.tcnt[q] = e->d_tcnt[q];
      g.toff[q] = e->d_toff[q];
      g.blo[q] = e->d_blo[q];
      g.blc[q] = e->d_blc[q];
      g.emc[q] = e->d_emc[q];
    }
    g.stg_off = e->d_stg_off;
    g.stg_cnt = e->d_stg_cnt;
    g.inb = e->A.m();
    g.ovf = e->d_ovf;
    g.cntb = e->d_cntb;
    g.heap_top = e->pw ? e->d_heap_top : nullptr;
    g.cap = e->acap;
    g.tstride = e->tstride;
    g.region = e->region;
  }
  if (!e->fused && e->R == 1) {  // multi-pass: the backlog stays in place (parity arenas bl / bl2)
    ba.em = em_arena(e, e->par).m();  // (tells by superstep parity: identity grouping reads the other one)
    if (e->ident_on) {
      ba.ident = e->d_ident;
      ba.in_alt = em_arena(e, e->par ^ 1u).c();
      ba.emmeta = e->d_emmeta;
    }
    ba.pstep = e->d_step;
    ba.cap = e->cap;
    ba.blpre = e->d_blpre;
    ba.bl_sbase = e->d_blpre + e->nb + kMaxBlSlices;
    ba.d_ninbox = e->d_ninbox;
    ba.g.bl[0] = e->bl.m();
    ba.g.bl[1] = e->bl2.m();
  }
  if (e->R > 1) {  // tells leave grouped by owner rank (phase 1 packs them for the exchange)
    ba.nx_shift = kOwnerShift;
    ba.nx_bits = std::max<uint32_t>(1, ceil_log2(e->R));
    ba.g.eg[0] = e->eg0.m();
    ba.g.tcnt[0] = e->d_tcnt[0];
    ba.g.toff[0] = e->d_toff[0];
    ba.g.tstride = e->tstride;
  }
  ba.dbg = e->d_dbg;
  ba.halt = e->R > 1 ? e->d_halt : nullptr;
  ba.tiny_max = e->tiny_max;
  ba.sk_rec = e->d_sk_rec;
  ba.sk_act = e->d_sk_act;
  if (e->ring_live) {
    ba.ring_of = e->d_ring_of;
    ba.ring_state = e->d_ring_state;
    ba.ring_src = e->d_ring_src;
    ba.ring_pay = e->d_ring_pay;
    ba.ring_next = e->d_ring_next;
    ba.ring_free = e->d_ring_free;
    ba.ring_total = e->d_ring_total;
    ba.ring_slots = e->ring_slots;
    ba.ring_c = e->ring_c;
    ba.ring_t = e->Traw;
    ba.ring_lo0 = (uint32_t)e->acap;
  }
  SkewArgs ska{e->d_sk_rec, e->d_sk_act, e->d_sk_pc, e->d_sk_meta, e->sk_budget, e->sk_rows};
  if (e->rg_on) {  // ring apply: one launch does admission, drains and ring appends (agx_ring.h)
    RingArgs ra{e->d_rg_state, e->d_rg_src, e->d_rg_pay, e->d_rg_dk, e->d_rg_ds, e->d_rg_dp, e->d_ring_total,
                e->d_rg_nz, e->rg_c, e->rg_dstride};
    const uint32_t vid = apply_variant(e);
    if (e->tiny_launch && e->tiny_max && !e->skew_only) {  // sparse buckets a wave each, then the marked ones
      ba.blist = e->d_blist;
      Scope s(e, K_TINY);
      HIP_TRY(agx_launch_ring(vid, true, dim3(grid_for((e->nb + kTinyWaves - 1) / kTinyWaves, kMaxApplyGrid)), e->stream,
                              ba, ra));
    }
    {
      Scope s(e, K_RINGAPPLY);
      HIP_TRY(agx_launch_ring(vid, false, dim3(grid_for(e->nb, e->apply_grid)), e->stream, ba, ra));
    }
    e->par ^= 1u;
    HIP_TRY(hipGetLastError());
    return AGX_OK;
  }
  {
    const uint32_t vid = apply_variant(e);
    const bool orm = vid == V_OR;  // ORSet-only full state: state effects in k_orset_merge
    if (orm) {
      if (!e->d_orw) return set_err(AGX_ESTATE, "ORSet work list not allocated (setup_orset)");
      ba.orw = e->d_orw;
      ba.orm = e->d_orm;
      ba.orw_n = e->d_orw_n;
      HIP_TRY(hipMemsetAsync(e->d_orw_n, 0, 8, e->stream));
    }
    const uint32_t mode = e->fused ? M_FUSED : e->R > 1 ? M_OWNER : M_BYPASS;
    const dim3 g(grid_for(e->nb, e->apply_grid));
    // dense buckets (one message per actor) first, in their own lean launch (k_dense_apply; fused
    // superstep: k_dense_fused); by default for ring populations, whose buckets all are
    // (AGX_DENSE_LAUNCH=1 / 0 forces it; AGX_DENSE_FUSED=0 keeps the fused superstep one launch)
    const bool dl = dense_on(e, vid) && !e->skew_only && !e->recover_dense;
    // fused strict replay: the dense launch alone is the superstep (a bucket it cannot take marks the
    // replay void from there, as a deferred skewed bucket does; run_single recovers it), until the
    // first such recovery (e->dense_alone cleared for the engine)
    const bool alone = dl && mode == M_FUSED && e->strict_cap && e->dense_alone;
    if (dl || e->recover_dense) {
      ba.blist = e->d_blist;
      // (owner mode: one word, [0] -- cleared by the superstep's k_mcompact_scan, before the dense launch)
      ba.dense_left = e->d_dense_left;
    }
    const bool persist = dl && alone && e->persist_steps > 0;
    if (dl) {
      Scope s(e, K_DENSE);
      BucketArgs bd = ba;
      bd.dense_alone = alone ? 1u : 0u;
      if (persist) {  // e->persist_steps supersteps in one launch, one block per bucket (persist_ok)
        bd.psteps = e->persist_steps;
        bd.pbar = e->d_pbar;
        if (bd.par) {  // the kernel's pointer arrays by LOGICAL parity: index 0 = the first superstep's write parity
          GatherArgs& q = bd.g;
          std::swap(q.bl[0], q.bl[1]);
          std::swap(q.eg[0], q.eg[1]);
          std::swap(q.tcnt[0], q.tcnt[1]);
          std::swap(q.toff[0], q.toff[1]);
          std::swap(q.blo[0], q.blo[1]);
          std::swap(q.blc[0], q.blc[1]);
          std::swap(q.emc[0], q.emc[1]);
        }
        HIP_TRY(agx_launch_dense(vid, M_PERSIST, dim3(e->nb), e->stream, bd));
      } else {
        HIP_TRY(agx_launch_dense(vid, mode, dim3(grid_for(e->nb, kMaxApplyGrid)), e->stream, bd));
      }
    }
    if (dl && e->prof && !persist && mode != M_OWNER) {
      // (profiling only: eager launches) the launch cleared the other parity's word and raised this
      // one's iff it left a bucket, so both words zero = it took every bucket and the wave / block
      // launches below return at entry (bench.py marks them returned_at_entry from this count)
      uint32_t w2[2] = {1u, 1u};
      HIP_TRY(hipMemcpyAsync(w2, e->d_dense_left, 8, hipMemcpyDeviceToHost, e->stream));
      HIP_TRY(hipStreamSynchronize(e->stream));
      if (w2[0] == 0u && w2[1] == 0u) ++e->prof_items[K_DENSE];
    }
    if (persist) {  // (nothing else runs in a dense-alone strict superstep)
      if (e->persist_steps & 1u) e->par ^= 1u;
      HIP_TRY(hipGetLastError());
      return AGX_OK;
    }
    const bool tl = mode == M_BYPASS && !kVariants[vid].wide && e->tiny_launch && e->tiny_max && !e->skew_only;
    if (tl) {  // wave-per-bucket launch first; the block launch then takes the buckets it marked
      ba.blist = e->d_blist;
      ba.dense_first = dl ? 1u : 0u;
      Scope s(e, K_TINY);
      const uint32_t gt = grid_for((e->nb + kTinyWaves - 1) / kTinyWaves, kMaxApplyGrid);
      HIP_TRY(agx_launch_tiny(vid, dim3(gt), e->stream, ba));
    }
    // skew list (grid-stride); ring buckets take the skew launch every superstep: a wider grid then
    const dim3 gs(grid_for(e->nb, std::min(e->apply_grid, e->ring_live ? std::max(e->skew_grid, 2048u) : e->skew_grid)));
    if (!e->skew_only && !alone) {
      Scope s(e, K_APPLY);
      BucketArgs bf = ba;
      if (e->stamps_skew) bf.dbg = nullptr;  // (diagnostic: stamps of the skew launch only)
      HIP_TRY(agx_launch_apply(vid, mode, false, g, e->stream, bf));
    }
    if (!(mode == M_FUSED && e->strict_cap)) {
      if (!kVariants[vid].wide && mode == M_BYPASS) {
        Scope s(e, K_SKEWPRE);  // (k_skew_plan / count / scan / scatter: their own profiling class)
        skew_prepass(e, ba, ska);
      }
      Scope s(e, K_SKEW);
      HIP_TRY(agx_launch_apply(vid, mode, true, gs, e->stream, ba));
    }
    if (orm) {
      Scope s(e, K_APPLY);
      hipLaunchKernelGGL(k_orset_merge, dim3(grid_for(e->n_local / 4 + 1, 4096)), dim3(kThreads), 0, e->stream, ba.P,
                         (const uint4*)e->d_orw, (const uint2*)e->d_orm, (const uint32_t*)e->d_orw_n);
    }
  }
  if (e->R == 1) e->par ^= 1u;  // the next superstep writes the other parity (fused and multi-pass)
  HIP_TRY(hipGetLastError());
  return AGX_OK;
}

// host-staged tells enter as chunk 2nb of the next single-rank step
agx_status launch_staged_chunk(agx_engine* e) {
  if (!e->n_staged_dev) return AGX_OK;
  hipLaunchKernelGGL(k_chunk_hist, dim3(kStagedChunks), dim3(kThreads), 0, e->stream, e->stg.key, e->n_staged_dev,
                     e->d_hist_c, e->cstride, 2 * e->ng, e->plan.shift[0], e->plan.bits[0], e->d_chunk_off,
                     e->d_chunk_cnt, 2 * e->nb);
  HIP_TRY(hipGetLastError());
  e->n_staged_dev = 0;
  return AGX_OK;
}

// Bounded-mailbox rings: allocate the pool at the first run whose configuration allows it (plain
// behaviours, every configured mailbox class bounded by <= kRingMaxC); from then on the classes
// are fixed (agx_set_mailbox_class refuses a capacity the rings cannot hold).
agx_status setup_rings(agx_engine* e) {
  if (e->ring_live || !e->ring_res || e->pw) return AGX_OK;
  uint32_t cmax = 0;
  for (uint32_t c = 0; c < AGX_MAX_MAILBOX_CLASSES; ++c) {
    if (!((e->mclass_set >> c) & 1u)) continue;
    if (e->mcap[c] == 0 || e->mcap[c] > kRingMaxC) return AGX_OK;  // an unbounded (or large) mailbox class
    cmax = std::max(cmax, e->mcap[c]);
  }
  uint64_t budget = kRingPoolBytes;
  if (const char* s = getenv("AGX_RING_MB")) budget = (uint64_t)std::max(0, atoi(s)) << 20;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) == hipSuccess) budget = std::min<uint64_t>(budget, fr / 4);
  const uint64_t per = (uint64_t)kBucket * (2ull * cmax + 1) * 4;
  const uint32_t slots = (uint32_t)std::min<uint64_t>(e->ring_res, budget / per);
  if (!slots) return AGX_OK;
  const uint64_t nst = (uint64_t)slots * kBucket, nmsg = nst * cmax;
  AGX_TRY(dalloc(&e->d_ring_of, e->nb));
  AGX_TRY(dalloc(&e->d_ring_state, nst));
  AGX_TRY(dalloc(&e->d_ring_src, nmsg));
  AGX_TRY(dalloc(&e->d_ring_pay, nmsg));
  AGX_TRY(dalloc(&e->d_ring_next, 2));
  AGX_TRY(dalloc(&e->d_ring_free, slots));
  AGX_TRY(dalloc(&e->d_ring_total, 2));
  HIP_TRY(hipMemsetAsync(e->d_ring_of, 0, e->nb * 4ull, e->stream));
  HIP_TRY(hipMemsetAsync(e->d_ring_state, 0, nst * 4, e->stream));
  HIP_TRY(hipMemsetAsync(e->d_ring_next, 0, 8, e->stream));
  HIP_TRY(hipMemsetAsync(e->d_ring_total, 0, 8, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->ring_slots = slots;
  e->ring_c = cmax;
  e->ring_live = true;
  drop_graphs(e);  // the ring arrays are kernel arguments of the captured supersteps
  return AGX_OK;
}

// Ring apply (agx_ring.h), decided once before the first superstep: a single-rank multi-pass engine
// with plain behaviours, one tell per message (max_emit 1) and every mailbox class bounded keeps its
// queued messages in per-actor rings of the largest capacity when they fit the HBM budget (at most
// half of the free memory: n_local x capacity x 8 B, C5's 10^8 actors x 64 = 51 GB of a 288 GB
// MI355X), so a queued message is written once and read once instead of being copied forward by every
// superstep it waits.  Each bucket's tells get a fixed slice of kBucket x throughput slots of the tell
// arenas (a bucket may drain more messages than it receives: its rings' heads).
constexpr uint32_t kRingAutoC = 256;  // ring apply by default from this mailbox capacity up (setup_ring_apply)
agx_status setup_ring_apply(agx_engine* e) {
  if (e->started || e->rg_on || e->ring_live || e->ring_res) return AGX_OK;
  if (e->fused || e->R != 1 || e->pw || e->kmax != 1 || e->n_local == 0) return AGX_OK;
  // AGX_RING_APPLY=1 / 0 forces rings on / off; unset: on when the largest bounded capacity is at
  // least kRingAutoC.  Deep queues are where re-copying the backlog every superstep costs most (C3,
  // BoundedMailbox(1000): 4.67e8 -> 6.7e8 msg/s with rings, the sparse buckets a wave each); at
  // C5's BoundedMailbox(64) the hub buckets' serial ring chain in one block still loses (2.9e9 with
  // the backlog arena vs 1.8e9).
  const char* rs = getenv("AGX_RING_APPLY");
  const int force = rs ? atoi(rs) : -1;
  if (force == 0) return AGX_OK;
  if (kVariants[apply_variant(e)].wide) return AGX_OK;
  uint32_t cmax = 0;
  for (uint32_t c = 0; c < AGX_MAX_MAILBOX_CLASSES; ++c) {
    if (!((e->mclass_set >> c) & 1u)) continue;
    if (e->mcap[c] == 0 || e->mcap[c] > kRingApplyMaxC) return AGX_OK;  // an unbounded (or huge) mailbox class
    cmax = std::max(cmax, e->mcap[c]);
  }
  if (force < 0 && cmax < kRingAutoC) return AGX_OK;
  const uint64_t dstr = e->Traw, slice = (uint64_t)kBucket * dstr;  // (drained per actor <= min(T, C) <= Traw)
  const uint64_t em_need = (uint64_t)e->nb * slice;
  if (em_need >= (1ull << 32)) return AGX_OK;
  const uint64_t ring_bytes = e->n_local * (uint64_t)cmax * 8 + e->n_local * 4;
  const uint64_t scratch_bytes = em_need * 12;
  const uint64_t em_bytes = em_need > e->em_cap ? 2 * em_need * 12 : 0;  // (bigger tell arenas, both parities)
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return AGX_OK;
  if (ring_bytes + scratch_bytes + em_bytes > fr / 2) return AGX_OK;  // the backlog arena, as before
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (em_need > e->em_cap) {
    free_msgs(e->em);
    free_msgs(e->em2);
    AGX_TRY(alloc_msgs(e->em, em_need));
    AGX_TRY(alloc_msgs(e->em2, em_need));
    e->em_cap = em_need;
  }
  AGX_TRY(dalloc(&e->d_rg_state, e->n_local));
  AGX_TRY(dalloc(&e->d_rg_nz, (uint64_t)e->nb * (kBucket / 32)));
  AGX_TRY(dalloc(&e->d_rg_src, e->n_local * (uint64_t)cmax));
  AGX_TRY(dalloc(&e->d_rg_pay, e->n_local * (uint64_t)cmax));
  AGX_TRY(dalloc(&e->d_rg_dk, em_need));
  AGX_TRY(dalloc(&e->d_rg_ds, em_need));
  AGX_TRY(dalloc(&e->d_rg_dp, em_need));
  if (!e->d_ring_total) AGX_TRY(dalloc(&e->d_ring_total, 2));
  HIP_TRY(hipMemsetAsync(e->d_rg_state, 0, e->n_local * 4, e->stream));
  HIP_TRY(hipMemsetAsync(e->d_rg_nz, 0, (size_t)e->nb * (kBucket / 32) * 4, e->stream));
  HIP_TRY(hipMemsetAsync(e->d_ring_total, 0, 16, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->rg_c = cmax;
  e->rg_dstride = (uint32_t)dstr;
  e->rg_on = true;
  drop_graphs(e);  // the arenas are kernel arguments of the captured supersteps
  return AGX_OK;
}

// ORSet-only full-state populations: k_orset_merge's work list (before any graph capture)
agx_status setup_orset(agx_engine* e) {
  if (e->d_orw || apply_variant(e) != V_OR) return AGX_OK;
  AGX_TRY(dalloc(&e->d_orw, e->n_local));
  AGX_TRY(dalloc(&e->d_orm, e->acap));
  AGX_TRY(dalloc(&e->d_orw_n, 2));
  return AGX_OK;
}

// upload host mirrors / staged tells before a run
agx_status prepare_run(agx_engine* e) {
  if (e->actors_dirty) {
    HIP_TRY(hipMemcpyAsync(e->d_kind, e->h_kind.data(), e->n_local, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_alive, e->h_alive.data(), e->n_local, hipMemcpyHostToDevice, e->stream));
    // first upload of a CRDT engine: actor-major rows from now on -- except delta-CRDT counter
    // populations, which stay word-major: there a lane walks its own replica's envelope and log,
    // and consecutive lanes then read consecutive words (same-box A/B: GCounter delta 3.25e9 ->
    // 3.93e9 word-major; ORSet delta 1.29e9 actor-major vs 1.17e9 word-major, its element rows
    // are read whole).  AGX_CRDT_LAYOUT=actor|word overrides.
    const char* lay = getenv("AGX_CRDT_LAYOUT");
    const bool word_major = apply_variant(e) != V_OR &&  // (k_orset_merge walks actor-major rows)
                            (lay ? lay[0] == 'w' : (e->delta_max && !(e->kinds_mask & kb(AGX_KIND_ORSET))));
    if (e->pw && !e->pitch && !word_major) {
      const uint32_t pitch = e->W <= 16 ? (e->W + 1u) & ~1u : (e->W + 15u) & ~15u;
      uint64_t* d = nullptr;
      AGX_TRY(dalloc(&d, (uint64_t)e->n_local * pitch));
      HIP_TRY(hipFree(e->d_state));
      e->d_state = d;
      e->pitch = pitch;
      drop_graphs(e);  // (the state array is a kernel argument)
    }
    if (e->pitch) {  // word-major mirror -> actor-major rows
      std::vector<uint64_t> rows((size_t)e->n_local * e->pitch, 0);
      for (uint64_t w = 0; w < e->W; ++w)
        for (uint64_t l = 0; l < e->n_local; ++l) rows[l * e->pitch + w] = e->h_state[w * e->n_local + l];
      HIP_TRY(hipMemcpyAsync(e->d_state, rows.data(), rows.size() * 8, hipMemcpyHostToDevice, e->stream));
      HIP_TRY(hipStreamSynchronize(e->stream));
    } else {
      HIP_TRY(hipMemcpyAsync(e->d_state, e->h_state.data(), e->n_local * e->W * 8, hipMemcpyHostToDevice, e->stream));
    }
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->actors_dirty = false;
  }
  if (e->fused && !e->hs_key.empty()) {
    // staged tells still on the device (a run of 0 supersteps) come first: staging order
    if (e->stg_pending) {
      e->hs_key.insert(e->hs_key.begin(), e->hd_key.begin(), e->hd_key.end());
      e->hs_src.insert(e->hs_src.begin(), e->hd_src.begin(), e->hd_src.end());
      e->hs_pay.insert(e->hs_pay.begin(), e->hd_pay.begin(), e->hd_pay.end());
    }
    const uint64_t n = e->hs_key.size();
    if (n > e->stg_cap) {
      free_msgs(e->stg);
      AGX_TRY(alloc_msgs(e->stg, n));
      e->stg_cap = n;
      drop_graphs(e);  // the staging arena is a kernel argument of the captured supersteps
    }
    // stable counting sort by destination bucket: each bucket's staged tells are one run
    std::vector<uint32_t> off(e->nb + 1, 0), cnt(e->nb, 0);
    for (uint64_t i = 0; i < n; ++i) cnt[e->hs_key[i] >> e->bb]++;
    for (uint32_t b = 0; b < e->nb; ++b) off[b + 1] = off[b] + cnt[b];
    std::vector<uint32_t> k(n), sv(n), pv(n), pos(off.begin(), off.end() - 1);
    for (uint64_t i = 0; i < n; ++i) {
      const uint32_t o = pos[e->hs_key[i] >> e->bb]++;
      k[o] = e->hs_key[i];
      sv[o] = e->hs_src[i];
      pv[o] = e->hs_pay[i];
    }
    HIP_TRY(hipMemcpyAsync(e->stg.key, k.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->stg.src, sv.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->stg.pay, pv.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_stg_off, off.data(), e->nb * 4ull, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_stg_cnt, cnt.data(), e->nb * 4ull, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->hd_key.swap(e->hs_key);
    e->hd_src.swap(e->hs_src);
    e->hd_pay.swap(e->hs_pay);
    e->hs_key.clear();
    e->hs_src.clear();
    e->hs_pay.clear();
    e->stg_pending = true;
  }
  if (!e->hs_key.empty()) {
    uint64_t n = e->hs_key.size();
    if (n > e->stg_cap) {
      free_msgs(e->stg);
      AGX_TRY(alloc_msgs(e->stg, n));
      e->stg_cap = n;
    }
    HIP_TRY(hipMemcpyAsync(e->stg.key, e->hs_key.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->stg.src, e->hs_src.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->stg.pay, e->hs_pay.data(), n * 4, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->n_staged_dev = (uint32_t)n;
    e->hs_key.clear();
    e->hs_src.clear();
    e->hs_pay.clear();
  }
  return AGX_OK;
}

// ----------------------------------------------------------- multi-rank step
// phase 1: backlog chunks -> front of A; the apply's owner-grouped tells -> s2, owner-major
// (the stable owner partition of the tells in chunk order); count vector
// [send counts..., n_backlog, n_staged] for the all-gather.
// direct: the device-resident replay of plain behaviours -- the peers' runs go straight into their send
// slabs (k_mcompact_copy), k_mr_pack copies only the own run
agx_status phase1(agx_engine* e, bool direct = false) {
  McompactArgs m{};
  m.ch = make_chunks(e);
  m.eg = e->eg0.c();
  m.tcnt = e->d_tcnt[0];
  m.toff = e->d_toff[0];
  m.out0 = e->A.m();
  m.out1 = e->s2.m();
  m.off0 = e->d_moff0;
  m.off1 = e->d_moff1;
  m.d_total = e->d_total;
  m.cvec = e->d_cvec;
  m.alive = e->d_alive;
  m.stopq = e->d_stopq;
  m.nstop = e->d_nstop;
  m.stats = e->d_stats;
  m.step = e->pw ? e->d_step : nullptr;
  m.heap_top = e->d_heap_top;
  m.skew_n = e->d_skew_n;
  m.cap0 = e->cap;
  m.cap1 = e->cap_emit;
  m.R = e->R;
  m.tstride = e->tstride;
  m.n_staged = e->n_staged_dev;
  m.halt = e->d_halt;  // (multi-rank only; zero outside device-resident replays)
  m.dense_left = e->d_dense_left;
  m.sslab = direct ? e->d_sslab : nullptr;
  m.slab = e->slab;
  m.rank = e->rank;
  {
    Scope s(e, K_MCOMPACT);
    hipLaunchKernelGGL(k_mcompact_scan, dim3(1), dim3(kScanThreads), 0, e->stream, m);
    hipLaunchKernelGGL(k_mcompact_copy, dim3(grid_for(e->nb, 4096)), dim3(kThreads), 0, e->stream, m);
  }
  if (e->pw) {
    Scope s(e, K_MCOMPACT);
    hipLaunchKernelGGL(k_pack_rows, dim3(grid_for(e->cap_emit / kThreads + 1, 2048)), dim3(kThreads), 0, e->stream,
                       e->s2.c(), e->d_total, make_params(e), e->d_s2rows);
  }
  HIP_TRY(hipGetLastError());
  return AGX_OK;
}

// phase 2: staged tells after the received mail, group by bucket, apply.
agx_status phase2(agx_engine* e, uint64_t n_sorted, uint64_t staged_at) {
  if (e->n_staged_dev) {
    HIP_TRY(hipMemcpyAsync(e->A.key + staged_at, e->stg.key, e->n_staged_dev * 4ull, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->A.src + staged_at, e->stg.src, e->n_staged_dev * 4ull, hipMemcpyDeviceToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->A.pay + staged_at, e->stg.pay, e->n_staged_dev * 4ull, hipMemcpyDeviceToDevice, e->stream));
    e->n_staged_dev = 0;
  }
  hipLaunchKernelGGL(k_set_u32, dim3(1), dim3(64), 0, e->stream, e->d_n, (uint32_t)n_sorted);  // no DMA round trip
  DevMsgs* sorted = nullptr;
  AGX_TRY(launch_bucket_sort(e, false, &sorted));
  AGX_TRY(launch_apply(e, *sorted));
  return AGX_OK;
}

struct Plan {
  uint64_t total_inflight = 0;
  uint64_t n_bl = 0, n_recv = 0, n_staged = 0;
  std::vector<uint64_t> send_cnt, send_off, recv_cnt, recv_off;
};

void make_plan(agx_engine* e, const uint64_t* mat, Plan& p) {
  const uint32_t R = e->R, S = R + 2;
  p.send_cnt.assign(R, 0);
  p.send_off.assign(R, 0);
  p.recv_cnt.assign(R, 0);
  p.recv_off.assign(R, 0);
  p.total_inflight = 0;
  for (uint32_t r = 0; r < R; ++r)
    for (uint32_t c = 0; c < S; ++c) p.total_inflight += mat[r * S + c];
  p.n_bl = mat[e->rank * S + R];
  p.n_staged = mat[e->rank * S + R + 1];
  uint64_t so = 0, ro = p.n_bl;
  for (uint32_t q = 0; q < R; ++q) {
    p.send_cnt[q] = mat[e->rank * S + q];
    p.send_off[q] = so;
    so += p.send_cnt[q];
    p.recv_cnt[q] = mat[q * S + e->rank];
    p.recv_off[q] = ro;
    ro += p.recv_cnt[q];
  }
  p.n_recv = ro - p.n_bl;
}

// host <-> device copies of the agx_set_* / read-back entry points: on the engine stream, waited for
// (ordered after any work still queued there -- never a null-stream copy racing the non-blocking
// engine stream)
agx_status copy_sync(agx_engine* e, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, kind, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return AGX_OK;
}

// the reply path: move the device outbox to the host queue (the engine is idle between calls); the
// appends past the outbox capacity were dropped on the device and are counted into outbox_lost
agx_status drain_outbox(agx_engine* e) {
  if (!e->d_outbox_n) return AGX_OK;
  HIP_TRY(hipStreamSynchronize(e->stream));
  uint32_t cnt = 0;
  AGX_TRY(copy_sync(e, &cnt, e->d_outbox_n, 4, hipMemcpyDeviceToHost));
  const uint64_t m = e->d_outbox ? std::min<uint64_t>(cnt, e->outbox_cap) : 0;
  if (m) {
    const size_t o = e->outq.size();
    e->outq.resize(o + 3 * m);
    AGX_TRY(copy_sync(e, e->outq.data() + o, e->d_outbox, 12 * m, hipMemcpyDeviceToHost));
  }
  e->outbox_lost += cnt - m;
  const uint32_t zero = 0;
  if (cnt) AGX_TRY(copy_sync(e, e->d_outbox_n, &zero, 4, hipMemcpyHostToDevice));
  return AGX_OK;
}

// bring the host mirrors up to date with the device (commits pending stops)
agx_status sync_mirrors(agx_engine* e) {
  if (e->actors_dirty) return AGX_OK;  // host mirror is newer than the device
  hipLaunchKernelGGL(k_commit_stops, dim3(1), dim3(kScanThreads), 0, e->stream, e->d_alive, e->d_stopq, e->d_nstop);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(e->stream));
  AGX_TRY(copy_sync(e, e->h_alive.data(), e->d_alive, e->n_local, hipMemcpyDeviceToHost));
  if (e->pitch) {  // actor-major rows -> word-major mirror
    std::vector<uint64_t> rows((size_t)e->n_local * e->pitch);
    AGX_TRY(copy_sync(e, rows.data(), e->d_state, rows.size() * 8, hipMemcpyDeviceToHost));
    for (uint64_t w = 0; w < e->W; ++w)
      for (uint64_t l = 0; l < e->n_local; ++l) e->h_state[w * e->n_local + l] = rows[l * e->pitch + w];
  } else {
    AGX_TRY(copy_sync(e, e->h_state.data(), e->d_state, e->n_local * e->W * 8, hipMemcpyDeviceToHost));
  }
  return AGX_OK;
}

// One read-back of every counter: the apply's per-block counters are summed and the messages in
// flight (backlog + tells of the last apply + staged) counted on the device, into the d_stats
// block, which comes back with ONE copy and ONE stream sync.
agx_status read_counters(agx_engine* e, uint64_t* s) {
  hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(kScanThreads), 0, e->stream, e->d_bstats, kMaxApplyGrid, e->d_sred);
  if (e->fused)
    hipLaunchKernelGGL(k_inflight_fused, dim3(1), dim3(kScanThreads), 0, e->stream, e->d_blc[0], e->d_blc[1],
                       e->d_emc[0], e->d_emc[1], e->d_stg_cnt, e->par ^ 1u, e->nb, (unsigned long long*)e->d_inflight);
  else
    hipLaunchKernelGGL(k_inflight, dim3(1), dim3(kScanThreads), 0, e->stream, e->d_chunk_cnt, e->nchunks,
                       (unsigned long long*)e->d_inflight, e->ring_live || e->rg_on ? e->d_ring_total : nullptr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(e->h_stat, e->d_stats, kStatBlk * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  memcpy(s, e->h_stat, kStatBlk * 8);
  return AGX_OK;
}

// The kernels' sticky error word -> status.  The bits are never cleared: after a capacity
// overflow mail was dropped, after a counter wrap a slot is wrong, so every later result of the
// engine is suspect -- each later agx_run / agx_get_stats reports the same error (agx_get_stats
// still fills its counters); destroy the engine and start over.
agx_status error_status(const agx_engine* e, uint64_t err) {
  if (err & kErrRange)
    return set_err(AGX_ERANGE, "a GCounter/PNCounter slot exceeded 2^64 - 1 (u64 slots; the reference uses BigInt)");
  if (err & kErrCapacity)
    return set_err(AGX_ECAPACITY, "in-flight messages exceeded engine capacity (msg_capacity=%llu)",
                   (unsigned long long)e->cap);
  if (err & kErrBarrier)
    return set_err(AGX_EDEVICE, "a persistent superstep launch's grid barrier timed out (not every block was "
                   "resident); unset AGX_PERSIST to avoid the persistent launch");
  return AGX_OK;
}

// counters -> agx_stats (filled even when an error is reported); check: report an error
// recorded by the kernels
agx_status collect_stats(agx_engine* e, agx_stats* out, bool check) {
  uint64_t s[kStatBlk];
  AGX_TRY(read_counters(e, s));
  e->inflight_dev = s[kStatInfl];  // (exact until the next agx_run: agx_stage_tells' capacity check)
  e->inflight_known = true;
  const agx_status est = check ? error_status(e, s[ST_ERROR]) : AGX_OK;
  const uint64_t* bs = s + kStatSred;
  agx_stats st{};
  st.delivered = bs[0];
  st.dead_letters = s[ST_DEAD] + bs[1] + e->staged_dead;
  st.unhandled = bs[2];
  st.emitted = bs[3];
  st.staged = e->staged_total;
  st.supersteps = s[ST_STEPS] + e->host_steps;
  // backlog + tells produced by the last apply, plus host tells not yet consumed
  st.in_flight = s[kStatInfl] + e->n_staged_dev + e->hs_key.size();
  // B = E_in + f_out*E_out + 2*S*(A/M); kind+alive bytes read per activation.
  // S = the state words a behaviour touches: words 0-1 (plain and compiled behaviours), a CRDT's
  // data words (a full-state merge reads and writes all of them), or with delta-CRDT replication
  // the envelope/selector words plus one element (a delta touches a few elements; rows not counted).
  uint64_t sw = std::min<uint64_t>(e->W, 2);
  const uint32_t km = e->kinds_mask;
  if (km & kb(AGX_KIND_GCOUNTER)) sw = std::max<uint64_t>(sw, AGX_GCOUNTER_WORDS);
  if (km & kb(AGX_KIND_PNCOUNTER)) sw = std::max<uint64_t>(sw, AGX_PNCOUNTER_WORDS);
  if (km & kb(AGX_KIND_ORSET)) sw = std::max<uint64_t>(sw, e->delta_max ? AGX_DELTA_ENV_WORDS + 4 : AGX_ORSET_WORDS);
  st.bytes_alg = 12ull * st.delivered + 12ull * st.emitted + (16ull * std::min<uint64_t>(sw, e->W) + 2ull) * bs[4];
  if (out) *out = st;
  return est;
}

// one superstep on one rank: [chunks] -> group by bucket -> in-bucket sort + drain + apply -> [chunks]
agx_status launch_step_single(agx_engine* e) {
  if (e->fused) return launch_apply(e, e->A);  // one kernel per superstep
  AGX_TRY(launch_staged_chunk(e));
  DevMsgs* sorted = nullptr;
  AGX_TRY(launch_bucket_sort(e, true, &sorted));
  AGX_TRY(launch_apply(e, *sorted));
  return AGX_OK;
}

// The persistent fused launch: a strict replay whose every superstep is the dense
// launch alone runs its K supersteps in ONE launch of k_dense_fused<.., true> -- one block per bucket,
// a grid barrier between supersteps, the actors' state words kept in registers -- instead of K
// launches.  Only when all nb blocks are resident at once (the barrier waits for every block): nb <=
// resident blocks per CU x CUs.  Opt-in (AGX_PERSIST=1): 3.8x slower than K graph-replayed launches on
// the 1M ring (47 vs 12.5 us per superstep) -- the grid barrier costs more than a
// kernel boundary.
bool persist_ok(agx_engine* e) {
  const uint32_t vid = apply_variant(e);
  if (e->persist >= 0 && e->persist_vid != vid) e->persist = -1;  // (kinds registered since: re-decide)
  if (e->persist < 0) {
    e->persist_vid = vid;
    e->persist = 0;
    const char* k = getenv("AGX_PERSIST");
    int per_cu = 0, dev = 0, ncu = 0;
    if (k && atoi(k) != 0 && e->R == 1 && e->fused &&
        agx_dense_persist_occupancy(vid, &per_cu) == hipSuccess && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      e->persist = (uint64_t)e->nb <= (uint64_t)per_cu * (uint64_t)ncu ? 1 : 0;
    (void)hipGetLastError();
  }
  return e->persist == 1 && e->fused && e->strict_cap && e->dense_alone && dense_on(e, vid) && !e->skew_only &&
         !e->recover_dense;
}

// hipGraph of `steps` supersteps (the launch-bound inner loop): replayed
// instead of 10+ eager launches per superstep.
agx_status capture_steps(agx_engine* e, uint32_t steps, hipGraphExec_t* out) {
  hipGraph_t g = nullptr;
  HIP_TRY(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
  agx_status st = AGX_OK;
  e->captured_persist = false;
  if (steps > 1 && persist_ok(e)) {  // one persistent launch for the replay's supersteps
    e->cur_slot = 0;
    e->persist_steps = steps;
    st = launch_step_single(e);
    e->persist_steps = 0;
    e->captured_persist = true;
  } else {
    for (uint32_t i = 0; i < steps && st == AGX_OK; ++i) {
      e->cur_slot = i;  // fused: the i-th superstep of the replay reports its inbox sizes in row i
      st = launch_step_single(e);
    }
  }
  e->cur_slot = 0;
  if (st == AGX_OK && e->fused)  // the replay's rows and abort marks -> host ring slot (no D2H copy)
    hipLaunchKernelGGL(k_replay_out, dim3(1), dim3(kScanThreads), 0, e->stream, e->d_cntb, steps * e->nb,
                       e->strict_cap ? e->d_abort : nullptr, (const unsigned long long*)(e->d_stats + ST_ERROR), e->d_ring,
                       e->d_rctr, agx_engine::kGraphSteps * e->nb + kRingTail);
  hipError_t ce = hipStreamEndCapture(e->stream, &g);
  if (st) {
    if (g) hipGraphDestroy(g);
    return st;
  }
  if (ce != hipSuccess) return set_err(AGX_EDEVICE, "hipStreamEndCapture: %s", hipGetErrorString(ce));
  hipError_t ie = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (ie != hipSuccess) return set_err(AGX_EDEVICE, "hipGraphInstantiate: %s", hipGetErrorString(ie));
  // upload now: a graph's first launch would otherwise pay the upload inside the budget that
  // first replays it (the 8-superstep graphs are first used by longer runs than the warmup)
  hipError_t ue = hipGraphUpload(*out, e->stream);
  if (ue != hipSuccess) return set_err(AGX_EDEVICE, "hipGraphUpload: %s", hipGetErrorString(ue));
  return AGX_OK;
}

agx_status run_single(agx_engine* e, uint32_t max_steps) {
  constexpr uint32_t kLag = 4;  // replays in flight before the host polls quiescence
  for (auto& x : e->lag_ev)
    if (!x) HIP_TRY(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  hipEvent_t* ev = e->lag_ev;
  agx_status st = AGX_OK;
  uint32_t left = max_steps;
  // fused with dense-alone strict replays: the superstep that consumes host-staged tells runs eagerly
  // (block launch beside the dense launch): every bucket with staged tells would otherwise leave the
  // dense launch and void the replay
  bool eager_first = left && e->fused && e->stg_pending && e->dense_alone && dense_on(e, apply_variant(e));
  // staged host tells enter through an eager step (the graphs assume none)
  if (left && e->fused && e->stg_pending) {  // the next superstep consumes the staged tells
    e->stg_pending = false;
    e->hd_key.clear();
    e->hd_src.clear();
    e->hd_pay.clear();
  }
  if (left && e->n_staged_dev) {
    st = launch_step_single(e);
    --left;
  }
  const bool use_graph = !e->prof && e->graphs_enabled;
  bool strict = e->fused && use_graph && e->strict_ok;  // replays without skew launches (see d_abort)
  const uint32_t max_si = e->max_replay_si;
  auto size_idx = [&](uint32_t l) -> uint32_t {
    uint32_t si = l >= 16 ? 4u : l >= 8 ? 3u : l >= 4 ? 2u : l >= 2 ? 1u : 0u;
    return si < max_si ? si : max_si;
  };
  auto graph = [&](uint32_t si) -> hipGraphExec_t& {
    return e->fused ? e->gx[strict][e->par][si] : e->gx[0][e->par][si];
  };
  // every replay size (and, fused, both starting parities) is captured at first use, so no
  // capture ever lands in the middle of a later budget
  auto ensure_graphs = [&]() -> agx_status {
    if (!use_graph) return AGX_OK;
    const uint32_t p0 = e->par;  // capturing advances the host parity: restore it
    e->strict_cap = strict;
    agx_status s2 = AGX_OK;
    for (uint32_t p = 0; p < 2u && s2 == AGX_OK; ++p)  // (both starting parities: arenas are kernel arguments)
      for (uint32_t si = 0; si < agx_engine::kNSizes && s2 == AGX_OK; ++si) {
        hipGraphExec_t& g = e->fused ? e->gx[strict][p][si] : e->gx[0][p][si];
        if (g) continue;
        e->par = p;
        s2 = capture_steps(e, kGraphSizes[si], &g);
        (e->fused ? e->gx_persist[strict][p][si] : e->gx_persist[0][p][si]) = s2 == AGX_OK && e->captured_persist;
      }
    e->par = p0;
    e->strict_cap = false;
    return s2;
  };
  // agx_run(0): capture the replay graphs now (setup, like building the kernels), so that a run
  // timed from its first superstep -- bench.py's C3 tree -- does not pay ~10 graph captures inside
  // (the replays assume no host-staged chunk: a pending one is set aside for the capture -- the first
  // superstep of the next run consumes it eagerly, as always)
  if (max_steps == 0 && use_graph) {
    const uint32_t nsd = e->n_staged_dev;
    e->n_staged_dev = 0;
    const agx_status s2 = ensure_graphs();
    e->n_staged_dev = nsd;
    return s2;
  }
  // fused: per-superstep inbox sizes of each replay (pinned ring); the host counts the supersteps
  // with mail and stops at the first replay whose last superstep had none (quiescent)
  uint32_t rep_steps[kLag] = {0, 0, 0, 0};
  uint32_t rep_start[kLag] = {0, 0, 0, 0}, rep_par[kLag] = {0, 0, 0, 0};  // supersteps launched before it; parity
  bool rep_strict[kLag] = {false, false, false, false}, rep_void[kLag] = {false, false, false, false};
  const size_t ring_row = (size_t)agx_engine::kGraphSteps * e->nb + kRingTail;  // rows, 2 abort marks, the error word
  uint32_t rep_ring[kLag] = {0, 0, 0, 0};  // host ring slot of each replay in flight
  const uint32_t left0 = left;
  uint32_t launched_steps = 0;
  bool recovered = false;
  int last_ring = -1;  // ring slot of the last fused replay launched (-1: eager work came last)
  auto fused_poll = [&](uint32_t slot) -> bool {
    const uint32_t* h = e->h_cntb + rep_ring[slot] * ring_row;
    bool last_empty = rep_steps[slot] > 0;
    for (uint32_t i = 0; i < rep_steps[slot]; ++i) {
      uint64_t t = 0;
      bool skew = false;  // a bucket's inbox over one LDS tile (it took the skew launch)
      for (uint32_t b = 0; b < e->nb; ++b) {
        const uint32_t v = h[(size_t)i * e->nb + b];
        t += v;
        skew |= v > (uint32_t)kBucket;
      }
      if (t) ++e->host_steps;
      e->clean_steps = skew ? 0u : e->clean_steps + 1u;
      last_empty = t == 0;
    }
    rep_steps[slot] = 0;
    return last_empty;
  };
  // A strict replay whose superstep k deferred a skewed bucket: supersteps after k (and every
  // replay launched after it) were no-ops.  Run k's skew launch, count k + 1 supersteps for this
  // replay, void the later ones, continue with the full graphs.
  // (A dense-alone strict replay -- k_dense_fused the whole superstep -- left its non-dense buckets
  // marked: k's block launch over the marks, then its skew launch; the strict graphs are recaptured
  // with the block launch from then on.)
  auto recover = [&](uint32_t slot, uint32_t k) -> agx_status {
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->par = rep_par[slot] ^ (k & 1u);
    e->cur_slot = k;
    const bool dense = e->dense_alone && dense_on(e, apply_variant(e));
    if (getenv("AGX_DEBUG_RECOVER")) {  // diagnostic: which buckets the aborting superstep left
      std::vector<uint32_t> bl(e->nb);
      if (dense) hipMemcpy(bl.data(), e->d_blist, e->nb * 4, hipMemcpyDeviceToHost);
      uint32_t nm = 0, first = ~0u;
      for (uint32_t b = 0; b < e->nb; ++b)
        if (bl[b]) {
          ++nm;
          if (first == ~0u) first = b;
        }
      fprintf(stderr, "[agx recover] replay slot %u superstep %u (launched %u): %s, %u buckets marked (first %u)\n", slot, k,
              rep_start[slot] + k, dense ? "dense-alone" : "skew", nm, first);
    }
    e->skew_only = !dense;
    e->recover_dense = dense;
    last_ring = -1;  // (eager launches after the replays: the error word is copied back)
    agx_status s2 = launch_apply(e, e->A);  // (advances e->par past superstep k)
    e->skew_only = false;
    e->recover_dense = false;
    e->cur_slot = 0;
    if (dense) {
      e->dense_alone = false;
      for (auto& a : e->gx[1])  // (strict graphs only: the replays in flight are full or void)
        for (auto& g : a) {
          if (g) hipGraphExecDestroy(g);
          g = nullptr;
        }
    }
    AGX_TRY(s2);
    HIP_TRY(hipMemcpyAsync(e->h_cntb + rep_ring[slot] * ring_row + (size_t)k * e->nb, e->d_cntb + (size_t)k * e->nb,
                           (size_t)e->nb * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemsetAsync(e->d_abort, 0, 8, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    rep_steps[slot] = k + 1u;
    for (uint32_t q = 0; q < kLag; ++q)
      if (q != slot && rep_steps[q]) rep_void[q] = true;
    left = left0 - (rep_start[slot] + k + 1u);
    strict = false;
    e->strict_ok = false;
    recovered = true;
    return AGX_OK;
  };
  auto poll = [&](uint32_t slot) -> bool {  // true: quiescent
    if (rep_void[slot]) {
      rep_void[slot] = false;
      rep_steps[slot] = 0;
      return false;
    }
    if (rep_strict[slot] && rep_steps[slot]) {
      const uint32_t* ha = e->h_cntb + rep_ring[slot] * ring_row + agx_engine::kGraphSteps * e->nb;
      const uint32_t ab = ha[0] ? ha[0] : ha[1];
      if (ab) {
        const agx_status s2 = recover(slot, ab - 1u);
        if (s2 != AGX_OK) {
          st = s2;
          return true;
        }
      }
    }
    return fused_poll(slot);
  };
  uint32_t launched = 0;
  bool quiet = false;
  for (uint32_t it = 0; st == AGX_OK && left > 0; ++it) {
    const uint32_t slot = it % kLag;
    if (it >= kLag) {
      hipEventSynchronize(ev[slot]);
      if (e->fused) {
        if (poll(slot)) {
          quiet = true;
          break;
        }
        if (left == 0) break;  // (a recovery recounted the supersteps run)
        // two full replays without a skewed bucket: back to the strict graphs (a workload whose
        // skew was transient -- a Zipf burst -- regains the cheaper replays)
        if (!strict && use_graph && e->strict_env && e->clean_steps >= 2 * agx_engine::kGraphSteps) {
          strict = true;
          e->strict_ok = true;
        }
      } else if (e->h_pin[slot] == 0) {
        break;  // that replay ended on a superstep with no mail: quiescent
      }
    }
    uint32_t cnt;
    const uint32_t par0 = e->par;
    const bool eager_now = eager_first;
    eager_first = false;
    if (use_graph && eager_now) {  // one eager superstep, reported through the replay ring like a replay of 1
      cnt = 1;
      st = launch_step_single(e);
      if (st == AGX_OK)
        hipLaunchKernelGGL(k_replay_out, dim3(1), dim3(kScanThreads), 0, e->stream, e->d_cntb, e->nb, nullptr,
                           (const unsigned long long*)(e->d_stats + ST_ERROR), e->d_ring, e->d_rctr,
                           agx_engine::kGraphSteps * e->nb + kRingTail);
    } else if (use_graph) {
      st = ensure_graphs();
      if (st != AGX_OK) break;
      const uint32_t si = size_idx(left);
      cnt = kGraphSizes[si];
      hipError_t ge = hipGraphLaunch(graph(si), e->stream);
      if (ge != hipSuccess) {  // nothing ran: no parity, ring slot or replay-counter change
        st = set_err(AGX_EDEVICE, "hipGraphLaunch: %s", hipGetErrorString(ge));
        break;
      }
      if (cnt & 1u) e->par ^= 1u;  // the replayed supersteps advanced the parity
      if (e->fused && e->gx_persist[strict][par0][si]) {
        ++e->persist_launches;
        e->persist_supersteps += cnt;
      }
    } else {
      cnt = 1;
      st = launch_step_single(e);
    }
    left -= cnt;
    ++launched;
    if (e->fused) {  // per-superstep inbox sizes of this replay
      rep_steps[slot] = cnt;
      rep_start[slot] = launched_steps;
      rep_par[slot] = par0;
      rep_strict[slot] = strict && !eager_now;
      rep_void[slot] = false;
      if (use_graph) {  // written by the graph's k_replay_out into ring slot (replay counter % kLag)
        rep_ring[slot] = (uint32_t)(e->replay_ctr++ % kLag);
        last_ring = (int)rep_ring[slot];
      } else {          // eager superstep: copied (the ring slots are all free between run_single calls)
        last_ring = -1;
        rep_ring[slot] = slot;
        uint32_t* hr = e->h_cntb + slot * ring_row;
        hipMemcpyAsync(hr, e->d_cntb, (size_t)cnt * e->nb * 4, hipMemcpyDeviceToHost, e->stream);
        hr[agx_engine::kGraphSteps * e->nb] = hr[agx_engine::kGraphSteps * e->nb + 1] = 0u;
      }
    } else {  // inbox total (sorted + backlog) of the replay's last superstep
      hipMemcpyAsync(&e->h_pin[slot], e->d_ninbox, 4, hipMemcpyDeviceToHost, e->stream);
    }
    launched_steps += cnt;
    hipEventRecord(ev[slot], e->stream);
  }
  if (e->timing) {  // (agx_run_timed: after the last replay, before the sync)
    hipEventRecord(e->tev[1], e->stream);
    e->tev1_recorded = true;
  }
  // the kernels' error word rides on the final sync (agx_run checks it even when out == NULL): in the
  // last replay's ring row (k_replay_out) when a fused replay ended the run, else copied back
  if (last_ring < 0) hipMemcpyAsync(e->h_stat + ST_ERROR, e->d_stats + ST_ERROR, 8, hipMemcpyDeviceToHost, e->stream);
  hipStreamSynchronize(e->stream);
  if (last_ring >= 0) {
    const uint32_t* t = e->h_cntb + (size_t)last_ring * ring_row + ring_row - 2;
    e->h_stat[ST_ERROR] = (uint64_t)t[0] | ((uint64_t)t[1] << 32);
  }
  if ((e->h_stat[ST_ERROR] & kErrBarrier) && e->persist != 0) {  // (never again on this engine)
    e->persist = 0;
    drop_graphs(e);
  }
  const bool rec0 = recovered;
  if (e->fused && !quiet)  // replays not polled yet, in launch order
    for (uint32_t k = launched > kLag ? launched - kLag : 0; k < launched && st == AGX_OK; ++k)
      if (poll(k % kLag)) {
        quiet = true;
        break;
      }
  if (recovered && !rec0) {  // (a recovery above launched more work: its errors too)
    hipMemcpyAsync(e->h_stat + ST_ERROR, e->d_stats + ST_ERROR, 8, hipMemcpyDeviceToHost, e->stream);
    hipStreamSynchronize(e->stream);
  }
  if (st == AGX_OK && recovered && !quiet && left > 0) return run_single(e, left);  // full graphs now
  return st;
}

// received state gossips -> rx rows (single kernel over the received range)
agx_status fix_rx(agx_engine* e, const Plan& p) {
  if (!e->pw || !p.n_recv) return AGX_OK;
  const uint32_t lo = (uint32_t)p.n_bl, hi = (uint32_t)(p.n_bl + p.n_recv);
  const uint32_t slo = (uint32_t)p.recv_off[e->rank], shi = (uint32_t)(p.recv_off[e->rank] + p.recv_cnt[e->rank]);
  hipLaunchKernelGGL(k_fix_rx, dim3(grid_for(p.n_recv / kThreads + 1, 2048)), dim3(kThreads), 0, e->stream, e->A.m(),
                     lo, hi, slo, shi, (uint32_t)e->heap_rows);
  HIP_TRY(hipGetLastError());
  return AGX_OK;
}

agx_status exchange_rccl(agx_engine* e, Plan& p) {
  // one contiguous (key, src, payload) run per peer: R sends instead of 3R (k_pack_aos / k_unpack_aos)
  hipLaunchKernelGGL(k_pack_aos, dim3(grid_for(e->cap_emit / kThreads + 1, 2048)), dim3(kThreads), 0, e->stream,
                     e->s2.c(), e->d_total, e->d_s2p);
  HIP_TRY(hipGetLastError());
  NCCL_TRY(ncclGroupStart());
  for (uint32_t q = 0; q < e->R; ++q) {
    if (p.send_cnt[q]) {
      const uint64_t o = p.send_off[q], n = p.send_cnt[q];
      NCCL_TRY(ncclSend(e->d_s2p + 3 * o, 3 * n, ncclUint32, (int)q, e->comm, e->stream));
      if (q != e->rank) {
        e->mr_sent_env += 12 * n;
        e->mr_sent_rows += 4ull * n * e->pw;
      }
      if (e->pw && q != e->rank)
        NCCL_TRY(ncclSend(e->d_s2rows + o * e->pw, n * e->pw, ncclUint32, (int)q, e->comm, e->stream));
    }
    if (p.recv_cnt[q]) {
      const uint64_t o = p.recv_off[q], n = p.recv_cnt[q];
      NCCL_TRY(ncclRecv(e->d_rcvp + 3 * (o - p.n_bl), 3 * n, ncclUint32, (int)q, e->comm, e->stream));
      if (e->pw && q != e->rank)
        NCCL_TRY(ncclRecv(e->d_rx + o * e->pw, n * e->pw, ncclUint32, (int)q, e->comm, e->stream));
    }
  }
  NCCL_TRY(ncclGroupEnd());
  if (p.n_recv) {  // received runs in sender-rank order after the local backlog (the sharded canonical order)
    hipLaunchKernelGGL(k_unpack_aos, dim3(grid_for(p.n_recv / kThreads + 1, 2048)), dim3(kThreads), 0, e->stream,
                       e->d_rcvp, (uint32_t)p.n_recv, e->A.m(), (uint32_t)p.n_bl);
    HIP_TRY(hipGetLastError());
  }
  return AGX_OK;
}

// ---- device-resident multi-rank supersteps (k_mr_pack / k_mr_unpack, agx_kernels.h)
// first slab: 17/16 of an even share of one superstep's tells per (sender, receiver) pair, + 1024
// (round 6; was 5/4): the wire bytes are slab-sized, and hash-sharded mail is even to within a few
// standard deviations (the 1M-per-rank ring: 125 K +- 0.35 K per pair at R = 8); skewed mail overflows
// once, takes the exact exchange for that superstep and grows the slabs to 5/4 of the largest count.
// Every rank must size it alike (the sends and receives are fixed-size): it depends on n_global,
// max_emit and R only, which the layout check compares (AGX_MR_SLAB overrides, on every rank).
uint32_t mr_initial_slab(const agx_engine* e) {
  if (const char* s = getenv("AGX_MR_SLAB")) return (uint32_t)std::max(1, atoi(s));
  const uint64_t share = e->n_global * e->kmax / ((uint64_t)e->R * e->R);
  return (uint32_t)std::min<uint64_t>(share + share / 16 + 1024, 1u << 30);
}

// (re)allocate the per-peer send / receive slabs (the same size on every rank: the decision to grow
// comes from the all-gathered counts, which every rank reads alike).  CRDT rows travel slab-sized
// too (R x slab rows of pw u32 to send and as many to receive): when they would leave the row handle
// space, pass the row budget (AGX_MR_ROW_MB, default 16384 MiB of the 288 GB HBM per rank) or fail
// to allocate on ANY rank -- all-gathered, so every rank decides alike -- every rank sets mr_host
// and runs the host-planned exchange (exact per-peer sizes) from then on.
agx_status mr_slabs(agx_engine* e, uint64_t want) {
  const uint32_t n = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(want, 64), 1u << 30);
  if (n <= e->slab) return AGX_OK;
  HIP_TRY(hipStreamSynchronize(e->stream));
  hipFree(e->d_sslab);
  hipFree(e->d_rslab);
  e->d_sslab = e->d_rslab = nullptr;
  e->slab = 0;
  drop_graphs(e);  // (the slabs are kernel and collective arguments of a captured replay)
  // this rank's verdict: 0 = the slabs fit, 1 = the envelope slabs fit but the CRDT row slabs do not
  // (host-planned exchange from now on), 2 = an allocation the exchange cannot do without failed.
  // No rank returns before the all-gather below: a rank that left early would leave its peers
  // blocked in the collective (every rank must take the same decision, from the same answers).
  uint64_t code = 0;
  if (dalloc(&e->d_sslab, (uint64_t)e->R * n * 3) != AGX_OK || dalloc(&e->d_rslab, (uint64_t)e->R * n * 3) != AGX_OK)
    code = 2;
  if (e->pw) {  // CRDT rows: row send slabs, and rx large enough to receive R slabs of rows
    const uint64_t rr = (uint64_t)e->R * n;
    const char* mb = getenv("AGX_MR_ROW_MB");
    const uint64_t budget = (mb ? (uint64_t)std::max(0, atoi(mb)) : 16384ull) << 20;
    hipFree(e->d_srows);
    e->d_srows = nullptr;
    bool fits = code == 0 && e->heap_rows + std::max<uint64_t>(rr, e->rx_rows) < kHandleMask &&
                2 * rr * e->pw * 4 <= budget;
    if (fits && dalloc(&e->d_srows, rr * e->pw) != AGX_OK) fits = false;
    if (fits && rr > e->rx_rows) {
      hipFree(e->d_rx);
      e->d_rx = nullptr;
      if (dalloc(&e->d_rx, rr * e->pw) == AGX_OK) {
        e->rx_rows = rr;
      } else {  // (the host-planned path needs rx of cap rows again)
        fits = false;
        e->rx_rows = 0;
        if (dalloc(&e->d_rx, e->cap * e->pw) == AGX_OK)
          e->rx_rows = e->cap;
        else
          code = 2;
      }
    }
    if (!fits && code == 0) code = 1;
  }
  (void)hipGetLastError();  // (a refused allocation is an answer here, not an error)
  set_err(AGX_OK, "");
  // every rank's verdict (the exchange sizes must agree)
  e->h_pin64[0] = code;
  HIP_TRY(hipMemcpyAsync(e->d_cvec, e->h_pin64, 8, hipMemcpyHostToDevice, e->stream));
  NCCL_TRY(ncclAllGather(e->d_cvec, e->d_cmat, 1, ncclUint64, e->comm, e->stream));
  HIP_TRY(hipMemcpyAsync(e->h_pin64, e->d_cmat, (size_t)e->R * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  uint64_t worst = 0;
  for (uint32_t r = 0; r < e->R; ++r) worst = std::max<uint64_t>(worst, e->h_pin64[r]);
  if (worst >= 2) {  // every rank fails alike
    hipFree(e->d_sslab);
    hipFree(e->d_rslab);
    hipFree(e->d_srows);
    e->d_sslab = e->d_rslab = nullptr;
    e->d_srows = nullptr;
    return set_err(AGX_ENOMEM, "rank %u: exchange slabs of %u envelopes per peer could not be allocated on %s",
                   e->rank, n, code >= 2 ? "this rank" : "a peer rank");
  }
  if (worst == 1) {
    hipFree(e->d_srows);
    e->d_srows = nullptr;
    e->mr_host = true;
    if (getenv("AGX_MR_DEBUG"))
      fprintf(stderr, "[agx rank %u] CRDT row slabs of %u rows per peer do not fit on every rank: host-planned "
              "exchange\n", e->rank, n);
  }
  e->slab = n;
  return AGX_OK;
}

agx_status mr_step_dev(agx_engine* e, uint32_t idx);

// All-or-nothing capture: every rank all-gathers its capture result before the first replay, and a
// rank keeps its graph only if every rank captured -- otherwise all of them replay eagerly.  (A rank
// replaying its captured collectives while a peer issues the same collectives eagerly is legal for
// RCCL, but one rank's failed capture must not leave the ranks on different paths whose first
// launches then wait on each other.)
agx_status mr_agree_capture(agx_engine* e) {
  e->h_pin64[0] = e->mr_gx ? 1u : 0u;
  HIP_TRY(hipMemcpyAsync(e->d_cvec, e->h_pin64, 8, hipMemcpyHostToDevice, e->stream));
  NCCL_TRY(ncclAllGather(e->d_cvec, e->d_cmat, 1, ncclUint64, e->comm, e->stream));
  HIP_TRY(hipMemcpyAsync(e->h_pin64, e->d_cmat, (size_t)e->R * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  uint32_t ok = 0;
  for (uint32_t r = 0; r < e->R; ++r) ok += e->h_pin64[r] ? 1u : 0u;
  if (getenv("AGX_MR_DEBUG"))
    fprintf(stderr, "[agx rank %u] multi-rank replay capture: %u of %u ranks captured%s\n", e->rank, ok, e->R,
            ok == e->R ? "" : " -> eager replays on every rank");
  if (ok != e->R) {
    if (e->mr_gx) hipGraphExecDestroy(e->mr_gx);
    e->mr_gx = nullptr;
    e->mr_graph_ok = false;
  }
  return AGX_OK;
}

// kMrReplay device-resident supersteps as one graph.  A failed capture (a collective that cannot be
// captured) ends the capture, clears mr_graph_ok and returns AGX_OK: the caller replays eagerly.
agx_status capture_mr(agx_engine* e, uint32_t steps) {
  hipGraph_t g = nullptr;
  if (hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    (void)hipGetLastError();
    e->mr_graph_ok = false;
    return AGX_OK;
  }
  agx_status st = AGX_OK;
  for (uint32_t i = 0; i < steps && st == AGX_OK; ++i) st = mr_step_dev(e, i);
  hipError_t ce = hipStreamEndCapture(e->stream, &g);
  hipGraphExec_t x = nullptr;
  if (st == AGX_OK && ce == hipSuccess && g && hipGraphInstantiate(&x, g, nullptr, nullptr, 0) == hipSuccess &&
      hipGraphUpload(x, e->stream) == hipSuccess) {
    hipGraphDestroy(g);
    e->mr_gx = x;
    if (getenv("AGX_MR_DEBUG")) fprintf(stderr, "[agx rank %u] multi-rank replay captured (%u supersteps)\n", e->rank, steps);
    return AGX_OK;
  }
  if (getenv("AGX_MR_DEBUG"))
    fprintf(stderr, "[agx rank %u] multi-rank replay capture failed (status %d, %s): eager replays\n", e->rank, (int)st,
            hipGetErrorString(ce));
  if (x) hipGraphExecDestroy(x);
  if (g) hipGraphDestroy(g);
  (void)hipGetLastError();
  e->mr_graph_ok = false;
  set_err(AGX_OK, "");  // (the eager replays report their own errors)
  return AGX_OK;
}

// one superstep with no host round trip: phase 1, count all-gather, the decision and the send
// slabs (k_mr_pack), one fixed-size send / receive per peer, unpack, bucket passes, apply
agx_status mr_step_dev(agx_engine* e, uint32_t idx) {
  const uint32_t S = e->R + 2;
  const bool direct = e->pw == 0 && !getenv("AGX_MR_NO_DIRECT");  // (CRDT rows are laid out beside s2's tells)
  AGX_TRY(phase1(e, direct));
  MrArgs a{};
  a.cmat = e->d_cmat;
  a.s2 = e->s2.c();
  a.sslab = e->d_sslab;
  a.rslab = e->d_rslab;
  a.A = e->A.m();
  a.d_n = e->d_n;
  a.halt = e->d_halt;
  a.stats = e->d_stats;
  a.cap = e->cap;
  a.R = e->R;
  a.rank = e->rank;
  a.slab = e->slab;
  a.step = idx;
  a.s2rows = e->d_s2rows;
  a.srows = e->d_srows;
  a.pw = e->pw;
  a.heap_rows = (uint32_t)e->heap_rows;
  a.direct = direct ? 1u : 0u;
  e->mr_direct = direct;
  const dim3 g(grid_for((uint64_t)e->R * e->slab / kThreads + 1, 2048));
  {
    Scope sc(e, K_EXCHANGE);
    NCCL_TRY(ncclAllGather(e->d_cvec, e->d_cmat, S, ncclUint64, e->comm, e->stream));
    hipLaunchKernelGGL(k_mr_pack, g, dim3(kThreads), 0, e->stream, a);
    NCCL_TRY(ncclGroupStart());
    for (uint32_t q = 0; q < e->R; ++q) {
      if (q == e->rank) continue;
      NCCL_TRY(ncclSend(e->d_sslab + (size_t)q * e->slab * 3, 3ull * e->slab, ncclUint32, (int)q, e->comm, e->stream));
      NCCL_TRY(ncclRecv(e->d_rslab + (size_t)q * e->slab * 3, 3ull * e->slab, ncclUint32, (int)q, e->comm, e->stream));
      if (e->pw) {  // the state gossips' rows, slab-sized as well
        NCCL_TRY(ncclSend(e->d_srows + (size_t)q * e->slab * e->pw, (size_t)e->slab * e->pw, ncclUint32, (int)q, e->comm,
                          e->stream));
        NCCL_TRY(ncclRecv(e->d_rx + (size_t)q * e->slab * e->pw, (size_t)e->slab * e->pw, ncclUint32, (int)q, e->comm,
                          e->stream));
      }
    }
    NCCL_TRY(ncclGroupEnd());
    hipLaunchKernelGGL(k_mr_unpack, g, dim3(kThreads), 0, e->stream, a);
  }
  HIP_TRY(hipGetLastError());
  DevMsgs* sorted = nullptr;
  AGX_TRY(launch_bucket_sort(e, false, &sorted));
  return launch_apply(e, *sorted);
}

agx_status run_multi_rccl(agx_engine* e, uint32_t max_steps) {
  const uint32_t S = e->R + 2;
  Plan p;
  if (!e->layout_checked) {  // every rank must size rows and tells alike (same register_range / set_* calls):
                             // the send/recv sizes of the exchange are derived from them
    const uint64_t sig[2] = {((uint64_t)e->pw << 32) | e->delta_max, ((uint64_t)e->kmax << 32) | e->W};
    e->h_pin64[0] = sig[0];  // (pinned: the async copy reads it after this call returns)
    e->h_pin64[1] = sig[1];
    HIP_TRY(hipMemcpyAsync(e->d_cvec, e->h_pin64, 16, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    NCCL_TRY(ncclAllGather(e->d_cvec, e->d_cmat, 2, ncclUint64, e->comm, e->stream));
    HIP_TRY(hipMemcpyAsync(e->h_pin64, e->d_cmat, (size_t)e->R * 16, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (uint32_t r = 0; r < e->R; ++r)
      if (e->h_pin64[2 * r] != sig[0] || e->h_pin64[2 * r + 1] != sig[1])
        return set_err(AGX_EINVAL, "rank %u and rank %u differ in row pitch / delta mode / max_emit / n_words "
                       "(make the same register_range and set_* calls on every rank)", e->rank, r);
    e->layout_checked = true;
  }
  // the host-planned exchange of a superstep whose phase 1 and count all-gather have run:
  // exact sizes from the count matrix (one host round trip); *quiet: nothing was in flight
  auto exact_rest = [&](bool* quiet) -> agx_status {
    HIP_TRY(hipMemcpyAsync(e->h_pin64, e->d_cmat, (size_t)e->R * S * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    make_plan(e, e->h_pin64, p);
    *quiet = p.total_inflight == 0;
    if (*quiet) return AGX_OK;
    if (p.n_bl + p.n_recv + p.n_staged > e->cap)
      return set_err(AGX_ECAPACITY, "rank %u: %llu messages in flight exceed capacity %llu", e->rank,
                     (unsigned long long)(p.n_bl + p.n_recv + p.n_staged), (unsigned long long)e->cap);
    {
      Scope sc(e, K_EXCHANGE);
      AGX_TRY(exchange_rccl(e, p));
    }
    AGX_TRY(fix_rx(e, p));
    return phase2(e, p.n_bl + p.n_recv + p.n_staged, p.n_bl + p.n_recv);
  };
  auto host_step = [&](bool* quiet) -> agx_status {
    AGX_TRY(phase1(e));
    {
      Scope sc(e, K_EXCHANGE);
      NCCL_TRY(ncclAllGather(e->d_cvec, e->d_cmat, S, ncclUint64, e->comm, e->stream));
    }
    return exact_rest(quiet);
  };
  uint32_t left = max_steps;
  bool quiet = false;
  // device-resident replays (CRDT rows travel in row slabs beside the envelope slabs); a staged
  // burst enters through one host-planned superstep (its staged count is a host number)
  const bool dev = !getenv("AGX_MR_HOST") && !e->mr_host;
  // whether ANY rank has staged tells: each rank knows only its own, and a rank that took the
  // host-planned superstep below while a peer went straight to the device replays would issue
  // different collectives than that peer (one all-gather per run, not per superstep)
  bool any_staged = e->n_staged_dev != 0;
  if (dev && left) {
    e->h_pin64[0] = e->n_staged_dev;
    HIP_TRY(hipMemcpyAsync(e->d_cvec, e->h_pin64, 8, hipMemcpyHostToDevice, e->stream));
    NCCL_TRY(ncclAllGather(e->d_cvec, e->d_cmat, 1, ncclUint64, e->comm, e->stream));
    HIP_TRY(hipMemcpyAsync(e->h_pin64, e->d_cmat, (size_t)e->R * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (uint32_t r = 0; r < e->R; ++r) any_staged = any_staged || e->h_pin64[r] != 0;
  }
  if (dev && any_staged && left) {
    AGX_TRY(host_step(&quiet));
    ++e->mr_host_steps;
    --left;
  }
  if (dev && !e->slab) AGX_TRY(mr_slabs(e, mr_initial_slab(e)));
  if (dev && !e->mr_host) {
    constexpr uint32_t kMrReplay = 8;  // supersteps enqueued before the host reads the stop word
    // kMrReplay supersteps captured as one graph (collectives included) and replayed: on by
    // default since round 5, AGX_MR_GRAPH=0 replays eagerly.  (Round 4 kept it opt-in after a run
    // "hung in its first launch"; the trace shows the replays completing and agx_destroy hanging in
    // ncclCommDestroy while the graph still held the communicator's persistent plans -- the graph
    // is now destroyed first, and the whole RCCL-rank suite passes with captured replays.)
    const char* mg = getenv("AGX_MR_GRAPH");
    const bool graphs = !e->prof && e->graphs_enabled && e->mr_graph_ok && (!mg || atoi(mg) != 0);
    while (left && !quiet && !e->mr_host) {
      const uint32_t k = std::min(left, kMrReplay);
      if (graphs && k == kMrReplay && !e->mr_gx) {
        AGX_TRY(capture_mr(e, kMrReplay));
        AGX_TRY(mr_agree_capture(e));
      }
      const bool dbg = getenv("AGX_MR_DEBUG") != nullptr;
      if (graphs && k == kMrReplay && e->mr_gx) {
        if (dbg) fprintf(stderr, "[agx rank %u] graph replay %llu: launch\n", e->rank, (unsigned long long)e->mr_replays);
        HIP_TRY(hipGraphLaunch(e->mr_gx, e->stream));
        ++e->mr_replays;
      } else {
        for (uint32_t i = 0; i < k; ++i) AGX_TRY(mr_step_dev(e, i));
      }
      HIP_TRY(hipMemcpyAsync(e->h_halt, e->d_halt, 8, hipMemcpyDeviceToHost, e->stream));
      HIP_TRY(hipStreamSynchronize(e->stream));
      const uint32_t code = e->h_halt[0], at = e->h_halt[1];
      if (dbg) fprintf(stderr, "[agx rank %u] %s of %u supersteps done: halt %u at %u\n", e->rank,
                       graphs && k == kMrReplay && e->mr_gx ? "graph replay" : "eager replay", k, code, at);
      const uint64_t sent = (uint64_t)(e->R - 1) * e->slab;  // fixed-size slabs per peer, per superstep
      if (!code) {
        left -= k;
        e->mr_dev_steps += k;
        e->mr_sent_env += k * 12 * sent;
        e->mr_sent_rows += k * 4 * sent * e->pw;
        continue;
      }
      left -= at;  // supersteps completed before the one that stopped (its phase 1 and all-gather ran)
      e->mr_dev_steps += at;
      e->mr_sent_env += at * 12 * sent;
      e->mr_sent_rows += at * 4 * sent * e->pw;
      HIP_TRY(hipMemsetAsync(e->d_halt, 0, 8, e->stream));
      if (code == 2u) break;  // nothing in flight (the host path's quiescence, same point)
      if (code == 3u)
        return set_err(AGX_ECAPACITY, "rank %u: messages in flight exceed capacity %llu", e->rank,
                       (unsigned long long)e->cap);
      // a sender -> receiver count over the slab: this superstep's exchange exactly, bigger slabs
      if (e->mr_direct) {  // (its peer runs went into the slabs: back into s2 for the exact exchange)
        hipLaunchKernelGGL(k_slab_to_s2, dim3(grid_for((uint64_t)e->R * e->slab / kThreads + 1, 2048)), dim3(kThreads), 0,
                           e->stream, (const uint64_t*)e->d_cmat, (const uint32_t*)e->d_sslab, e->s2.m(), e->R, e->rank,
                           e->slab);
        HIP_TRY(hipGetLastError());
      }
      AGX_TRY(exact_rest(&quiet));
      ++e->mr_exact;
      ++e->mr_host_steps;
      --left;
      uint64_t mx = 0;
      for (uint32_t r = 0; r < e->R; ++r)
        for (uint32_t q = 0; q < e->R; ++q)
          if (q != r) mx = std::max<uint64_t>(mx, e->h_pin64[r * S + q]);
      AGX_TRY(mr_slabs(e, mx + mx / 4 + 1024));
    }
  }
  // host-planned supersteps: AGX_MR_HOST, or CRDT row slabs that do not fit (mr_slabs)
  for (; left && !quiet; --left) {
    AGX_TRY(host_step(&quiet));
    ++e->mr_host_steps;
  }
  HIP_TRY(hipMemcpyAsync(e->h_stat + ST_ERROR, e->d_stats + ST_ERROR, 8, hipMemcpyDeviceToHost, e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream));
  return AGX_OK;
}

void drop_graphs(agx_engine* e) {
  if (e->mr_gx && getenv("AGX_MR_DEBUG")) fprintf(stderr, "[agx rank %u] multi-rank replay graph dropped\n", e->rank);
  for (auto& a : e->gx)
    for (auto& b : a)
      for (auto& g : b) {
        if (g) hipGraphExecDestroy(g);
        g = nullptr;
      }
  if (e->mr_gx) hipGraphExecDestroy(e->mr_gx);
  e->mr_gx = nullptr;
}

// First CRDT kind (or a wider one): size the snapshot heap for `kind`'s rows (full state, plus
// deltaVersions and DeltaPropagation rows in delta-CRDT mode; include/akka_gpu.h).
agx_status enable_crdt(agx_engine* e, uint32_t kind) {
  const uint32_t words = kind == AGX_KIND_GCOUNTER ? AGX_GCOUNTER_WORDS
                         : kind == AGX_KIND_PNCOUNTER ? AGX_PNCOUNTER_WORDS : AGX_ORSET_WORDS;
  const uint32_t need = !e->delta_max ? words
                        : kind == AGX_KIND_GCOUNTER ? AGX_GCOUNTER_DELTA_WORDS
                        : kind == AGX_KIND_PNCOUNTER ? AGX_PNCOUNTER_DELTA_WORDS : AGX_ORSET_DELTA_WORDS;
  if (e->W < need) return set_err(AGX_EINVAL, "behaviour kind %u needs n_words >= %u", kind, need);
  const uint32_t ru = !e->delta_max ? 2 * words : kind == AGX_KIND_ORSET ? AGX_ORSET_DELTA_ROW_U32
                                                                          : 2 * words + AGX_CRDT_NODES;
  // row pitch in u32: rows wider than one 128-B line start on a line boundary (ORSet: 2080 B
  // rows padded to 2176 B), so a merge's batched row loads never split a line between rows
  const uint32_t pw = ru > kRowAlign ? (ru + kRowAlign - 1) / kRowAlign * kRowAlign : ru;
  if (pw <= e->pw) return AGX_OK;
  if (e->started) return set_err(AGX_ESTATE, "register CRDT kinds before the first agx_run");
  const uint64_t rows = ((uint64_t)e->nb << e->bb) + e->cap;
  if (rows + e->cap > kHandleMask) return set_err(AGX_EINVAL, "CRDT kinds need msg_capacity < 2^28 - n_actors");
  hipFree(e->d_heap);
  hipFree(e->d_rx);
  hipFree(e->d_s2rows);
  e->d_heap = e->d_rx = e->d_s2rows = nullptr;
  e->pw = 0;
  AGX_TRY(dalloc(&e->d_heap, 2 * rows * pw));
  e->heap_rows = rows;
  if (e->R > 1) {
    AGX_TRY(dalloc(&e->d_rx, e->cap * pw));
    AGX_TRY(dalloc(&e->d_s2rows, e->cap_emit * pw));
    e->rx_rows = e->cap;
    hipFree(e->d_srows);
    e->d_srows = nullptr;
    e->slab = 0;  // (the row slabs are sized with the envelope slabs, for this pitch)
  }
  e->pw = pw;
  drop_graphs(e);
  return AGX_OK;
}

agx_status validate_cfg(const agx_cfg* c) {
  if (!c) return set_err(AGX_EINVAL, "null cfg");
  if (c->abi_version != AGX_ABI_VERSION) return set_err(AGX_EINVAL, "abi_version %u != %u", c->abi_version, AGX_ABI_VERSION);
  if (c->n_actors == 0 || c->n_actors >= (1ull << 31)) return set_err(AGX_EINVAL, "n_actors out of range");
  if (c->n_words == 0 || c->n_words > AGX_MAX_WORDS) return set_err(AGX_EINVAL, "n_words must be 1..%u", AGX_MAX_WORDS);
  uint32_t R = c->n_ranks ? c->n_ranks : 1;
  if (R > AGX_MAX_RANKS || c->rank >= R) return set_err(AGX_EINVAL, "bad rank %u / n_ranks %u", c->rank, R);
  if (c->num_shards > (uint32_t)INT32_MAX) return set_err(AGX_EINVAL, "num_shards must be < 2^31 (maxNumberOfShards is an Int)");
  const uint32_t ba = c->bucket_actors;
  if (ba && (ba & (ba - 1) || ba < (1u << kMinBucketBits) || ba > (uint32_t)kBucket))
    return set_err(AGX_EINVAL, "bucket_actors must be 0 or a power of two in [%d, %d]", 1 << kMinBucketBits, kBucket);
  return AGX_OK;
}

}  // namespace

// =========================================================================
// C ABI
// =========================================================================
extern "C" {

const char* agx_last_error(void) { return g_err.c_str(); }
uint32_t agx_abi_version(void) { return AGX_ABI_VERSION; }

// The source hash this library was built from (__graft_entry__.source_hash, passed by build_native);
// the stamp is found in the file's bytes without loading it, so a stale library is rebuilt.
#ifndef AGX_BUILD_HASH
#define AGX_BUILD_HASH "unstamped000000"
#endif
extern "C" __attribute__((used, visibility("default"))) const char agx_build_stamp[] = "AGX_BUILD_HASH=" AGX_BUILD_HASH;
const char* agx_build_hash(void) { return agx_build_stamp + 15; }

int32_t agx_shard_id(uint32_t id, uint32_t num_shards) {
  if (num_shards == 0 || num_shards > (uint32_t)INT32_MAX) return 0;  // (maxNumberOfShards is an Int)
  int32_t h = java_hash_decimal(id);
  int32_t a = (h == INT32_MIN) ? INT32_MIN : (h < 0 ? -h : h);  // math.abs(Int.MinValue) stays negative
  return a % (int32_t)num_shards;
}

uint32_t agx_owner(uint32_t id, uint32_t num_shards, uint32_t n_ranks) {
  if (n_ranks <= 1) return 0;
  int32_t m = agx_shard_id(id, num_shards) % (int32_t)n_ranks;
  return (uint32_t)(m < 0 ? m + (int32_t)n_ranks : m);
}

agx_status agx_create(const agx_cfg* cfg, agx_engine** out) {
  AGX_TRY(validate_cfg(cfg));
  if (!out) return set_err(AGX_EINVAL, "null out");
  auto* e = new agx_engine();
  e->cfg = *cfg;
  e->n_global = cfg->n_actors;
  e->T = cfg->throughput == 0 || (int32_t)cfg->throughput < 0 ? 1u : cfg->throughput;  // Mailbox.scala:261
  e->Traw = e->T;
  e->C = cfg->capacity;
  e->mcap[0] = e->C;
  if (e->C && e->T > e->C) e->T = e->C;  // a bounded queue never holds more than C: drain <= min(T, C)
  e->W = cfg->n_words;
  e->kmax = std::max<uint32_t>(1, cfg->max_emit);
  e->R = cfg->n_ranks ? cfg->n_ranks : 1;
  e->rank = cfg->rank;
  e->num_shards = cfg->num_shards ? cfg->num_shards : 1000;
  e->bb = cfg->bucket_actors ? ceil_log2(cfg->bucket_actors) : (uint32_t)kBucketBits;
  if (const char* s = getenv("AGX_TINY")) e->tiny_max = std::min<uint32_t>(kTinyMax, (uint32_t)std::max(0, atoi(s)));
  if (const char* s = getenv("AGX_TINY_LAUNCH")) e->tiny_launch = atoi(s) != 0;
  if (const char* s = getenv("AGX_DENSE_LAUNCH")) e->dense_launch = atoi(s) != 0 ? 1 : 0;
  if (const char* s = getenv("AGX_DENSE_FUSED")) e->dense_fused = atoi(s) != 0;
  if (const char* s = getenv("AGX_DENSE_OWNER")) e->dense_owner = atoi(s) != 0;
  if (const char* s = getenv("AGX_BUCKET_ACTORS")) {  // diagnostic: override the bucket width (power of two)
    const uint32_t ba = (uint32_t)atoi(s);
    if (ba >= (1u << kMinBucketBits) && ba <= (uint32_t)kBucket && !(ba & (ba - 1))) e->bb = ceil_log2(ba);
  }
  e->graphs_enabled = getenv("AGX_NO_GRAPH") == nullptr && getenv("AGX_STAMPS") == nullptr;
  agx_status st = ensure_dev(e);
  if (st) { delete e; return st; }

  // ShardRegion hash sharding: owner(id) = floor-mod(shardId(id), R); local index = rank among owned ids
  if (e->R > 1) {
    e->h_route.resize(e->n_global);
    uint64_t nl = 0;
    std::vector<uint32_t> cnt(e->R, 0);
    for (uint64_t id = 0; id < e->n_global; ++id) {
      uint32_t o = agx_owner((uint32_t)id, e->num_shards, e->R);
      e->h_route[id] = (o << kOwnerShift) | cnt[o];
      if (o == e->rank) e->h_gid.push_back((uint32_t)id);
      cnt[o]++;
    }
    nl = cnt[e->rank];
    for (uint32_t o = 0; o < e->R; ++o)
      if (cnt[o] > kLocalMask) { delete e; return set_err(AGX_EINVAL, "too many actors per rank"); }
    e->n_local = nl;
  } else {
    if (e->n_global > kLocalMask) { delete e; return set_err(AGX_EINVAL, "n_actors exceeds 2^28 per rank"); }
    e->n_local = e->n_global;
  }
  const uint64_t nl = std::max<uint64_t>(e->n_local, 1);
  e->key_bits = std::max<uint32_t>(1, ceil_log2(nl));
  e->cap = cfg->msg_capacity ? cfg->msg_capacity : std::max<uint64_t>(4 * nl, 1u << 16);
  if (e->cap >= (1ull << 32) - kTile) { delete e; return set_err(AGX_EINVAL, "msg_capacity too large"); }
  e->cap_emit = e->cap * e->kmax;  // bucket b's tells live at [lo*kmax, (lo+cnt)*kmax)
  if (e->cap_emit >= (1ull << 32)) { delete e; return set_err(AGX_EINVAL, "msg_capacity * max_emit must be < 2^32"); }
  {  // largest super-tile of the dense sort passes: about 1024+ workgroups at full capacity; each pass
     // picks its own size from its input (pass_super), down to one tile, so the histogram table is
     // sized for one-tile super-tiles
    const uint64_t mx = std::max(e->cap, e->cap_emit);
    e->dsub = (uint32_t)std::min<uint64_t>(kSub, std::max<uint64_t>(1, mx / ((uint64_t)kTile * 1024)));
  }
  e->max_supers = (uint32_t)((std::max(e->cap, e->cap_emit) + kTile - 1) / kTile + 1);
  e->dstride = (e->max_supers + 3) & ~3u;
  // buckets of 2^bb actors; LSD passes over key bits [bb, key_bits), <= kRadixBits each
  e->nb = (uint32_t)((nl + (1ull << e->bb) - 1) >> e->bb);
  e->nchunks = 2 * e->nb + kStagedChunks;
  // first-pass histogram columns: ~2048 units per arena at most (G buckets per unit)
  e->G = (e->nb + 2047) / 2048;
  if (const char* s = getenv("AGX_UNIT_G")) e->G = (uint32_t)std::max(1, atoi(s));  // test knob
  e->G = std::min<uint32_t>(e->G, kMaxUnitChunks);
  e->ng = (e->nb + e->G - 1) / e->G;
  e->nunits = 2 * e->ng + kStagedChunks;
  e->cstride = (e->nunits + 3) & ~3u;
  {
    const uint32_t lo = e->bb, hi = std::max<uint32_t>(e->key_bits, e->bb + 1);
    // AGX_RADIX_BITS (test knob): narrower digits, so that small populations take the multi-pass path
    uint32_t rb = kRadixBits;
    if (const char* s = getenv("AGX_RADIX_BITS")) rb = std::min<uint32_t>(kRadixBits, std::max(1, atoi(s)));
    e->plan.npass = (hi - lo + rb - 1) / rb;
    if (e->plan.npass > 4) { delete e; return set_err(AGX_EINVAL, "AGX_RADIX_BITS=%u needs more than 4 passes", rb); }
    for (uint32_t p = 0, sh = lo; p < e->plan.npass; ++p) {
      const uint32_t b = (hi - sh + (e->plan.npass - p) - 1) / (e->plan.npass - p);  // spread bits evenly
      e->plan.shift[p] = sh;
      e->plan.bits[p] = b;
      sh += b;
    }
    // AGX_PASS0_BITS (A/B knob): the first (chunk-list) pass's digit width, the rest spread over the
    // dense passes -- fewer first-pass digits make longer per-digit runs out of its small tiles
    if (const char* s = getenv("AGX_PASS0_BITS"); s && e->plan.npass > 1) {
      const uint32_t b0 = std::min<uint32_t>(rb, std::max(1, atoi(s)));
      if (b0 < hi - lo) {
        const uint32_t rest = hi - lo - b0, np = (rest + rb - 1) / rb;
        if (1 + np <= 4) {
          e->plan.npass = 1 + np;
          e->plan.shift[0] = lo;
          e->plan.bits[0] = b0;
          for (uint32_t p = 1, sh = lo + b0; p < e->plan.npass; ++p) {
            const uint32_t b = (hi - sh + (e->plan.npass - p) - 1) / (e->plan.npass - p);
            e->plan.shift[p] = sh;
            e->plan.bits[p] = b;
            sh += b;
          }
        }
      }
    }
  }

  // fused superstep when one radix digit covers every bucket of a single rank
  e->fused = e->R == 1 && e->plan.npass == 1 && getenv("AGX_NO_FUSED") == nullptr;
  // identity grouping (k_ident_combine): single-rank multi-pass with a bucket-bounds search
  e->ident_on = !e->fused && e->R == 1 && e->plan.npass > 1 && getenv("AGX_NO_IDENT") == nullptr;
  if (!e->fused && e->R == 1) e->par = 1u;  // multi-pass: parity of the first superstep's counter value (1)
  e->tstride = (e->nb + 3) & ~3u;
  // fused: bucket b's inbox (and its backlog / tell slices) live at [b*region, ...) of the
  // arenas; an inbox larger than the region (skew) takes a slot of the overflow area that
  // follows, sized like the whole message capacity — no shared counter on the common path
  e->region = kBucket;
  if (getenv("AGX_NO_STRICT")) e->strict_ok = e->strict_env = false;
  if (const char* s = getenv("AGX_MAX_REPLAY")) {  // diagnostic: cap the replay length (1, 2, 4, 8)
    const uint32_t m = (uint32_t)std::max(1, atoi(s));
    e->max_replay_si = m >= 16 ? 4u : m >= 8 ? 3u : m >= 4 ? 2u : m >= 2 ? 1u : 0u;
  }
  e->stamps_skew = getenv("AGX_STAMPS_SKEW") != nullptr;
  if (const char* s = getenv("AGX_SKEW_GRID"))
    e->skew_grid = (uint32_t)std::min<int>(kMaxApplyGrid, std::max(1, atoi(s)));
  if (const char* s = getenv("AGX_APPLY_GRID"))
    e->apply_grid = (uint32_t)std::min<int>(kMaxApplyGrid, std::max(1, atoi(s)));
  e->acap = e->fused ? (uint64_t)e->nb * e->region + e->cap : e->cap;
  if (e->acap * e->kmax >= (1ull << 32)) { delete e; return set_err(AGX_EINVAL, "msg_capacity * max_emit too large"); }
  // bounded-mailbox rings: drain scratch / tell slices of kBucket x throughput messages per pool slot
  // after the arenas (AGX_RING_SLOTS: how many; CRDT kinds are registered later and turn the pool off
  // at the first run; class 0 is agx_cfg.capacity, so an unbounded default never has rings).
  // Opt-in: measured same-box against the backlog arena they cost C5 -2 % and C3 -6 % (every ring
  // bucket takes the four-kernel skew path each superstep)
  if (!e->fused && e->R == 1 && e->Traw <= kRingMaxT && e->mcap[0] && e->mcap[0] <= kRingMaxC) {
    uint64_t want = 0;
    if (const char* s = getenv("AGX_RING_SLOTS")) want = (uint64_t)std::max(0, atoi(s));
    const uint64_t per = (uint64_t)kBucket * e->Traw;
    const uint64_t room = ((1ull << 32) / e->kmax - 1 - e->acap) / per;
    e->ring_res = (uint32_t)std::min<uint64_t>({want, e->nb, room});
  }
  const uint64_t ring_extra = (uint64_t)e->ring_res * kBucket * e->Traw;

  e->h_kind.assign(e->n_local, 0);
  e->h_alive.assign(e->n_local, 0);
  e->h_state.assign(e->n_local * e->W, 0);

#define CREATE_TRY(x)            \
  do {                           \
    agx_status _s = (x);         \
    if (_s) { agx_destroy(e); return _s; } \
  } while (0)
  CREATE_TRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) == hipSuccess
                 ? AGX_OK
                 : set_err(AGX_EDEVICE, "hipStreamCreate failed"));
  CREATE_TRY(dalloc(&e->d_kind, nl));
  // (padded to whole buckets: the apply loads every bucket's flags as u32 words, masked past n_local)
  const uint64_t alive_sz = ((uint64_t)e->nb << e->bb) + kBucket + 64;
  CREATE_TRY(dalloc(&e->d_alive, alive_sz));
  CREATE_TRY(hipMemset(e->d_alive, 0, alive_sz) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(dalloc(&e->d_stopq, nl));
  CREATE_TRY(dalloc(&e->d_nstop, 4));
  CREATE_TRY(hipMemset(e->d_nstop, 0, 16) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(dalloc(&e->d_state, nl * e->W));
  // two-word engines (the plain behaviours' count + cursor / sum): actor-major pairs on the device
  // (DevParams::sa / sw; the host mirror stays word-major, transposed at upload / read-back).
  // A CRDT kind needs n_words >= 8, so a two-word engine never becomes a CRDT engine.
  if (e->W == 2 && !getenv("AGX_STATE_SOA")) e->pitch = 2;
  if (e->R > 1) {
    CREATE_TRY(dalloc(&e->d_gid, nl));
    CREATE_TRY(dalloc(&e->d_route, e->n_global));
    CREATE_TRY(hipMemcpy(e->d_gid, e->h_gid.data(), e->n_local * 4, hipMemcpyHostToDevice) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "upload gid"));
    CREATE_TRY(hipMemcpy(e->d_route, e->h_route.data(), e->n_global * 4, hipMemcpyHostToDevice) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "upload route"));
  }
  CREATE_TRY(alloc_msgs(e->A, e->acap));
  CREATE_TRY(alloc_msgs(e->B, e->fused ? 1 : e->cap));
  CREATE_TRY(alloc_msgs(e->scr, e->acap + ring_extra));
  CREATE_TRY(alloc_msgs(e->bl, e->acap));
  e->em_cap = (e->acap + ring_extra) * e->kmax;
  CREATE_TRY(alloc_msgs(e->em, e->em_cap));
  if (e->R > 1) {  // tells grouped by owner per bucket (eg0 + [R][tstride] tables), send buffer s2
    const uint64_t tsz = (uint64_t)e->R * e->tstride;
    CREATE_TRY(alloc_msgs(e->eg0, e->cap_emit));
    CREATE_TRY(alloc_msgs(e->s2, e->cap_emit));
    CREATE_TRY(dalloc(&e->d_s2p, 3 * e->cap_emit));
    CREATE_TRY(dalloc(&e->d_rcvp, 3 * e->cap));
    CREATE_TRY(dalloc(&e->d_halt, 2));
    CREATE_TRY(hipMemset(e->d_halt, 0, 8) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    CREATE_TRY(hipHostMalloc((void**)&e->h_halt, 8, hipHostMallocDefault) == hipSuccess ? AGX_OK : set_err(AGX_ENOMEM, "pinned"));
    CREATE_TRY(dalloc(&e->d_tcnt[0], tsz));
    CREATE_TRY(dalloc(&e->d_toff[0], tsz));
    CREATE_TRY(hipMemset(e->d_tcnt[0], 0, tsz * 4) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    CREATE_TRY(dalloc(&e->d_moff0, e->nb));
    CREATE_TRY(dalloc(&e->d_moff1, tsz));
  }
  if (!e->fused && e->R == 1) {  // multi-pass: backlog and tell arenas by superstep parity
    CREATE_TRY(alloc_msgs(e->bl2, e->acap));
    CREATE_TRY(alloc_msgs(e->em2, e->em_cap));
    if (e->ident_on) {
      CREATE_TRY(dalloc(&e->d_emmeta, e->nb));
      CREATE_TRY(dalloc(&e->d_slsum, (uint64_t)(kMaxBlSlices + 1) * kSlSum));
      CREATE_TRY(dalloc(&e->d_ident, 4));
      CREATE_TRY(hipMemset(e->d_emmeta, 0, e->nb * sizeof(uint4)) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
      CREATE_TRY(hipMemset(e->d_ident, 0, 16) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    }
    CREATE_TRY(dalloc(&e->d_blpre, e->nb + 2 * kMaxBlSlices));  // [nb] prefixes, [64] slice totals, [64] bases
    CREATE_TRY(dalloc(&e->d_ninbox, 1));
    CREATE_TRY(hipMemset(e->d_ninbox, 0, 4) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    // skewed-bucket partitions: a skewed bucket holds > kBucket messages, so at most cap / kBucket
    // of them; parts of >= kSkSpan positions.  k_skew_plan rounds a bucket's backlog parts and its
    // new-mail parts up separately, so each skewed bucket adds up to TWO parts beyond the budget:
    // at most sk_budget + 2 x (skewed buckets) rows of pc
    const uint64_t nsk = std::min<uint64_t>(e->nb, e->cap / kBucket + 1);
    e->sk_budget = (uint32_t)std::min<uint64_t>(8192, e->cap / kSkSpan + 1);
    e->sk_rows = e->sk_budget + 2 * (uint32_t)nsk;
    CREATE_TRY(dalloc(&e->d_sk_rec, (uint64_t)e->nb * kSkRec));
    CREATE_TRY(dalloc(&e->d_sk_act, nsk * kSkActPlanes * kBucket));
    CREATE_TRY(dalloc(&e->d_sk_pc, (uint64_t)e->sk_rows * kBucket));
    CREATE_TRY(dalloc(&e->d_sk_meta, 4));
  }
  if (e->fused) {
    const uint64_t tsz = (uint64_t)kRadix * e->tstride;
    CREATE_TRY(alloc_msgs(e->bl2, e->acap));
    CREATE_TRY(alloc_msgs(e->eg0, e->acap * e->kmax));
    CREATE_TRY(alloc_msgs(e->eg1, e->acap * e->kmax));
    for (int q = 0; q < 2; ++q) {
      CREATE_TRY(dalloc(&e->d_tcnt[q], tsz));
      CREATE_TRY(dalloc(&e->d_toff[q], tsz));
      CREATE_TRY(dalloc(&e->d_blo[q], e->nb));
      CREATE_TRY(dalloc(&e->d_blc[q], e->nb));
      CREATE_TRY(dalloc(&e->d_emc[q], e->nb));
      CREATE_TRY(hipMemset(e->d_tcnt[q], 0, tsz * 4) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
      CREATE_TRY(hipMemset(e->d_blc[q], 0, e->nb * 4ull) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
      CREATE_TRY(hipMemset(e->d_emc[q], 0, e->nb * 4ull) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    }
    CREATE_TRY(dalloc(&e->d_stg_off, e->nb));
    CREATE_TRY(dalloc(&e->d_stg_cnt, e->nb));
    CREATE_TRY(dalloc(&e->d_ovf, 2));
    CREATE_TRY(dalloc(&e->d_cntb, (uint64_t)agx_engine::kGraphSteps * e->nb));
    CREATE_TRY(hipHostMalloc((void**)&e->h_cntb, 4ull * (agx_engine::kGraphSteps * e->nb + kRingTail) * 4, hipHostMallocDefault) ==
                       hipSuccess ? AGX_OK : set_err(AGX_ENOMEM, "pinned"));
    CREATE_TRY(dalloc(&e->d_parv, 2));
    const uint32_t parv[2] = {0u, 1u};
    CREATE_TRY(hipMemcpy(e->d_parv, parv, 8, hipMemcpyHostToDevice) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "upload"));
    CREATE_TRY(hipMemset(e->d_stg_cnt, 0, e->nb * 4ull) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    CREATE_TRY(hipMemset(e->d_ovf, 0, 8) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    CREATE_TRY(hipHostGetDevicePointer((void**)&e->d_ring, e->h_cntb, 0) == hipSuccess ? AGX_OK
                   : set_err(AGX_EDEVICE, "hipHostGetDevicePointer"));
    CREATE_TRY(dalloc(&e->d_rctr, 1));
    CREATE_TRY(hipMemset(e->d_rctr, 0, 4) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    CREATE_TRY(dalloc(&e->d_abort, 2));
    CREATE_TRY(hipMemset(e->d_abort, 0, 8) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    CREATE_TRY(dalloc(&e->d_pbar, 4));
    CREATE_TRY(hipMemset(e->d_pbar, 0, 16) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
    CREATE_TRY(hipHostMalloc((void**)&e->h_abort, 4 * 2 * 4, hipHostMallocDefault) == hipSuccess
                   ? AGX_OK : set_err(AGX_ENOMEM, "pinned"));
  }
  CREATE_TRY(dalloc(&e->d_skew_list, e->nb));
  CREATE_TRY(dalloc(&e->d_skew_n, 4));
  CREATE_TRY(hipMemset(e->d_skew_n, 0, 16) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(dalloc(&e->d_blist, e->nb));
  CREATE_TRY(dalloc(&e->d_dense_left, 2));
  CREATE_TRY(hipMemset(e->d_dense_left, 0, 8) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(dalloc(&e->d_chunk_off, e->nchunks));
  CREATE_TRY(dalloc(&e->d_chunk_cnt, e->nchunks));
  CREATE_TRY(hipMemset(e->d_chunk_off, 0, e->nchunks * 4ull) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(hipMemset(e->d_chunk_cnt, 0, e->nchunks * 4ull) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(dalloc(&e->d_hist_c, (uint64_t)kRadix * e->cstride));
  CREATE_TRY(hipMemset(e->d_hist_c, 0, (uint64_t)kRadix * e->cstride * 4) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(dalloc(&e->d_bstart, std::max<uint64_t>(kRadix, e->nb) + 1));
  if (getenv("AGX_STAMPS")) {
    CREATE_TRY(dalloc(&e->d_dbg, (uint64_t)std::min<uint64_t>(e->nb, 4096) * 16));
    CREATE_TRY(hipMemset(e->d_dbg, 0, std::min<uint64_t>(e->nb, 4096) * 16 * 8) == hipSuccess ? AGX_OK
                                                                                       : set_err(AGX_EDEVICE, "memset"));
  }
  CREATE_TRY(dalloc(&e->d_hist_d, (uint64_t)kRadix * e->dstride));
  CREATE_TRY(dalloc(&e->d_tot, kRadix));
  CREATE_TRY(dalloc(&e->d_n, 4));
  CREATE_TRY(dalloc(&e->d_total, 4));
  CREATE_TRY(dalloc(&e->d_stats, kStatBlk));
  e->d_sred = (unsigned long long*)(e->d_stats + kStatSred);
  e->d_inflight = e->d_stats + kStatInfl;
  CREATE_TRY(dalloc(&e->d_bstats, (uint64_t)kMaxApplyGrid * kBStats));
  CREATE_TRY(hipMemset(e->d_bstats, 0, (uint64_t)kMaxApplyGrid * kBStats * 8) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(dalloc(&e->d_heap_top, 2));
  CREATE_TRY(dalloc(&e->d_step, 1));
  CREATE_TRY(hipMemset(e->d_heap_top, 0, 8) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(hipMemset(e->d_step, 0, 4) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(dalloc(&e->d_cvec, AGX_MAX_RANKS + 2));
  CREATE_TRY(dalloc(&e->d_cmat, (uint64_t)AGX_MAX_RANKS * (AGX_MAX_RANKS + 2)));
  CREATE_TRY(hipMemset(e->d_n, 0, 16) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(hipMemset(e->d_total, 0, 16) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(hipMemset(e->d_stats, 0, kStatBlk * 8) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  CREATE_TRY(hipHostMalloc((void**)&e->h_stat, kStatBlk * 8, hipHostMallocDefault) == hipSuccess ? AGX_OK : set_err(AGX_ENOMEM, "pinned"));
  CREATE_TRY(hipHostMalloc((void**)&e->h_pin, 64 * 4, hipHostMallocDefault) == hipSuccess ? AGX_OK : set_err(AGX_ENOMEM, "pinned"));
  CREATE_TRY(hipHostMalloc((void**)&e->h_pin64, (AGX_MAX_RANKS * (AGX_MAX_RANKS + 2) + 8) * 8, hipHostMallocDefault) == hipSuccess ? AGX_OK : set_err(AGX_ENOMEM, "pinned"));
  // empty graph rows so FORWARD_RR on an engine without a graph is well defined
  e->h_row.assign(e->n_local + 1, 0);
  CREATE_TRY(dalloc(&e->d_row, e->n_local + 1));
  CREATE_TRY(hipMemset(e->d_row, 0, (e->n_local + 1) * 8) == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "memset"));
  // the hipMemsets above run on the null stream, which a non-blocking engine stream does not wait
  // for: without this, the first upload (prepare_run, on e->stream) could land before a memset of
  // the same buffer (seen: alive flags zeroed after their upload -> every tell a dead letter)
  CREATE_TRY(hipDeviceSynchronize() == hipSuccess ? AGX_OK : set_err(AGX_EDEVICE, "hipDeviceSynchronize"));
#undef CREATE_TRY
  *out = e;
  return AGX_OK;
}

agx_status agx_destroy(agx_engine* e) {
  if (!e) return AGX_OK;
  hipSetDevice((int)e->cfg.device);
  if (e->stream) hipStreamSynchronize(e->stream);
  // graphs first: a captured replay holds RCCL's persistent plans of this communicator, and
  // ncclCommDestroy with such a graph still alive never returned (round 5: the opt-in captured
  // multi-rank replay ran to quiescence, then the engine's destroy hung -- DESIGN.md §3.3)
  drop_graphs(e);
  const bool dbg = e->comm && getenv("AGX_MR_DEBUG");
  if (dbg) fprintf(stderr, "[agx rank %u] destroy: communicator\n", e->rank);
  if (e->comm) ncclCommDestroy(e->comm);
  if (dbg) fprintf(stderr, "[agx rank %u] destroy: communicator destroyed\n", e->rank);
  hipFree(e->d_kind); hipFree(e->d_alive); hipFree(e->d_stopq); hipFree(e->d_nstop); hipFree(e->d_state); hipFree(e->d_gid); hipFree(e->d_route);
  hipFree(e->d_zcdf); hipFree(e->d_zperm); hipFree(e->d_zent); hipFree(e->d_row); hipFree(e->d_col);
  free_msgs(e->A); free_msgs(e->B); free_msgs(e->scr); free_msgs(e->bl); free_msgs(e->em); free_msgs(e->stg);
  free_msgs(e->s2); free_msgs(e->bl2); free_msgs(e->eg0); free_msgs(e->eg1); free_msgs(e->em2);
  hipFree(e->d_emmeta); hipFree(e->d_slsum); hipFree(e->d_ident);
  hipFree(e->d_outbox); hipFree(e->d_outbox_n);
  hipFree(e->d_s2p); hipFree(e->d_rcvp); hipFree(e->d_sslab); hipFree(e->d_rslab); hipFree(e->d_halt);
  if (e->h_halt) hipHostFree(e->h_halt);
  for (int q = 0; q < 2; ++q) {
    hipFree(e->d_tcnt[q]); hipFree(e->d_toff[q]); hipFree(e->d_blo[q]); hipFree(e->d_blc[q]); hipFree(e->d_emc[q]);
  }
  hipFree(e->d_stg_off); hipFree(e->d_stg_cnt); hipFree(e->d_ovf); hipFree(e->d_cntb);
  if (e->h_cntb) hipHostFree(e->h_cntb); hipFree(e->d_parv);
  hipFree(e->d_abort); hipFree(e->d_rctr);
  hipFree(e->d_pbar);
  for (auto& ev : e->tev)
    if (ev) hipEventDestroy(ev);
  if (e->h_abort) hipHostFree(e->h_abort);
  hipFree(e->d_skew_list); hipFree(e->d_skew_n); hipFree(e->d_blist); hipFree(e->d_dense_left);
  hipFree(e->d_sk_rec); hipFree(e->d_sk_act); hipFree(e->d_sk_pc); hipFree(e->d_sk_meta);
  hipFree(e->d_ring_of); hipFree(e->d_ring_state); hipFree(e->d_ring_src); hipFree(e->d_ring_pay);
  hipFree(e->d_rg_state); hipFree(e->d_rg_nz); hipFree(e->d_rg_src); hipFree(e->d_rg_pay); hipFree(e->d_rg_dk); hipFree(e->d_rg_ds);
  hipFree(e->d_rg_dp);
  hipFree(e->d_ring_next); hipFree(e->d_ring_free); hipFree(e->d_ring_total);
  hipFree(e->d_orw); hipFree(e->d_orm); hipFree(e->d_orw_n);
  hipFree(e->d_chunk_off); hipFree(e->d_chunk_cnt); hipFree(e->d_hist_c); hipFree(e->d_hist_d); hipFree(e->d_tot); hipFree(e->d_bstart); hipFree(e->d_dbg);
  hipFree(e->d_moff0); hipFree(e->d_moff1); hipFree(e->d_blpre); hipFree(e->d_ninbox); hipFree(e->d_n); hipFree(e->d_total);
  hipFree(e->d_stats); hipFree(e->d_bstats); hipFree(e->d_cvec); hipFree(e->d_cmat);
  if (e->h_stat) hipHostFree(e->h_stat);
  for (auto ev : e->lag_ev)
    if (ev) hipEventDestroy(ev);
  hipFree(e->d_heap); hipFree(e->d_heap_top); hipFree(e->d_step); hipFree(e->d_rx); hipFree(e->d_s2rows); hipFree(e->d_srows);
  hipFree(e->d_bcase); hipFree(e->d_bact); hipFree(e->d_bfirst);
  if (e->h_pin) hipHostFree(e->h_pin);
  if (e->h_pin64) hipHostFree(e->h_pin64);
  for (auto ev : e->ev_pool) hipEventDestroy(ev);
  if (e->stream) hipStreamDestroy(e->stream);
  delete e;
  return AGX_OK;
}

agx_status agx_register_range(agx_engine* e, uint64_t first_id, uint64_t count, uint32_t kind, const void* init,
                              size_t stride) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  AGX_TRY(ensure_dev(e));
  AGX_TRY(sync_mirrors(e));  // device state is authoritative after a run
  const bool compiled = kind >= AGX_KIND_COMPILED && kind < AGX_KIND_COMPILED + AGX_MAX_BEHAVIORS;
  if (first_id + count > e->n_global || (kind >= AGX_KIND_MAX && !compiled)) return set_err(AGX_EINVAL, "bad range or kind");
  const uint32_t kCrdtMask = kb(AGX_KIND_GCOUNTER) | kb(AGX_KIND_PNCOUNTER) | kb(AGX_KIND_ORSET);
  if (count && ((compiled && (e->kinds_mask & kCrdtMask)) ||
                (kind >= AGX_KIND_GCOUNTER && kind <= AGX_KIND_ORSET && (e->kinds_mask & kb(AGX_KIND_COMPILED)))))
    return set_err(AGX_EINVAL, "compiled behaviours and CRDT replicas need separate engines");
  if ((kind == AGX_KIND_FORWARD_RR || kind == AGX_KIND_STOP_AFTER) && e->W < 2)
    return set_err(AGX_EINVAL, "behaviour kind %u needs n_words >= 2", kind);
  if (init && stride < e->W * 8ull) return set_err(AGX_EINVAL, "state_stride smaller than n_words*8");
  if (kind >= AGX_KIND_GCOUNTER && kind <= AGX_KIND_ORSET) AGX_TRY(enable_crdt(e, kind));
  if (count && !(e->kinds_mask & kb(kind))) {  // the apply variant is captured in the superstep graphs
    e->kinds_mask |= kb(kind);
    drop_graphs(e);
  }
  const uint8_t* ib = (const uint8_t*)init;
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t id = first_id + i, l;
    if (e->R > 1) {
      uint32_t r = e->h_route[id];
      if ((r >> kOwnerShift) != e->rank) continue;
      l = r & kLocalMask;
    } else {
      l = id;
    }
    e->h_kind[l] = (uint8_t)kind;
    e->h_alive[l] = (uint8_t)((e->h_alive[l] & 0xFEu) | (kind != AGX_KIND_NONE ? 1u : 0u));  // (bits 1..3: mailbox class)
    for (uint32_t w = 0; w < e->W; ++w) {
      uint64_t v = 0;
      if (ib) memcpy(&v, ib + i * stride + w * 8, 8);
      e->h_state[(uint64_t)w * e->n_local + l] = v;
    }
  }
  e->actors_dirty = true;
  return AGX_OK;
}

agx_status agx_set_mailbox_class(agx_engine* e, uint32_t cls, uint32_t capacity) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  if (cls == 0 || cls >= AGX_MAX_MAILBOX_CLASSES)
    return set_err(AGX_EINVAL, "mailbox class %u: classes 1..%u are configurable (0 is agx_cfg.capacity)", cls,
                   AGX_MAX_MAILBOX_CLASSES - 1);
  if (e->ring_live && (capacity == 0 || capacity > e->ring_c))
    return set_err(AGX_EINVAL,
                   "mailbox class %u capacity %u: this engine keeps queued messages in rings of %u (set every "
                   "mailbox class before the first run, or AGX_RING_SLOTS=0)", cls, capacity, e->ring_c);
  if (e->rg_on && (capacity == 0 || capacity > e->rg_c))
    return set_err(AGX_EINVAL,
                   "mailbox class %u capacity %u: this engine keeps queued messages in per-actor rings of %u (set "
                   "every mailbox class before the first run, or AGX_RING_APPLY=0)", cls, capacity, e->rg_c);
  e->mcap[cls] = capacity;
  e->mclass_set |= 1u << cls;
  e->mclasses = true;
  drop_graphs(e);  // the class table is a kernel parameter captured in the superstep graphs
  return AGX_OK;
}

agx_status agx_set_mailbox(agx_engine* e, uint64_t first_id, uint64_t count, uint32_t cls) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  if (cls >= AGX_MAX_MAILBOX_CLASSES || !((e->mclass_set >> cls) & 1u))
    return set_err(AGX_EINVAL, "mailbox class %u is not configured (agx_set_mailbox_class)", cls);
  if (first_id + count > e->n_global) return set_err(AGX_EINVAL, "bad actor range");
  AGX_TRY(ensure_dev(e));
  AGX_TRY(sync_mirrors(e));  // device state is authoritative after a run
  for (uint64_t i = 0; i < count; ++i) {
    const uint64_t id = first_id + i;
    uint64_t l = id;
    if (e->R > 1) {
      const uint32_t r = e->h_route[id];
      if ((r >> kOwnerShift) != e->rank) continue;
      l = r & kLocalMask;
    }
    e->h_alive[l] = (uint8_t)((e->h_alive[l] & 1u) | (cls << 1));
  }
  e->actors_dirty = true;
  return AGX_OK;
}

agx_status agx_set_outbound(agx_engine* e, uint32_t first_host_id, uint32_t n_host, uint64_t capacity) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  if (n_host && (first_host_id < e->n_global || (uint64_t)first_host_id + n_host > (1ull << 31)))
    return set_err(AGX_EINVAL, "host ids must lie in [n_actors, 2^31) (bit 31 of a sender tags CRDT state gossips)");
  if (n_host && (capacity == 0 || capacity > 0x3FFFFFFFull))
    return set_err(AGX_EINVAL, "outbox capacity must be in [1, 2^30)");
  AGX_TRY(ensure_dev(e));
  HIP_TRY(hipStreamSynchronize(e->stream));
  if (!e->d_outbox_n) {
    AGX_TRY(dalloc(&e->d_outbox_n, 1));
    HIP_TRY(hipMemsetAsync(e->d_outbox_n, 0, 4, e->stream));
  }
  if (n_host && capacity != e->outbox_cap) {
    AGX_TRY(drain_outbox(e));  // tells still in the old buffer move to the host queue first
    hipFree(e->d_outbox);
    e->d_outbox = nullptr;
    AGX_TRY(dalloc(&e->d_outbox, 3 * capacity));
    e->outbox_cap = capacity;
  }
  HIP_TRY(hipDeviceSynchronize());  // (null-stream allocation / memset before the engine stream uses them)
  e->host_lo = first_host_id;
  e->host_n = n_host;
  drop_graphs(e);  // the host-id range is a kernel parameter captured in the superstep graphs
  return AGX_OK;
}

agx_status agx_take_outbound(agx_engine* e, uint32_t* dst, uint32_t* src, uint32_t* payload, uint64_t cap,
                             uint64_t* n) {
  if (!e || !n || (cap && (!dst || !src || !payload))) return set_err(AGX_EINVAL, "bad take_outbound args");
  *n = 0;
  AGX_TRY(ensure_dev(e));
  AGX_TRY(drain_outbox(e));
  if (e->outbox_lost) {  // reported once, then cleared: the engine stays usable after an overflow
    const uint64_t lost = e->outbox_lost;
    e->outbox_lost = 0;
    return set_err(AGX_ECAPACITY, "%llu outbound tells dropped: more than the outbox capacity %llu between two "
                   "agx_take_outbound calls", (unsigned long long)lost, (unsigned long long)e->outbox_cap);
  }
  const uint64_t k = std::min<uint64_t>(cap, e->outq.size() / 3);
  for (uint64_t i = 0; i < k; ++i) {
    dst[i] = e->outq[3 * i];
    src[i] = e->outq[3 * i + 1];
    payload[i] = e->outq[3 * i + 2];
  }
  e->outq.erase(e->outq.begin(), e->outq.begin() + 3 * k);
  *n = k;
  return AGX_OK;
}

agx_status agx_set_gossip(agx_engine* e, uint32_t fanout, uint64_t seed) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  if (fanout + 1 > e->kmax) return set_err(AGX_EINVAL, "gossip fanout %u needs max_emit >= %u", fanout, fanout + 1);
  e->gossip_f = fanout;
  e->gossip_seed = seed;
  drop_graphs(e);  // behaviour parameters are captured in the superstep graphs
  return AGX_OK;
}

agx_status agx_set_behaviors(agx_engine* e, const agx_case* cases, uint32_t n_cases, const agx_act* acts,
                             uint32_t n_acts, const uint32_t* first, uint32_t n_beh) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  if (e->started) return set_err(AGX_ESTATE, "set compiled behaviours before agx_run");
  if (n_beh == 0 || n_beh > AGX_MAX_BEHAVIORS || n_cases > AGX_MAX_CASES || n_acts > AGX_MAX_ACTS || !first ||
      (n_cases && !cases) || (n_acts && !acts))
    return set_err(AGX_EINVAL, "compiled behaviours: bad table sizes");
  if (first[0] != 0 || first[n_beh] != n_cases) return set_err(AGX_EINVAL, "first[] must run from 0 to n_cases");
  for (uint32_t b = 0; b < n_beh; ++b)
    if (first[b] > first[b + 1]) return set_err(AGX_EINVAL, "first[] must be non-decreasing");
  auto opnd_ok = [](uint32_t src, uint32_t word) { return src <= AGX_V_SELF && word <= 1u; };
  for (uint32_t c = 0; c < n_cases; ++c) {
    const agx_case& C = cases[c];
    if (!opnd_ok(C.src1, C.word1) || !opnd_ok(C.src2, C.word2) || !opnd_ok(C.src3, C.word3) ||
        !opnd_ok(C.src4, C.word4) || C.cmp1 > AGX_CMP_GE || C.cmp2 > AGX_CMP_GE || C.result > AGX_RES_BECOME ||
        (C.result == AGX_RES_BECOME && C.next >= n_beh) || (uint32_t)C.act_first + C.act_count > n_acts)
      return set_err(AGX_EINVAL, "compiled behaviours: bad case %u", c);
  }
  for (uint32_t i = 0; i < n_acts; ++i) {
    const agx_act& A = acts[i];
    if (A.op < AGX_A_SET || A.op > AGX_A_TELL || A.word > 1u || !opnd_ok(A.src, A.sword) ||
        (A.op == AGX_A_TELL && !opnd_ok(A.dsrc, A.dword)))
      return set_err(AGX_EINVAL, "compiled behaviours: bad action %u (state words 0..1)", i);
  }
  // the apply kernels reserve kmax tell slots per message (single pass: the tell overwrites the
  // message's own consumed LDS slot; otherwise a bucket's tells live in [lo*kmax, (lo+cnt)*kmax)):
  // a case that tells more often would overwrite unprocessed mail or the next bucket's tells
  for (uint32_t c = 0; c < n_cases; ++c) {
    uint32_t tells = 0;
    for (uint32_t i = cases[c].act_first; i < (uint32_t)cases[c].act_first + cases[c].act_count; ++i)
      tells += acts[i].op == AGX_A_TELL;
    if (tells > e->kmax)
      return set_err(AGX_EINVAL, "compiled behaviours: case %u tells %u times per message, max_emit is %u", c, tells,
                     e->kmax);
  }
  AGX_TRY(ensure_dev(e));
  hipFree(e->d_bcase);
  hipFree(e->d_bact);
  hipFree(e->d_bfirst);
  e->d_bcase = nullptr;
  e->d_bact = nullptr;
  e->d_bfirst = nullptr;
  AGX_TRY(dalloc(&e->d_bcase, std::max<uint32_t>(n_cases, 1)));
  AGX_TRY(dalloc(&e->d_bact, std::max<uint32_t>(n_acts, 1)));
  AGX_TRY(dalloc(&e->d_bfirst, n_beh + 1));
  if (n_cases) AGX_TRY(copy_sync(e, e->d_bcase, cases, n_cases * sizeof(agx_case), hipMemcpyHostToDevice));
  if (n_acts) AGX_TRY(copy_sync(e, e->d_bact, acts, n_acts * sizeof(agx_act), hipMemcpyHostToDevice));
  AGX_TRY(copy_sync(e, e->d_bfirst, first, (n_beh + 1) * 4ull, hipMemcpyHostToDevice));
  e->n_beh = n_beh;
  drop_graphs(e);  // the tables are kernel parameters captured in the superstep graphs
  return AGX_OK;
}

agx_status agx_set_delta_crdt(agx_engine* e, uint32_t max_delta_size) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  if (max_delta_size > AGX_DELTA_MAX_SIZE)
    return set_err(AGX_EINVAL, "max_delta_size %u > %u (DeltaPropagation rows are sized for it)", max_delta_size,
                   AGX_DELTA_MAX_SIZE);
  if (max_delta_size && e->kmax < 4) return set_err(AGX_EINVAL, "delta-CRDT replicas need max_emit >= 4");
  if (max_delta_size && e->n_global >= (1ull << 30)) return set_err(AGX_EINVAL, "delta-CRDT needs n_actors < 2^30");
  if (e->started && max_delta_size != e->delta_max) return set_err(AGX_ESTATE, "set delta-CRDT mode before agx_run");
  e->delta_max = max_delta_size;
  for (uint32_t k = AGX_KIND_GCOUNTER; k <= AGX_KIND_ORSET; ++k)
    if (e->kinds_mask & kb(k)) AGX_TRY(enable_crdt(e, k));
  drop_graphs(e);
  return AGX_OK;
}

agx_status agx_set_ring(agx_engine* e, uint32_t stride) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  e->ring_stride = stride;
  drop_graphs(e);
  return AGX_OK;
}

agx_status agx_set_fanout(agx_engine* e, uint32_t k, uint64_t seed, const uint32_t* cdf, const uint32_t* perm,
                          uint64_t n) {
  if (!e || !cdf || !perm || n == 0) return set_err(AGX_EINVAL, "bad fanout args");
  if (k > e->kmax) return set_err(AGX_EINVAL, "fanout k=%u exceeds max_emit=%u", k, e->kmax);
  for (uint64_t i = 0; i < n; ++i)
    if (perm[i] >= e->n_global) return set_err(AGX_EINVAL, "perm entry out of range");
  AGX_TRY(ensure_dev(e));
  if (n >= (1ull << 32)) return set_err(AGX_EINVAL, "fanout table too large");
  for (uint64_t i = 1; i < n; ++i)
    if (cdf[i] < cdf[i - 1]) return set_err(AGX_EINVAL, "fanout cdf not monotone at %llu", (unsigned long long)i);
  // range index (zipf_dest): zidx[t] = first i with cdf[i] >= t << (32 - kZipfBits), clamped to n - 1,
  // zidx[Z] = n - 1; entry t = {perm[i], kZipfDirect} when zidx[t] == zidx[t + 1] = i (every u of the
  // range answers i), else the search range {zidx[t], zidx[t + 1]}
  const uint64_t Z = 1ull << kZipfBits;
  std::vector<uint32_t> zidx(Z + 1);
  for (uint64_t t = 0, i = 0; t < Z; ++t) {
    const uint64_t u = t << (32 - kZipfBits);
    while (i < n && cdf[i] < u) ++i;
    zidx[t] = (uint32_t)std::min<uint64_t>(i, n - 1);
  }
  zidx[Z] = (uint32_t)(n - 1);
  std::vector<uint2> zent(Z);
  for (uint64_t t = 0; t < Z; ++t)
    zent[t] = zidx[t] == zidx[t + 1] ? make_uint2(perm[zidx[t]], kZipfDirect) : make_uint2(zidx[t], zidx[t + 1]);
  hipFree(e->d_zcdf);
  hipFree(e->d_zperm);
  hipFree(e->d_zent);
  e->d_zcdf = e->d_zperm = nullptr;
  e->d_zent = nullptr;
  AGX_TRY(dalloc(&e->d_zcdf, n));
  AGX_TRY(dalloc(&e->d_zperm, n));
  AGX_TRY(dalloc(&e->d_zent, Z));
  AGX_TRY(copy_sync(e, e->d_zent, zent.data(), Z * sizeof(uint2), hipMemcpyHostToDevice));
  AGX_TRY(copy_sync(e, e->d_zcdf, cdf, n * 4, hipMemcpyHostToDevice));
  AGX_TRY(copy_sync(e, e->d_zperm, perm, n * 4, hipMemcpyHostToDevice));
  e->fan_k = k;
  e->fan_seed = seed;
  e->zipf_n = n;
  drop_graphs(e);
  return AGX_OK;
}

agx_status agx_set_graph(agx_engine* e, const uint64_t* row_ptr, const uint32_t* col) {
  if (!e || !row_ptr) return set_err(AGX_EINVAL, "bad graph args");
  // the whole row_ptr is checked before col is read: then col[0, row_ptr[n_actors]) is every index
  // read below, the length a binding checks its array against (agx_jni.c setGraph)
  for (uint64_t id = 0; id < e->n_global; ++id)
    if (row_ptr[id + 1] < row_ptr[id]) return set_err(AGX_EINVAL, "row_ptr not monotone at %llu", (unsigned long long)id);
  if (row_ptr[e->n_global] > row_ptr[0] && !col) return set_err(AGX_EINVAL, "bad graph args: null col");
  AGX_TRY(ensure_dev(e));
  // keep only the rows of local actors (rows indexed by local id)
  std::vector<uint64_t> row(e->n_local + 1, 0);
  std::vector<uint32_t> c;
  for (uint64_t l = 0; l < e->n_local; ++l) {
    uint64_t id = e->R > 1 ? e->h_gid[l] : l;
    uint64_t b = row_ptr[id], en = row_ptr[id + 1];
    for (uint64_t j = b; j < en; ++j) c.push_back(col[j]);
    row[l + 1] = c.size();
  }
  hipFree(e->d_row);
  hipFree(e->d_col);
  e->d_row = nullptr;
  e->d_col = nullptr;
  AGX_TRY(dalloc(&e->d_row, row.size()));
  AGX_TRY(dalloc(&e->d_col, c.size()));
  AGX_TRY(copy_sync(e, e->d_row, row.data(), row.size() * 8, hipMemcpyHostToDevice));
  if (!c.empty()) AGX_TRY(copy_sync(e, e->d_col, c.data(), c.size() * 4, hipMemcpyHostToDevice));
  e->graph_set = true;
  drop_graphs(e);
  return AGX_OK;
}

agx_status agx_set_graph_rmat(agx_engine* e, const uint64_t* row_ptr, uint32_t bits, uint32_t ta, uint32_t tb,
                              uint32_t tc, uint64_t seed) {
  if (!e || !row_ptr || bits == 0 || bits > 40) return set_err(AGX_EINVAL, "bad rmat graph args");
  AGX_TRY(ensure_dev(e));
  std::vector<uint64_t> lrow(e->n_local + 1, 0), gstart(std::max<uint64_t>(e->n_local, 1), 0);
  for (uint64_t l = 0; l < e->n_local; ++l) {
    const uint64_t id = e->R > 1 ? e->h_gid[l] : l;
    const uint64_t b = row_ptr[id], en = row_ptr[id + 1];
    if (en < b) return set_err(AGX_EINVAL, "row_ptr not monotone at %llu", (unsigned long long)id);
    gstart[l] = b;
    lrow[l + 1] = lrow[l] + (en - b);
  }
  hipFree(e->d_row);
  hipFree(e->d_col);
  e->d_row = nullptr;
  e->d_col = nullptr;
  uint64_t* d_gs = nullptr;
  AGX_TRY(dalloc(&e->d_row, lrow.size()));
  AGX_TRY(dalloc(&e->d_col, lrow.back()));
  AGX_TRY(dalloc(&d_gs, gstart.size()));
  AGX_TRY(copy_sync(e, e->d_row, lrow.data(), lrow.size() * 8, hipMemcpyHostToDevice));
  AGX_TRY(copy_sync(e, d_gs, gstart.data(), gstart.size() * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_gen_rmat, dim3(grid_for(e->n_local / kThreads + 1, 8192)), dim3(kThreads), 0, e->stream,
                     e->d_row, d_gs, e->d_col, (uint32_t)e->n_local, bits, ta, tb, tc, seed, (uint32_t)e->n_global);
  hipError_t le = hipGetLastError();
  hipError_t se = hipStreamSynchronize(e->stream);
  hipFree(d_gs);
  if (le != hipSuccess || se != hipSuccess) return set_err(AGX_EDEVICE, "rmat generation failed");
  e->graph_set = true;
  drop_graphs(e);
  return AGX_OK;
}

// Host tells.  All or nothing: the tells are validated and counted before any is staged, so an
// AGX_EINVAL or AGX_ECAPACITY leaves the engine exactly as it was (no tell staged, no counter moved).
// Capacity: the messages in flight after staging -- the device's backlog and undelivered tells, the
// staged tells not yet consumed, and these -- must fit msg_capacity, or the first superstep's inbox
// would overflow its arenas.
agx_status in_flight_now(agx_engine* e, uint64_t* out);
agx_status agx_stage_tells(agx_engine* e, const uint32_t* dst, const uint32_t* src, const uint32_t* payload, size_t n) {
  if (!e || (n && (!dst || !payload))) return set_err(AGX_EINVAL, "bad tells");
  uint64_t take = 0;  // tells this rank stages (unknown refs are dead letters, other ranks' tells ignored)
  for (size_t i = 0; i < n; ++i) {
    const uint32_t d = dst[i];
    if (d >= e->n_global || (e->R > 1 && (e->h_route[d] >> kOwnerShift) != e->rank)) continue;
    const uint32_t sv = src ? src[i] : AGX_NO_SENDER;
    if ((sv & AGX_WIDE_BIT) && sv != AGX_NO_SENDER)
      return set_err(AGX_EINVAL, "tell %zu: sender %u is not an actor id (bit 31 tags CRDT state gossips)", i, sv);
    ++take;
  }
  if (take) {
    uint64_t infl = 0;
    AGX_TRY(in_flight_now(e, &infl));
    if (infl + take > e->cap)
      return set_err(AGX_ECAPACITY, "%llu staged tells do not fit: %llu messages in flight, msg_capacity %llu "
                     "(nothing staged)", (unsigned long long)take, (unsigned long long)infl, (unsigned long long)e->cap);
  }
  for (size_t i = 0; i < n; ++i) {
    const uint32_t d = dst[i];
    if (d >= e->n_global) {  // unknown ref -> deadLetters (counted once, on rank 0)
      if (e->rank == 0) { e->staged_total++; e->staged_dead++; }
      continue;
    }
    uint32_t key = d;
    if (e->R > 1) {
      uint32_t r = e->h_route[d];
      if ((r >> kOwnerShift) != e->rank) continue;
      key = r;
    }
    e->staged_total++;
    e->hs_key.push_back(key);
    e->hs_src.push_back(src ? src[i] : AGX_NO_SENDER);
    e->hs_pay.push_back(payload[i]);
  }
  return AGX_OK;
}

// Messages in flight on this rank right now (what agx_stats.in_flight would report): the device's
// backlog, undelivered tells and consumed-later staged chunks (one counter read-back, only once the
// engine has run), plus the host-staged tells not yet uploaded.
agx_status in_flight_now(agx_engine* e, uint64_t* out) {
  uint64_t dev = 0;
  if (e->started) {
    if (e->inflight_known) {
      dev = e->inflight_dev;
    } else {
      uint64_t s[kStatBlk];
      AGX_TRY(read_counters(e, s));
      dev = s[kStatInfl];
      e->inflight_dev = dev;
      e->inflight_known = true;  // (valid until the next agx_run)
    }
  }
  *out = dev + e->n_staged_dev + e->hs_key.size();
  return AGX_OK;
}

// The lock-free tell path: take the published tells (producer by producer, each in its order) into
// the host staging, exactly as agx_stage_tells would stage them -- but only as many as fit the
// message capacity.  The rest stay in the producers' queues (none is refused or lost: the
// reference's unbounded MPSC queue never refuses, AbstractNodeQueue.java:79-82) and
// agx_pump_idle reschedules the pump while any remain, so a burst larger than msg_capacity enters
// over several pumps as the engine drains (back-pressure across pumps).
agx_status take_tells(agx_engine* e) {
  if (!e->tq.pending()) return AGX_OK;
  uint64_t infl = 0;
  AGX_TRY(in_flight_now(e, &infl));
  uint64_t room = e->cap > infl ? e->cap - infl : 0;
  e->tq.take_while([&](uint32_t d, uint32_t s, uint32_t p) {
    const bool local = d < e->n_global && (e->R == 1 || (e->h_route[d] >> kOwnerShift) == e->rank);
    if (local) {
      if (!room) return false;  // stays queued for the next pump
      --room;
    }
    // (agx_tell rejected wide senders already; unknown refs and other ranks' tells take no room)
    const agx_status r = agx_stage_tells(e, &d, &s, &p, 1);
    (void)r;
    return true;
  });
  return AGX_OK;
}

agx_status agx_tell(agx_engine* e, uint32_t dst, uint32_t src, uint32_t payload, int32_t* schedule) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  if ((src & AGX_WIDE_BIT) && src != AGX_NO_SENDER)
    return set_err(AGX_EINVAL, "tell: sender %u is not an actor id (bit 31 tags CRDT state gossips)", src);
  const bool sched = e->tq.tell(dst, src, payload);
  if (schedule) *schedule = sched ? 1 : 0;
  return AGX_OK;
}

// The pump's last call (Mailbox.run's finally, Mailbox.scala:227-240: setAsIdle, then
// registerForExecution if the mailbox still has messages).  "Still has messages" is, here, either
// tells published but not taken (the queue re-check after the idle store) or mail in flight on the
// device after a run that stopped at its superstep budget (gpu.supersteps-per-pump) -- then the
// engine stays scheduled and the pump is submitted again.  After a failed run only the queue
// re-check applies (a broken engine must not spin its pump).
agx_status agx_pump_idle(agx_engine* e, int32_t* reschedule) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  bool again = false;
  if (e->last_run_ok && e->started) {
    uint64_t infl = 0;
    AGX_TRY(in_flight_now(e, &infl));
    again = infl > 0;  // (status stays "scheduled": this pump hands over to the next)
  }
  if (!again) again = e->tq.pump_idle();
  if (reschedule) *reschedule = again ? 1 : 0;
  return AGX_OK;
}

agx_status agx_pump_cancel(agx_engine* e) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  e->tq.cancel_schedule();
  return AGX_OK;
}

agx_status agx_run(agx_engine* e, uint32_t max_supersteps, agx_stats* out) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  e->last_run_ok = false;
  AGX_TRY(ensure_dev(e));
  AGX_TRY(take_tells(e));
  e->inflight_known = false;  // (the supersteps below change the device's in-flight count)
  if (e->R > 1 && !e->comm) return set_err(AGX_ESTATE, "n_ranks > 1 needs agx_comm_init (or agx_group_run)");
  AGX_TRY(prepare_run(e));
  AGX_TRY(setup_rings(e));
  AGX_TRY(setup_ring_apply(e));
  AGX_TRY(setup_orset(e));
  e->started = true;
  if (e->R > 1) {
    AGX_TRY(run_multi_rccl(e, max_supersteps));
  } else {
    AGX_TRY(run_single(e, max_supersteps));
  }
  prof_collect(e);
  if (e->ident_on && getenv("AGX_IDENT_DEBUG")) {  // diagnostic: the last superstep's slice summaries
    const uint32_t nsl = (e->nb + kBlSlice - 1) / kBlSlice;
    std::vector<uint32_t> h((kMaxBlSlices + 1) * kSlSum), id(4);
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipMemcpy(h.data(), e->d_slsum, h.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(id.data(), e->d_ident, 16, hipMemcpyDeviceToHost));
    fprintf(stderr, "[agx ident] on=%u rot=%u total=%u staged=%u |", id[0], id[1], id[2], h[kMaxBlSlices * kSlSum]);
    for (uint32_t i = 0; i < nsl; ++i)
      fprintf(stderr, " s%u{tot=%u fl=%u d=%u nd=%u pos=%u first=%u last=%u}", i, h[i * kSlSum], h[i * kSlSum + 1],
              h[i * kSlSum + 2], h[i * kSlSum + 3], h[i * kSlSum + 4], h[i * kSlSum + 5], h[i * kSlSum + 6]);
    fprintf(stderr, "\n");
  }
  if (e->d_dbg) {  // diagnostic: mean phase durations of k_bucket_apply blocks (last superstep)
    const uint64_t nbk = std::min<uint64_t>(e->nb, 4096);
    std::vector<unsigned long long> h(nbk * 16);
    HIP_TRY(hipMemcpy(h.data(), e->d_dbg, h.size() * 8, hipMemcpyDeviceToHost));
    double acc[8] = {0};
    unsigned long long t0min = ~0ull, t8max = 0;
    uint64_t nst = 0;  // blocks that recorded stamps (the skew launch runs fewer blocks)
    for (uint64_t b = 0; b < nbk; ++b) {
      if (!h[b * 16] || !h[b * 16 + 8]) continue;
      ++nst;
      for (int k = 0; k < 8; ++k) acc[k] += (double)(h[b * 16 + k + 1] - h[b * 16 + k]);
      t0min = std::min(t0min, h[b * 16]);
      t8max = std::max(t8max, h[b * 16 + 8]);
    }
    fprintf(stderr, "[agx stamps%s] mean cycles per phase over %llu blocks:", e->stamps_skew ? " (skew launch)" : "",
            (unsigned long long)nst);
    const char* nm[8] = {"range+alive", "sort", "->finish", "classify+backlog", "prefetch+phaseA", "scan", "phaseB", "hist+stats"};
    const char* nr[8] = {"count", "admission", "ring_heads", "placement", "prefetch", "drain", "tells", "words+hist"};
    for (int k = 0; k < 8; ++k) fprintf(stderr, " %s=%.0f", (e->rg_on ? nr : nm)[k], nst ? acc[k] / nst : 0.0);
    fprintf(stderr, " | kernel span=%llu cycles\n", t8max - t0min);
    std::vector<std::pair<unsigned long long, uint64_t>> slow;
    for (uint64_t b = 0; b < nbk; ++b) slow.push_back({h[b * 16 + 10], b});
    std::sort(slow.rbegin(), slow.rend());
    fprintf(stderr, "[agx stamps] slowest buckets (cycles bucket inbox):");
    for (size_t i = 0; i < std::min<size_t>(6, slow.size()); ++i)
      fprintf(stderr, " %llu:%llu:%llu", slow[i].first, h[slow[i].second * 16 + 11], h[slow[i].second * 16 + 12]);
    fprintf(stderr, "\n");
    {  // device-clock (100 MHz) block start / end offsets within the launch (k_dense_fused only: slots 13 / 14)
      std::vector<double> st, en;
      unsigned long long s0 = ~0ull;
      for (uint64_t b = 0; b < nbk; ++b)
        if (h[b * 16 + 13] && h[b * 16 + 14]) s0 = std::min(s0, h[b * 16 + 13]);
      for (uint64_t b = 0; b < nbk; ++b)
        if (h[b * 16 + 13] && h[b * 16 + 14]) {
          st.push_back((h[b * 16 + 13] - s0) * 0.01);
          en.push_back((h[b * 16 + 14] - s0) * 0.01);
        }
      if (!st.empty()) {
        std::vector<double> du(st.size());
        for (size_t i = 0; i < st.size(); ++i) du[i] = en[i] - st[i];
        std::sort(st.begin(), st.end());
        std::sort(en.begin(), en.end());
        std::sort(du.begin(), du.end());
        auto q = [](const std::vector<double>& v, double f) { return v[std::min(v.size() - 1, (size_t)(f * v.size()))]; };
        fprintf(stderr, "[agx stamps] block start us (p0/p50/p90/max): %.2f %.2f %.2f %.2f | end: %.2f %.2f %.2f %.2f | "
                "duration: %.2f %.2f %.2f %.2f\n", q(st, 0), q(st, .5), q(st, .9), st.back(), q(en, 0), q(en, .5), q(en, .9),
                en.back(), q(du, 0), q(du, .5), q(du, .9), du.back());
      }
    }
    HIP_TRY(hipMemsetAsync(e->d_dbg, 0, h.size() * 8, e->stream));
  }
  // out == NULL: no counter read-back (one stream round trip less; agx_get_stats reads them
  // later), but the error word came back with the run's final sync
  const agx_status rs = out ? collect_stats(e, out, true) : error_status(e, e->h_stat[ST_ERROR]);
  e->last_run_ok = rs == AGX_OK;
  return rs;
}

agx_status agx_identity_supersteps(agx_engine* e, uint64_t* out) {
  if (!e || !out) return set_err(AGX_EINVAL, "bad identity_supersteps args");
  AGX_TRY(ensure_dev(e));
  uint64_t s[kStatBlk];
  AGX_TRY(read_counters(e, s));
  *out = s[ST_IDENT];
  return AGX_OK;
}

agx_status agx_ring_buckets(agx_engine* e, uint64_t* out) {
  if (!e || !out) return set_err(AGX_EINVAL, "bad ring_buckets args");
  AGX_TRY(ensure_dev(e));
  *out = 0;
  if (!e->ring_live) return AGX_OK;
  uint32_t n = 0;  // pool slots handed out (high-water mark: released slots are reused first)
  HIP_TRY(hipStreamSynchronize(e->stream));
  AGX_TRY(copy_sync(e, &n, e->d_ring_next, 4, hipMemcpyDeviceToHost));
  *out = std::min(n, e->ring_slots);
  return AGX_OK;
}

// agx_run with the run's device time on the engine stream: HIP events recorded before the first
// launch and after the last replay (single rank), so the host's own time around the run is not in it
agx_status agx_run_timed(agx_engine* e, uint32_t max_supersteps, agx_stats* out, float* device_ms) {
  if (!e || !device_ms) return set_err(AGX_EINVAL, "bad run_timed args");
  AGX_TRY(ensure_dev(e));
  for (auto& ev : e->tev)
    if (!ev) HIP_TRY(hipEventCreate(&ev));
  HIP_TRY(hipEventRecord(e->tev[0], e->stream));
  e->timing = e->R == 1;
  e->tev1_recorded = false;
  const agx_status st = agx_run(e, max_supersteps, out);
  e->timing = false;
  if (st != AGX_OK) return st;
  // multi-rank, and a single-rank run that launched nothing through the replay loop (agx_run(0)
  // captures graphs and returns before it): the end event is recorded here, after the run's work
  if (!e->tev1_recorded) HIP_TRY(hipEventRecord(e->tev[1], e->stream));
  HIP_TRY(hipEventSynchronize(e->tev[1]));
  HIP_TRY(hipEventElapsedTime(device_ms, e->tev[0], e->tev[1]));
  return st;
}

agx_status agx_persist_info(agx_engine* e, uint64_t out[2]) {
  if (!e || !out) return set_err(AGX_EINVAL, "bad persist_info args");
  out[0] = e->persist_launches;
  out[1] = e->persist_supersteps;
  return AGX_OK;
}

agx_status agx_exchange_info(agx_engine* e, uint64_t out[6]) {
  if (!e || !out) return set_err(AGX_EINVAL, "bad exchange_info args");
  out[0] = e->mr_dev_steps;
  out[1] = e->mr_host_steps;
  out[2] = e->mr_sent_env;
  out[3] = e->mr_sent_rows;
  out[4] = e->mr_host ? 1u : 0u;
  out[5] = e->slab;
  return AGX_OK;
}

agx_status agx_get_stats(agx_engine* e, agx_stats* out) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  AGX_TRY(ensure_dev(e));
  return collect_stats(e, out, true);
}

agx_status agx_get_shape(agx_engine* e, uint64_t* n_actors, uint32_t* n_words) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  if (n_actors) *n_actors = e->n_global;
  if (n_words) *n_words = e->W;
  return AGX_OK;
}

agx_status agx_read_state(agx_engine* e, uint64_t first_id, uint64_t count, uint64_t* words, uint8_t* alive) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  if (first_id + count > e->n_global) return set_err(AGX_EINVAL, "range out of bounds");
  AGX_TRY(ensure_dev(e));
  AGX_TRY(sync_mirrors(e));
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t id = first_id + i, l;
    if (e->R > 1) {
      uint32_t r = e->h_route[id];
      if ((r >> kOwnerShift) != e->rank) continue;
      l = r & kLocalMask;
    } else {
      l = id;
    }
    if (words)
      for (uint32_t w = 0; w < e->W; ++w) words[i * e->W + w] = e->h_state[(uint64_t)w * e->n_local + l];
    if (alive) alive[i] = e->h_alive[l] & 1u;
  }
  return AGX_OK;
}

agx_status agx_comm_unique_id(uint8_t out[128]) {
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  memcpy(out, &id, 128);
  return AGX_OK;
}

agx_status agx_comm_init(agx_engine* e, const uint8_t id[128]) {
  if (!e || !id) return set_err(AGX_EINVAL, "bad comm args");
  AGX_TRY(ensure_dev(e));
  ncclUniqueId uid;
  memcpy(&uid, id, 128);
  NCCL_TRY(ncclCommInitRank(&e->comm, (int)e->R, uid, (int)e->rank));
  return AGX_OK;
}

agx_status agx_group_run(agx_engine** engs, uint32_t n, uint32_t max_steps, agx_stats* out) {
  if (!engs || n == 0) return set_err(AGX_EINVAL, "bad group");
  if (n == 1) return agx_run(engs[0], max_steps, out);
  for (uint32_t i = 0; i < n; ++i) {
    if (!engs[i] || engs[i]->R != n || engs[i]->rank != i || engs[i]->n_global != engs[0]->n_global)
      return set_err(AGX_EINVAL, "group engines must be ranks 0..n-1 of one population");
    if (engs[i]->pw != engs[0]->pw || engs[i]->delta_max != engs[0]->delta_max || engs[i]->kmax != engs[0]->kmax ||
        engs[i]->W != engs[0]->W)
      return set_err(AGX_EINVAL, "group engines differ in row pitch / delta mode / max_emit / n_words");
    AGX_TRY(ensure_dev(engs[i]));
    AGX_TRY(prepare_run(engs[i]));
    AGX_TRY(setup_orset(engs[i]));
    engs[i]->started = true;
    engs[i]->inflight_known = false;
  }
  const uint32_t S = n + 2;
  std::vector<uint64_t> mat((size_t)n * S);
  std::vector<Plan> plans(n);
  for (uint32_t s = 0; s < max_steps; ++s) {
    for (uint32_t i = 0; i < n; ++i) AGX_TRY(phase1(engs[i]));
    for (uint32_t i = 0; i < n; ++i) {
      agx_engine* e = engs[i];
      HIP_TRY(hipMemcpyAsync(&mat[(size_t)i * S], e->d_cvec, S * 8, hipMemcpyDeviceToHost, e->stream));
      HIP_TRY(hipStreamSynchronize(e->stream));
    }
    uint64_t total = 0;
    for (auto v : mat) total += v;
    if (total == 0) break;
    for (uint32_t i = 0; i < n; ++i) {
      make_plan(engs[i], mat.data(), plans[i]);
      if (plans[i].n_bl + plans[i].n_recv + plans[i].n_staged > engs[i]->cap)
        return set_err(AGX_ECAPACITY, "rank %u over capacity", i);
    }
    // loopback exchange: receiver i pulls its slice of every sender's partitioned buffer
    for (uint32_t i = 0; i < n; ++i) {
      agx_engine* r = engs[i];
      for (uint32_t q = 0; q < n; ++q) {
        uint64_t cnt = plans[i].recv_cnt[q];
        if (!cnt) continue;
        agx_engine* snd = engs[q];
        uint64_t so = plans[q].send_off[i], ro = plans[i].recv_off[q];
        HIP_TRY(hipMemcpyAsync(r->A.key + ro, snd->s2.key + so, cnt * 4, hipMemcpyDeviceToDevice, r->stream));
        HIP_TRY(hipMemcpyAsync(r->A.src + ro, snd->s2.src + so, cnt * 4, hipMemcpyDeviceToDevice, r->stream));
        HIP_TRY(hipMemcpyAsync(r->A.pay + ro, snd->s2.pay + so, cnt * 4, hipMemcpyDeviceToDevice, r->stream));
        if (r->pw && q != i)
          HIP_TRY(hipMemcpyAsync(r->d_rx + ro * r->pw, snd->d_s2rows + so * snd->pw, cnt * r->pw * 4ull,
                                 hipMemcpyDeviceToDevice, r->stream));
      }
      AGX_TRY(fix_rx(r, plans[i]));
    }
    for (uint32_t i = 0; i < n; ++i) {
      Plan& p = plans[i];
      AGX_TRY(phase2(engs[i], p.n_bl + p.n_recv + p.n_staged, p.n_bl + p.n_recv));
    }
    for (uint32_t i = 0; i < n; ++i) HIP_TRY(hipStreamSynchronize(engs[i]->stream));
  }
  agx_stats tot{};
  for (uint32_t i = 0; i < n; ++i) {
    prof_collect(engs[i]);
    agx_stats st{};
    AGX_TRY(collect_stats(engs[i], &st, true));
    tot.delivered += st.delivered;
    tot.dead_letters += st.dead_letters;
    tot.unhandled += st.unhandled;
    tot.emitted += st.emitted;
    tot.staged += st.staged;
    tot.supersteps = std::max(tot.supersteps, st.supersteps);
    tot.in_flight += st.in_flight;
    tot.bytes_alg += st.bytes_alg;
  }
  if (out) *out = tot;
  return AGX_OK;
}

agx_status agx_mr_plan(const uint64_t* mat, uint32_t R, uint32_t rank, uint32_t slab, uint64_t cap, uint32_t* code,
                       uint64_t* send_off, uint64_t* recv_off, uint64_t* n_backlog) {
  if (!mat || !code || R == 0 || R > AGX_MAX_RANKS || rank >= R) return set_err(AGX_EINVAL, "bad mr_plan args");
  MrPlan p;
  mr_decide(mat, R, rank, slab, cap, p);
  *code = p.code;
  for (uint32_t q = 0; q <= R; ++q) {
    if (send_off) send_off[q] = p.soff[q];
    if (recv_off) recv_off[q] = p.roff[q];
  }
  if (n_backlog) *n_backlog = p.nbl;
  return AGX_OK;
}

agx_status agx_exchange_plan(const uint64_t* mat, uint32_t R, uint32_t rank, uint64_t* send_cnt, uint64_t* send_off,
                             uint64_t* recv_cnt, uint64_t* recv_off, uint64_t* inflight) {
  if (!mat || R == 0 || R > AGX_MAX_RANKS || rank >= R) return set_err(AGX_EINVAL, "bad plan args");
  agx_engine tmp;
  tmp.R = R;
  tmp.rank = rank;
  Plan p;
  make_plan(&tmp, mat, p);
  for (uint32_t q = 0; q < R; ++q) {
    if (send_cnt) send_cnt[q] = p.send_cnt[q];
    if (send_off) send_off[q] = p.send_off[q];
    if (recv_cnt) recv_cnt[q] = p.recv_cnt[q];
    if (recv_off) recv_off[q] = p.recv_off[q];
  }
  if (inflight) *inflight = p.total_inflight;
  return AGX_OK;
}

agx_status agx_profile_enable(agx_engine* e, int on) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  e->prof = on != 0;
  return AGX_OK;
}

agx_status agx_profile_reset(agx_engine* e) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  prof_collect(e);
  for (int i = 0; i < K_NCLASS; ++i) {
    e->prof_ms[i] = 0;
    e->prof_n[i] = 0;
    e->prof_items[i] = 0;
  }
  return AGX_OK;
}

agx_status agx_profile_read(agx_engine* e, char (*names)[32], double* total_ms, uint64_t* launches, uint64_t* items,
                            uint32_t cap, uint32_t* n) {
  if (!e) return set_err(AGX_EINVAL, "null engine");
  prof_collect(e);
  uint32_t k = 0;
  for (int i = 0; i < K_NCLASS && k < cap; ++i, ++k) {
    if (names) {
      strncpy(names[k], kClassNames[i], 31);
      names[k][31] = 0;
    }
    if (total_ms) total_ms[k] = e->prof_ms[i];
    if (launches) launches[k] = e->prof_n[i];
    if (items) items[k] = e->prof_items[i];
  }
  if (n) *n = K_NCLASS;
  return AGX_OK;
}

}  // extern "C"
