/*
 * bsp_ref.c — TEST INFRASTRUCTURE ONLY.  CPU oracle for the batched actor
 * dispatcher.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this; the product path (akka_amd/) never does.
 *
 * A deterministic restatement of the reference's
 * Dispatcher/Mailbox drain loop as bulk-synchronous supersteps
 * (SURVEY.md §7 "Execution model").  Each step follows these reference
 * functions (paths relative to /root/reference):
 *
 *  - inbox formation: the per-actor FIFO queue, backlog first, new arrivals
 *    appended in emission order — Mailbox.enqueue / NodeMessageQueue
 *    (akka-actor/src/main/scala/akka/dispatch/Mailbox.scala:89,392-409;
 *    akka-actor/src/main/java/akka/dispatch/AbstractNodeQueue.java:79-82).
 *  - bounded admission: BoundedMailbox with pushTimeOut 0 tail-drops into
 *    deadLetters (Mailbox.scala:551-565,699-720; AbstractBoundedNodeQueue.java:92-113;
 *    typed MailboxSelector.bounded -> BoundedMailbox(n, 0) Mailboxes.scala:212-216).
 *    An arrival of rank r is admitted iff len(backlog) + r < C, i.e. iff its
 *    position p in the inbox is < C.
 *  - drain: processMailbox(left = max(throughput, 1)) (Mailbox.scala:260-277):
 *    the first min(len, max(T,1)) messages are invoked in order, the rest
 *    stay queued (the backlog for the next step).
 *  - invoke: ActorCell.invoke -> receiveMessage (akka-actor/.../actor/ActorCell.scala:539-577)
 *    -> typed Behavior.interpretMessage / ActorAdapter.next
 *    (akka-actor-typed/.../Behavior.scala:229-278, .../adapter/ActorAdapter.scala:152-168):
 *    same / stopped / unhandled.
 *  - stop: context.stop(self) takes effect after the current message
 *    (Mailbox.scala:273); remaining drained messages and all later arrivals
 *    are dead letters (AbstractDispatcher.scala:221-227, Mailbox.scala:337-351).
 *    Messages of a stopping actor that were already queued beyond the
 *    throughput cap are dead-lettered at the next inbox formation (same
 *    totals; see DESIGN.md "stop").
 *  - tell to an unknown ref / noSender -> deadLetters (ActorRef.scala:546,687-695).
 *  - shard ownership: HashCodeMessageExtractor.shardId
 *    (akka-cluster-sharding/.../ShardRegion.scala:154-158) with JLS String.hashCode.
 *
 * Canonical order (what makes the BSP schedule deterministic): arrivals to an
 * actor are ordered by (owner rank of sender, sender id, per-sender emission
 * index), then host-staged tells in staging order.  With n_ranks = 1 this is
 * (sender id, emission index).  It preserves per-sender FIFO, the only order
 * Akka guarantees (akka-docs/.../general/message-delivery-reliability.md:110-131).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/akka_gpu.h"
#include "behaviors_ref.h"

/* ---------------------------------------------------------------- helpers */

/* SplitMix64 finaliser — the counter RNG shared with the device code. */
uint64_t bsp_splitmix64(uint64_t x) { return ref_splitmix64(x); }

/* JLS String.hashCode of the decimal representation of id (s[0]*31^(n-1)+...). */
int32_t bsp_java_hash_decimal(uint32_t id) {
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

/* HashCodeMessageExtractor.shardId: (math.abs(id.hashCode) % maxNumberOfShards)
 * (ShardRegion.scala:154-158).  math.abs(Int.MinValue) == Int.MinValue, so the
 * result can be negative (e.g. "-648" for hash -2147483648 at 1000 shards).  */
int32_t bsp_shard_id(uint32_t id, uint32_t num_shards) {
  int32_t h = bsp_java_hash_decimal(id);
  int32_t a = (h == INT32_MIN) ? INT32_MIN : (h < 0 ? -h : h);
  return a % (int32_t)num_shards; /* Java '%' truncates toward zero like C */
}

uint32_t bsp_owner(uint32_t id, uint32_t num_shards, uint32_t n_ranks) {
  if (n_ranks <= 1) return 0;
  int32_t s = bsp_shard_id(id, num_shards);
  int32_t m = s % (int32_t)n_ranks;
  if (m < 0) m += (int32_t)n_ranks;
  return (uint32_t)m;
}

uint64_t bsp_fanout_rand(uint64_t seed, uint32_t self, uint32_t h, uint32_t j) {
  return ref_fanout_rand(seed, self, h, j);
}

/* ---------------------------------------------------------------- sim */

typedef struct {
  uint32_t dst, src, payload;
} env_t;

/* Envelopes; CRDT state gossips carry their snapshot inline (`rw` u64 per
 * envelope in `rows`, allocated once a CRDT kind is registered). */
typedef struct {
  env_t* v;
  uint64_t* rows;
  uint64_t n, cap;
  uint32_t rw;
} envvec;

static int ev_push(envvec* e, uint32_t d, uint32_t s, uint32_t p, const uint64_t* row, uint32_t row_words) {
  if (e->n == e->cap) {
    uint64_t nc = e->cap ? e->cap * 2 : 1024;
    env_t* nv = (env_t*)realloc(e->v, nc * sizeof(env_t));
    if (!nv) return -1;
    e->v = nv;
    if (e->rw) {
      uint64_t* nr = (uint64_t*)realloc(e->rows, nc * e->rw * 8);
      if (!nr) return -1;
      e->rows = nr;
    }
    e->cap = nc;
  }
  e->v[e->n].dst = d;
  e->v[e->n].src = s;
  e->v[e->n].payload = p;
  if (e->rw) {
    uint64_t* r = e->rows + e->n * e->rw;
    uint32_t k = row ? (row_words < e->rw ? row_words : e->rw) : 0;
    if (k) memcpy(r, row, (size_t)k * 8);
    if (k < e->rw) memset(r + k, 0, (size_t)(e->rw - k) * 8);
  }
  e->n++;
  return 0;
}

/* enable inline snapshots of `rw` u64 per envelope (only before any mail exists) */
static int ev_set_rw(envvec* e, uint32_t rw) {
  if (rw <= e->rw) return 0;
  if (e->n) return -1;
  free(e->rows);
  e->rows = e->cap ? (uint64_t*)calloc(e->cap * rw, 8) : (uint64_t*)0;
  if (e->cap && !e->rows) return -1;
  e->rw = rw;
  return 0;
}

typedef struct bsp_sim {
  uint64_t n;
  uint32_t T, C, W, n_ranks, num_shards;
  uint8_t* kind;
  uint8_t* alive;
  uint64_t* state; /* actor-major: state[a*W + w] */
  uint32_t* order; /* apply order: by (owner, id) */
  uint32_t* pos;   /* its inverse (built at the first superstep) */
  /* params */
  ref_params P;
  uint32_t* zipf_cdf;
  uint32_t* zipf_perm;
  uint64_t* row_ptr;
  uint32_t* col;
  agx_case* bcase;
  agx_act* bact;
  uint32_t* bfirst;
  /* mail */
  /* mail in flight: runs of backlog then runs of emitted tells (one run per apply thread of the last
   * superstep, in canonical order: concatenated without a copy), then the host-staged tells */
  envvec* seg;
  uint32_t nseg, nbl; /* runs; the first nbl are backlog */
  uint32_t rw;        /* inline snapshot words per envelope (CRDT state gossips) */
  envvec staged;
  agx_stats st;
  /* per-actor mailboxes (Mailboxes.lookupConfigurator, Mailboxes.scala:204-260): class per actor,
   * capacity per class (class 0 = the dispatcher default), Tr = throughput before the bound clamp */
  uint8_t* mcls;
  uint32_t mcap[AGX_MAX_MAILBOX_CLASSES];
  uint32_t Tr;
  /* the reply path: tells to host-side ids [host_lo, host_lo + host_n) go to the outbox
   * (sender() ! reply to a JVM actor, ActorCell.scala:583-587) */
  uint32_t host_lo, host_n;
  uint32_t* outbox;
  uint64_t outbox_n, outbox_cap;
  /* the engine's overflow rule (agx_take_outbound, include/akka_gpu.h): at most outbox_cap appends
   * between two takes are kept, later ones are dropped and counted; the next take reports the drop
   * once (AGX_ECAPACITY) and clears it -- the run itself goes on */
  uint64_t outbox_since, outbox_lost;
} bsp_sim;

bsp_sim* bsp_create(uint64_t n_actors, uint32_t throughput, uint32_t capacity, uint32_t n_words,
                    uint32_t n_ranks, uint32_t num_shards) {
  if (n_words == 0 || n_words > AGX_MAX_WORDS || n_actors == 0 || n_actors >= (1ull << 31)) return NULL;
  bsp_sim* s = (bsp_sim*)calloc(1, sizeof(bsp_sim));
  if (!s) return NULL;
  s->n = n_actors;
  s->T = throughput == 0 ? 1 : throughput; /* max(throughput, 1), Mailbox.scala:261 */
  if ((int32_t)throughput < 0) s->T = 1;
  s->Tr = s->T;
  s->C = capacity;
  s->mcap[0] = capacity;
  /* a bounded queue never holds more than C messages: drain <= min(T, C) */
  if (capacity && s->T > capacity) s->T = capacity;
  s->W = n_words;
  s->n_ranks = n_ranks ? n_ranks : 1;
  s->num_shards = num_shards ? num_shards : 1000;
  s->kind = (uint8_t*)calloc(n_actors, 1);
  s->alive = (uint8_t*)calloc(n_actors, 1);
  s->state = (uint64_t*)calloc(n_actors * n_words, 8);
  s->order = (uint32_t*)malloc(n_actors * 4);
  s->mcls = (uint8_t*)calloc(n_actors, 1);
  s->P.n = n_actors;
  s->P.W = n_words;
  s->P.ring_stride = 1;
  if (!s->kind || !s->alive || !s->state || !s->order || !s->mcls) return NULL;
  if (s->n_ranks == 1) {
    for (uint64_t a = 0; a < n_actors; ++a) s->order[a] = (uint32_t)a;
  } else {
    /* counting sort of ids by owner, stable in id */
    uint64_t cnt[AGX_MAX_RANKS + 1];
    memset(cnt, 0, sizeof cnt);
    uint8_t* own = (uint8_t*)malloc(n_actors);
    for (uint64_t a = 0; a < n_actors; ++a) {
      own[a] = (uint8_t)bsp_owner((uint32_t)a, s->num_shards, s->n_ranks);
      cnt[own[a] + 1]++;
    }
    for (uint32_t r = 0; r < s->n_ranks; ++r) cnt[r + 1] += cnt[r];
    for (uint64_t a = 0; a < n_actors; ++a) s->order[cnt[own[a]]++] = (uint32_t)a;
    free(own);
  }
  return s;
}

void bsp_destroy(bsp_sim* s) {
  if (!s) return;
  free(s->kind); free(s->alive); free(s->state); free(s->order); free(s->pos); free(s->mcls); free(s->outbox);
  free(s->zipf_cdf); free(s->zipf_perm); free(s->row_ptr); free(s->col);
  free(s->bcase); free(s->bact); free(s->bfirst);
  for (uint32_t i = 0; i < s->nseg; ++i) { free(s->seg[i].v); free(s->seg[i].rows); }
  free(s->seg);
  free(s->staged.v); free(s->staged.rows);
  free(s);
}

static uint64_t bsp_in_flight(const bsp_sim* s) {
  uint64_t n = s->staged.n;
  for (uint32_t i = 0; i < s->nseg; ++i) n += s->seg[i].n;
  return n;
}

/* inline snapshot rows of `rw` u64 per envelope (only before any mail exists) */
static int bsp_set_rw(bsp_sim* s, uint32_t rw) {
  if (rw <= s->rw) return 0;
  if (bsp_in_flight(s)) return -1;
  if (ev_set_rw(&s->staged, rw)) return -1;
  s->rw = rw;
  return 0;
}

int bsp_register_range(bsp_sim* s, uint64_t first, uint64_t count, uint32_t kind, const uint64_t* init,
                       uint64_t stride_words) {
  const int compiled = kind >= AGX_KIND_COMPILED && kind < AGX_KIND_COMPILED + AGX_MAX_BEHAVIORS;
  if (first + count > s->n || (kind >= AGX_KIND_MAX && !compiled)) return 1;
  if ((kind == AGX_KIND_FORWARD_RR || kind == AGX_KIND_STOP_AFTER) && s->W < 2) return 1;
  uint32_t rw = ref_crdt_words(kind);
  if (rw) {
    if (s->W < rw) return 1;
    if (bsp_set_rw(s, rw)) return 1;
  }
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t a = first + i;
    s->kind[a] = (uint8_t)kind;
    s->alive[a] = kind != AGX_KIND_NONE;
    for (uint32_t w = 0; w < s->W; ++w) s->state[a * s->W + w] = init ? init[i * stride_words + w] : 0;
  }
  return 0;
}

void bsp_set_ring(bsp_sim* s, uint32_t stride) { s->P.ring_stride = stride; }

/* agx_set_mailbox_class / agx_set_mailbox: a mailbox type per actor */
int bsp_set_mailbox_class(bsp_sim* s, uint32_t cls, uint32_t capacity) {
  if (cls == 0 || cls >= AGX_MAX_MAILBOX_CLASSES) return 1;
  s->mcap[cls] = capacity;
  return 0;
}
int bsp_set_mailbox(bsp_sim* s, uint64_t first, uint64_t count, uint32_t cls) {
  if (cls >= AGX_MAX_MAILBOX_CLASSES || first + count > s->n) return 1;
  for (uint64_t i = 0; i < count; ++i) s->mcls[first + i] = (uint8_t)cls;
  return 0;
}

/* agx_set_outbound / agx_take_outbound (the outbox keeps the canonical emission order) */
int bsp_set_outbound(bsp_sim* s, uint32_t first, uint32_t n, uint64_t cap) {
  if (n && first < s->n) return 1;
  s->host_lo = first;
  s->host_n = n;
  if (n && cap != s->outbox_cap) s->outbox_since = 0; /* the engine drains its device outbox here */
  if (n) s->outbox_cap = cap;
  return 0;
}
/* returns 0, or 5 (AGX_ECAPACITY: tells were dropped since the last take; nothing is taken then) */
int bsp_take_outbound(bsp_sim* s, uint32_t* dst, uint32_t* src, uint32_t* pay, uint64_t cap, uint64_t* n) {
  *n = 0;
  s->outbox_since = 0;
  if (s->outbox_lost) {
    s->outbox_lost = 0;
    return 5;
  }
  const uint64_t k = s->outbox_n < cap ? s->outbox_n : cap;
  for (uint64_t i = 0; i < k; ++i) {
    dst[i] = s->outbox[3 * i];
    src[i] = s->outbox[3 * i + 1];
    pay[i] = s->outbox[3 * i + 2];
  }
  memmove(s->outbox, s->outbox + 3 * k, (size_t)(s->outbox_n - k) * 12);
  s->outbox_n -= k;
  *n = k;
  return 0;
}

void bsp_set_gossip(bsp_sim* s, uint32_t fanout, uint64_t seed) {
  s->P.gossip_f = fanout;
  s->P.gossip_seed = seed;
}

/* compiled behaviour tables (include/akka_gpu.h agx_set_behaviors; copied) */
int bsp_set_behaviors(bsp_sim* s, const agx_case* cases, uint32_t n_cases, const agx_act* acts, uint32_t n_acts,
                      const uint32_t* first, uint32_t n_beh) {
  free(s->bcase); free(s->bact); free(s->bfirst);
  s->bcase = (agx_case*)malloc((n_cases ? n_cases : 1) * sizeof(agx_case));
  s->bact = (agx_act*)malloc((n_acts ? n_acts : 1) * sizeof(agx_act));
  s->bfirst = (uint32_t*)malloc((n_beh + 1) * 4);
  if (!s->bcase || !s->bact || !s->bfirst) return 2;
  memcpy(s->bcase, cases, n_cases * sizeof(agx_case));
  memcpy(s->bact, acts, n_acts * sizeof(agx_act));
  memcpy(s->bfirst, first, (n_beh + 1) * 4);
  s->P.bcase = s->bcase;
  s->P.bact = s->bact;
  s->P.bfirst = s->bfirst;
  s->P.n_beh = n_beh;
  return 0;
}

/* delta-crdt.enabled / max-delta-size (include/akka_gpu.h agx_set_delta_crdt) */
int bsp_set_delta_crdt(bsp_sim* s, uint32_t max_delta_size) {
  if (max_delta_size > AGX_DELTA_MAX_SIZE) return 1;
  s->P.delta_max = max_delta_size;
  uint32_t rw = 0;
  for (uint64_t a = 0; a < s->n; ++a) {
    const uint32_t k = s->kind[a];
    const uint32_t need = k == AGX_KIND_GCOUNTER ? AGX_GCOUNTER_DELTA_WORDS
                          : k == AGX_KIND_PNCOUNTER ? AGX_PNCOUNTER_DELTA_WORDS
                          : k == AGX_KIND_ORSET ? AGX_ORSET_DELTA_WORDS : 0u;
    if (max_delta_size && need > s->W) return 1;
    const uint32_t r = ref_row_words(k, max_delta_size);
    if (r > rw) rw = r;
  }
  if (bsp_set_rw(s, rw)) return 1;
  return 0;
}

int bsp_set_fanout(bsp_sim* s, uint32_t k, uint64_t seed, const uint32_t* cdf, const uint32_t* perm, uint64_t n) {
  s->P.fan_k = k;
  s->P.fan_seed = seed;
  free(s->zipf_cdf); free(s->zipf_perm);
  s->zipf_cdf = (uint32_t*)malloc(n * 4);
  s->zipf_perm = (uint32_t*)malloc(n * 4);
  if (!s->zipf_cdf || !s->zipf_perm) return 2;
  memcpy(s->zipf_cdf, cdf, n * 4);
  memcpy(s->zipf_perm, perm, n * 4);
  s->P.zipf_cdf = s->zipf_cdf;
  s->P.zipf_perm = s->zipf_perm;
  s->P.zipf_n = n;
  return 0;
}

int bsp_set_graph(bsp_sim* s, const uint64_t* row_ptr, const uint32_t* col) {
  free(s->row_ptr); free(s->col);
  s->row_ptr = (uint64_t*)malloc((s->n + 1) * 8);
  uint64_t e = row_ptr[s->n];
  s->col = (uint32_t*)malloc((e ? e : 1) * 4);
  if (!s->row_ptr || !s->col) return 2;
  memcpy(s->row_ptr, row_ptr, (s->n + 1) * 8);
  memcpy(s->col, col, e * 4);
  s->P.row_ptr = s->row_ptr;
  s->P.col = s->col;
  return 0;
}

/* Workload setup (not the dispatcher): the R-MAT destinations agx_set_graph_rmat generates on the
 * device, restated from its formula in include/akka_gpu.h -- edge e's destination takes `bits`
 * quadrant draws q = splitmix64(e*64 + bit + seed) & 0xFFFF, bit = (ta <= q < tb) | (q >= tc), MSB
 * first, reduced mod n (workloads.rmat_cols is the numpy form; tests/test_oracle_golden.py checks
 * they agree).  Split over `threads` host threads so a 10^8-actor graph (~3.6e8 edges) takes
 * seconds, not minutes, in the full-size parity tests. */
typedef struct {
  uint32_t* col;
  uint64_t lo, hi, seed, n;
  uint32_t bits, ta, tb, tc;
} rmat_job;

static void* rmat_worker(void* arg) {
  const rmat_job* j = (const rmat_job*)arg;
  for (uint64_t e = j->lo; e < j->hi; ++e) {
    uint64_t c = 0;
    for (uint32_t bit = 0; bit < j->bits; ++bit) {
      const uint32_t q = (uint32_t)(ref_splitmix64(e * 64ull + bit + j->seed) & 0xFFFFull);
      c |= (uint64_t)(((q >= j->ta && q < j->tb) || q >= j->tc) ? 1u : 0u) << (j->bits - 1 - bit);
    }
    j->col[e] = (uint32_t)(c % j->n);
  }
  return 0;
}

int bsp_set_graph_rmat(bsp_sim* s, const uint64_t* row_ptr, uint32_t bits, uint32_t ta, uint32_t tb, uint32_t tc,
                       uint64_t seed, uint32_t threads) {
  free(s->row_ptr); free(s->col);
  s->row_ptr = (uint64_t*)malloc((s->n + 1) * 8);
  const uint64_t m = row_ptr[s->n];
  s->col = (uint32_t*)malloc((m ? m : 1) * 4);
  if (!s->row_ptr || !s->col) return 2;
  memcpy(s->row_ptr, row_ptr, (s->n + 1) * 8);
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  rmat_job jobs[64];
  pthread_t th[64];
  int live[64] = {0};
  for (uint32_t t = 0; t < threads; ++t) {
    jobs[t] = (rmat_job){s->col, m * t / threads, m * (t + 1) / threads, seed, s->n, bits, ta, tb, tc};
    /* the last slice (and any whose thread could not start) runs on this thread */
    live[t] = t + 1 < threads && pthread_create(&th[t], 0, rmat_worker, &jobs[t]) == 0;
    if (!live[t]) rmat_worker(&jobs[t]);
  }
  for (uint32_t t = 0; t < threads; ++t)
    if (live[t]) pthread_join(th[t], 0);
  s->P.row_ptr = s->row_ptr;
  s->P.col = s->col;
  return 0;
}

int bsp_stage(bsp_sim* s, const uint32_t* dst, const uint32_t* src, const uint32_t* payload, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    s->st.staged++;
    uint32_t sv = src ? src[i] : AGX_NO_SENDER;
    if (ref_is_wide(sv)) return 1; /* host tells are never state gossips */
    if (dst[i] >= s->n) { s->st.dead_letters++; continue; }
    if (ev_push(&s->staged, dst[i], sv, payload[i], 0, 0)) return 2;
  }
  return 0;
}

/* ---------------------------------------------------------------- one superstep
 * Inbox formation is a stable sort of the message list [backlog ++ emitted ++ staged] by the
 * destination's position in the canonical apply order (the counting sort of the restatement; a
 * radix sort of the message indices when the mail is sparse against the population, so a
 * superstep costs O(mail), not O(actors)).  The actors with mail are then applied in canonical
 * order, split over host threads into contiguous runs: each run collects its own emitted tells,
 * backlog, outbox and counters, and the runs are concatenated in order afterwards -- exactly the
 * sequence one thread produces (every behaviour touches only its own actor's state).
 * BSP_THREADS=1 restores a single thread; the tests compare 1 and N threads. */

typedef struct {
  bsp_sim* s;
  ref_params P;  /* per-thread copy: ref_apply may set P.error */
  envvec emitted, backlog;
  uint32_t* outbox;
  uint64_t outbox_n;
  agx_stats st;
  int error;
} bsp_part;

/* emit: tell(dst, payload) from `self`; unknown dst -> deadLetters now. */
static void emit_cb(void* ctx, uint32_t dst, uint32_t self, uint32_t payload, const uint64_t* row, uint32_t rw) {
  bsp_part* t = (bsp_part*)ctx;
  bsp_sim* s = t->s;
  if (dst >= s->n && dst - s->host_lo < s->host_n) { /* a host-side actor: the outbox (not emitted here) */
    uint32_t* o = (uint32_t*)realloc(t->outbox, (size_t)(t->outbox_n + 1) * 12);
    if (!o) { t->error = 1; return; }
    t->outbox = o;
    o[3 * t->outbox_n] = dst;
    o[3 * t->outbox_n + 1] = self;
    o[3 * t->outbox_n + 2] = payload;
    t->outbox_n++;
    return;
  }
  t->st.emitted++;
  if (dst >= s->n) { t->st.dead_letters++; return; }
  if (ev_push(&t->emitted, dst, row ? (self | AGX_WIDE_BIT) : self, payload, row, rw)) t->error = 1;
}

/* a message of the run list [backlog runs ++ emitted runs ++ staged], named (run << 40) | index */
#define MSG_RUN_SHIFT 40
typedef struct {
  const envvec** v;
} msgview;
static inline const env_t* mv_env(const msgview* m, uint64_t q, const uint64_t** row) {
  const envvec* e = m->v[q >> MSG_RUN_SHIFT];
  const uint64_t i = q & ((1ull << MSG_RUN_SHIFT) - 1);
  *row = e->rw ? e->rows + i * e->rw : (const uint64_t*)0;
  return &e->v[i];
}
/* every message id of the run list, in order */
#define FOR_EACH_MSG(mv, nruns, q)                                               \
  for (uint64_t _r = 0; _r < (nruns); ++_r)                                     \
    for (uint64_t _i = 0, q = (_r << MSG_RUN_SHIFT); _i < (mv).v[_r]->n; ++_i, ++q)

typedef struct {
  bsp_sim* s;
  bsp_part* part;
  const msgview* mv;
  const uint64_t* perm;   /* message indices in inbox order */
  const uint64_t* abeg;   /* per active actor: first inbox position (abeg[k+1] = end) */
  const uint32_t* aact;   /* per active actor: its id */
  uint64_t k0, k1;        /* this run's active actors */
} bsp_job;

static void* bsp_apply_run(void* arg) {
  const bsp_job* j = (const bsp_job*)arg;
  bsp_sim* s = j->s;
  bsp_part* t = j->part;
  const uint32_t rw = s->rw;
  for (uint64_t k = j->k0; k < j->k1; ++k) {
    const uint32_t a = j->aact[k];
    const uint64_t b = j->abeg[k], L = j->abeg[k + 1] - b;
    if (!s->alive[a]) { t->st.dead_letters += L; continue; }
    /* this actor's mailbox: capacity C (0 = unbounded), drain <= min(throughput, C) */
    const uint32_t C = s->mcap[s->mcls[a]];
    const uint32_t T = C && s->Tr > C ? C : s->Tr;
    const uint64_t nd = L < T ? L : T;
    uint32_t kcur = s->kind[a];
    for (uint64_t p = 0; p < nd; ++p) {
      const uint64_t* row;
      const env_t* m = mv_env(j->mv, j->perm[b + p], &row);
      const uint32_t r = ref_apply(&t->P, &kcur, a, &s->state[(uint64_t)a * s->W], m->src, m->payload, row, emit_cb, t);
      s->kind[a] = (uint8_t)kcur;
      t->st.delivered++;
      if (r == AGX_RES_UNHANDLED) t->st.unhandled++;
      if (r == AGX_RES_STOPPED) {
        s->alive[a] = 0;
        t->st.dead_letters += nd - p - 1;
        break;
      }
    }
    for (uint64_t p = nd; p < L; ++p) {
      if (C == 0 || p < C) {
        const uint64_t* row;
        const env_t* m = mv_env(j->mv, j->perm[b + p], &row);
        if (ev_push(&t->backlog, m->dst, m->src, m->payload, row, rw)) t->error = 1;
      } else {
        t->st.dead_letters++;
      }
    }
  }
  return 0;
}

static uint32_t bsp_threads(void) {
  const char* e = getenv("BSP_THREADS");
  int t = e ? atoi(e) : 16;
  return t < 1 ? 1u : t > 64 ? 64u : (uint32_t)t;
}

/* One BSP superstep.  Returns 1 if any message was in flight. */
static int bsp_step(bsp_sim* s) {
  const uint64_t total = bsp_in_flight(s);
  if (total == 0) return 0;
  const uint32_t nruns = s->nseg + 1;
  const envvec** runs = (const envvec**)malloc(nruns * sizeof(envvec*));
  if (!runs) return s->P.error = 1, 1;
  for (uint32_t i = 0; i < s->nseg; ++i) runs[i] = &s->seg[i];
  runs[s->nseg] = &s->staged;
  msgview mv = {runs};
  if (!s->pos) { /* position of each actor in the canonical apply order */
    s->pos = (uint32_t*)malloc(s->n * 4);
    if (!s->pos) { free(runs); return s->P.error = 1, 1; }
    for (uint64_t i = 0; i < s->n; ++i) s->pos[s->order[i]] = (uint32_t)i;
  }
  uint64_t* perm = (uint64_t*)malloc(total * 8);
  uint64_t* abeg = (uint64_t*)malloc((total + 1) * 8);
  uint32_t* aact = (uint32_t*)malloc(total * 4);
  if (!perm || !abeg || !aact) { free(perm); free(abeg); free(aact); free(runs); s->P.error = 1; return 1; }
  uint64_t nact = 0;
  if (total * 4 >= s->n) { /* dense: counting sort over the positions */
    uint64_t* off = (uint64_t*)calloc(s->n + 1, 8);
    if (!off) { free(perm); free(abeg); free(aact); free(runs); s->P.error = 1; return 1; }
    FOR_EACH_MSG(mv, nruns, q) {
      const uint64_t* row;
      off[s->pos[mv_env(&mv, q, &row)->dst] + 1]++;
    }
    for (uint64_t i = 0; i < s->n; ++i) {
      if (off[i + 1]) {
        aact[nact] = s->order[i];
        abeg[nact++] = off[i];
      }
      off[i + 1] += off[i];
    }
    abeg[nact] = total;
    FOR_EACH_MSG(mv, nruns, q) {
      const uint64_t* row;
      perm[off[s->pos[mv_env(&mv, q, &row)->dst]]++] = q;
    }
    free(off);
  } else { /* sparse: stable LSD radix sort of (position, message id) in 11-bit digits */
    uint32_t* key = (uint32_t*)malloc(total * 4);
    uint32_t* key2 = (uint32_t*)malloc(total * 4);
    uint64_t* perm2 = (uint64_t*)malloc(total * 8);
    if (!key || !key2 || !perm2) {
      free(key); free(key2); free(perm2); free(perm); free(abeg); free(aact); free(runs);
      s->P.error = 1;
      return 1;
    }
    uint64_t o = 0;
    FOR_EACH_MSG(mv, nruns, q) {
      const uint64_t* row;
      key[o] = s->pos[mv_env(&mv, q, &row)->dst];
      perm[o++] = q;
    }
    uint32_t bits = 1;
    while (bits < 32 && (1ull << bits) < s->n) ++bits;
    for (uint32_t sh = 0; sh < bits; sh += 11) {
      uint64_t cnt[2049];
      memset(cnt, 0, sizeof cnt);
      for (uint64_t q = 0; q < total; ++q) cnt[((key[q] >> sh) & 2047u) + 1]++;
      for (int d = 0; d < 2048; ++d) cnt[d + 1] += cnt[d];
      for (uint64_t q = 0; q < total; ++q) {
        const uint64_t x = cnt[(key[q] >> sh) & 2047u]++;
        key2[x] = key[q];
        perm2[x] = perm[q];
      }
      uint32_t* tk = key; key = key2; key2 = tk;
      uint64_t* tp = perm; perm = perm2; perm2 = tp;
    }
    for (uint64_t q = 0; q < total; ++q)
      if (q == 0 || key[q] != key[q - 1]) {
        aact[nact] = s->order[key[q]];
        abeg[nact++] = q;
      }
    abeg[nact] = total;
    free(key); free(key2); free(perm2);
  }

  /* runs of active actors, balanced by messages */
  uint32_t nt = bsp_threads();
  if ((uint64_t)nt > nact) nt = (uint32_t)(nact ? nact : 1);
  if (total < 4096) nt = 1;
  bsp_part* parts = (bsp_part*)calloc(nt, sizeof(bsp_part));
  bsp_job* jobs = (bsp_job*)calloc(nt, sizeof(bsp_job));
  pthread_t* th = (pthread_t*)calloc(nt, sizeof(pthread_t));
  int* live = (int*)calloc(nt, sizeof(int));
  envvec* seg = (envvec*)calloc(2 * nt, sizeof(envvec));
  if (!parts || !jobs || !th || !live || !seg) {
    free(parts); free(jobs); free(th); free(live); free(seg); free(perm); free(abeg); free(aact); free(runs);
    s->P.error = 1;
    return 1;
  }
  uint64_t k = 0;
  for (uint32_t t = 0; t < nt; ++t) {
    parts[t].s = s;
    parts[t].P = s->P;
    ev_set_rw(&parts[t].emitted, s->rw);
    ev_set_rw(&parts[t].backlog, s->rw);
    const uint64_t goal = total * (t + 1) / nt;
    uint64_t k1 = k;
    if (t + 1 == nt) k1 = nact;
    else while (k1 < nact && abeg[k1] < goal) ++k1;
    jobs[t] = (bsp_job){s, &parts[t], &mv, perm, abeg, aact, k, k1};
    k = k1;
  }
  for (uint32_t t = 0; t < nt; ++t) {
    live[t] = t + 1 < nt && pthread_create(&th[t], 0, bsp_apply_run, &jobs[t]) == 0;
    if (!live[t]) bsp_apply_run(&jobs[t]);
  }
  for (uint32_t t = 0; t < nt; ++t)
    if (live[t]) pthread_join(th[t], 0);
  free(th); free(live); free(jobs);
  free(perm); free(abeg); free(aact); free(runs);

  /* the runs become the mail in flight, in canonical order (backlog runs, then emitted runs) */
  for (uint32_t i = 0; i < s->nseg; ++i) { free(s->seg[i].v); free(s->seg[i].rows); }
  free(s->seg);
  s->staged.n = 0;
  for (uint32_t t = 0; t < nt; ++t) {
    bsp_part* x = &parts[t];
    if (x->error || x->P.error) s->P.error = 1;
    seg[t] = x->backlog;
    seg[nt + t] = x->emitted;
    s->st.delivered += x->st.delivered;
    s->st.dead_letters += x->st.dead_letters;
    s->st.unhandled += x->st.unhandled;
    s->st.emitted += x->st.emitted;
    for (uint64_t i = 0; i < x->outbox_n; ++i) {
      if (s->outbox_since++ >= s->outbox_cap) { /* past the capacity: dropped, reported by the next take */
        s->outbox_lost++;
        continue;
      }
      uint32_t* o = (uint32_t*)realloc(s->outbox, (size_t)(s->outbox_n + 1) * 12);
      if (!o) { s->P.error = 1; break; }
      s->outbox = o;
      memcpy(o + 3 * s->outbox_n, x->outbox + 3 * i, 12);
      s->outbox_n++;
    }
    free(x->outbox);
  }
  s->seg = seg;
  s->nseg = 2 * nt;
  s->nbl = nt;
  free(parts);
  s->st.supersteps++;
  return 1;
}

int bsp_run(bsp_sim* s, uint32_t max_steps, agx_stats* out) {
  for (uint32_t i = 0; i < max_steps && !s->P.error; ++i)
    if (!bsp_step(s)) break;
  s->st.in_flight = bsp_in_flight(s);
  if (out) *out = s->st;
  return s->P.error ? AGX_ECAPACITY : 0;
}

void bsp_read_state(bsp_sim* s, uint64_t first, uint64_t count, uint64_t* words, uint8_t* alive) {
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t a = first + i;
    if (words) memcpy(&words[i * s->W], &s->state[a * s->W], s->W * 8);
    if (alive) alive[i] = s->alive[a];
  }
}

/* ------------------------------------------------ CRDT restatements (KATs) */

/* GCounter over R node slots (node index 0..R-1 in UniqueAddress order,
 * akka-cluster/.../Member.scala:303-311).  increment: slot += n
 * (DD GCounter.scala:97-111); merge: slot-wise max (GCounter.scala:113-125);
 * value: sum of slots (GCounter.scala:62-64).  BigInt there, u64 here.     */
void bsp_gcounter_increment(uint64_t* c, uint32_t slot, uint64_t n) { c[slot] += n; }
void bsp_gcounter_merge(uint64_t* out, const uint64_t* a, const uint64_t* b, uint32_t r) {
  for (uint32_t i = 0; i < r; ++i) out[i] = a[i] > b[i] ? a[i] : b[i];
}
uint64_t bsp_gcounter_value(const uint64_t* c, uint32_t r) {
  uint64_t v = 0;
  for (uint32_t i = 0; i < r; ++i) v += c[i];
  return v;
}
/* ORSet restatement on the engine layout (crdt_ref.h), for the ORSetSpec KATs. */
void bsp_orset_merge(uint64_t* self, const uint64_t* that) { orset_merge(self, that); }
void bsp_orset_add(uint64_t* w, uint32_t node, uint32_t e) { orset_add(w, node, e); }
void bsp_orset_remove(uint64_t* w, uint32_t e) { orset_remove(w, e); }
void bsp_orset_subtract_dots(uint32_t* out, const uint32_t* dot, const uint32_t* vv) { orset_subtract_dots(out, dot, vv); }
uint32_t bsp_crdt_peer(uint64_t seed, uint32_t self, uint32_t round, uint32_t j, uint64_t n) {
  return crdt_peer(seed, self, round, j, n);
}

/* PNCounter = (increments, decrements) GCounters; merge each (PNCounter.scala:178). */
void bsp_pncounter_merge(uint64_t* out_p, uint64_t* out_n, const uint64_t* ap, const uint64_t* an,
                         const uint64_t* bp, const uint64_t* bn, uint32_t r) {
  bsp_gcounter_merge(out_p, ap, bp, r);
  bsp_gcounter_merge(out_n, an, bn, r);
}

/* ORSet deltas and VersionVector (crdt_ref.h), for the ORSetSpec delta / VersionVectorSpec KATs. */
uint32_t bsp_orset_delta_bytes(void) { return (uint32_t)sizeof(orset_delta); }
void bsp_orset_add_d(uint64_t* w, orset_delta* d, uint32_t node, uint32_t e, uint32_t ver) { orset_add_d(w, d, node, e, ver); }
void bsp_orset_remove_d(uint64_t* w, orset_delta* d, uint32_t node, uint32_t e) { orset_remove_d(w, d, node, e); }
void bsp_orset_clear_d(uint64_t* w, orset_delta* d) { orset_clear_d(w, d); }
int bsp_orset_delta_merge(orset_delta* d1, const orset_delta* d2) { return orset_delta_merge(d1, d2); }
void bsp_orset_merge_delta(uint64_t* w, const orset_delta* d) { orset_merge_delta(w, d); }
uint32_t bsp_vv_compare(const uint32_t* a, const uint32_t* b) { return vv_compare(a, b); }
