// fjp_ref.cpp — TEST INFRASTRUCTURE / CPU BASELINE ONLY.  Never linked by akka_amd/.
//
// A multi-threaded restatement of the reference's Dispatcher + Mailbox +
// ForkJoinPool hot loop ("restatement of the reference algorithm", not Akka):
//   - per-actor Vyukov MPSC node queue: add = getAndSet(head) + link,
//     poll spins while a producer is mid-publish
//     (akka-actor/src/main/java/akka/dispatch/AbstractNodeQueue.java:79-82,155-173);
//   - bounded variant: capacity check before add, overflow -> DeadLetter
//     (AbstractBoundedNodeQueue.java:92-113; Mailbox.scala:415-443);
//   - mailbox status word with a Scheduled bit set by CAS in
//     registerForExecution (Mailbox.scala:185-203, Dispatcher.scala:120-143);
//   - Mailbox.run: drain up to max(throughput,1) messages, setAsIdle, re-register
//     if messages remain (Mailbox.scala:227-277);
//   - stop: context.stop(self) closes the mailbox after the current message;
//     the rest and later tells go to deadLetters (Mailbox.scala:273,337-351);
//   - executor: a lock-free work-stealing pool like the JDK ForkJoinPool that
//     AkkaForkJoinPool extends (ForkJoinExecutorConfigurator.scala:16-37), one
//     worker per host thread, in asyncMode (FIFO): each worker owns a Chase-Lev
//     deque (owner pushes at the bottom; the owner and the thieves take from the
//     top with a CAS, so local tasks run in submission order, as asyncMode = true
//     makes the JDK WorkQueue poll FIFO).  Growable circular arrays (Chase & Lev,
//     SPAA'05; C11 orderings after Lê et al., PPoPP'13).  No locks anywhere on the
//     per-message path.
//   - quiescence (the JMH harness waits on a latch instead): per-worker sent /
//     processed counters on their own cache lines, and Mattern's four-counter
//     wave test when a worker finds no work -- no shared counter per message.
// Behaviours: the shared table in behaviors_ref.h (CRDT state gossips carry a
// heap copy of the sender's state, like the immutable ddata value objects).
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "behaviors_ref.h"

namespace {

struct Node {
  std::atomic<Node*> next{nullptr};
  uint32_t src = 0, payload = 0;
  uint64_t* row = nullptr;  // CRDT state gossip snapshot (owned by the message)
};

// Vyukov non-intrusive MPSC queue with a stub node (AbstractNodeQueue).
struct MpscQueue {
  std::atomic<Node*> head;  // producers swap here
  Node* tail;               // consumer side
  Node stub;
  MpscQueue() {
    head.store(&stub, std::memory_order_relaxed);
    tail = &stub;
  }
  void add(Node* n) {
    n->next.store(nullptr, std::memory_order_relaxed);
    Node* prev = head.exchange(n, std::memory_order_acq_rel);  // getAndSet (AbstractNodeQueue.java:79-82)
    prev->next.store(n, std::memory_order_release);
  }
  // returns a node whose (src,payload,row) is the dequeued value; the node handed
  // back is the old tail (value moved into it), to be recycled by the caller.
  Node* poll() {
    Node* t = tail;
    Node* next = t->next.load(std::memory_order_acquire);
    if (!next) {
      if (head.load(std::memory_order_acquire) == t) return nullptr;
      // producer mid-publish: spin until visible (AbstractNodeQueue.java:158-164)
      while (!(next = t->next.load(std::memory_order_acquire))) std::this_thread::yield();
    }
    tail = next;
    t->src = next->src;
    t->payload = next->payload;
    t->row = next->row;
    next->row = nullptr;
    return t;  // t is free (unless it is the stub)
  }
};

enum : uint32_t { kScheduled = 1u, kClosed = 2u };

struct alignas(64) Actor {
  MpscQueue q;
  std::atomic<uint32_t> status{0};
  std::atomic<int64_t> size{0};
  uint32_t kind = 0;
};

// ---------------------------------------------------------------- Chase-Lev deque
struct TaskArray {
  int64_t cap;  // power of two
  std::atomic<uint32_t>* buf;
  explicit TaskArray(int64_t c) : cap(c), buf(new std::atomic<uint32_t>[c]) {}
  ~TaskArray() { delete[] buf; }
  uint32_t get(int64_t i) const { return buf[i & (cap - 1)].load(std::memory_order_relaxed); }
  void put(int64_t i, uint32_t v) { buf[i & (cap - 1)].store(v, std::memory_order_relaxed); }
};

struct alignas(64) Deque {
  alignas(64) std::atomic<int64_t> top{0};
  alignas(64) std::atomic<int64_t> bottom{0};
  std::atomic<TaskArray*> arr;
  std::vector<TaskArray*> retired;  // old arrays stay valid until the pool is torn down
  Deque() : arr(new TaskArray(1024)) {}
  ~Deque() {
    delete arr.load();
    for (auto* a : retired) delete a;
  }
  // owner only
  void push(uint32_t v) {
    const int64_t b = bottom.load(std::memory_order_relaxed);
    const int64_t t = top.load(std::memory_order_acquire);
    TaskArray* a = arr.load(std::memory_order_relaxed);
    if (b - t > a->cap - 1) {  // grow: copy the live range into a twice larger array
      TaskArray* na = new TaskArray(a->cap * 2);
      for (int64_t i = t; i < b; ++i) na->put(i, a->get(i));
      retired.push_back(a);
      arr.store(na, std::memory_order_release);
      a = na;
    }
    a->put(b, v);
    bottom.store(b + 1, std::memory_order_release);  // publishes the task (a release store, not a
                                                     // standalone fence: ThreadSanitizer models it)
  }
  // owner (FIFO, asyncMode) and thieves: take the oldest task.  0 = empty, 1 = got one, 2 = lost a race
  int take(uint32_t* out) {
    int64_t t = top.load(std::memory_order_acquire);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const int64_t b = bottom.load(std::memory_order_acquire);
    if (t >= b) return 0;
    TaskArray* a = arr.load(std::memory_order_acquire);
    const uint32_t v = a->get(t);
    if (!top.compare_exchange_strong(t, t + 1, std::memory_order_seq_cst, std::memory_order_relaxed)) return 2;
    *out = v;
    return 1;
  }
  bool empty() const {
    return top.load(std::memory_order_acquire) >= bottom.load(std::memory_order_acquire);
  }
};

struct alignas(64) Worker {
  Deque dq;
  std::vector<Node*> free_nodes;
  // termination counters (written by this worker only; read by the wave test)
  alignas(64) std::atomic<uint64_t> sent{0};       // messages this worker enqueued (or dead-lettered at send)
  std::atomic<uint64_t> processed{0};              // messages this worker dequeued (invoked or dead-lettered)
  uint64_t delivered = 0, dead = 0, unhandled = 0, emitted = 0;
  uint64_t rng = 0;
};

struct Pool {
  uint32_t nthreads = 1;
  std::vector<Worker*> workers;
  std::atomic<bool> done{false};
  uint64_t ext_sent = 0;  // tells staged by the calling thread before the workers start
};

struct Sim {
  ref_params P{};
  uint32_t T = 1, C = 0, W = 1, rw = 0;
  uint64_t n = 0;
  std::vector<Actor> actors;
  std::vector<uint64_t> state;  // actor-major
  std::vector<uint32_t> zipf_cdf, zipf_perm, col;
  std::vector<uint64_t> row_ptr;
  std::vector<agx_case> bcase;  // compiled behaviours
  std::vector<agx_act> bact;
  std::vector<uint32_t> bfirst;
  Pool pool;
  std::vector<uint32_t> st_dst, st_src, st_pay;  // staged tells
  agx_stats st{};
};

thread_local Worker* tl_worker = nullptr;

inline void bump(std::atomic<uint64_t>& c) {  // single writer: no read-modify-write on the hot path
  c.store(c.load(std::memory_order_relaxed) + 1, std::memory_order_release);
}

Node* alloc_node(Worker* w) {
  if (w && !w->free_nodes.empty()) {
    Node* n = w->free_nodes.back();
    w->free_nodes.pop_back();
    return n;
  }
  return new Node();
}

void schedule(Sim* s, uint32_t a) {
  Worker* w = tl_worker;
  // outside the pool (the staging thread, before the workers start): the deque of the worker whose
  // contiguous id range holds the actor.  (Round-robin homes, a % threads, put neighbouring actors --
  // a ring's sender and receiver -- on different workers, so every hand-off moved the receiver's
  // mailbox line between cores: 1M ring 1.7e7 msg/s on 1 thread, 2.8e7 on 8; contiguous homes
  // 1.65e7 / 6.6e7.  Either is a legal initial placement: the JDK pool takes external submissions
  // through its submission queues and spreads them by stealing.)
  if (!w) w = s->pool.workers[(uint32_t)((uint64_t)a * s->pool.nthreads / s->n)];
  w->dq.push(a);
}

// Dispatcher.registerForExecution: CAS the Scheduled bit, then execute(mbox)
void register_for_execution(Sim* s, uint32_t a) {
  Actor& ac = s->actors[a];
  uint32_t cur = ac.status.load(std::memory_order_acquire);
  while (true) {
    if (cur & kScheduled) return;
    if (ac.size.load(std::memory_order_acquire) <= 0) return;
    if (ac.status.compare_exchange_weak(cur, cur | kScheduled, std::memory_order_acq_rel)) break;
  }
  schedule(s, a);
}

// tell: Dispatcher.dispatch -> Mailbox.enqueue -> registerForExecution
void tell(Sim* s, uint32_t dst, uint32_t src, uint32_t payload, const uint64_t* row, Worker* w) {
  if (dst >= s->n) {
    if (w) w->dead++;
    else s->st.dead_letters++;
    return;
  }
  Actor& ac = s->actors[dst];
  if (s->C) {
    int64_t prev = ac.size.fetch_add(1, std::memory_order_acq_rel);
    if (prev >= (int64_t)s->C) {  // bounded overflow -> DeadLetter
      ac.size.fetch_sub(1, std::memory_order_acq_rel);
      if (w) w->dead++;
      else s->st.dead_letters++;
      return;
    }
  } else {
    ac.size.fetch_add(1, std::memory_order_acq_rel);
  }
  if (w) bump(w->sent);
  else s->pool.ext_sent++;
  Node* n = alloc_node(w);
  n->src = row ? (src | AGX_WIDE_BIT) : src;
  n->payload = payload;
  n->row = nullptr;
  if (row) {  // the gossip carries its own immutable copy of the sender's state
    n->row = (uint64_t*)malloc((size_t)s->rw * 8);
    memcpy(n->row, row, (size_t)s->rw * 8);
  }
  ac.q.add(n);
  register_for_execution(s, dst);
}

struct EmitCtx {
  Sim* s;
  Worker* w;
};
void emit_cb(void* ctx, uint32_t dst, uint32_t self, uint32_t payload, const uint64_t* row, uint32_t) {
  EmitCtx* c = (EmitCtx*)ctx;
  c->w->emitted++;
  tell(c->s, dst, self, payload, row, c->w);
}

// Mailbox.run -> processMailbox(left = max(throughput, 1))
void run_mailbox(Sim* s, uint32_t a, Worker* w) {
  Actor& ac = s->actors[a];
  EmitCtx ctx{s, w};
  for (uint32_t left = s->T; left > 0; --left) {
    Node* n = ac.q.poll();
    if (!n) break;
    const uint32_t src = n->src, pay = n->payload;
    uint64_t* row = n->row;
    n->row = nullptr;
    if (n != &ac.q.stub) w->free_nodes.push_back(n);
    ac.size.fetch_sub(1, std::memory_order_acq_rel);
    if (ac.status.load(std::memory_order_acquire) & kClosed) {
      w->dead++;  // cleanUp -> deadLetters
    } else {
      uint32_t r = ref_apply(&s->P, &ac.kind, a, &s->state[(uint64_t)a * s->W], src, pay, row, emit_cb, &ctx);
      w->delivered++;
      if (r == AGX_RES_UNHANDLED) w->unhandled++;
      if (r == AGX_RES_STOPPED) ac.status.fetch_or(kClosed, std::memory_order_acq_rel);
    }
    free(row);
    bump(w->processed);  // after the children's sends were counted (the wave test relies on it)
    if (ac.status.load(std::memory_order_acquire) & kClosed) left = 0xFFFFFFFFu;  // closed: drain all to dead
  }
  ac.status.fetch_and(~kScheduled, std::memory_order_acq_rel);  // setAsIdle
  register_for_execution(s, a);
}

bool take(Sim* s, Worker* self, uint32_t idx, uint32_t* out) {
  for (;;) {
    int r = self->dq.take(out);
    if (r == 1) return true;
    if (r == 0) break;
  }
  const uint32_t nw = s->pool.nthreads;
  if (nw == 1) return false;
  // steal sweep from a random victim (FJP scans from a random index)
  self->rng = self->rng * 6364136223846793005ull + 1442695040888963407ull;
  const uint32_t start = (uint32_t)(self->rng >> 33) % nw;
  for (uint32_t k = 0; k < nw; ++k) {
    const uint32_t v = (start + k) % nw;
    if (v == idx) continue;
    for (int tries = 0; tries < 4; ++tries) {
      int r = s->pool.workers[v]->dq.take(out);
      if (r == 1) return true;
      if (r == 0) break;
    }
  }
  return false;
}

// Mattern's four-counter test: two waves over the per-worker counters; terminated iff the
// processed total of the first wave equals the sent total of the second (and no deque holds
// a task).  Counters are monotonic; a message's children are counted as sent before the
// message is counted as processed.
bool quiescent(Sim* s) {
  auto wave = [&](uint64_t* sent, uint64_t* proc) {
    uint64_t p = 0, q = s->pool.ext_sent;
    for (Worker* w : s->pool.workers) p += w->processed.load(std::memory_order_acquire);
    for (Worker* w : s->pool.workers) q += w->sent.load(std::memory_order_acquire);
    *sent = q;
    *proc = p;
  };
  for (Worker* w : s->pool.workers)
    if (!w->dq.empty()) return false;
  uint64_t s1, p1, s2, p2;
  wave(&s1, &p1);
  if (s1 != p1) return false;
  wave(&s2, &p2);
  return p1 == s2;
}

void worker_main(Sim* s, uint32_t idx) {
  Worker* w = s->pool.workers[idx];
  tl_worker = w;
  w->rng = 0x9E3779B97F4A7C15ull * (idx + 1);
  uint32_t a;
  uint32_t idle = 0;
  while (!s->pool.done.load(std::memory_order_acquire)) {
    if (take(s, w, idx, &a)) {
      idle = 0;
      run_mailbox(s, a, w);
    } else {
      if (quiescent(s)) {
        s->pool.done.store(true, std::memory_order_release);
        break;
      }
      if (++idle > 64) std::this_thread::yield();
    }
  }
  tl_worker = nullptr;
}

void free_pool(Sim* s) {
  for (auto* w : s->pool.workers) {
    for (Node* n : w->free_nodes) delete n;
    delete w;
  }
  s->pool.workers.clear();
}

}  // namespace

extern "C" {

void* fjp_create(uint64_t n_actors, uint32_t throughput, uint32_t capacity, uint32_t n_words) {
  if (!n_actors || !n_words || n_words > AGX_MAX_WORDS) return nullptr;
  Sim* s = new Sim();
  s->n = n_actors;
  s->T = (throughput == 0 || (int32_t)throughput < 0) ? 1u : throughput;
  s->C = capacity;
  if (s->C && s->T > s->C) s->T = s->C;  // as the engine / bsp_ref: drain <= min(T, C)
  s->W = n_words;
  s->actors = std::vector<Actor>(n_actors);
  s->state.assign(n_actors * n_words, 0);
  s->P.n = n_actors;
  s->P.W = n_words;
  s->P.ring_stride = 1;
  return s;
}

void fjp_destroy(void* h) {
  Sim* s = (Sim*)h;
  if (!s) return;
  // messages still queued (a run that was not taken to quiescence) own their rows
  for (auto& ac : s->actors)
    while (Node* n = ac.q.poll()) {
      free(n->row);
      if (n != &ac.q.stub) delete n;
    }
  free_pool(s);
  delete s;
}

int fjp_register_range(void* h, uint64_t first, uint64_t count, uint32_t kind, const uint64_t* init,
                       uint64_t stride_words) {
  Sim* s = (Sim*)h;
  const bool compiled = kind >= AGX_KIND_COMPILED && kind < AGX_KIND_COMPILED + AGX_MAX_BEHAVIORS;
  if (first + count > s->n || (kind >= AGX_KIND_MAX && !compiled)) return 1;
  const uint32_t rw = ref_crdt_words(kind);
  if (rw) {
    if (s->W < rw) return 1;
    if (rw > s->rw) s->rw = rw;
  }
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t a = first + i;
    s->actors[a].kind = kind;
    s->actors[a].status.store(kind == AGX_KIND_NONE ? kClosed : 0u);
    for (uint32_t w = 0; w < s->W; ++w) s->state[a * s->W + w] = init ? init[i * stride_words + w] : 0;
  }
  return 0;
}

void fjp_set_ring(void* h, uint32_t stride) { ((Sim*)h)->P.ring_stride = stride; }

void fjp_set_gossip(void* h, uint32_t fanout, uint64_t seed) {
  Sim* s = (Sim*)h;
  s->P.gossip_f = fanout;
  s->P.gossip_seed = seed;
}

// compiled behaviour tables (see bsp_set_behaviors)
int fjp_set_behaviors(void* h, const agx_case* cases, uint32_t n_cases, const agx_act* acts, uint32_t n_acts,
                      const uint32_t* first, uint32_t n_beh) {
  Sim* s = (Sim*)h;
  s->bcase.assign(cases, cases + n_cases);
  s->bact.assign(acts, acts + n_acts);
  s->bfirst.assign(first, first + n_beh + 1);
  s->P.bcase = s->bcase.data();
  s->P.bact = s->bact.data();
  s->P.bfirst = s->bfirst.data();
  s->P.n_beh = n_beh;
  return 0;
}

// delta-crdt.enabled / max-delta-size (see bsp_set_delta_crdt)
int fjp_set_delta_crdt(void* h, uint32_t max_delta_size) {
  Sim* s = (Sim*)h;
  if (max_delta_size > AGX_DELTA_MAX_SIZE) return 1;
  s->P.delta_max = max_delta_size;
  for (uint64_t a = 0; a < s->P.n; ++a) {
    const uint32_t r = ref_row_words(s->actors[a].kind, max_delta_size);
    if (r > s->rw) s->rw = r;
  }
  return 0;
}

void fjp_set_fanout(void* h, uint32_t k, uint64_t seed, const uint32_t* cdf, const uint32_t* perm, uint64_t n) {
  Sim* s = (Sim*)h;
  s->zipf_cdf.assign(cdf, cdf + n);
  s->zipf_perm.assign(perm, perm + n);
  s->P.fan_k = k;
  s->P.fan_seed = seed;
  s->P.zipf_cdf = s->zipf_cdf.data();
  s->P.zipf_perm = s->zipf_perm.data();
  s->P.zipf_n = n;
}

void fjp_set_graph(void* h, const uint64_t* row_ptr, const uint32_t* col) {
  Sim* s = (Sim*)h;
  s->row_ptr.assign(row_ptr, row_ptr + s->n + 1);
  s->col.assign(col, col + row_ptr[s->n]);
  s->P.row_ptr = s->row_ptr.data();
  s->P.col = s->col.data();
}

void fjp_stage(void* h, const uint32_t* dst, const uint32_t* src, const uint32_t* payload, uint64_t n) {
  Sim* s = (Sim*)h;
  for (uint64_t i = 0; i < n; ++i) {
    s->st_dst.push_back(dst[i]);
    s->st_src.push_back(src ? src[i] : AGX_NO_SENDER);
    s->st_pay.push_back(payload[i]);
  }
}

// Runs until quiescent on `threads` workers; returns wall seconds of the run
// (the staged tells are enqueued by the calling thread inside the timed region,
// like the JMH benchmark's initial tells).
double fjp_run(void* h, uint32_t threads, agx_stats* out) {
  Sim* s = (Sim*)h;
  if (threads == 0) threads = 1;
  free_pool(s);
  s->pool.nthreads = threads;
  for (uint32_t i = 0; i < threads; ++i) s->pool.workers.push_back(new Worker());
  s->pool.done.store(false);
  s->pool.ext_sent = 0;
  auto t0 = std::chrono::steady_clock::now();
  // the calling thread is "outside the pool" (tl_worker == nullptr): it schedules into the
  // actors' home deques before the workers start (thread creation publishes them)
  for (size_t i = 0; i < s->st_dst.size(); ++i) {
    s->st.staged++;
    tell(s, s->st_dst[i], s->st_src[i], s->st_pay[i], nullptr, nullptr);
  }
  s->st_dst.clear();
  s->st_src.clear();
  s->st_pay.clear();
  std::vector<std::thread> th;
  for (uint32_t i = 0; i < threads; ++i) th.emplace_back(worker_main, s, i);
  for (auto& t : th) t.join();
  auto t1 = std::chrono::steady_clock::now();
  uint64_t sent = s->pool.ext_sent, proc = 0;
  for (auto* w : s->pool.workers) {
    s->st.delivered += w->delivered;
    s->st.dead_letters += w->dead;
    s->st.unhandled += w->unhandled;
    s->st.emitted += w->emitted;
    sent += w->sent.load();
    proc += w->processed.load();
  }
  s->st.in_flight = sent - proc;
  if (out) *out = s->st;
  return std::chrono::duration<double>(t1 - t0).count();
}

void fjp_read_state(void* h, uint64_t first, uint64_t count, uint64_t* words, uint8_t* alive) {
  Sim* s = (Sim*)h;
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t a = first + i;
    if (words) memcpy(&words[i * s->W], &s->state[a * s->W], s->W * 8);
    if (alive) alive[i] = (s->actors[a].kind != AGX_KIND_NONE) && !(s->actors[a].status.load() & kClosed);
  }
}

}  // extern "C"
