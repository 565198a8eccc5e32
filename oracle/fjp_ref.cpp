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
//   - executor: a work-stealing pool, one worker per host core, FIFO local
//     queues (asyncMode), like AkkaForkJoinPool (ForkJoinExecutorConfigurator.scala:16-37).
// Behaviours: the shared table in behaviors_ref.h.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "behaviors_ref.h"

namespace {

struct Node {
  std::atomic<Node*> next{nullptr};
  uint32_t src = 0, payload = 0;
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
  // returns a node whose (src,payload) is the dequeued value; the node handed
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
    return t;  // t is free (unless it is the stub)
  }
};

enum : uint32_t { kScheduled = 1u, kClosed = 2u };

struct Actor {
  MpscQueue q;
  std::atomic<uint32_t> status{0};
  std::atomic<int64_t> size{0};
  uint32_t kind = 0;
};

struct Worker;

struct Pool {
  uint32_t nthreads = 1;
  std::vector<Worker*> workers;
  std::mutex ext_mu;
  std::deque<uint32_t> ext;  // external submission queue
  std::atomic<int64_t> inflight{0};
  std::atomic<bool> done{false};
};

struct Worker {
  std::mutex mu;
  std::deque<uint32_t> dq;  // FIFO (asyncMode)
  std::vector<Node*> free_nodes;
  uint64_t delivered = 0, dead = 0, unhandled = 0, emitted = 0;
};

struct Sim {
  ref_params P{};
  uint32_t T = 1, C = 0, W = 1;
  uint64_t n = 0;
  std::vector<Actor> actors;
  std::vector<uint64_t> state;  // actor-major
  std::vector<uint32_t> zipf_cdf, zipf_perm, col;
  std::vector<uint64_t> row_ptr;
  Pool pool;
  std::vector<uint32_t> st_dst, st_src, st_pay;  // staged tells
  agx_stats st{};
};

thread_local Worker* tl_worker = nullptr;

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
  if (w) {
    std::lock_guard<std::mutex> g(w->mu);
    w->dq.push_back(a);
  } else {
    std::lock_guard<std::mutex> g(s->pool.ext_mu);
    s->pool.ext.push_back(a);
  }
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
void tell(Sim* s, uint32_t dst, uint32_t src, uint32_t payload, Worker* w) {
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
  s->pool.inflight.fetch_add(1, std::memory_order_acq_rel);
  Node* n = alloc_node(w);
  n->src = src;
  n->payload = payload;
  ac.q.add(n);
  register_for_execution(s, dst);
}

struct EmitCtx {
  Sim* s;
  Worker* w;
};
void emit_cb(void* ctx, uint32_t dst, uint32_t self, uint32_t payload, const uint64_t*, uint32_t) {
  EmitCtx* c = (EmitCtx*)ctx;
  c->w->emitted++;
  tell(c->s, dst, self, payload, c->w);
}

// Mailbox.run -> processMailbox(left = max(throughput, 1))
void run_mailbox(Sim* s, uint32_t a, Worker* w) {
  Actor& ac = s->actors[a];
  EmitCtx ctx{s, w};
  for (uint32_t left = s->T; left > 0; --left) {
    Node* n = ac.q.poll();
    if (!n) break;
    uint32_t src = n->src, pay = n->payload;
    if (n != &ac.q.stub) w->free_nodes.push_back(n);
    ac.size.fetch_sub(1, std::memory_order_acq_rel);
    if (ac.status.load(std::memory_order_acquire) & kClosed) {
      w->dead++;  // cleanUp -> deadLetters
    } else {
      uint32_t r = ref_apply(&s->P, ac.kind, a, &s->state[(uint64_t)a * s->W], src, pay, nullptr, emit_cb, &ctx);
      w->delivered++;
      if (r == AGX_RES_UNHANDLED) w->unhandled++;
      if (r == AGX_RES_STOPPED) ac.status.fetch_or(kClosed, std::memory_order_acq_rel);
    }
    s->pool.inflight.fetch_sub(1, std::memory_order_acq_rel);
    if (ac.status.load(std::memory_order_acquire) & kClosed) left = 0xFFFFFFFFu;  // closed: drain all to dead
  }
  ac.status.fetch_and(~kScheduled, std::memory_order_acq_rel);  // setAsIdle
  register_for_execution(s, a);
}

bool take(Sim* s, Worker* self, uint32_t idx, uint32_t* out) {
  {
    std::lock_guard<std::mutex> g(self->mu);
    if (!self->dq.empty()) {
      *out = self->dq.front();
      self->dq.pop_front();
      return true;
    }
  }
  {
    std::lock_guard<std::mutex> g(s->pool.ext_mu);
    if (!s->pool.ext.empty()) {
      *out = s->pool.ext.front();
      s->pool.ext.pop_front();
      return true;
    }
  }
  uint32_t nw = s->pool.nthreads;
  for (uint32_t k = 1; k < nw; ++k) {  // steal
    Worker* v = s->pool.workers[(idx + k) % nw];
    std::unique_lock<std::mutex> g(v->mu, std::try_to_lock);
    if (g.owns_lock() && !v->dq.empty()) {
      *out = v->dq.front();
      v->dq.pop_front();
      return true;
    }
  }
  return false;
}

void worker_main(Sim* s, uint32_t idx) {
  Worker* w = s->pool.workers[idx];
  tl_worker = w;
  uint32_t a;
  uint32_t idle = 0;
  while (!s->pool.done.load(std::memory_order_acquire)) {
    if (take(s, w, idx, &a)) {
      idle = 0;
      run_mailbox(s, a, w);
    } else {
      if (s->pool.inflight.load(std::memory_order_acquire) == 0) {
        s->pool.done.store(true, std::memory_order_release);
        break;
      }
      if (++idle > 64) std::this_thread::yield();
    }
  }
  tl_worker = nullptr;
}

}  // namespace

extern "C" {

void* fjp_create(uint64_t n_actors, uint32_t throughput, uint32_t capacity, uint32_t n_words) {
  if (!n_actors || !n_words || n_words > AGX_MAX_WORDS) return nullptr;
  Sim* s = new Sim();
  s->n = n_actors;
  s->T = (throughput == 0 || (int32_t)throughput < 0) ? 1u : throughput;
  s->C = capacity;
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
  for (auto* w : s->pool.workers) {
    for (Node* n : w->free_nodes) delete n;
    delete w;
  }
  delete s;
}

int fjp_register_range(void* h, uint64_t first, uint64_t count, uint32_t kind, const uint64_t* init,
                       uint64_t stride_words) {
  Sim* s = (Sim*)h;
  if (first + count > s->n || kind >= AGX_KIND_MAX) return 1;
  if (ref_crdt_words(kind)) return 1; /* CRDT replicas are checked by the BSP oracle only */
  for (uint64_t i = 0; i < count; ++i) {
    uint64_t a = first + i;
    s->actors[a].kind = kind;
    s->actors[a].status.store(kind == AGX_KIND_NONE ? kClosed : 0u);
    for (uint32_t w = 0; w < s->W; ++w) s->state[a * s->W + w] = init ? init[i * stride_words + w] : 0;
  }
  return 0;
}

void fjp_set_ring(void* h, uint32_t stride) { ((Sim*)h)->P.ring_stride = stride; }

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
  for (auto* w : s->pool.workers) delete w;
  s->pool.workers.clear();
  s->pool.nthreads = threads;
  for (uint32_t i = 0; i < threads; ++i) s->pool.workers.push_back(new Worker());
  s->pool.done.store(false);
  auto t0 = std::chrono::steady_clock::now();
  // the calling thread is "outside the pool" (tl_worker == nullptr): its tells go to the submission queue
  s->pool.inflight.fetch_add(1);  // hold the pool open while staging
  for (size_t i = 0; i < s->st_dst.size(); ++i) {
    s->st.staged++;
    tell(s, s->st_dst[i], s->st_src[i], s->st_pay[i], nullptr);
  }
  s->st_dst.clear();
  s->st_src.clear();
  s->st_pay.clear();
  std::vector<std::thread> th;
  for (uint32_t i = 0; i < threads; ++i) th.emplace_back(worker_main, s, i);
  s->pool.inflight.fetch_sub(1);
  for (auto& t : th) t.join();
  auto t1 = std::chrono::steady_clock::now();
  for (auto* w : s->pool.workers) {
    s->st.delivered += w->delivered;
    s->st.dead_letters += w->dead;
    s->st.unhandled += w->unhandled;
    s->st.emitted += w->emitted;
    w->delivered = w->dead = w->unhandled = w->emitted = 0;
  }
  s->st.in_flight = (uint64_t)s->pool.inflight.load();
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
