// agx_tellq.h — the lock-free tell path of the C ABI (agx_tell / agx_pump_idle), host code only.
//
// ActorRef.! may be called from any thread (AbstractDispatcher contract).  The reference enqueues
// with one atomic getAndSet on an MPSC node queue (akka-actor/src/main/java/akka/dispatch/
// AbstractNodeQueue.java:79-82) and schedules the mailbox behind a CAS on its status word
// (akka-actor/src/main/scala/akka/dispatch/Mailbox.scala:185-194, Dispatcher.scala:120-128), so N
// tells to an idle mailbox submit ONE task.  Here every producer thread appends to a queue of its
// own (a chain of single-producer segments: one store of the tail per tell, to the thread's own
// line -- no contended atomic -- and each sender's tells in order), and the engine has one status
// word:
//   tell:      append, then (seq_cst) if status == idle and CAS idle -> scheduled: "submit the pump";
//   pump end:  (seq_cst) status = idle, then if any producer has untaken tells and CAS idle ->
//              scheduled: "submit the pump again" (Mailbox.run's finally: setAsIdle +
//              registerForExecution).
// The two seq_cst store -> load pairs make a lost wake-up impossible: either the producer sees the
// idle status (and schedules) or the pump sees the producer's tail (and reschedules); at most one
// of them wins the CAS.  The consumer (the one pump thread, agx_run) takes every published tell of
// every producer; a segment is freed only after its producer moved on to the next one.
#pragma once
#include <atomic>
#include <cstdint>
#include <utility>
#include <vector>

namespace agx {

struct TellSeg {
  static constexpr uint32_t kCap = 4096;
  uint32_t dst[kCap], src[kCap], pay[kCap];
  std::atomic<uint32_t> tail{0};        // published entries (producer: seq_cst store)
  uint32_t head = 0;                    // taken entries (consumer only)
  std::atomic<TellSeg*> next{nullptr};  // set by the producer when this segment is full
};

struct TellProducer {
  TellSeg* wseg;        // producer: the segment it appends to
  TellSeg* rseg;        // consumer: the oldest segment not fully taken
  TellProducer* link;   // registry (push-front, never unlinked before the queue dies)
};

class TellQueue {
 public:
  TellQueue() : id_(next_id().fetch_add(1) + 1) {}
  ~TellQueue() {
    for (TellProducer* p = producers_.load(); p;) {
      for (TellSeg* s = p->rseg; s;) {
        TellSeg* n = s->next.load();
        delete s;
        s = n;
      }
      TellProducer* n = p->link;
      delete p;
      p = n;
    }
  }
  TellQueue(const TellQueue&) = delete;
  TellQueue& operator=(const TellQueue&) = delete;

  // any thread; returns true iff the caller must submit the pump (idle -> scheduled)
  bool tell(uint32_t dst, uint32_t src, uint32_t pay) {
    TellProducer* p = mine();
    TellSeg* s = p->wseg;
    uint32_t t = s->tail.load(std::memory_order_relaxed);
    if (t == TellSeg::kCap) {
      TellSeg* n = new TellSeg;
      s->next.store(n, std::memory_order_seq_cst);  // (seq_cst: pending() must see it, as the tail below)
      p->wseg = s = n;
      t = 0;
    }
    s->dst[t] = dst;
    s->src[t] = src;
    s->pay[t] = pay;
    s->tail.store(t + 1, std::memory_order_seq_cst);
    return try_schedule();
  }

  // the pump's last call: status idle, then a re-check for tells published meanwhile
  bool pump_idle() {
    status_.store(0, std::memory_order_seq_cst);
    return pending() && try_schedule();
  }

  // consumer (the pump thread): every published tell, producer by producer, each in its order
  template <typename F>
  void take(F&& f) {
    take_while([&](uint32_t d, uint32_t s, uint32_t p) {
      f(d, s, p);
      return true;
    });
  }

  // consumer, bounded: offers published tells to f in order (per producer) and stops at the first one
  // f refuses -- that tell and everything after it stay queued for a later take (back-pressure, not
  // loss: an unbounded mailbox never refuses an enqueue, AbstractNodeQueue.java:79-82).  The next
  // take starts at the producer this one stopped at, so a refusing pump serves the producers round
  // robin instead of starving the ones at the end of the registry.  Returns false iff f refused.
  template <typename F>
  bool take_while(F&& f) {
    TellProducer* const head = producers_.load(std::memory_order_acquire);
    TellProducer* const first = resume_ ? resume_ : head;
    resume_ = nullptr;
    // first .. end of the registry, then head .. first (producers are only ever pushed at the head,
    // so `first` stays reachable and every producer is visited once)
    for (int pass = 0; pass < 2; ++pass)
      for (TellProducer* p = pass ? head : first; p && !(pass && p == first); p = p->link)
        if (!take_one(p, f)) {
          resume_ = p;
          return false;
        }
    return true;
  }

  // tells published and not taken (the pump's re-check; agx_pump_idle)
  bool pending() const {
    for (TellProducer* p = producers_.load(std::memory_order_seq_cst); p; p = p->link) {
      TellSeg* s = p->rseg;
      if (s->tail.load(std::memory_order_seq_cst) != s->head) return true;
      if (s->head == TellSeg::kCap && s->next.load(std::memory_order_seq_cst)) return true;
    }
    return false;
  }
  bool scheduled() const { return status_.load() != 0; }
  // the pump could not be submitted (the executor rejected it): back to idle WITHOUT the re-check,
  // so the next tell schedules again (Dispatcher.registerForExecution's catch: setAsIdle, rethrow,
  // Dispatcher.scala:130-138)
  void cancel_schedule() { status_.store(0, std::memory_order_seq_cst); }

 private:
  bool try_schedule() {
    uint32_t idle = 0;
    return status_.load(std::memory_order_seq_cst) == 0 &&
           status_.compare_exchange_strong(idle, 1u, std::memory_order_seq_cst);
  }
  template <typename F>
  bool take_one(TellProducer* p, F& f) {
    for (;;) {
      TellSeg* s = p->rseg;
      const uint32_t t = s->tail.load(std::memory_order_acquire);
      for (uint32_t i = s->head; i < t; ++i)
        if (!f(s->dst[i], s->src[i], s->pay[i])) {
          s->head = i;
          return false;
        }
      s->head = t;
      TellSeg* n = t == TellSeg::kCap ? s->next.load(std::memory_order_acquire) : nullptr;
      if (!n) return true;
      p->rseg = n;  // the producer has moved on: it never touches s again
      delete s;
    }
  }
  // this thread's producer for this queue (registered on its first tell)
  TellProducer* mine() {
    thread_local std::vector<std::pair<uint64_t, TellProducer*>> tl;  // (queue id: never reused)
    for (auto& x : tl)
      if (x.first == id_) return x.second;
    TellSeg* s = new TellSeg;
    TellProducer* p = new TellProducer{s, s, nullptr};
    TellProducer* h = producers_.load(std::memory_order_relaxed);
    do p->link = h;
    while (!producers_.compare_exchange_weak(h, p, std::memory_order_release, std::memory_order_relaxed));
    tl.emplace_back(id_, p);
    return p;
  }
  static std::atomic<uint64_t>& next_id() {
    static std::atomic<uint64_t> n{0};
    return n;
  }

  const uint64_t id_;
  std::atomic<TellProducer*> producers_{nullptr};
  std::atomic<uint32_t> status_{0};  // 0 idle, 1 scheduled
  TellProducer* resume_ = nullptr;    // consumer only: where the last refused take stopped
};

}  // namespace agx
