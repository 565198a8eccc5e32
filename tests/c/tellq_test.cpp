// CPU test of the lock-free tell path (akka_amd/csrc/agx_tellq.h; test infrastructure).
//   1. a burst of tells to an idle engine asks for exactly ONE pump submission
//      (Mailbox.setAsScheduled, akka-actor/.../dispatch/Mailbox.scala:185-194);
//   2. K producer threads against a pump thread that submits itself again only when
//      pump_idle() says so: every tell is taken exactly once, each producer's tells in order, and
//      no wake-up is lost (the pump drains everything after the producers stop);
//   3. segment hand-off (more than one 4096-tell segment per producer) under concurrency.
// Exit 0 = pass; prints one line per check.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../akka_amd/csrc/agx_tellq.h"

#define CHECK(c, ...)                 \
  do {                                \
    if (!(c)) {                       \
      std::printf("FAIL: " __VA_ARGS__); \
      std::printf("\n");              \
      std::exit(1);                   \
    }                                 \
  } while (0)

int main() {
  {  // 1. one burst, one submission; the pump takes it all and goes idle
    agx::TellQueue q;
    int sub = 0;
    for (uint32_t i = 0; i < 100000; ++i) sub += q.tell(i, 7, i) ? 1 : 0;
    CHECK(sub == 1, "burst: %d pump submissions for 100000 tells to an idle engine (want 1)", sub);
    uint64_t n = 0, bad = 0;
    q.take([&](uint32_t d, uint32_t s, uint32_t p) {
      bad += (d != n || s != 7 || p != n);
      ++n;
    });
    CHECK(n == 100000 && bad == 0, "burst: took %llu (bad %llu)", (unsigned long long)n, (unsigned long long)bad);
    CHECK(!q.pump_idle(), "burst: nothing pending, yet pump_idle asked for another run");
    CHECK(q.tell(1, 2, 3), "idle again: the next tell must ask for a submission");
    std::printf("burst: one submission per burst OK\n");
  }
  {  // 2 + 3. K producers, one pump (the executor is a counter of submissions)
    constexpr int K = 8;
    constexpr uint32_t M = 200000;  // ~49 segments per producer
    agx::TellQueue q;
    std::atomic<uint64_t> submitted{0};
    std::atomic<bool> done{false};
    std::vector<uint32_t> last(K, 0);
    std::vector<uint64_t> got(K, 0);
    uint64_t bad = 0, runs = 0;
    std::thread pump([&] {
      uint64_t ran = 0;
      auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        if (submitted.load() == ran) {  // not scheduled: wait for a submission
          if (done.load() && submitted.load() == ran) break;
          std::this_thread::yield();
          if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) break;
          continue;
        }
        ++ran;  // one pump run: take everything published, then the idle protocol
        ++runs;
        q.take([&](uint32_t d, uint32_t s, uint32_t p) {
          const uint32_t k = s, seq = p;
          if (k >= (uint32_t)K || seq != last[k] + 1 || d != (k << 24 | seq)) ++bad;
          last[k < (uint32_t)K ? k : 0] = seq;
          ++got[k < (uint32_t)K ? k : 0];
        });
        if (q.pump_idle()) submitted.fetch_add(1);
      }
    });
    std::vector<std::thread> prod;
    for (int k = 0; k < K; ++k)
      prod.emplace_back([&, k] {
        for (uint32_t i = 1; i <= M; ++i)
          if (q.tell((uint32_t)k << 24 | i, (uint32_t)k, i)) submitted.fetch_add(1);
      });
    for (auto& t : prod) t.join();
    done.store(true);
    pump.join();
    uint64_t total = 0;
    for (int k = 0; k < K; ++k) total += got[k];
    CHECK(bad == 0, "stress: %llu tells out of order or corrupted", (unsigned long long)bad);
    CHECK(total == (uint64_t)K * M, "stress: took %llu of %llu tells (a lost wake-up leaves tells behind)",
          (unsigned long long)total, (unsigned long long)K * M);
    CHECK(!q.pending() && !q.scheduled(), "stress: tells pending or still scheduled after the last run");
    std::printf("stress: %d producers x %u tells, %llu pump runs, FIFO per producer, none lost OK\n", K, M,
                (unsigned long long)runs);
  }
  {  // 4. bounded takes (the pump takes only what fits msg_capacity): nothing lost or reordered, the
     //    refused tell stays queued, and successive takes resume where the last one stopped
    agx::TellQueue q;
    constexpr int K = 3;
    constexpr uint32_t M = 10000;  // 3 segments per producer
    std::vector<std::thread> prod;
    for (int k = 0; k < K; ++k)
      prod.emplace_back([&, k] {
        for (uint32_t i = 1; i <= M; ++i) q.tell((uint32_t)k, (uint32_t)k, i);
      });
    for (auto& t : prod) t.join();
    std::vector<uint32_t> last(K, 0);
    uint64_t total = 0, bad = 0, takes = 0;
    std::vector<int> first_of_take;
    for (;;) {
      uint32_t room = 777;
      int first = -1;
      const bool all = q.take_while([&](uint32_t d, uint32_t s, uint32_t p) {
        if (!room) return false;
        --room;
        if (first < 0) first = (int)s;
        if (d != s || s >= (uint32_t)K || p != last[s] + 1) ++bad;
        if (s < (uint32_t)K) last[s] = p;
        ++total;
        return true;
      });
      ++takes;
      first_of_take.push_back(first);
      CHECK(all == !q.pending(), "bounded: take_while's answer disagrees with pending()");
      if (all) break;
      CHECK(takes < 1000, "bounded: no progress");
    }
    CHECK(bad == 0 && total == (uint64_t)K * M, "bounded: took %llu of %llu (bad %llu)", (unsigned long long)total,
          (unsigned long long)K * M, (unsigned long long)bad);
    // a take that stopped inside producer p's tells starts the next take at p
    CHECK(takes == (K * M + 776) / 777, "bounded: %llu takes", (unsigned long long)takes);
    std::printf("bounded: %llu takes of <= 777, FIFO per producer, none lost OK\n", (unsigned long long)takes);
  }
  return 0;
}
