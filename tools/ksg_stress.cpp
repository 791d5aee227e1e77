// ksg_stress.cpp — concurrency driver of libksgather (include/ksgather.h) for
// the sanitizer builds (make -C k8s-1m_amd sanitize): built with the library's
// source under -fsanitize=thread and under -fsanitize=address,undefined.
//
// Phase 1: blocking recorders (ksg_record_and_wait), asynchronous recorders
//   (ksg_record) and one ksg_next_fired driver run against each other on
//   overlapping keys, with fires by member count and by deadline; every
//   recorder's answer is checked against the evaluation's reported winner.
// Phase 2: ksg_shutdown while all of them are running: every call after it
//   returns -1 (next_fired drains what fired before), the threads finish, then
//   ksg_close frees the evaluator.
// Phase 3: recorders parked inside ksg_record_and_wait when ksg_close starts
//   (no call starts after it): close fires their pods, waits for them to
//   leave, frees.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "ksgather.h"

static std::atomic<int> failures{0};
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      failures++;                                                    \
    }                                                                \
  } while (0)

int main() {
  using namespace std::chrono_literals;
  // ---- phases 1 + 2
  {
    ksg_evaluator *ev = ksg_open(3, 20, KSG_TIE_LOWEST_NAME, 7);
    CHECK(ev != nullptr);
    std::atomic<bool> shut{false};
    std::atomic<long> blocking_calls{0}, async_calls{0}, fired_reports{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 6; ++t)
      th.emplace_back([&, t] {
        std::mt19937 r(t);
        char win[64];
        int32_t ws = 0;
        for (int i = 0;; ++i) {
          const std::string key = "ns/p" + std::to_string(r() % 50);
          const std::string node = "n" + std::to_string(t);
          const int32_t sc = (int32_t)(r() % 5);
          const int32_t rc = ksg_record_and_wait(ev, key.c_str(), node.c_str(), sc, win, sizeof win, &ws);
          if (rc < 0) {
            CHECK(shut.load());
            return;
          }
          blocking_calls++;
          CHECK(rc == (std::strcmp(win, node.c_str()) == 0 ? 1 : 0));
        }
      });
    for (int t = 0; t < 3; ++t)
      th.emplace_back([&, t] {
        std::mt19937 r(100 + t);
        char win[64];
        int32_t ws = 0;
        uint64_t id = 0;
        for (;;) {
          const std::string key = "ns/p" + std::to_string(r() % 50);
          const int32_t rc = ksg_record(ev, key.c_str(), ("a" + std::to_string(t)).c_str(), (int32_t)(r() % 5), &id,
                                        win, sizeof win, &ws);
          if (rc < 0) {
            CHECK(shut.load());
            return;
          }
          async_calls++;
          std::this_thread::sleep_for(50us);
        }
      });
    th.emplace_back([&] {
      char win[64];
      int32_t ws = 0;
      uint64_t id = 0;
      for (;;) {
        const int32_t rc = ksg_next_fired(ev, 5, &id, win, sizeof win, &ws);
        if (rc < 0) return;  // shut down and drained
        if (rc == 1) fired_reports++;
      }
    });
    std::this_thread::sleep_for(1500ms);
    shut = true;
    ksg_shutdown(ev);
    for (auto &x : th) x.join();
    CHECK(ksg_pending(ev) == 0);
    ksg_close(ev);
    std::printf("phase 1+2: %ld blocking, %ld async records, %ld fired reports\n", blocking_calls.load(),
                async_calls.load(), fired_reports.load());
    CHECK(blocking_calls > 100 && async_calls > 100 && fired_reports > 0);
  }
  // ---- phase 3
  for (int rep = 0; rep < 20; ++rep) {
    ksg_evaluator *ev = ksg_open(5, 60000, KSG_TIE_RANDOM, rep);
    std::vector<std::thread> th;
    std::atomic<int> returned{0}, entering{0};
    for (int t = 0; t < 4; ++t)
      th.emplace_back([&, t] {
        char win[64];
        int32_t ws = 0;
        entering++;
        const int32_t rc = ksg_record_and_wait(ev, "ns/parked", ("n" + std::to_string(t)).c_str(), 10 + t, win,
                                               sizeof win, &ws);
        CHECK(rc == 0 || rc == 1);
        returned++;
      });
    // every recorder must be inside its call before ksg_close starts (no
    // call may start after it): wait for all four, then give them 5 ms to
    // pass the entry check
    while (entering < 4 || ksg_pending(ev) == 0) std::this_thread::sleep_for(100us);
    std::this_thread::sleep_for(5ms);
    ksg_close(ev);  // the 4 recorders entered before it: released, then freed
    for (auto &x : th) x.join();
    CHECK(returned == 4);
  }
  std::printf("phase 3: 20 closes with parked recorders\n");
  std::printf("%s\n", failures ? "ksg_stress FAILED" : "ksg_stress ok");
  return failures ? 1 : 0;
}
