// ksched_sync.hpp — libksched's host-thread protocols, HIP-free so that
// tools/sync_stress.cpp can drive them under ThreadSanitizer and
// AddressSanitizer on the CPU (make -C k8s-1m_amd sanitize):
//
//   Rendezvous    the in-process communicator's exchange (ks_comm_init_local):
//                 every rank posts, all receive the same snapshot; a timeout
//                 fails the group for good
//   RunQueue      ks_batch_submit / ks_batch_wait / drain: batches run in
//                 submission order on one worker thread
//   parallel_chunks  the event-log pool: [0, n) split over T threads
//
// ksched_host.cpp instantiates them with its own types (hipEvent_t posts,
// ks_batch jobs); nothing here touches the device.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace ks {

// All ranks of a group post one entry per collective and receive every
// rank's entry (the same snapshot for all).  A rank that waits longer than
// `timeout` fails the group: a late post would otherwise pair with the next
// collective's.
template <class Post>
class Rendezvous {
 public:
  explicit Rendezvous(uint32_t world, std::chrono::milliseconds timeout = std::chrono::seconds(300))
      : world_(world), timeout_(timeout), posts_(world), snap_(world) {}
  uint32_t world() const { return world_; }
  // false: the group failed (this or an earlier exchange timed out)
  bool exchange(uint32_t rank, Post p, std::vector<Post> &out) {
    std::unique_lock<std::mutex> g(mu_);
    if (failed_) return false;
    posts_[rank] = std::move(p);
    const uint64_t my = gen_;
    if (++arrived_ == world_) {
      snap_ = posts_;
      arrived_ = 0;
      ++gen_;
      cv_.notify_all();
    } else if (!cv_.wait_for(g, timeout_, [&] { return gen_ != my || failed_; }) || failed_) {
      failed_ = true;
      cv_.notify_all();
      return false;
    }
    out = snap_;
    return true;
  }

 private:
  const uint32_t world_;
  const std::chrono::milliseconds timeout_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Post> posts_, snap_;
  uint32_t arrived_ = 0;
  uint64_t gen_ = 0;
  bool failed_ = false;
};

// Jobs run in submission order on one worker thread, started by the first
// submit.  Job has `bool queued, done; int32_t run_status; std::string
// run_err` (ks_batch).  The run callback returns the job's status and error
// text; stop() lets the worker finish the queued jobs, then joins it.
template <class Job>
class RunQueue {
 public:
  using RunFn = int32_t (*)(void *ctx, Job *job, std::string *err);
  using InitFn = void (*)(void *ctx);
  RunQueue(void *ctx, RunFn run, InitFn init = nullptr) : ctx_(ctx), run_(run), init_(init) {}
  ~RunQueue() { stop(); }
  RunQueue(const RunQueue &) = delete;
  RunQueue &operator=(const RunQueue &) = delete;

  // false: the job is already queued and not done
  bool submit(Job *b) {
    std::lock_guard<std::mutex> g(mu_);
    if (b->queued && !b->done) return false;
    if (!worker_.joinable()) worker_ = std::thread([this] { loop(); });
    b->queued = true;
    b->done = false;
    b->run_status = 0;
    b->run_err.clear();
    q_.push_back(b);
    ++inflight_;
    qcv_.notify_one();
    return true;
  }
  // waits for a submitted job; false: it was never submitted
  bool wait(Job *b) {
    std::unique_lock<std::mutex> lk(mu_);
    if (!b->queued) return false;
    dcv_.wait(lk, [&] { return b->done; });
    return true;
  }
  // waits for the job if it was submitted (ks_batch_free)
  void settle(Job *b) {
    std::unique_lock<std::mutex> lk(mu_);
    if (b->queued) dcv_.wait(lk, [&] { return b->done; });
  }
  bool running(const Job *b) {
    std::lock_guard<std::mutex> g(mu_);
    return b->queued && !b->done;
  }
  bool idle() {
    std::lock_guard<std::mutex> g(mu_);
    return inflight_ == 0;
  }
  // every submitted job done
  void drain() {
    std::unique_lock<std::mutex> lk(mu_);
    dcv_.wait(lk, [&] { return inflight_ == 0; });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      qcv_.notify_all();
    }
    if (worker_.joinable()) worker_.join();
  }
  // worker time: [0] in runs, [1] idle between runs with another one queued soon, [2] runs
  void profile(double out[3]) {
    std::lock_guard<std::mutex> g(mu_);
    for (int i = 0; i < 3; ++i) out[i] = prof_[i];
  }

 private:
  void loop() {
    if (init_) init_(ctx_);
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      const auto ti = std::chrono::steady_clock::now();
      qcv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stop requested, nothing queued
      if (prof_[2] > 0) prof_[1] += std::chrono::duration<double>(std::chrono::steady_clock::now() - ti).count();
      Job *b = q_.front();
      q_.pop_front();
      lk.unlock();
      const auto t0 = std::chrono::steady_clock::now();
      std::string e;
      const int32_t st = run_(ctx_, b, &e);
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      lk.lock();
      prof_[0] += dt;
      prof_[2] += 1;
      b->run_status = st;
      b->run_err = st ? e : std::string();
      b->done = true;
      --inflight_;
      dcv_.notify_all();
    }
  }

  void *const ctx_;
  const RunFn run_;
  const InitFn init_;
  std::mutex mu_;
  std::condition_variable qcv_, dcv_;
  std::deque<Job *> q_;
  uint32_t inflight_ = 0;
  bool stop_ = false;
  double prof_[3] = {0, 0, 0};
  std::thread worker_;
};

// f(t, lo, hi) on T threads over the contiguous chunks of [0, n) (thread t
// takes [n t / T, n (t + 1) / T)); returns once all have finished.
template <class F>
void parallel_chunks(uint32_t n, uint32_t T, F f) {
  if (T <= 1) {
    f(0u, 0u, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T);
  for (uint32_t t = 0; t < T; ++t)
    th.emplace_back([&f, n, T, t] { f(t, (uint32_t)((uint64_t)n * t / T), (uint32_t)((uint64_t)n * (t + 1) / T)); });
  for (auto &x : th) x.join();
}

}  // namespace ks
