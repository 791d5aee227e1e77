// Concurrency driver for libksched's host-thread protocols
// (k8s-1m_amd/csrc/ksched_sync.hpp), built under ThreadSanitizer and under
// AddressSanitizer + UBSan by `make -C k8s-1m_amd sanitize`:
//
//  1. Rendezvous: 8 ranks x 20,000 collectives, every rank receiving the same
//     snapshot of the same collective; then a group whose last rank never
//     arrives: every waiting rank times out, and the group stays failed.
//  2. RunQueue: 4 submitter threads, each submitting its own jobs and
//     waiting for them, while a fifth thread drains and polls idle(); jobs
//     run one at a time in each submitter's order; jobs resubmitted after
//     they finish; a failing job's status and error text; stop() with
//     queued jobs (the worker finishes them first).
//  3. parallel_chunks: disjoint chunks covering [0, n), per-thread partials.
#include <atomic>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "ksched_sync.hpp"

using namespace ks;

static int failures = 0;
#define CHECK(x)                                                              \
  do {                                                                        \
    if (!(x)) {                                                               \
      std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #x, __LINE__);     \
      ++failures;                                                             \
    }                                                                         \
  } while (0)

struct Post {
  uint32_t rank = 0;
  uint64_t iter = 0;
  std::vector<double> vals;
};

static void rendezvous() {
  const uint32_t W = 8, N = 20000;
  Rendezvous<Post> g(W);
  std::vector<std::thread> th;
  std::atomic<uint64_t> bad{0};
  for (uint32_t r = 0; r < W; ++r)
    th.emplace_back([&, r] {
      std::vector<Post> out;
      for (uint64_t i = 0; i < N; ++i) {
        Post p;
        p.rank = r;
        p.iter = i;
        p.vals.assign(1 + (i % 3), (double)(r * 1000 + i));
        if (!g.exchange(r, p, out)) {
          ++bad;
          return;
        }
        for (uint32_t j = 0; j < W; ++j)
          if (out[j].rank != j || out[j].iter != i || out[j].vals.size() != 1 + (i % 3) ||
              out[j].vals[0] != (double)(j * 1000 + i))
            ++bad;
      }
    });
  for (auto &t : th) t.join();
  CHECK(bad == 0);
  // a rank that never arrives: the others time out, the group stays failed
  Rendezvous<Post> h(4, std::chrono::milliseconds(200));
  std::atomic<int> failed{0};
  th.clear();
  for (uint32_t r = 0; r < 3; ++r)
    th.emplace_back([&, r] {
      std::vector<Post> out;
      Post p;
      p.rank = r;
      if (!h.exchange(r, p, out)) ++failed;
    });
  for (auto &t : th) t.join();
  CHECK(failed == 3);
  std::vector<Post> out;
  CHECK(!h.exchange(3, Post{}, out));
  std::printf("rendezvous: %u ranks x %u exchanges, timeout group ok\n", W, N);
}

struct Job {
  bool queued = false, done = false;
  int32_t run_status = 0;
  std::string run_err;
  uint32_t owner = 0, seq = 0;
  bool fail = false;
  uint32_t runs = 0;  // written by the worker only, read after wait()
};

struct Ctx {
  std::atomic<int> active{0};
  std::atomic<uint64_t> order_bad{0}, overlap{0}, total{0}, inits{0};
  std::vector<uint32_t> last_seq;  // per owner: written by the worker only
};

static int32_t run_job(void *ctx, Job *j, std::string *err) {
  Ctx *c = static_cast<Ctx *>(ctx);
  if (c->active.fetch_add(1) != 0) ++c->overlap;  // one job at a time
  if (j->seq != 0 && j->seq <= c->last_seq[j->owner] && j->runs == 0) ++c->order_bad;
  c->last_seq[j->owner] = j->seq;
  j->runs += 1;
  volatile uint64_t spin = 0;
  for (int k = 0; k < 200; ++k) spin = spin + k;
  ++c->total;
  c->active.fetch_sub(1);
  if (j->fail) {
    *err = "job " + std::to_string(j->owner) + "/" + std::to_string(j->seq) + " failed";
    return 7;
  }
  return 0;
}
static void init_worker(void *ctx) { ++static_cast<Ctx *>(ctx)->inits; }

static void run_queue() {
  const uint32_t S = 4, J = 3000;
  Ctx ctx;
  ctx.last_seq.assign(S, 0);
  std::vector<std::vector<Job>> jobs(S, std::vector<Job>(J));
  {
    RunQueue<Job> q(&ctx, &run_job, &init_worker);
    std::atomic<bool> done{false};
    std::vector<std::thread> th;
    for (uint32_t s = 0; s < S; ++s)
      th.emplace_back([&, s] {
        for (uint32_t i = 0; i < J; ++i) {
          Job &j = jobs[s][i];
          j.owner = s;
          j.seq = i + 1;
          j.fail = (i % 97) == 5;
          CHECK(q.submit(&j));
          if (i % 4 == 3)  // waits lag the submits (several jobs of this thread in flight)
            for (uint32_t k = i - 3; k <= i; ++k) {
              Job &w = jobs[s][k];
              CHECK(q.wait(&w));
              CHECK(w.done && w.runs == 1);
              CHECK(w.run_status == (w.fail ? 7 : 0));
              CHECK(w.fail == !w.run_err.empty());
              CHECK(!q.running(&w));
            }
        }
      });
    th.emplace_back([&] {
      while (!done) {
        q.drain();
        (void)q.idle();
        std::this_thread::yield();
      }
    });
    for (uint32_t s = 0; s < S; ++s) th[s].join();
    done = true;
    th.back().join();
    // resubmit finished jobs; settle() waits like ks_batch_free
    for (uint32_t i = 0; i < 64; ++i) {
      Job &j = jobs[0][i];
      CHECK(q.submit(&j));
      // refused while j is queued and unfinished, accepted once the worker
      // has finished it (no unlocked read of j's state here)
      const bool again = q.submit(&j);
      q.settle(&j);
      CHECK(j.done && j.runs >= (again ? 3 : 2));
    }
    Job never;
    CHECK(!q.wait(&never));
    q.drain();
    CHECK(q.idle());
    // stop with jobs queued: they still run
    std::vector<Job> tail(200);
    for (uint32_t i = 0; i < tail.size(); ++i) {
      tail[i].owner = 1;
      tail[i].seq = 0;
      CHECK(q.submit(&tail[i]));
    }
    q.stop();
    for (auto &t : tail) CHECK(t.done && t.runs == 1);
    double prof[3];
    q.profile(prof);
    CHECK(prof[2] == (double)ctx.total.load());
  }
  CHECK(ctx.overlap == 0);
  CHECK(ctx.order_bad == 0);
  CHECK(ctx.inits == 1);
  std::printf("run queue: %llu runs, %u submitters, in order, one at a time\n", (unsigned long long)ctx.total.load(), S);
}

static void chunks() {
  for (uint32_t n : {0u, 1u, 7u, 8192u, 150001u})
    for (uint32_t T : {1u, 3u, 8u}) {
      std::vector<uint8_t> hit(n, 0);
      std::vector<uint64_t> part(T, 0);
      parallel_chunks(n, T, [&](uint32_t t, uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i) {
          hit[i] += 1;
          part[t] += i;
        }
      });
      uint64_t sum = 0;
      for (uint64_t v : part) sum += v;
      bool once = true;
      for (uint8_t h : hit) once &= h == 1;
      CHECK(once);
      CHECK(sum == (uint64_t)n * (n ? n - 1 : 0) / 2);
    }
  std::printf("parallel_chunks: ok\n");
}

int main() {
  rendezvous();
  run_queue();
  chunks();
  std::printf("sync_stress: %s\n", failures ? "FAILED" : "ok");
  return failures ? 1 : 0;
}
