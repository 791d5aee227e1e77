// ksgather.cpp — the cross-host gather of SURVEY.md §8(f) F3 (include/ksgather.h):
// the gatherer's per-pod score evaluation (ScoreEvaluator.RecordAndWait / fire,
// dist-scheduler/pkg/scoreevaluator/scoreevaluator.go:45-126) and the
// member-side gatherer choice (SchedulerSet.GetTargetForScoring,
// pkg/schedulerset/schedulerset.go:107-143).  Host code; the gRPC wire is
// ksched/relay.py.
#include "ksgather.h"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

namespace {

constexpr size_t MAX_TIED = 100;  // candidates kept at the highest score (scoreevaluator.go:100)
const char *const RELAY_PREFIX = "dist-scheduler-relay";  // schedulerset.go:34

struct Score {
  std::string node;
  int32_t score;
};

// One pod's evaluation.  Instead of the reference's ticker goroutine, the
// waiters themselves wait until first-score + delay and the first to wake
// then fires: every recorder waits until its pod fires, so one always does.
struct One {
  std::mutex m;
  std::condition_variable cv;
  uint32_t limit = 0;
  std::vector<Score> scores;
  bool fired = false;
  Score winner{"", -1};
  std::chrono::steady_clock::time_point deadline;
};

}  // namespace

struct ksg_evaluator {
  std::mutex lock;
  std::map<std::string, std::shared_ptr<One>> pods;
  uint32_t members = 0;
  std::chrono::milliseconds delay{5000};
  int32_t tie = KSG_TIE_RANDOM;
  std::mt19937_64 rng;
  std::mutex rng_lock;

  // fire(): o.m is held by the caller
  void fire(const std::string &key, const std::shared_ptr<One> &o) {
    if (o->fired) return;
    int32_t best = -1;
    std::vector<const Score *> cand;
    cand.reserve(MAX_TIED);
    for (const Score &s : o->scores) {
      if (s.score > best) {
        best = s.score;
        cand.clear();
        cand.push_back(&s);
      } else if (s.score == best && cand.size() < MAX_TIED) {
        cand.push_back(&s);
      }
    }
    const Score *w = nullptr;
    if (!cand.empty()) {
      if (tie == KSG_TIE_LOWEST_NAME) {
        w = *std::min_element(cand.begin(), cand.end(), [](const Score *a, const Score *b) { return a->node < b->node; });
      } else {
        std::lock_guard<std::mutex> g(rng_lock);
        w = cand[std::uniform_int_distribution<size_t>(0, cand.size() - 1)(rng)];
      }
      o->winner = *w;
    }
    o->fired = true;
    {
      std::lock_guard<std::mutex> g(lock);
      auto it = pods.find(key);
      if (it != pods.end() && it->second == o) pods.erase(it);
    }
    o->cv.notify_all();
  }
};

extern "C" {

ksg_evaluator *ksg_open(uint32_t members, uint32_t delay_ms, int32_t tie_mode, uint64_t seed) {
  if (tie_mode != KSG_TIE_RANDOM && tie_mode != KSG_TIE_LOWEST_NAME) return nullptr;
  auto *e = new ksg_evaluator();
  e->members = members;
  e->delay = std::chrono::milliseconds(delay_ms);
  e->tie = tie_mode;
  e->rng.seed(seed);
  return e;
}

void ksg_close(ksg_evaluator *ev) { delete ev; }

void ksg_set_members(ksg_evaluator *ev, uint32_t members) {
  if (!ev) return;
  std::lock_guard<std::mutex> g(ev->lock);
  ev->members = members;
}

int32_t ksg_record_and_wait(ksg_evaluator *ev, const char *key, const char *node_name, int32_t score, char *winner,
                            uint32_t winner_cap, int32_t *winner_score) {
  if (!ev || !key || !node_name) return -1;
  const std::string k(key);
  std::shared_ptr<One> o;
  {
    std::lock_guard<std::mutex> g(ev->lock);
    auto it = ev->pods.find(k);
    if (it == ev->pods.end()) {
      o = std::make_shared<One>();
      o->limit = ev->members;
      o->deadline = std::chrono::steady_clock::now() + ev->delay;
      ev->pods.emplace(k, o);
    } else {
      o = it->second;
    }
  }
  std::unique_lock<std::mutex> l(o->m);
  o->scores.push_back(Score{node_name, score});
  if (o->scores.size() >= o->limit) {
    ev->fire(k, o);  // every member's score is in: fire early
  } else {
    while (!o->fired) {
      if (o->cv.wait_until(l, o->deadline) == std::cv_status::timeout && !o->fired) ev->fire(k, o);
    }
  }
  if (winner && winner_cap) {
    const size_t n = std::min<size_t>(o->winner.node.size(), winner_cap - 1);
    std::memcpy(winner, o->winner.node.data(), n);
    winner[n] = 0;
  }
  if (winner_score) *winner_score = o->winner.score;
  return o->winner.node == node_name ? 1 : 0;
}

uint32_t ksg_pending(ksg_evaluator *ev) {
  if (!ev) return 0;
  std::lock_guard<std::mutex> g(ev->lock);
  return (uint32_t)ev->pods.size();
}

uint32_t ksg_fnv1_32(const char *data, uint32_t n) {
  uint32_t h = 2166136261u;
  for (uint32_t i = 0; i < n; ++i) {
    h *= 16777619u;
    h ^= (uint8_t)data[i];
  }
  return h;
}

uint32_t ksg_target_index(const char *key, const char *const *members, uint32_t n, const char *leader) {
  if (!key || !members || n == 0) return UINT32_MAX;
  if (n == 1) return 0;
  const std::string lead = leader ? leader : "";
  std::vector<uint32_t> order(n);
  for (uint32_t i = 0; i < n; ++i) order[i] = i;
  // podNameSort: the leader first, relay pods ("a" + name) before the rest, by name
  auto sort_key = [&](const std::string &s) { return s.rfind(RELAY_PREFIX, 0) == 0 ? "a" + s : s; };
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    const std::string sa = members[a], sb = members[b];
    if (!lead.empty() && sa == lead) return sb != lead;
    if (!lead.empty() && sb == lead) return false;
    return sort_key(sa) < sort_key(sb);
  });
  const uint32_t h = ksg_fnv1_32(key, (uint32_t)std::strlen(key)) % n;
  return order[h];
}

}  // extern "C"
