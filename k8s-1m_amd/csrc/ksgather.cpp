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
#include <deque>
#include <map>
#include <unordered_map>
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
  bool async = false;  // a ksg_record caller waits for ksg_next_fired to report it
  uint64_t id = 0;     // evaluation id (a key's later evaluation gets a new one)
  Score winner{"", -1};
  std::chrono::steady_clock::time_point deadline;
};

struct Fired {
  uint64_t id;
  Score winner;
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
  uint64_t next_id = 1;
  // KSG_TIE_LOWEST_INDEX: node name -> global index (ksg_set_node_order, under lock)
  std::unordered_map<std::string, uint64_t> order;
  // evaluations with asynchronous recorders, fired and not yet reported
  std::deque<Fired> fired_q;
  std::condition_variable fired_cv;  // with `lock`: fired_q grew, or closing
  bool closing = false;
  uint32_t inside = 0;  // threads inside record_and_wait / record / next_fired (ksg_close waits for 0)
  std::condition_variable idle_cv;

  // Entry into an API call that may touch the evaluator after ksg_close
  // began: refused once closing, else counted in `inside` until the guard
  // goes out of scope (the last one out lets ksg_close free the evaluator).
  struct Inside {
    ksg_evaluator *ev = nullptr;
    ~Inside() {
      if (!ev) return;
      std::lock_guard<std::mutex> g(ev->lock);
      if (--ev->inside == 0) ev->idle_cv.notify_all();
    }
  };
  // caller holds `lock`
  bool enter(Inside &in, bool allow_closing = false) {
    if (closing && !allow_closing) return false;
    inside++;
    in.ev = this;
    return true;
  }

  uint64_t rank_of(const std::string &node) {  // caller holds `lock`
    auto it = order.find(node);
    return it == order.end() ? UINT64_MAX : it->second;
  }

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
      } else if (tie == KSG_TIE_LOWEST_INDEX) {
        // the lowest global node index (the hosts' own lowest-slot rule
        // across hosts); names outside the table after every listed one
        std::lock_guard<std::mutex> g(lock);
        w = *std::min_element(cand.begin(), cand.end(), [&](const Score *a, const Score *b) {
          const uint64_t ra = rank_of(a->node), rb = rank_of(b->node);
          return ra != rb ? ra < rb : a->node < b->node;
        });
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
      if (o->async) {
        fired_q.push_back(Fired{o->id, o->winner});
        fired_cv.notify_all();
      }
    }
    o->cv.notify_all();
  }

  // The evaluation of `key` the next score joins (a fired one is gone from
  // `pods`: a late score starts a new evaluation).  Caller holds `lock`.
  std::shared_ptr<One> evaluation(const std::string &k) {
    auto it = pods.find(k);
    if (it != pods.end()) return it->second;
    auto o = std::make_shared<One>();
    o->limit = members;
    o->deadline = std::chrono::steady_clock::now() + delay;
    o->id = next_id++;
    pods.emplace(k, o);
    return o;
  }

  // Fire every pending evaluation whose deadline has passed (all of them when
  // closing); never called with `lock` held (fire takes it after o->m).
  void fire_expired(bool all) {
    std::vector<std::pair<std::string, std::shared_ptr<One>>> due;
    {
      std::lock_guard<std::mutex> g(lock);
      const auto now = std::chrono::steady_clock::now();
      for (auto &kv : pods)
        if (all || kv.second->deadline <= now) due.push_back(kv);
    }
    for (auto &kv : due) {
      std::lock_guard<std::mutex> l(kv.second->m);
      fire(kv.first, kv.second);
    }
  }
};

extern "C" {

ksg_evaluator *ksg_open(uint32_t members, uint32_t delay_ms, int32_t tie_mode, uint64_t seed) {
  if (tie_mode != KSG_TIE_RANDOM && tie_mode != KSG_TIE_LOWEST_NAME && tie_mode != KSG_TIE_LOWEST_INDEX) return nullptr;
  auto *e = new ksg_evaluator();
  e->members = members;
  e->delay = std::chrono::milliseconds(delay_ms);
  e->tie = tie_mode;
  e->rng.seed(seed);
  return e;
}

// Close: fire every pending evaluation (its waiters return with the scores
// recorded so far), wake ksg_next_fired, and free once no thread is inside.
void ksg_shutdown(ksg_evaluator *ev) {
  if (!ev) return;
  {
    std::lock_guard<std::mutex> g(ev->lock);
    ev->closing = true;
  }
  ev->fire_expired(true);
  std::lock_guard<std::mutex> g(ev->lock);
  ev->fired_cv.notify_all();
}

void ksg_close(ksg_evaluator *ev) {
  if (!ev) return;
  {
    std::lock_guard<std::mutex> g(ev->lock);
    ev->closing = true;
  }
  for (;;) {  // an evaluation a racing recorder created meanwhile is fired on the next pass
    ev->fire_expired(true);
    std::unique_lock<std::mutex> g(ev->lock);
    ev->fired_cv.notify_all();
    if (ev->idle_cv.wait_for(g, std::chrono::milliseconds(10), [&] { return ev->inside == 0; })) break;
  }
  delete ev;
}

void ksg_set_node_order(ksg_evaluator *ev, const char *const *names, uint32_t n) {
  if (!ev || (n && !names)) return;
  std::lock_guard<std::mutex> g(ev->lock);
  ev->order.clear();
  for (uint32_t i = 0; i < n; ++i)
    if (names[i]) ev->order.emplace(names[i], i);
}

void ksg_set_members(ksg_evaluator *ev, uint32_t members) {
  if (!ev) return;
  std::lock_guard<std::mutex> g(ev->lock);
  ev->members = members;
}

int32_t ksg_record_and_wait(ksg_evaluator *ev, const char *key, const char *node_name, int32_t score, char *winner,
                            uint32_t winner_cap, int32_t *winner_score) {
  if (!ev || !key || !node_name) return -1;
  const std::string k(key);
  ksg_evaluator::Inside in;
  {
    std::lock_guard<std::mutex> g(ev->lock);
    if (!ev->enter(in)) return -1;
  }
  std::shared_ptr<One> o;
  std::unique_lock<std::mutex> l;
  for (;;) {  // an evaluation that fired before we locked it: the score starts a new one
    {
      std::lock_guard<std::mutex> g(ev->lock);
      o = ev->evaluation(k);
    }
    l = std::unique_lock<std::mutex>(o->m);
    if (!o->fired) break;
    l.unlock();
  }
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

int32_t ksg_record(ksg_evaluator *ev, const char *key, const char *node_name, int32_t score, uint64_t *eval_id,
                   char *winner, uint32_t winner_cap, int32_t *winner_score) {
  if (!ev || !key || !node_name || !eval_id) return -1;
  const std::string k(key);
  // counted in `inside` like the other calls: ksg_close must not free the
  // evaluator while this call still locks o->m / fires / takes ev->lock
  ksg_evaluator::Inside in;
  {
    std::lock_guard<std::mutex> g(ev->lock);
    if (!ev->enter(in)) return -1;
  }
  std::shared_ptr<One> o;
  std::unique_lock<std::mutex> l;
  for (;;) {  // as ksg_record_and_wait: never join an evaluation that already fired
    {
      std::lock_guard<std::mutex> g(ev->lock);
      o = ev->evaluation(k);
    }
    l = std::unique_lock<std::mutex>(o->m);
    if (!o->fired) break;
    l.unlock();
  }
  *eval_id = o->id;
  o->scores.push_back(Score{node_name, score});
  if (o->scores.size() < o->limit) {
    o->async = true;  // reported by ksg_next_fired when it fires
    return 2;
  }
  ev->fire(k, o);
  if (winner && winner_cap) {
    const size_t n = std::min<size_t>(o->winner.node.size(), winner_cap - 1);
    std::memcpy(winner, o->winner.node.data(), n);
    winner[n] = 0;
  }
  if (winner_score) *winner_score = o->winner.score;
  return o->winner.node == node_name ? 1 : 0;
}

int32_t ksg_next_fired(ksg_evaluator *ev, uint32_t timeout_ms, uint64_t *eval_id, char *winner, uint32_t winner_cap,
                       int32_t *winner_score) {
  if (!ev || !eval_id) return -1;
  const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  ksg_evaluator::Inside in;
  {
    std::lock_guard<std::mutex> g(ev->lock);
    if (ev->closing && ev->fired_q.empty()) return -1;
    ev->enter(in, true);  // still drains evaluations fired by the close
  }
  for (;;) {
    ev->fire_expired(false);  // deadlines of evaluations nobody waits on synchronously
    std::unique_lock<std::mutex> g(ev->lock);
    if (!ev->fired_q.empty()) {
      const Fired f = ev->fired_q.front();
      ev->fired_q.pop_front();
      *eval_id = f.id;
      if (winner && winner_cap) {
        const size_t n = std::min<size_t>(f.winner.node.size(), winner_cap - 1);
        std::memcpy(winner, f.winner.node.data(), n);
        winner[n] = 0;
      }
      if (winner_score) *winner_score = f.winner.score;
      return 1;
    }
    if (ev->closing) return -1;
    const auto now = std::chrono::steady_clock::now();
    if (now >= until) return 0;
    auto wake = until;
    for (auto &kv : ev->pods) wake = std::min(wake, kv.second->deadline);
    ev->fired_cv.wait_until(g, std::max(wake, now + std::chrono::microseconds(100)));
  }
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
