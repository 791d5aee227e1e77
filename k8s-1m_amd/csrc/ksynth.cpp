// ksynth.cpp — seeded synthetic kwok-shaped clusters / pod streams (see include/ksynth.h).
//
// Every node and pod is a pure function of (seed, index): node i draws from
// rng(seed, i), pod j from rng(seed, j).  Any prefix or slice of a stream can
// therefore be regenerated exactly by the oracle harness, the tests and the
// bench without sharing files.
#include "ksynth.h"

#include <cstdio>
#include <cstring>
#include <deque>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

inline uint64_t splitmix64(uint64_t &x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// xoshiro256** seeded from splitmix64(seed ^ mix(index)).
struct Rng {
  uint64_t s[4];
  Rng(uint64_t seed, uint64_t index, uint64_t stream = 0) {
    uint64_t x = seed ^ (index * 0xD1B54A32D192ED03ull) ^ (stream * 0x8CB92BA72F3D8DD7ull);
    for (auto &v : s) v = splitmix64(x);
  }
  static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * (uint64_t)n >> 32); }
  double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  bool chance(double p) { return unit() < p; }
};

constexpr int64_t kGi = 1024ll * 1024 * 1024;
constexpr int64_t kMi = 1024ll * 1024;

}  // namespace

struct ksynth {
  std::vector<ks_node> nodes;
  std::vector<ks_pod> pods;
  std::vector<uint32_t> slots;
  // Backing storage, reserved up-front so element pointers stay stable.
  std::vector<ks_label> labels;
  std::vector<ks_taint> taints;
  std::vector<ks_container> containers;
  std::vector<ks_toleration> tolerations;
  std::vector<ks_requirement> reqs;
  std::vector<ks_term> terms;
  std::vector<ks_preferred_term> prefs;
  std::vector<const char *> values;
  std::vector<ks_spread_constraint> spread;
  std::vector<ks_pod_affinity_term> affinity;
  std::deque<std::string> strings;
  std::unordered_map<std::string, const char *> interned;

  const char *intern(const std::string &s) {
    auto it = interned.find(s);
    if (it != interned.end()) return it->second;
    strings.push_back(s);
    const char *p = strings.back().c_str();
    interned.emplace(s, p);
    return p;
  }
  const char *own(const std::string &s) {  // not interned (unique strings)
    strings.push_back(s);
    return strings.back().c_str();
  }
  template <class T>
  static T *push(std::vector<T> &v, const T &x) {
    if (v.size() == v.capacity()) {
      std::fprintf(stderr, "ksynth: reserve exceeded\n");
      std::abort();
    }
    v.push_back(x);
    return &v.back();
  }
};

namespace {

// ---------------------------------------------------------------- nodes

struct Shape {
  int64_t cpu, mem, pods;
};

Shape node_shape(int32_t kind, uint64_t seed, uint32_t i) {
  if (kind == KSYNTH_KWOK) return {32000, 256 * kGi, 32};  // make_nodes/main.go:155-158, :64
  Rng r(seed, i, 1);
  static const int64_t cpus[5] = {8, 16, 32, 64, 96};
  static const int64_t mems[5] = {32, 64, 128, 256, 512};
  Shape s;
  s.cpu = cpus[r.below(5)] * 1000;
  s.mem = mems[r.below(5)] * kGi;
  s.pods = r.chance(0.5) ? 32 : 110;  // make_nodes default 32; test_manifests/node.yaml:26 uses 110
  return s;
}

void add_kwok_labels(ksynth *s, uint32_t i, const char *name) {
  // kwok/make_nodes/main.go:130-141
  static const char *fixed[][2] = {{"beta.kubernetes.io/arch", "amd64"},
                                   {"beta.kubernetes.io/os", "linux"},
                                   {"kubernetes.io/arch", "amd64"},
                                   {"kubernetes.io/os", "linux"},
                                   {"kubernetes.io/role", "agent"},
                                   {"node-role.kubernetes.io/agent", ""},
                                   {"type", "kwok"}};
  for (auto &kv : fixed) ksynth::push(s->labels, ks_label{s->intern(kv[0]), s->intern(kv[1])});
  ksynth::push(s->labels, ks_label{s->intern("kubernetes.io/hostname"), name});
  ksynth::push(s->labels,
               ks_label{s->intern("kwok-group"), s->intern(std::to_string(i / 10000))});
}

}  // namespace

extern "C" ksynth *ksynth_nodes(int32_t kind, uint32_t n, uint64_t seed) {
  auto *s = new ksynth();
  s->nodes.reserve(n);
  s->labels.reserve((size_t)n * 24);
  s->taints.reserve((size_t)n * 6);
  for (uint32_t i = 0; i < n; ++i) {
    Shape sh = node_shape(kind, seed, i);
    ks_node nd{};
    nd.name = s->own("kwok-node-" + std::to_string(i));
    nd.alloc_milli_cpu = sh.cpu;
    nd.alloc_memory = sh.mem;
    nd.alloc_pods = sh.pods;
    nd.labels = s->labels.data() + s->labels.size();
    add_kwok_labels(s, i, nd.name);
    nd.taints = s->taints.data() + s->taints.size();
    ksynth::push(s->taints, ks_taint{s->intern("kwok.x-k8s.io/node"), s->intern("fake"),
                                     KS_EFFECT_NO_SCHEDULE, 0});
    if (kind == KSYNTH_ZONED) {
      Rng r(seed, i, 2);
      ksynth::push(s->labels, ks_label{s->intern("topology.kubernetes.io/zone"),
                                       s->intern("zone-" + std::to_string(r.below(32)))});
    }
    if (kind == KSYNTH_LABELED) {
      Rng r(seed, i, 2);
      auto lab = [&](const std::string &k, const std::string &v) {
        ksynth::push(s->labels, ks_label{s->intern(k), s->intern(v)});
      };
      uint32_t pool = r.below(8);
      lab("topology.kubernetes.io/zone", "zone-" + std::to_string(r.below(16)));
      lab("node.kubernetes.io/instance-type", "it-" + std::to_string(r.below(32)));
      lab("pool", "pool-" + std::to_string(pool));
      for (int f = 0; f < 8; ++f)
        if (r.chance(0.3)) lab("feature-" + std::to_string(f), "true");
      static const int gpus[5] = {0, 1, 2, 4, 8};
      uint32_t g = r.below(6);
      if (g < 5) lab("gpu-count", std::to_string(gpus[g]));
      else lab("gpu-count", "many");  // unparseable for Gt/Lt
      auto taint = [&](const std::string &k, const std::string &v, int32_t eff) {
        ksynth::push(s->taints, ks_taint{s->intern(k), s->intern(v), eff, 0});
      };
      if (r.chance(0.10)) taint("dedicated", "pool-" + std::to_string(pool), KS_EFFECT_NO_SCHEDULE);
      if (r.chance(0.02)) taint("maint", "true", KS_EFFECT_NO_EXECUTE);
      if (r.chance(0.05)) taint("spot", "true", KS_EFFECT_PREFER_NO_SCHEDULE);
      if (r.chance(0.03)) taint("batch", "true", KS_EFFECT_PREFER_NO_SCHEDULE);
      nd.unschedulable = r.chance(0.01) ? 1u : 0u;
    }
    nd.n_labels = (uint32_t)(s->labels.data() + s->labels.size() - nd.labels);
    nd.n_taints = (uint32_t)(s->taints.data() + s->taints.size() - nd.taints);
    s->nodes.push_back(nd);
  }
  return s;
}

// ---------------------------------------------------------------- pods

namespace {

void reserve_pods(ksynth *s, size_t n) {
  s->pods.reserve(n);
  s->containers.reserve(n);
  s->tolerations.reserve(n * 8);
  s->reqs.reserve(n * 8);
  s->terms.reserve(n * 4);
  s->prefs.reserve(n * 2);
  s->values.reserve(n * 16);
  s->labels.reserve(n * 2);
  s->spread.reserve(n * 2);
  s->affinity.reserve(n * 2);
}

// Resource requests of the C1 stream: cpu in {50..4000 step 50}m,
// memory = 64Mi x U{1..256}; 10% best-effort (no requests at all).
void draw_requests(Rng &r, ks_container &c) {
  c = ks_container{};
  if (r.chance(0.10)) return;  // best-effort: requests map empty
  c.milli_cpu = 50 * (1 + (int64_t)r.below(80));
  c.memory = 64 * kMi * (1 + (int64_t)r.below(256));
  c.flags = KS_REQ_HAS_CPU | KS_REQ_HAS_MEMORY;
}

void kwok_tolerations(ksynth *s) {
  // kwok/make_pods/main.go:128-144
  ksynth::push(s->tolerations, ks_toleration{s->intern("kwok.x-k8s.io/node"), s->intern(""),
                                             KS_TOL_EXISTS, KS_EFFECT_NO_SCHEDULE});
  ksynth::push(s->tolerations, ks_toleration{s->intern("node.kubernetes.io/not-ready"),
                                             s->intern(""), KS_TOL_EXISTS, KS_EFFECT_NO_SCHEDULE});
  ksynth::push(s->tolerations, ks_toleration{s->intern("node.kubernetes.io/not-ready"),
                                             s->intern(""), KS_TOL_EXISTS, KS_EFFECT_NO_EXECUTE});
}

ks_pod base_pod(ksynth *s, uint32_t j, const char *prefix) {
  ks_pod p{};
  p.ns = s->intern("default");
  p.name = s->own(std::string(prefix) + std::to_string(j));
  return p;
}

const char *const *values(ksynth *s, std::initializer_list<std::string> vs) {
  const char **first = nullptr;
  for (auto &v : vs) {
    const char **p = ksynth::push(s->values, s->intern(v));
    if (!first) first = p;
  }
  return first;
}

}  // namespace

extern "C" ksynth *ksynth_pods(int32_t kind, uint32_t n, uint64_t seed) {
  auto *s = new ksynth();
  reserve_pods(s, n);
  for (uint32_t j = 0; j < n; ++j) {
    Rng r(seed, j, 3);
    ks_pod p = base_pod(s, j, "res-");
    ks_container c;
    draw_requests(r, c);
    p.containers = ksynth::push(s->containers, c);
    p.n_containers = 1;
    p.tolerations = s->tolerations.data() + s->tolerations.size();
    kwok_tolerations(s);
    if (kind == KSYNTH_LABELED) {
      Rng q(seed, j, 4);
      auto tol = [&](const std::string &k, int32_t op, const std::string &v, int32_t eff) {
        ksynth::push(s->tolerations, ks_toleration{s->intern(k), s->intern(v), op, eff});
      };
      if (q.chance(0.15)) tol("dedicated", KS_TOL_EQUAL, "pool-" + std::to_string(q.below(8)), KS_EFFECT_NO_SCHEDULE);
      if (q.chance(0.05)) tol("", KS_TOL_EXISTS, "", KS_EFFECT_ALL);
      if (q.chance(0.20)) tol("spot", KS_TOL_EXISTS, "", KS_EFFECT_PREFER_NO_SCHEDULE);
      if (q.chance(0.05)) tol("batch", KS_TOL_EQUAL, "true", KS_EFFECT_ALL);
      if (q.chance(0.30)) {
        p.node_selector = ksynth::push(
            s->labels, ks_label{s->intern("topology.kubernetes.io/zone"),
                     s->intern("zone-" + std::to_string(q.below(16)))});
        p.n_node_selector = 1;
      }
      bool aff = q.chance(0.20), gpu = q.chance(0.10), byname = q.chance(0.01);
      bool bad = q.chance(0.005);
      if (aff || gpu || byname || bad) {
        p.has_required = 1;
        int nterms = (aff && q.chance(0.25)) ? 2 : 1;
        p.required_terms = s->terms.data() + s->terms.size();
        for (int t = 0; t < nterms; ++t) {
          ks_term term{};
          term.match_expressions = s->reqs.data() + s->reqs.size();
          if (t == 0 && aff) {
            ksynth::push(s->reqs, ks_requirement{s->intern("node.kubernetes.io/instance-type"),
                                                 values(s, {"it-" + std::to_string(q.below(32)),
                                                            "it-" + std::to_string(q.below(32)),
                                                            "it-" + std::to_string(q.below(32)),
                                                            "it-" + std::to_string(q.below(32))}),
                                                 4, KS_OP_IN});
            ksynth::push(s->reqs, ks_requirement{s->intern("pool"),
                                                 values(s, {"pool-" + std::to_string(q.below(8))}), 1,
                                                 KS_OP_NOT_IN});
            ksynth::push(s->reqs, ks_requirement{s->intern("feature-" + std::to_string(q.below(8))),
                                                 nullptr, 0, KS_OP_EXISTS});
          }
          if (t == 1) {
            ksynth::push(s->reqs, ks_requirement{s->intern("topology.kubernetes.io/zone"),
                                                 values(s, {"zone-" + std::to_string(q.below(16)),
                                                            "zone-" + std::to_string(q.below(16))}),
                                                 2, KS_OP_IN});
          }
          if (gpu) {
            ksynth::push(s->reqs, ks_requirement{s->intern("gpu-count"), values(s, {"1"}), 1,
                                                 KS_OP_GT});
          }
          if (bad && t == 0) {
            ksynth::push(s->reqs, ks_requirement{s->intern("gpu-count"), values(s, {"two"}), 1,
                                                 KS_OP_LT});
          }
          term.n_expressions =
              (uint32_t)(s->reqs.data() + s->reqs.size() - term.match_expressions);
          if (byname && t == 0) {
            term.match_fields = s->reqs.data() + s->reqs.size();
            ksynth::push(s->reqs,
                         ks_requirement{s->intern("metadata.name"),
                                        values(s, {"kwok-node-" + std::to_string(q.below(1000))}),
                                        1, KS_OP_IN});
            term.n_fields = 1;
          }
          if (term.n_expressions == 0) term.match_expressions = nullptr;
          ksynth::push(s->terms, term);
        }
        p.n_required_terms = (uint32_t)nterms;
      }
      if (q.chance(0.15)) {
        p.has_preferred = 1;
        p.preferred = s->prefs.data() + s->prefs.size();
        int np = 1 + (int)q.below(2);
        for (int t = 0; t < np; ++t) {
          ks_preferred_term pt{};
          pt.weight = 1 + (int32_t)q.below(100);
          pt.preference.match_expressions = s->reqs.data() + s->reqs.size();
          if (t == 0) {
            ksynth::push(s->reqs, ks_requirement{s->intern("topology.kubernetes.io/zone"),
                                                 values(s, {"zone-" + std::to_string(q.below(16)),
                                                            "zone-" + std::to_string(q.below(16)),
                                                            "zone-" + std::to_string(q.below(16)),
                                                            "zone-" + std::to_string(q.below(16))}),
                                                 4, KS_OP_IN});
          } else {
            ksynth::push(s->reqs, ks_requirement{s->intern("feature-" + std::to_string(q.below(8))),
                                                 nullptr, 0, KS_OP_EXISTS});
          }
          pt.preference.n_expressions = 1;
          ksynth::push(s->prefs, pt);
        }
        p.n_preferred = (uint32_t)np;
      }
    }
    p.n_tolerations = (uint32_t)(s->tolerations.data() + s->tolerations.size() - p.tolerations);
    s->pods.push_back(p);
  }
  return s;
}

extern "C" ksynth *ksynth_besteffort_pods(uint32_t n) {
  auto *s = new ksynth();
  reserve_pods(s, n);
  for (uint32_t j = 0; j < n; ++j) {
    ks_pod p = base_pod(s, j, "res-");
    p.containers = ksynth::push(s->containers, ks_container{});
    p.n_containers = 1;
    p.tolerations = s->tolerations.data() + s->tolerations.size();
    kwok_tolerations(s);
    p.n_tolerations = 3;
    s->pods.push_back(p);
  }
  return s;
}

extern "C" ksynth *ksynth_spread_pods(uint32_t n, uint32_t n_apps, uint64_t seed) {
  auto *s = new ksynth();
  reserve_pods(s, n);
  if (n_apps == 0) n_apps = 1;
  for (uint32_t j = 0; j < n; ++j) {
    Rng r(seed, j, 6);
    ks_pod p = base_pod(s, j, "spread-");
    ks_container c;
    draw_requests(r, c);
    p.containers = ksynth::push(s->containers, c);
    p.n_containers = 1;
    p.tolerations = s->tolerations.data() + s->tolerations.size();
    kwok_tolerations(s);
    p.n_tolerations = 3;
    const std::string app = "app-" + std::to_string(r.below(n_apps));
    const ks_label *lab = ksynth::push(s->labels, ks_label{s->intern("app"), s->intern(app)});
    p.labels = lab;
    p.n_labels = 1;
    ks_spread_constraint a{}, b{};
    a.selector.match_labels = lab;
    a.selector.n_match_labels = 1;
    b.selector = a.selector;
    if (r.chance(0.5)) {  // system defaults (podtopologyspread systemDefaultConstraints)
      a.topology_key = s->intern("kubernetes.io/hostname");
      a.max_skew = 3;
      a.when_unsatisfiable = KS_SCHEDULE_ANYWAY;
      b.topology_key = s->intern("topology.kubernetes.io/zone");
      b.max_skew = 5;
      b.when_unsatisfiable = KS_SCHEDULE_ANYWAY;
      p.spread_defaulted = 1;
    } else {
      a.topology_key = s->intern("topology.kubernetes.io/zone");
      a.max_skew = 1;
      a.when_unsatisfiable = KS_DO_NOT_SCHEDULE;
      b.topology_key = s->intern("kubernetes.io/hostname");
      b.max_skew = 1;
      b.when_unsatisfiable = KS_SCHEDULE_ANYWAY;
    }
    p.spread = ksynth::push(s->spread, a);
    ksynth::push(s->spread, b);
    p.n_spread = 2;
    s->pods.push_back(p);
  }
  return s;
}

// Deployment replicas under the system default spread constraints (ksynth.h):
// the replica set's pod template, so a deployment's pods are identical.
static ksynth *deploy_stream(uint32_t n, uint32_t replicas, uint64_t seed, bool dns) {
  auto *s = new ksynth();
  reserve_pods(s, n);
  if (replicas == 0) replicas = 1;
  for (uint32_t j = 0; j < n; ++j) {
    const uint32_t d = j / replicas;
    Rng r(seed, d, 7);  // per deployment: every replica draws the same requests
    ks_pod p = base_pod(s, j, "deploy-");
    ks_container c;
    draw_requests(r, c);
    p.containers = ksynth::push(s->containers, c);
    p.n_containers = 1;
    p.tolerations = s->tolerations.data() + s->tolerations.size();
    kwok_tolerations(s);
    p.n_tolerations = 3;
    const ks_label *lab =
        ksynth::push(s->labels, ks_label{s->intern("app"), s->intern("deploy-" + std::to_string(d))});
    p.labels = lab;
    p.n_labels = 1;
    ks_spread_constraint a{}, b{};
    a.selector.match_labels = lab;
    a.selector.n_match_labels = 1;
    b.selector = a.selector;
    if (dns) {  // the pod's own constraints: zone DoNotSchedule, hostname ScheduleAnyway
      a.topology_key = s->intern("topology.kubernetes.io/zone");
      a.max_skew = 1;
      a.when_unsatisfiable = KS_DO_NOT_SCHEDULE;
      b.topology_key = s->intern("kubernetes.io/hostname");
      b.max_skew = 1;
      b.when_unsatisfiable = KS_SCHEDULE_ANYWAY;
    } else {  // the system defaults
      a.topology_key = s->intern("kubernetes.io/hostname");
      a.max_skew = 3;
      a.when_unsatisfiable = KS_SCHEDULE_ANYWAY;
      b.topology_key = s->intern("topology.kubernetes.io/zone");
      b.max_skew = 5;
      b.when_unsatisfiable = KS_SCHEDULE_ANYWAY;
      p.spread_defaulted = 1;
    }
    p.spread = ksynth::push(s->spread, a);
    ksynth::push(s->spread, b);
    p.n_spread = 2;
    s->pods.push_back(p);
  }
  return s;
}

extern "C" ksynth *ksynth_deploy_pods(uint32_t n, uint32_t replicas, uint64_t seed) {
  return deploy_stream(n, replicas, seed, false);
}

extern "C" ksynth *ksynth_deploy_dns_pods(uint32_t n, uint32_t replicas, uint64_t seed) {
  return deploy_stream(n, replicas, seed, true);
}

// Deployment pods with pod (anti-)affinity (InterPodAffinity, the one-pod
// path): app-k pods with, alternately, required hostname anti-affinity to
// their own app + preferred zone affinity to it (weight 50), and preferred
// hostname anti-affinity to their own app (weight 100) + required zone
// affinity to app-(k+1) (the zoned prefill holds pods of every app).
extern "C" ksynth *ksynth_affinity_pods(uint32_t n, uint32_t n_apps, uint64_t seed) {
  auto *s = new ksynth();
  reserve_pods(s, n);
  if (n_apps == 0) n_apps = 1;
  for (uint32_t j = 0; j < n; ++j) {
    Rng r(seed, j, 7);
    ks_pod p = base_pod(s, j, "aff-");
    ks_container c;
    draw_requests(r, c);
    p.containers = ksynth::push(s->containers, c);
    p.n_containers = 1;
    p.tolerations = s->tolerations.data() + s->tolerations.size();
    kwok_tolerations(s);
    p.n_tolerations = 3;
    const uint32_t k = r.below(n_apps);
    const ks_label *own = ksynth::push(s->labels, ks_label{s->intern("app"), s->intern("app-" + std::to_string(k))});
    const ks_label *next =
        ksynth::push(s->labels, ks_label{s->intern("app"), s->intern("app-" + std::to_string((k + 1) % n_apps))});
    p.labels = own;
    p.n_labels = 1;
    ks_pod_affinity_term a{}, b{};
    a.namespace_selector.is_nil = b.namespace_selector.is_nil = 1;
    a.selector.match_labels = own;
    a.selector.n_match_labels = 1;
    if (j % 2 == 0) {
      a.topology_key = s->intern("kubernetes.io/hostname");
      a.kind = KS_POD_ANTI_AFFINITY_REQUIRED;
      b.selector = a.selector;
      b.topology_key = s->intern("topology.kubernetes.io/zone");
      b.kind = KS_POD_AFFINITY_PREFERRED;
      b.weight = 50;
    } else {
      a.topology_key = s->intern("kubernetes.io/hostname");
      a.kind = KS_POD_ANTI_AFFINITY_PREFERRED;
      a.weight = 100;
      b.selector.match_labels = next;
      b.selector.n_match_labels = 1;
      b.topology_key = s->intern("topology.kubernetes.io/zone");
      b.kind = KS_POD_AFFINITY_REQUIRED;
    }
    p.affinity_terms = ksynth::push(s->affinity, a);
    ksynth::push(s->affinity, b);
    p.n_affinity_terms = 2;
    s->pods.push_back(p);
  }
  return s;
}

extern "C" ksynth *ksynth_prefill(int32_t kind, uint32_t n_nodes, uint64_t nodes_seed,
                                  uint64_t seed, double max_fill) {
  auto *s = new ksynth();
  // First pass: count to reserve exactly.
  std::vector<ks_container> reqs;
  std::vector<uint32_t> slots;
  reqs.reserve((size_t)n_nodes * 6);
  for (uint32_t i = 0; i < n_nodes; ++i) {
    Shape sh = node_shape(kind, nodes_seed, i);
    Rng r(seed, i, 5);
    const double frac = r.unit() * max_fill;
    const int64_t cpu_target = (int64_t)(frac * (double)sh.cpu);
    const int64_t mem_target = (int64_t)(frac * (double)sh.mem);
    int64_t cpu = 0, mem = 0, cnt = 0;
    for (int attempt = 0; attempt < 64 && cnt + 1 < sh.pods; ++attempt) {
      ks_container c;
      draw_requests(r, c);
      int64_t ncpu = cpu + (c.flags ? c.milli_cpu : 100);
      int64_t nmem = mem + (c.flags ? c.memory : 200 * kMi);
      if (ncpu > cpu_target || nmem > mem_target) break;
      cpu = ncpu;
      mem = nmem;
      ++cnt;
      reqs.push_back(c);
      slots.push_back(i);
    }
  }
  reserve_pods(s, reqs.size());
  for (size_t j = 0; j < reqs.size(); ++j) {
    ks_pod p = base_pod(s, (uint32_t)j, "prefill-");
    if (kind == KSYNTH_ZONED) {  // bound pods of 64 apps (spread selectors count them)
      p.labels = ksynth::push(s->labels, ks_label{s->intern("app"), s->intern("app-" + std::to_string(j % 64))});
      p.n_labels = 1;
    }
    p.containers = ksynth::push(s->containers, reqs[j]);
    p.n_containers = 1;
    p.tolerations = s->tolerations.data() + s->tolerations.size();
    kwok_tolerations(s);
    p.n_tolerations = 3;
    s->pods.push_back(p);
  }
  s->slots = std::move(slots);
  return s;
}

extern "C" const ks_node *ksynth_node_array(const ksynth *s, uint32_t *n) {
  if (n) *n = (uint32_t)s->nodes.size();
  return s->nodes.data();
}
extern "C" const ks_pod *ksynth_pod_array(const ksynth *s, uint32_t *n) {
  if (n) *n = (uint32_t)s->pods.size();
  return s->pods.data();
}
extern "C" const uint32_t *ksynth_slots(const ksynth *s, uint32_t *n) {
  if (n) *n = (uint32_t)s->slots.size();
  return s->slots.data();
}
extern "C" void ksynth_free(ksynth *s) { delete s; }

extern "C" uint64_t ksynth_fnv64(const void *data, uint64_t len, uint64_t seed) {
  uint64_t h = 0xcbf29ce484222325ull ^ seed;
  const unsigned char *p = (const unsigned char *)data;
  for (uint64_t i = 0; i < len; ++i) {
    h ^= p[i];
    h *= 0x100000001b3ull;
  }
  return h;
}
