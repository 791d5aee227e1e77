// jacobi_sim.cpp — CPU model of a round's in-order commit, used to size the
// parallel proposal / verify resolve before writing the kernel.
//
// For windows of P pods over a kwok-shaped cluster (libksynth), it computes
// every pod's top-K keys under the round-start state, resolves the round
// sequentially (the serial resolve's rules, §5.1), and then runs the
// proposal / verify fixed point:
//   proposals w_j = first listed key; repeat { every unfixed pod j computes
//   its exact winner given the proposals of the pods before it; the first
//   pod whose winner differs from its proposal (or that stops the round) is
//   fixed; all pods before it are verified; proposals := computed winners }
// and checks that it ends at the sequential result.  Prints per-round pass
// counts, changed proposals per pass and distinct proposed nodes.
// Resource-only scoring (Fit + LeastAllocated + BalancedAllocation + the
// constant TaintToleration), not bit-exact: a model, not a checker.
//
// g++ -O2 -fopenmp -std=c++17 -Iinclude tools/jacobi_sim.cpp
//     -Lk8s-1m_amd/ksched/lib -lksynth -Wl,-rpath,$PWD/k8s-1m_amd/ksched/lib
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "ksynth.h"

struct Node { int64_t acpu, amem, apods, rc, rm, zc, zm, np; };
struct Pod { int64_t rc, rm, zc, zm; };

static Pod pod_req(const ks_pod &p) {
  Pod q{0, 0, 0, 0};
  for (uint32_t c = 0; c < p.n_containers; ++c) {
    const ks_container &k = p.containers[c];
    q.rc += k.milli_cpu;
    q.rm += k.memory;
    q.zc += (k.flags & KS_REQ_HAS_CPU) ? k.milli_cpu : 100;
    q.zm += (k.flags & KS_REQ_HAS_MEMORY) ? k.memory : 200ll * 1024 * 1024;
  }
  return q;
}

static uint64_t key(const Node &n, const Pod &p, uint32_t slot) {
  if (n.np + 1 > n.apods) return 0;
  if (p.rc > 0 && p.rc > n.acpu - n.rc) return 0;
  if (p.rm > 0 && p.rm > n.amem - n.rm) return 0;
  auto la = [](int64_t cap, int64_t req) -> int64_t { return req > cap ? 0 : (cap - req) * 100 / cap; };
  const int64_t l = (la(n.acpu, n.zc + p.zc) + la(n.amem, n.zm + p.zm)) / 2;
  const double fc = std::min(1.0, (double)(n.rc + p.rc) / (double)n.acpu);
  const double fm = std::min(1.0, (double)(n.rm + p.rm) / (double)n.amem);
  const int64_t b = (int64_t)((1.0 - std::abs((fc - fm) / 2)) * 100);
  const int64_t t = l + b + 300;
  return (uint64_t)(t + 1) << 32 | (0xFFFFFFFFu - slot);
}
static uint32_t kslot(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }

struct List { std::vector<uint64_t> keys; uint64_t bound; };

int main(int argc, char **argv) {
  const uint32_t N = argc > 1 ? atoi(argv[1]) : 100000;
  const uint32_t rounds = argc > 2 ? atoi(argv[2]) : 8;
  const uint32_t P = argc > 3 ? atoi(argv[3]) : 256;
  const uint32_t K = argc > 4 ? atoi(argv[4]) : 256;
  const int kind = argc > 5 ? atoi(argv[5]) : KSYNTH_HETERO;
  const double fill = argc > 6 ? atof(argv[6]) : 0.5;
  ksynth *ns = ksynth_nodes(kind, N, 1);
  uint32_t nn;
  const ks_node *na = ksynth_node_array(ns, &nn);
  std::vector<Node> nodes(N);
  for (uint32_t i = 0; i < N; ++i) nodes[i] = {na[i].alloc_milli_cpu, na[i].alloc_memory, na[i].alloc_pods, 0, 0, 0, 0, 0};
  if (fill > 0) {
    ksynth *pf = ksynth_prefill(kind, N, 1, 3, fill);
    uint32_t np;
    const ks_pod *pp = ksynth_pod_array(pf, &np);
    const uint32_t *sl = ksynth_slots(pf, &np);
    for (uint32_t i = 0; i < np; ++i) {
      const Pod q = pod_req(pp[i]);
      Node &n = nodes[sl[i]];
      n.rc += q.rc; n.rm += q.rm; n.zc += q.zc; n.zm += q.zm; n.np += 1;
    }
  }
  ksynth *ps = ksynth_pods(kind == KSYNTH_KWOK ? KSYNTH_KWOK : KSYNTH_HETERO, P * rounds, 2);
  uint32_t npods;
  const ks_pod *pa = ksynth_pod_array(ps, &npods);
  std::vector<Pod> pods(npods);
  for (uint32_t i = 0; i < npods; ++i) pods[i] = pod_req(pa[i]);

  uint32_t start = 0;
  long tot_pass = 0, tot_rounds = 0, hist[64] = {0};
  while (start < npods && tot_rounds < rounds * 2) {
    const uint32_t n = std::min(P, npods - start);
    std::vector<List> L(n);
#pragma omp parallel for schedule(dynamic)
    for (uint32_t j = 0; j < n; ++j) {
      std::vector<uint64_t> all;
      all.reserve(N);
      for (uint32_t s = 0; s < N; ++s) {
        const uint64_t k = key(nodes[s], pods[start + j], s);
        if (k) all.push_back(k);
      }
      const uint32_t m = std::min<uint32_t>(K, all.size());
      std::partial_sort(all.begin(), all.begin() + std::min<size_t>(m + 1, all.size()), all.end(), std::greater<uint64_t>());
      L[j].bound = all.size() > m ? all[m] : 0;
      L[j].keys.assign(all.begin(), all.begin() + m);
    }
    // F_j: pod j's decision given the winners of pods 0..j-1 (win[i], 0 = none)
    auto decide = [&](uint32_t j, const std::vector<uint64_t> &win, bool &stop) -> uint64_t {
      std::unordered_map<uint32_t, Node> mod;
      for (uint32_t i = 0; i < j; ++i) {
        if (!win[i]) continue;
        const uint32_t s = kslot(win[i]);
        auto it = mod.find(s);
        if (it == mod.end()) it = mod.emplace(s, nodes[s]).first;
        Node &x = it->second;
        const Pod &q = pods[start + i];
        x.rc += q.rc; x.rm += q.rm; x.zc += q.zc; x.zm += q.zm; x.np += 1;
      }
      uint64_t ku = 0;
      for (uint64_t k : L[j].keys)
        if (!mod.count(kslot(k))) { ku = k; break; }
      uint64_t bm = 0;
      for (auto &kv : mod) bm = std::max(bm, key(kv.second, pods[start + j], kv.first));
      stop = false;
      if (L[j].keys.empty() && bm == 0) return 0;  // unschedulable (model: no feasible node)
      if (ku) return std::max(ku, bm);
      if (bm > L[j].bound) return bm;
      stop = true;
      return 0;
    };
    // sequential
    std::vector<uint64_t> seq(n, 0);
    uint32_t seq_stop = n;
    for (uint32_t j = 0; j < n; ++j) {
      bool st;
      seq[j] = decide(j, seq, st);
      if (st) { seq_stop = j; break; }
    }
    // proposal / verify
    std::vector<uint64_t> w(n), c(n);
    const int mode = getenv("SIM_MODE") ? atoi(getenv("SIM_MODE")) : 1;
    // greedy matching from pod f on: each pod takes its first listed node no
    // earlier pod (fixed or proposed) takes -- no re-scoring
    std::vector<uint32_t> hint(n, 0xFFFFFFFFu);
    auto greedy = [&](uint32_t from) {
      std::unordered_map<uint32_t, int> taken;
      for (uint32_t i = 0; i < from; ++i) if (w[i]) taken[kslot(w[i])] = 1;
      for (uint32_t j = from; j < n; ++j) {
        uint64_t g = 0;
        if (mode == 2 && hint[j] != 0xFFFFFFFFu && taken.count(hint[j])) { w[j] = c[j]; continue; }
        for (uint64_t k : L[j].keys) if (!taken.count(kslot(k))) { g = k; break; }
        w[j] = g;
        if (g) taken[kslot(g)] = 1;
      }
    };
    if (mode == 0) { for (uint32_t j = 0; j < n; ++j) w[j] = L[j].keys.empty() ? 0 : L[j].keys[0]; }
    else greedy(0);
    uint32_t f = 0, passes = 0, jstop = n;
    std::vector<uint32_t> changed;
    std::vector<size_t> ndistinct;
    while (f < n) {
      ++passes;
      std::vector<char> stp(n, 0);
#pragma omp parallel for schedule(dynamic)
      for (uint32_t j = f; j < n; ++j) {
        bool st;
        c[j] = decide(j, w, st);
        stp[j] = st;
      }
      uint32_t m = f;
      while (m < n && !stp[m] && c[m] == w[m]) ++m;
      if (m < n && stp[m]) { jstop = m; for (uint32_t j = m; j < n; ++j) w[j] = 0; break; }
      uint32_t ch = 0;
      if (mode == 0) { for (uint32_t j = m; j < n; ++j) { ch += c[j] != w[j]; w[j] = c[j]; } }
      else if (m < n) {
        std::vector<uint64_t> old(w);
        if (mode == 2) {
          std::unordered_map<uint32_t, int> tk;
          for (uint32_t j = 0; j < n; ++j) {
            hint[j] = (j > m && c[j] && tk.count(kslot(c[j]))) ? kslot(c[j]) : 0xFFFFFFFFu;
            if (old[j]) tk[kslot(old[j])] = 1;
          }
        }
        w[m] = c[m];
        greedy(m + 1);
        for (uint32_t j = m; j < n; ++j) ch += old[j] != w[j];
      }
      changed.push_back(ch);
      std::unordered_map<uint32_t, int> dd;
      for (uint32_t j = 0; j < n; ++j) if (w[j]) dd[kslot(w[j])]++;
      ndistinct.push_back(dd.size());
      f = m < n ? m + 1 : n;
    }
    // chunked proposal / verify: the fixed prefix's modified
    // nodes are exact for every later pod (Rpre); a chunk's proposals are the
    // greedy matching with Rpre; only in-chunk re-takes can mismatch
    for (uint32_t C : {16u, 32u, 64u}) {
      std::vector<uint64_t> fx(n, 0);
      uint32_t ff = 0, iters = 0, cstop = n;
      while (ff < n) {
        ++iters;
        const uint32_t ce = std::min(n, ff + C);
        std::vector<uint64_t> pr(fx);
        // proposals: decision given fixed prefix + earlier chunk proposals, ignoring in-chunk re-scores
        std::unordered_map<uint32_t, int> fixed_taken;
        for (uint32_t i = 0; i < ff; ++i) if (fx[i]) fixed_taken[kslot(fx[i])] = 1;
        std::unordered_map<uint32_t, int> tk(fixed_taken);
        for (uint32_t j = ff; j < ce; ++j) {
          // Rpre: max over fixed modified nodes at their live state
          std::vector<uint64_t> pre(fx.begin(), fx.begin() + ff);
          pre.resize(j, 0);
          bool st;
          // decide with only the fixed prefix's commits but the chunk's taken set for the list
          std::unordered_map<uint32_t, Node> mod;
          for (uint32_t i = 0; i < ff; ++i) if (fx[i]) {
            const uint32_t s = kslot(fx[i]);
            auto it = mod.find(s);
            if (it == mod.end()) it = mod.emplace(s, nodes[s]).first;
            Node &x = it->second; const Pod &q = pods[start + i];
            x.rc += q.rc; x.rm += q.rm; x.zc += q.zc; x.zm += q.zm; x.np += 1;
          }
          uint64_t rp = 0;
          for (auto &kv : mod) rp = std::max(rp, key(kv.second, pods[start + j], kv.first));
          uint64_t ku = 0;
          for (uint64_t k : L[j].keys) if (!tk.count(kslot(k))) { ku = k; break; }
          uint64_t p = ku ? std::max(ku, rp) : (rp > L[j].bound ? rp : 0);
          pr[j] = p;
          if (p) tk[kslot(p)] = 1;
          (void)st;
        }
        uint32_t m = ff;
        bool stopped = false;
        for (; m < ce; ++m) {
          bool st;
          const uint64_t d = decide(m, pr, st);
          if (st) { stopped = true; break; }
          if (d != pr[m]) { fx[m] = d; break; }
          fx[m] = d;
        }
        if (stopped) { cstop = m; break; }
        ff = m < ce ? m + 1 : ce;
      }
      bool okc = cstop == seq_stop;
      for (uint32_t j = 0; j < seq_stop && okc; ++j) okc = fx[j] == seq[j];
      printf(" C%u:%u%s", C, iters, okc ? "" : "(MISMATCH)");
    }
    // rewin-aware proposals (chunk 64): after the greedy matching, every pod
    // re-scores the nodes lower chunk pods claimed (with those pods' requests)
    // and proposes the best of that and its greedy proposal; R alternations
    // of greedy (rewinners keep their node) and re-score
    for (uint32_t R : {1u, 2u, 3u}) {
      const uint32_t C = 64;
      std::vector<uint64_t> fx(n, 0);
      uint32_t ff = 0, iters = 0, cstop = n;
      while (ff < n) {
        ++iters;
        const uint32_t ce = std::min(n, ff + C);
        std::unordered_map<uint32_t, Node> mod;  // the fixed prefix's nodes, live
        for (uint32_t i = 0; i < ff; ++i) if (fx[i]) {
          const uint32_t s = kslot(fx[i]);
          auto it = mod.find(s);
          if (it == mod.end()) it = mod.emplace(s, nodes[s]).first;
          Node &x = it->second; const Pod &q = pods[start + i];
          x.rc += q.rc; x.rm += q.rm; x.zc += q.zc; x.zm += q.zm; x.np += 1;
        }
        std::vector<uint64_t> rp(n, 0);
        for (uint32_t j = ff; j < ce; ++j)
          for (auto &kv : mod) rp[j] = std::max(rp[j], key(kv.second, pods[start + j], kv.first));
        std::vector<uint64_t> pr(fx);
        std::vector<char> rw(n, 0);  // pr[j] is a rewin
        for (uint32_t r = 0; r < R; ++r) {
          // greedy: the first listed node no lower pod claims (rewinners keep theirs)
          std::unordered_map<uint32_t, int> tk;
          for (uint32_t i = 0; i < ff; ++i) if (fx[i]) tk[kslot(fx[i])] = 1;
          for (uint32_t j = ff; j < ce; ++j) {
            if (!rw[j]) {
              uint64_t ku = 0;
              for (uint64_t k : L[j].keys) if (!tk.count(kslot(k))) { ku = k; break; }
              pr[j] = ku ? std::max(ku, rp[j]) : (rp[j] > L[j].bound ? rp[j] : 0);
            }
            if (pr[j]) tk[kslot(pr[j])] = 1;
          }
          // re-score (in parallel: from this iteration's claims)
          std::vector<uint64_t> np(pr);
          std::vector<char> nrw(n, 0);
          for (uint32_t j = ff; j < ce; ++j) {
            std::unordered_map<uint32_t, Node> ch;
            for (uint32_t i = ff; i < j; ++i) if (pr[i]) {
              const uint32_t s = kslot(pr[i]);
              auto it = ch.find(s);
              if (it == ch.end()) {
                auto m2 = mod.find(s);
                it = ch.emplace(s, m2 != mod.end() ? m2->second : nodes[s]).first;
              }
              Node &x = it->second; const Pod &q = pods[start + i];
              x.rc += q.rc; x.rm += q.rm; x.zc += q.zc; x.zm += q.zm; x.np += 1;
            }
            uint64_t best = 0;
            for (auto &kv : ch) best = std::max(best, key(kv.second, pods[start + j], kv.first));
            if (best > pr[j] && (pr[j] || best > L[j].bound)) { np[j] = best; nrw[j] = 1; }
          }
          pr = np;
          rw = nrw;
          if (getenv("SIM_FINAL")) {
            // final greedy with the rewin as a non-exclusive extra candidate:
            // max(first unclaimed listed node, the rewin key of the re-score)
            std::unordered_map<uint32_t, int> tk2;
            for (uint32_t i = 0; i < ff; ++i) if (fx[i]) tk2[kslot(fx[i])] = 1;
            for (uint32_t j = ff; j < ce; ++j) {
              uint64_t ku = 0;
              for (uint64_t k : L[j].keys) if (!tk2.count(kslot(k))) { ku = k; break; }
              uint64_t g = ku ? std::max(ku, rp[j]) : (rp[j] > L[j].bound ? rp[j] : 0);
              const uint64_t rk2 = rw[j] ? np[j] : 0;
              if (rk2 > g) { g = rk2; rw[j] = 1; } else rw[j] = 0;
              pr[j] = g;
              if (g && !rw[j]) tk2[kslot(g)] = 1;
            }
          }
        }
        uint32_t m = ff;
        bool stopped = false;
        for (; m < ce; ++m) {
          bool st;
          const uint64_t d = decide(m, pr, st);
          if (st) { stopped = true; break; }
          if (d != pr[m]) {
            fx[m] = d;
            if (R == (uint32_t)atoi(getenv("SIM_R") ? getenv("SIM_R") : "1")) {  // why: d / pr claimed by a lower chunk pod (rewin) or not; their list ranks
              bool drw = false, prw = false;
              for (uint32_t i = ff; i < m; ++i) { drw |= pr[i] && kslot(pr[i]) == kslot(d); prw |= pr[i] && kslot(pr[i]) == kslot(pr[m]); }
              int rd = -1, rpp = -1;
              for (size_t q = 0; q < L[m].keys.size(); ++q) { if (kslot(L[m].keys[q]) == kslot(d)) rd = (int)q; if (kslot(L[m].keys[q]) == kslot(pr[m])) rpp = (int)q; }
              fprintf(stderr, "mm pod %u (chunk+%u): d %s rank %d key %llu | pr %s rank %d key %llu | rp %llu\n", m, m - ff,
                      drw ? "REWIN" : (mod.count(kslot(d)) ? "M" : "list"), rd, (unsigned long long)(d >> 32),
                      prw ? "REWIN" : (mod.count(kslot(pr[m])) ? "M" : "list"), rpp, (unsigned long long)(pr[m] >> 32),
                      (unsigned long long)(rp[m] >> 32));
            }
            break;
          }
          fx[m] = d;
        }
        if (stopped) { cstop = m; break; }
        ff = m < ce ? m + 1 : ce;
      }
      bool okc = cstop == seq_stop;
      for (uint32_t j = 0; j < seq_stop && okc; ++j) okc = fx[j] == seq[j];
      printf(" RW%u:%u%s", R, iters, okc ? "" : "(MISMATCH)");
    }
    bool ok = jstop == seq_stop;
    for (uint32_t j = 0; j < seq_stop && ok; ++j) ok = w[j] == seq[j];
    printf("round %ld start %u: seq %u pods, passes %u, changed/pass", tot_rounds, start, seq_stop, passes);
    for (size_t i = 0; i < changed.size() && i < 16; ++i) printf(" %u", changed[i]);
    std::unordered_map<uint32_t, int> sd;
    for (uint32_t j = 0; j < seq_stop; ++j) if (seq[j]) sd[kslot(seq[j])]++;
    uint32_t rewins = 0;
    {
      std::unordered_map<uint32_t, int> tk;
      for (uint32_t j = 0; j < seq_stop; ++j) {
        if (seq[j] && tk.count(kslot(seq[j]))) ++rewins;
        if (seq[j]) tk[kslot(seq[j])] = 1;
      }
    }
    printf(" rewins %u", rewins);
    {
      uint32_t dmax = 0; double dsum = 0; uint32_t cnt = 0, d64 = 0, d32 = 0;
      for (uint32_t j = 0; j < seq_stop; ++j) {
        uint32_t d = 0;
        for (; d < L[j].keys.size(); ++d) if (L[j].keys[d] == seq[j]) break;
        if (d == L[j].keys.size()) continue;  // rewin of a node not listed at this depth
        dmax = std::max(dmax, d); dsum += d; ++cnt; d64 += d >= 64; d32 += d >= 32;
      }
      printf(" depth mean %.1f max %u >=32 %u >=64 %u", dsum / std::max(1u, cnt), dmax, d32, d64);
    }
    uint32_t firstwin = 0;
    for (uint32_t j = 0; j < seq_stop; ++j) firstwin += !L[j].keys.empty() && seq[j] == L[j].keys[0];
    printf(" | distinct %zu, seq distinct %zu, first-listed wins %u %s\n", ndistinct.empty() ? 0 : ndistinct[0], sd.size(), firstwin, ok ? "OK" : "MISMATCH");
    hist[std::min<uint32_t>(passes, 63)]++;
    tot_pass += passes;
    ++tot_rounds;
    // commit the sequential result
    for (uint32_t j = 0; j < seq_stop; ++j)
      if (seq[j]) {
        Node &x = nodes[kslot(seq[j])];
        const Pod &q = pods[start + j];
        x.rc += q.rc; x.rm += q.rm; x.zc += q.zc; x.zm += q.zm; x.np += 1;
      }
    start += seq_stop;
  }
  printf("mean passes %.2f over %ld rounds\n", (double)tot_pass / tot_rounds, tot_rounds);
  return 0;
}
