// ksched_kernels.hip — gfx950 kernels of the dist-scheduler shard hot path.
//
// One scheduling ROUND evaluates a window of P pending pods against the node
// snapshot and then commits them in queue order:
//
//   sweep     Filter + Score of every (pod, node) pair; per pod and block the
//             best BLOCK_KEYS packed keys plus a bound      -> BlockRec
//   merge     per pod: blocks -> sorted candidate prefix    -> shard record
//   [normalising plugins: RCCL all-reduce(max) of the measured maxima,
//    norm_check, FIX-mode sweep + merge of the pods scored with a wrong guess]
//   [RCCL all-gather of shard records across GPUs]
//   merge_shards  per pod: shards -> final candidate prefix
//   resolve   one workgroup walks the window in order; pod i's winner is the
//             best of (a) its first listed candidate not modified by pods < i
//             and (b) every modified node re-scored against the live state.
//             If neither is provably the max the round ends at pod i.
//
// Exact arithmetic: int64 resource checks; the
// LeastAllocated quotient floor((cap-req)*100/cap) is computed in binary64 and
// corrected with an exact FMA remainder (all operands < 2^53); the
// BalancedAllocation fractions use IEEE binary64 division; compiled with
// -ffp-contract=off so that no product/sum is fused.  References:
// upstream k8s.io/kubernetes v1.31.3 pkg/scheduler/framework/plugins/
// noderesources/{fit.go, least_allocated.go, balanced_allocation.go,
// resource_allocation.go}, tainttoleration/taint_toleration.go,
// nodeaffinity/node_affinity.go, helper/normalize_score.go.
#include <hip/hip_runtime.h>

#include <utility>

#include "ksched_dev.hpp"
#include "ksched_eval.hpp"
#include "ksched_kernels.hpp"
#include "ksched_instr.hpp"
#include "ksched_util.hpp"

namespace ks {

// ============================================================ device helpers



// A wave-uniform pod descriptor.  SCALAR (the resource-only sweep): through
// the constant address space, i.e. s_load into SGPRs -- the generic pointer
// gave three vector loads per pod and a compare + readfirstlane per request
// test (round 5: C3 sweep 0.358 -> 0.355 ms).  The EXT sweep keeps the
// generic load (the copy took 48 B of scratch there).  Batches are never
// written while kernels read them.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) u32x4 *const_words;
template <bool SCALAR = false>
__device__ __forceinline__ PodDev load_pod(const PodDev *pods, uint32_t i) {
  if constexpr (SCALAR) {
    const const_words src = (const_words)(pods + i);
    u32x4 w[sizeof(PodDev) / 16];
#pragma unroll
    for (int k = 0; k < (int)(sizeof(PodDev) / 16); ++k) w[k] = src[k];
    PodDev p;
    __builtin_memcpy(&p, w, sizeof p);
    return p;
  } else {
    return pods[i];
  }
}


// ------------------------------------------------ sweep: EXT pods, NPL nodes
// The sweep evaluates a pod's label programs term-outer, node-inner: each
// term's words are read once per pod (scalar loads) and applied to the
// lane's NPL nodes.  Label words beyond the dictionary's (LWU, a template
// parameter) are not read: straight-line AND / XOR / OR over the words in
// use, no per-word branches.  Results are 0 / 1 vector values.
template <int NPL, int LWU>
__device__ __forceinline__ const uint64_t *term_pass_n(const uint64_t *t, const NodeExt (&e)[NPL],
                                                       const NodeRegs (&nr)[NPL], uint32_t (&ok)[NPL]) {
  const uint64_t w0 = t[0];
  const uint32_t ng = uniform_u32((uint32_t)w0 & 0xFF), nn = uniform_u32(((uint32_t)w0 >> 8) & 0xFF),
                 nm = uniform_u32(((uint32_t)w0 >> 16) & 0xFF);
  uint64_t must[LWU], mf[LWU];
#pragma unroll
  for (int k = 0; k < LWU; ++k) {
    must[k] = t[1 + k];
    mf[k] = t[1 + LW + k];
  }
  static_for<NPL>([&](auto J) {
    constexpr int j = J;
    uint64_t diff = 0;
#pragma unroll
    for (int k = 0; k < LWU; ++k) diff |= (e[j].lab[k] & mf[k]) ^ must[k];
    ok[j] = diff == 0 ? 1u : 0u;
  });
  const uint64_t *g = t + TERM_HDR_WORDS;
  for (uint32_t i = 0; i < ng; ++i, g += LW) {
    uint64_t gm[LWU];
#pragma unroll
    for (int k = 0; k < LWU; ++k) gm[k] = g[k];
    static_for<NPL>([&](auto J) {
      constexpr int j = J;
      uint64_t any = 0;
#pragma unroll
      for (int k = 0; k < LWU; ++k) any |= e[j].lab[k] & gm[k];
      ok[j] &= any != 0 ? 1u : 0u;
    });
  }
  for (uint32_t i = 0; i < nn; ++i, g += 2) {  // rare: Gt / Lt
    const bool col1 = g[0] & 0xFF, gt = ((g[0] >> 8) & 0xFF) == TO_GT;
    const int64_t x = (int64_t)g[1];
    static_for<NPL>([&](auto J) {
      constexpr int j = J;
      const int64_t v = col1 ? e[j].num[1] : e[j].num[0];
      ok[j] &= (gt ? v > x : v < x) ? 1u : 0u;
    });
  }
  for (uint32_t i = 0; i < nm; ++i, g += 2) {  // rare: metadata.name
    const bool in = g[0] == TO_NAME_IN;
    const int64_t x = (int64_t)g[1];
    static_for<NPL>([&](auto J) {
      constexpr int j = J;
      ok[j] &= (((int64_t)nr[j].slot == x) == in) ? 1u : 0u;
    });
  }
  return g;
}

// required_match for NPL nodes at once
template <int NPL, int LWU>
__device__ __forceinline__ void required_match_n(const PodDev &p, const uint64_t *prog, const NodeExt (&e)[NPL],
                                                 const NodeRegs (&nr)[NPL], bool (&out)[NPL]) {
  uint32_t any[NPL];
  static_for<NPL>([&](auto J) { any[J] = 0u; });
  const uint64_t *t = prog + p.req_off;
  for (uint32_t k = 0; k < p.req_len; ++k) {
    uint32_t ok[NPL];
    t = term_pass_n<NPL, LWU>(t, e, nr, ok);
    static_for<NPL>([&](auto J) { any[J] |= ok[J]; });
  }
  static_for<NPL>([&](auto J) { out[J] = any[J] != 0u; });
}

// preferred_raw for NPL nodes at once
template <int NPL, int LWU>
__device__ __forceinline__ void preferred_raw_n(const PodDev &p, const uint64_t *prog, const NodeExt (&e)[NPL],
                                                const NodeRegs (&nr)[NPL], uint32_t (&raw)[NPL]) {
  static_for<NPL>([&](auto J) { raw[J] = 0u; });
  const uint64_t *t = prog + p.pref_off;
  for (uint32_t k = 0; k < p.pref_len; ++k) {
    const uint32_t w = uniform_u32((uint32_t)(t[0] >> 32));
    uint32_t ok[NPL];
    t = term_pass_n<NPL, LWU>(t, e, nr, ok);
    static_for<NPL>([&](auto J) { raw[J] += ok[J] * w; });
  }
}

// DefaultNormalizeScore's floor(100 * raw / max) for 0 <= raw <= max < 2^25
// from inv = RN(1 / max) (0 for max == 0, giving 0): the product is within
// 2^-44 of the quotient (<= 100), whose fractional part is 0 or >= 2^-25, so
// 2^-40 lifts exact quotients above the rounding error without reaching the
// next integer: truncation is the exact floor.
constexpr double NORM_EPS = 0x1p-40;
__device__ __forceinline__ uint32_t normalize_inv(uint32_t raw, double inv) {
  return (uint32_t)__builtin_fma((double)(100u * raw), inv, NORM_EPS);
}


// =================================================================== sweep
// Normalising plugins (TaintToleration with PreferNoSchedule taints, NodeAffinity
// preferred terms) score against max raw over the feasible nodes, which is
// only known after the sweep.  The sweep scores with the pod's guess of it
// (PodDev::tt_guess / na_guess) and measures the true maxima on the way; the
// merge reduces them and norm_check flags the pods whose guess was wrong,
// which a second, FIX-mode launch re-sweeps with the measured maxima.  With a
// right guess (the usual case) one pass over the nodes suffices.
// grid: x = block within shard, y = pod group, z = local shard.
constexpr uint32_t KEY32_POS_BITS = 9, KEY32_POS_MASK = (1u << KEY32_POS_BITS) - 1;

template <int NPL, bool EXT, int LWU = LW>
// EXT with 2 nodes per lane: 5 waves per SIMD (91 VGPRs) runs the C4 sweep
// 5 % faster than 4 (103 VGPRs); 6 waves spill 72 B; the resource-only
// kernel at 5 waves spills 20 B and measured 9 % slower (kept at 4)
__global__ __launch_bounds__(SWEEP_THREADS) __attribute__((amdgpu_waves_per_eu(EXT && NPL == 2 ? 5 : 1)))
void sweep_kernel(RoundArgs a) {
  static_assert(NPL * WAVE <= (1 << KEY32_POS_BITS), "wave-local key position field");
  constexpr int NW = SWEEP_THREADS / WAVE;
  __shared__ uint64_t s_keys[MAX_PG][NW][3];
  // per pod and wave: feasible, first failures per plugin, #at max (tt, na), max raw (tt, na)
  constexpr int NCNT = NFILT + 5;
  __shared__ uint32_t s_cnt[MAX_PG][NW][NCNT];

  const uint32_t start = uniform_u32(*a.sstart);
  const uint32_t sh = blockIdx.z;
  const Shard s = a.shards[a.shard0 + sh];
  const uint32_t wid = threadIdx.x / WAVE;
  const uint32_t kw = blockIdx.x * NW + wid;  // kernel wave
  const uint32_t kwaves = s.waves * a.sub;
  const uint32_t lane = threadIdx.x % WAVE;
  const uint32_t lwave = kw / a.sub, j0 = (kw % a.sub) * NPL;  // layout wave / first step
  const uint32_t p0 = start + blockIdx.y * a.pg;
  uint32_t p1 = min(min(p0 + a.pg, start + a.P), a.npods);
  // FIX mode: only the pods norm_check flagged (pod groups of MAX_PG)
  const bool fix = EXT && a.fix;
  // identical pods: the groups walk the round's representatives (ulist)
  const bool dedup = !fix && a.ulist != nullptr;
  if (dedup) p1 = min(p1, start + uniform_u32(*a.nuniq));
  if (p0 >= p1 || blockIdx.x * NW >= kwaves) return;
  if (fix && uniform_u32(a.fix_group[blockIdx.y]) == 0) return;

  NodeRegs nr[NPL];
  NodeExt ne[EXT ? NPL : 1];
  static_for<NPL>([&](auto J) {
    constexpr int j = J;
    const uint32_t l = (j0 + (uint32_t)j) * WAVE * s.waves + lane * s.waves + lwave;
    const uint32_t pos = s.base + kw * WAVE * NPL + (uint32_t)j * WAVE + lane;
    load_core(a.t, pos, s.lo + l, kw < kwaves && l < s.count, nr[j]);
    if constexpr (EXT) load_ext<LWU>(a.t, pos, nr[j].bits & 1u, ne[j]);
  });

  // per node, pod-independent: pod-count fit (also false for empty slots), and
  // the wave-local key position ~(step * 64 + lane)
  bool podfit[NPL];
  uint64_t podfit_m[NPL];  // as wave masks (SGPR pairs)
  uint32_t vcount = 0;  // valid nodes of the wave
  static_for<NPL>([&](auto J) {
    constexpr int j = J;
    podfit[j] = nr[j].bits & 2u;
    podfit_m[j] = __builtin_amdgcn_ballot_w64(podfit[j]);
    vcount += popc_ballot(nr[j].bits & 1u);
  });
  const uint32_t kpos0 = KEY32_POS_MASK - lane;
  // resource-only batches: the pod-independent part of each node's key,
  // (TaintToleration 100 * weight + 1) << 9 | ~(step * 64 + lane)
  uint32_t kc[EXT ? 1 : NPL];
  const uint32_t wf9 = (uint32_t)a.w.fit << KEY32_POS_BITS, wb9 = (uint32_t)a.w.ba << KEY32_POS_BITS;
  const uint32_t wt9 = (uint32_t)a.w.tt << KEY32_POS_BITS, wn9 = (uint32_t)a.w.na << KEY32_POS_BITS;
  const uint32_t kpos1 = (1u << KEY32_POS_BITS) + kpos0;  // the + 1 of the key, and the position
  if constexpr (!EXT) {
    const uint32_t cplus = (uint32_t)(a.w.tt * 100) + 1u;
    static_for<NPL>([&](auto J) { kc[J] = (cplus << KEY32_POS_BITS) + (kpos0 - (uint32_t)J * WAVE); });
  }

  for (uint32_t it = p0; it < p1; ++it) {
    // FIX mode: slice entry it - start of the compacted flagged-pod list
    const uint32_t r = fix ? uniform_u32(a.fix_list[it - start]) : dedup ? uniform_u32(a.ulist[it - start]) : it - start;
    if (fix && r == FIX_NONE) continue;
    const uint32_t pi = start + r;
    const PodDev p = load_pod<!EXT>(a.pods, pi);
    uint32_t tt_max = 0, na_max = 0;
    if (EXT && (p.flags & (PF_TT | PF_NA))) {
      tt_max = uniform_u32(fix ? a.norm_max[2 * r + 0] : p.tt_guess);
      na_max = uniform_u32(fix ? a.norm_max[2 * r + 1] : p.na_guess);
    }
    // lane top-2 of wave-local 32-bit keys (TotalScore + 1) << 9 | ~(step * 64 + lane):
    // within a wave slot order is (step, lane) order, so these sort like packed keys
    uint32_t b1 = 0, b2 = 0;
    uint32_t feas = 0, f0 = 0, f1 = 0, f2 = 0, f3 = 0, f4 = 0, ttc = 0, nac = 0;
    uint32_t tmx = 0, nmx = 0;  // max raw over this lane's feasible nodes
    uint64_t over_m = 0;        // lanes where a feasible node's raw score exceeds the max used
    if constexpr (!EXT) {
      // Resource-only pods: only NodeResourcesFit can fail (a batch without
      // PF_EXT pods tolerates every hard taint and names no node).  A zero
      // request skips its check (fitsRequest), encoded as a -inf request.
      // (requests are >= 0, compile_pod refuses others: `!= 0` is a SALU
      // compare where `> 0` is a 64-bit VALU one; PF_HAS_REQ is implied)
      // Fit as Requested + request > Allocatable on the sums BalancedAllocation
      // divides (exact integers in binary64), so the free columns need no
      // registers; a zero request's check is masked off (all-ones lane mask)
      // (lane masks of the wave-uniform conditions: SGPR pairs)
      const uint64_t zc = __builtin_amdgcn_ballot_w64(p.req_cpu == 0), zm = __builtin_amdgcn_ballot_w64(p.req_mem == 0);
      static_for<NPL>([&](auto J) {
        constexpr int j = J;
        const double sc = nr[j].rcpu + p.req_cpu_d, sm = nr[j].rmem + p.req_mem_d;
        // the wave's feasibility mask, ANDed from the compares' lane masks
        // (SALU), selects the key and is counted by s_bcnt1: a bool here
        // made the compiler copy the mask through a VGPR per node
        const uint64_t fm = podfit_m[j] & (zc | __builtin_amdgcn_ballot_w64(!(sc > nr[j].acpu_d))) &
                            (zm | __builtin_amdgcn_ballot_w64(!(sm > nr[j].amem_d)));
        // key = (w_fit LA + w_ba BA) << 9 + kc[j]: two 24-bit multiply-adds
        // with the weights pre-shifted (10000 << 9 < 2^24; the key < 2^31)
        const uint32_t key = sel_mask(fm, wmad_s(wf9, (uint32_t)score_la(p, nr[j]),
                                                 wmad_s(wb9, (uint32_t)score_ba_sum(sc, sm, nr[j]), kc[j])));
        b2 = max(b2, min(b1, key));
        b1 = max(b1, key);
        feas += (uint32_t)__popcll(fm);
      });
      f4 = vcount - feas;
    } else {
      // label programs once per pod for the lane's NPL nodes
      bool aff[NPL], pre[NPL];
      uint32_t praw[NPL];
      static_for<NPL>([&](auto J) { aff[J] = true; pre[J] = true; praw[J] = 0u; });
      if (p.flags & PF_AFF) required_match_n<NPL, LWU>(p, a.clauses, ne, nr, aff);
      if (p.flags & PF_PREFILTER) {  // rare: pods naming their nodes by metadata.name
        static_for<NPL>([&](auto J) { pre[J] = false; });
        for (uint32_t k = 0; k < p.pre_len; ++k) {
          const uint64_t x = a.clauses[p.pre_off + k];
          static_for<NPL>([&](auto J) { pre[J] |= (uint64_t)nr[J].slot == x; });
        }
      }
      const bool conflict = p.flags & PF_NA_CONFLICT;
      if (p.flags & PF_NA) preferred_raw_n<NPL, LWU>(p, a.clauses, ne, nr, praw);
      const double *ip = fix ? a.norm_inv + 2 * r : a.guess_inv + 2 * (size_t)pi;  // RN(1 / max)
      const double inv_tt = (p.flags & PF_TT) ? ip[0] : 0.0;
      const double inv_na = (p.flags & PF_NA) ? ip[1] : 0.0;
      // request > Allocatable - Requested as Requested + request > Allocatable
      // (exact integers in binary64): the sums BalancedAllocation divides,
      // so the free columns need no registers (96 -> 91 VGPRs, no spill at 5 waves)
      const bool hc = p.req_cpu != 0, hm = p.req_mem != 0;  // as rq_c / rq_m above
      const bool ext = p.flags & PF_EXT;
      const bool named = p.name_slot != -1;
      static_for<NPL>([&](auto J) {
        constexpr int j = J;
        const bool valid = nr[j].bits & 1u;
        // filter chain in profile order (NodeUnschedulable, NodeName,
        // TaintToleration, NodeAffinity, NodeResourcesFit), branch-free:
        // every lane scores its node and the feasibility mask selects
        int st = ST_FEASIBLE;
        const double sc = nr[j].rcpu + p.req_cpu_d, sm = nr[j].rmem + p.req_mem_d;
        const bool fitfail = !podfit[j] || (hc && sc > nr[j].acpu_d) || (hm && sm > nr[j].amem_d);
        if (fitfail) st = 4;
        if (ext) {
          const uint64_t untol = ne[j].hard & ~p.tol_hard;
          if (!aff[j]) st = 3;
          if (untol) st = 2;
          if (named && (int64_t)nr[j].slot != (int64_t)p.name_slot) st = 1;
          if (untol & UNSCHED_BIT) st = 0;
          if (conflict) st = 3;
          if (!pre[j]) st = ST_PREFILTERED;  // not evaluated, no plugin blamed
        }
        if (!valid) st = ST_EMPTY;
        const bool feasible = st == ST_FEASIBLE;
        // feasibility and the normaliser tallies as wave masks (SGPR pairs):
        // bools here are copied through VGPRs and compared again per node
        const uint64_t fb = __builtin_amdgcn_ballot_w64(feasible);
        // key = (TotalScore + 1) << 9 | position, accumulated by 24-bit
        // multiply-adds with pre-shifted weights (10000 << 9 < 2^24; < 2^31)
        uint32_t acc = kpos1 - (uint32_t)j * WAVE;
        uint32_t tts = 100u;
        if (p.flags & PF_TT) {
          const uint32_t raw = (uint32_t)__popcll(ne[j].prefer & ~p.tol_prefer);
          tts = 100u - normalize_inv(raw, inv_tt);
          ttc += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(raw == tt_max) & fb);
          over_m |= __builtin_amdgcn_ballot_w64(raw > tt_max) & fb;
          tmx = max(tmx, feasible ? raw : 0u);
        }
        acc = wmad_s(wt9, tts, acc);
        if (p.flags & PF_NA) {  // (PF_HAS_PREF without PF_NA scores 0)
          const uint32_t nas = normalize_inv(praw[j], inv_na);
          nac += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(praw[j] == na_max) & fb);
          over_m |= __builtin_amdgcn_ballot_w64(praw[j] > na_max) & fb;
          nmx = max(nmx, feasible ? praw[j] : 0u);
          acc = wmad_s(wn9, nas, acc);
        }
        acc = wmad_s(wb9, (uint32_t)score_ba_sum(sc, sm, nr[j]), acc);
        acc = wmad_s(wf9, (uint32_t)score_la(p, nr[j]), acc);
        const uint32_t key = sel_mask(fb, acc);
        b2 = max(b2, min(b1, key));
        b1 = max(b1, key);
        const uint64_t vb = __builtin_amdgcn_ballot_w64(valid);
        feas += (uint32_t)__popcll(fb);
        if (fb != vb) {  // some node failed a filter: per-plugin diagnosis counts
          f0 += popc_ballot(st == 0);
          f1 += popc_ballot(st == 1);
          f2 += popc_ballot(st == 2);
          f3 += popc_ballot(st == 3);
          f4 += popc_ballot(st == 4);
        }
      });
    }
    if (EXT && (p.flags & (PF_TT | PF_NA))) {
      // the wave's max raw is the max used when some feasible node reaches it
      // and none exceeds it (the usual case): reduce only otherwise
      const bool exceeded = over_m != 0;
      if (p.flags & PF_TT) tmx = (!exceeded && ttc) ? tt_max : wave_max_u32_dpp(tmx);
      if (p.flags & PF_NA) nmx = (!exceeded && nac) ? na_max : wave_max_u32_dpp(nmx);
    }
    const uint32_t best = b1, second = b2;
    // Wave list: the lane bests above every lane's second best (top 2) + bound,
    // DPP reductions, skipping those the candidate count makes unnecessary.
    uint32_t bound32 = wave_max_u32_dpp(second);
    uint32_t c = best > bound32 ? best : 0u;
    const uint32_t ncand = popc_ballot(c != 0u);
    uint32_t c1 = 0, c2 = 0;
    if (ncand) {
      c1 = wave_max_u32_dpp(c);
      if (ncand > 1) {
        if (c == c1) c = 0;
        c2 = wave_max_u32_dpp(c);
        if (ncand > 2) {
          if (c == c2) c = 0;
          bound32 = max(bound32, wave_max_u32_dpp(c));
        }
      }
    }
    if (lane == 0) {
      // back to packed keys ((score + 1) << 32 | ~slot)
      auto widen = [&](uint32_t k) -> uint64_t {
        if (!k) return 0ull;
        const uint32_t q = KEY32_POS_MASK - (k & KEY32_POS_MASK);
        const uint32_t slot = s.lo + (j0 + q / WAVE) * WAVE * s.waves + (q % WAVE) * s.waves + lwave;
        return ((uint64_t)(k >> KEY32_POS_BITS) << 32) | (uint64_t)(0xFFFFFFFFu - slot);
      };
      const uint64_t k1 = widen(c1), k2 = widen(c2), bound = widen(bound32);
      const uint32_t pl = it - p0;
      s_keys[pl][wid][0] = k1;
      s_keys[pl][wid][1] = k2;
      s_keys[pl][wid][2] = bound;
      s_cnt[pl][wid][0] = feas;
      s_cnt[pl][wid][1] = f0;
      s_cnt[pl][wid][2] = f1;
      s_cnt[pl][wid][3] = f2;
      s_cnt[pl][wid][4] = f3;
      s_cnt[pl][wid][5] = f4;
      s_cnt[pl][wid][6] = ttc;
      s_cnt[pl][wid][7] = nac;
      s_cnt[pl][wid][8] = tmx;
      s_cnt[pl][wid][9] = nmx;
    }
  }
  __syncthreads();
  // Block list per pod: top BLOCK_KEYS of the 4 wave lists above every bound.
  const uint32_t npl = p1 - p0;
  for (uint32_t pl = threadIdx.x; pl < npl; pl += blockDim.x) {
    const uint32_t r = fix ? a.fix_list[p0 + pl - start] : dedup ? a.ulist[p0 + pl - start] : p0 + pl - start;
    if (fix && r == FIX_NONE) continue;
    uint64_t k[2 * NW];
    uint64_t bound = 0;
    const uint32_t nwaves = min((uint32_t)NW, kwaves - blockIdx.x * NW);
    static_for<NW>([&](auto W) {
      constexpr int w = W;
      const bool on = (uint32_t)w < nwaves;
      k[2 * w] = on ? s_keys[pl][w][0] : 0ull;
      k[2 * w + 1] = on ? s_keys[pl][w][1] : 0ull;
      const uint64_t b = on ? s_keys[pl][w][2] : 0ull;
      bound = b > bound ? b : bound;
    });
    sort8_desc(k);
    bound = max(bound, k[BLOCK_KEYS]);
    const uint32_t nk = 2 * NW;
    BlockRec br;
#pragma unroll
    for (int i = 0; i < BLOCK_KEYS; ++i) br.keys[i] = (i < (int)nk && k[i] > bound) ? k[i] : 0ull;
    br.bound = bound;
    uint32_t cnt[NFILT + 3] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t tmx = 0, nmx = 0;
    for (uint32_t w = 0; w < nwaves; ++w) {
      for (int q = 0; q < NFILT + 3; ++q) cnt[q] += s_cnt[pl][w][q];
      tmx = max(tmx, s_cnt[pl][w][8]);
      nmx = max(nmx, s_cnt[pl][w][9]);
    }
    br.feasible = cnt[0];
    for (int q = 0; q < NFILT; ++q) br.fails[q] = cnt[1 + q];
    br.tt_cnt = cnt[6];
    br.na_cnt = cnt[7];
    br.tt_max = tmx;
    br.na_max = nmx;
    if (EXT && a.pstat_sweep && !fix && cnt[0]) {
      // measured normaliser maxima straight from the sweep, so norm_check and
      // the FIX sweep follow it on its own stream.  Blocks with a feasible node
      // raise tt_max / na_max to max raw + 1 (0: no feasible node anywhere);
      // one coherent 64-bit pre-check keeps the atomics to the few blocks that
      // raise a maximum
      uint32_t *pm = &a.pstat[r].tt_max;  // tt_max, na_max adjacent (8-B aligned)
      const uint64_t cur = __hip_atomic_load((uint64_t *)pm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tmx + 1u > (uint32_t)cur) atomicMax(pm, tmx + 1u);
      if (nmx + 1u > (uint32_t)(cur >> 32)) atomicMax(pm + 1, nmx + 1u);
    }
    a.brec[((size_t)sh * a.P + r) * a.bstride + blockIdx.x] = br;
  }
}

// =================================================================== merge
// Bitonic sort (descending) of s[0..m) in LDS, m a power of two: every
// thread takes whole compare-exchange pairs (p -> i, i + j), so a pass over m
// keys is m / 2 exchanges spread over the block, one barrier per pass.
__device__ void bitonic_desc(uint64_t *s, uint32_t m) {
  for (uint32_t k = 2; k <= m; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t p = threadIdx.x; p < m / 2; p += blockDim.x) {
        const uint32_t i = ((p & ~(j - 1)) << 1) | (p & (j - 1));
        const uint64_t x = s[i], y = s[i + j];
        const bool desc = (i & k) == 0;
        if (desc ? (x < y) : (x > y)) { s[i] = y; s[i + j] = x; }
      }
      __syncthreads();
    }
  }
}

__device__ uint64_t block_max_u64(uint64_t v, uint64_t *scratch) {
  v = wave_max_u64(v);
  const uint32_t wid = threadIdx.x / WAVE, nw = (blockDim.x + WAVE - 1) / WAVE;
  __syncthreads();
  if (threadIdx.x % WAVE == 0) scratch[wid] = v;
  __syncthreads();
  uint64_t m = 0;
  for (uint32_t i = 0; i < nw; ++i) m = scratch[i] > m ? scratch[i] : m;
  __syncthreads();
  return m;
}

__device__ uint32_t block_sum_u32(uint32_t v, uint32_t *scratch) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, WAVE);
  const uint32_t wid = threadIdx.x / WAVE, nw = (blockDim.x + WAVE - 1) / WAVE;
  __syncthreads();
  if (threadIdx.x % WAVE == 0) scratch[wid] = v;
  __syncthreads();
  uint32_t s = 0;
  for (uint32_t i = 0; i < nw; ++i) s += scratch[i];
  __syncthreads();
  return s;
}

// Combine `nl` sorted lists of `len` keys (each listing every key above its
// own bound) into one sorted prefix of <= K keys with a single bound.
// Writes header + keys to out.  Uses blockDim.x threads.
__device__ void merge_lists(const uint64_t *keys, size_t list_stride, const uint64_t *bounds,
                            size_t bound_stride, uint32_t nl, uint32_t len, uint32_t K, uint64_t *out,
                            uint64_t *s_sort, uint64_t *s_scr, uint32_t *s_cnt, uint32_t *s_u32) {
  uint64_t b = 0;
  for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x) b = max(b, bounds[i * bound_stride]);
  b = block_max_u64(b, s_scr);
  // Count candidates above the common bound; if more than MERGE_CAP, cut every
  // list to c entries (raising the bound to the largest dropped key).
  uint32_t cnt = 0;
  for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x)
    for (uint32_t q = 0; q < len; ++q) cnt += keys[i * list_stride + q] > b;
  cnt = block_sum_u32(cnt, s_u32);
  if (cnt > MERGE_CAP) {
    const uint32_t c = MERGE_CAP / nl;  // >= 1 whenever nl <= MERGE_CAP
    uint64_t b2 = b;
    for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x)
      if (c < len) b2 = max(b2, keys[i * list_stride + c]);
    b = block_max_u64(b2, s_scr);
  }
  if (threadIdx.x == 0) *s_cnt = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x)
    for (uint32_t q = 0; q < len; ++q) {
      const uint64_t k = keys[i * list_stride + q];
      if (k > b) {
        const uint32_t at = atomicAdd(s_cnt, 1u);
        if (at < MERGE_CAP) s_sort[at] = k;
      }
    }
  __syncthreads();
  const uint32_t n = min(*s_cnt, (uint32_t)MERGE_CAP);
  uint32_t m = 64;
  while (m < n) m <<= 1;
  for (uint32_t i = n + threadIdx.x; i < m; i += blockDim.x) s_sort[i] = 0;
  __syncthreads();
  bitonic_desc(s_sort, m);
  const uint32_t keep = min(n, K);
  if (n > K) b = max(b, s_sort[K]);
  for (uint32_t i = threadIdx.x; i < K; i += blockDim.x) out[REC_HDR_WORDS + i] = i < keep ? s_sort[i] : 0ull;
  if (threadIdx.x == 0) {
    out[0] = b;
    ((uint32_t *)out)[2] = keep;
  }
}

// grid: x = pod in round, y = local shard.  Blocks -> shard record.
constexpr int MERGE_THREADS = 1024;
__global__ __launch_bounds__(MERGE_THREADS) void merge_kernel(RoundArgs a) {
  __shared__ uint64_t s_sort[MERGE_CAP];
  __shared__ uint64_t s_scr[16];
  __shared__ uint32_t s_u32[16];
  __shared__ uint32_t s_cnt;
  __shared__ uint32_t s_wc[MERGE_THREADS / WAVE][NFILT + 5];
  const uint32_t start = uniform_u32(*a.sstart);
  const uint32_t r = blockIdx.x;
  if (start + r >= a.npods || r >= a.P) return;
  if (a.fix && a.fix_flag[r] == 0) return;  // FIX mode: re-merge the re-swept pods only
  if (a.rep != nullptr && a.rep[r] != r) return;  // an identical pod's record serves it
  const uint32_t sh = blockIdx.y;
  const Shard s = a.shards[a.shard0 + sh];
  const uint32_t nb = (s.waves * a.sub + 3) / 4;
  const BlockRec *br = a.brec + ((size_t)sh * a.P + r) * a.bstride;
  uint64_t *out = a.srec + ((size_t)(a.shard0 + sh) * a.P + r) * rec_words(a.K);
  merge_lists(&br[0].keys[0], sizeof(BlockRec) / 8, &br[0].bound, sizeof(BlockRec) / 8, nb, BLOCK_KEYS, a.K,
              out, s_sort, s_scr, &s_cnt, s_u32);
  // counts, and the normalising maxima measured by the sweep: per wave by DPP,
  // then one barrier and thread 0 over the waves
  int32_t c[NFILT + 3];
  for (int q = 0; q < NFILT + 3; ++q) c[q] = 0;
  uint32_t tmx = 0, nmx = 0;
  for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) {
    c[0] += br[i].feasible;
    for (int q = 0; q < NFILT; ++q) c[1 + q] += br[i].fails[q];
    c[6] += br[i].tt_cnt;
    c[7] += br[i].na_cnt;
    tmx = max(tmx, br[i].tt_max);
    nmx = max(nmx, br[i].na_max);
  }
  const uint32_t wid = threadIdx.x / WAVE;
#pragma unroll
  for (int q = 0; q < NFILT + 3; ++q) c[q] = wave_sum_i32_dpp(c[q]);
  tmx = wave_max_u32_dpp(tmx);
  nmx = wave_max_u32_dpp(nmx);
  if (threadIdx.x % WAVE == 0) {
    for (int q = 0; q < NFILT + 3; ++q) s_wc[wid][q] = (uint32_t)c[q];
    s_wc[wid][NFILT + 3] = tmx;
    s_wc[wid][NFILT + 4] = nmx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t[NFILT + 5] = {};
    for (uint32_t w = 0; w < blockDim.x / WAVE; ++w) {
      for (int q = 0; q < NFILT + 3; ++q) t[q] += s_wc[w][q];
      t[NFILT + 3] = max(t[NFILT + 3], s_wc[w][NFILT + 3]);
      t[NFILT + 4] = max(t[NFILT + 4], s_wc[w][NFILT + 4]);
    }
    ShardRecHdr *h = (ShardRecHdr *)out;
    h->feasible = t[0];
    for (int q = 0; q < NFILT; ++q) h->fails[q] = t[1 + q];
    h->tt_cnt = t[6];
    h->na_cnt = t[7];
    if (a.pstat != nullptr && !a.fix && !a.pstat_sweep) {  // across local shards (atomics) and ranks (RCCL all-reduce max)
      PodStat *ps = a.pstat + r;
      if (t[NFILT + 3]) atomicMax(&ps->tt_max, t[NFILT + 3]);
      if (t[NFILT + 4]) atomicMax(&ps->na_max, t[NFILT + 4]);
      if (t[0]) atomicMax(&ps->any_feasible, 1u);
    }
  }
}

// One block: per pod of the round, the normalising maxima the rest of the
// round uses (measured when some node is feasible, else the guess, which is
// then unused) and whether the sweep's guess was wrong (FIX flags, per pod
// and per MAX_PG-pod group; counters[4] counts re-swept pods).

__global__ __launch_bounds__(MAX_P) void norm_check_kernel(RoundArgs a) {
  __shared__ uint32_t s_wn[MAX_P / WAVE];
  const uint32_t start = uniform_u32(*a.sstart);
  const uint32_t r = threadIdx.x;
  bool wrong = false, listed = false;
  if (r < a.P && start + r < a.npods) {
    const PodDev &p = a.pods[start + r];
    // identical pods: the representative's measured maxima (only it was swept)
    const uint32_t rr = a.rep != nullptr ? a.rep[r] : r;
    PodStat st = a.pstat[rr];
    if (a.pstat_sweep) {  // sweep encoding: max raw + 1 over blocks with a feasible node
      st.any_feasible = st.tt_max != 0u;
      st.tt_max = st.tt_max ? st.tt_max - 1u : 0u;
      st.na_max = st.na_max ? st.na_max - 1u : 0u;
    }
    uint32_t tt = p.tt_guess, na = p.na_guess;
    if (st.any_feasible) {
      wrong = ((p.flags & PF_TT) && st.tt_max != tt) || ((p.flags & PF_NA) && st.na_max != na);
      tt = st.tt_max;
      na = st.na_max;
    }
    a.norm_max[2 * r] = tt;
    a.norm_max[2 * r + 1] = na;
    a.norm_inv[2 * r] = tt ? 1.0 / (double)tt : 0.0;
    a.norm_inv[2 * r + 1] = na ? 1.0 / (double)na : 0.0;
    a.fix_flag[r] = wrong ? 1u : 0u;
    if (wrong) mark_pod(a.marks, start + r, MARK_FIX);
    listed = wrong && rr == r;  // the FIX sweep re-sweeps representatives
  }
  // compacted list of the flagged pods (round order): the FIX sweep runs
  // ceil(count / MAX_PG) pod groups, so node rows are re-read once per 64
  // flagged pods rather than once per 64-pod slice holding one
  const uint64_t wb = __ballot(listed);
  const uint32_t nw = (uint32_t)__popcll(wb), nwrong = (uint32_t)__popcll(__ballot(wrong));
  const uint32_t wid = threadIdx.x / WAVE, lane = threadIdx.x % WAVE;
  if (lane == 0) s_wn[wid] = nw;
  if (nwrong && lane == 0) atomicAdd((unsigned long long *)&a.counters[4], (unsigned long long)nwrong);
  __syncthreads();
  uint32_t idx = (uint32_t)__popcll(wb & ((1ull << lane) - 1ull)), total = 0;
#pragma unroll
  for (int w = 0; w < MAX_P / WAVE; ++w) {
    idx += (uint32_t)w < wid ? s_wn[w] : 0u;
    total += s_wn[w];
  }
  if (listed) a.fix_list[idx] = r;
  if (r >= total) a.fix_list[r] = FIX_NONE;
  if (r < MAX_P / MAX_PG) a.fix_group[r] = r * MAX_PG < total ? 1u : 0u;
}

// grid: x = pod in round.  Shard records -> final record.
__global__ __launch_bounds__(256) void merge_shards_kernel(RoundArgs a) {
  __shared__ uint64_t s_sort[MERGE_CAP];
  __shared__ uint64_t s_scr[16];
  __shared__ uint32_t s_u32[16];
  __shared__ uint32_t s_cnt;
  const uint32_t start = uniform_u32(*a.sstart);
  const uint32_t r = blockIdx.x;
  if (start + r >= a.npods || r >= a.P) return;
  if (a.rep != nullptr && a.rep[r] != r) return;
  const uint32_t W = rec_words(a.K);
  const uint64_t *in = a.srec + (size_t)r * W;
  const size_t stride = (size_t)a.P * W;  // between shards
  uint64_t *out = a.frec + (size_t)r * W;
  merge_lists(in + REC_HDR_WORDS, stride, in, stride, a.total_shards, a.K, a.K, out, s_sort, s_scr, &s_cnt, s_u32);
  if (threadIdx.x == 0) {
    ShardRecHdr *h = (ShardRecHdr *)out;
    uint32_t f = 0, ttc = 0, nac = 0, fl[NFILT] = {0, 0, 0, 0, 0};
    for (uint32_t q = 0; q < a.total_shards; ++q) {
      const ShardRecHdr *x = (const ShardRecHdr *)(in + q * stride);
      f += x->feasible;
      ttc += x->tt_cnt;
      nac += x->na_cnt;
      for (int z = 0; z < NFILT; ++z) fl[z] += x->fails[z];
    }
    h->feasible = f;
    h->tt_cnt = ttc;
    h->na_cnt = nac;
    for (int z = 0; z < NFILT; ++z) h->fails[z] = fl[z];
  }
}

// ============================================================ gather rows
__device__ __forceinline__ CandRow cand_row(int64_t acpu, int64_t amem, int64_t rc, int64_t rm, int64_t zc, int64_t zm,
                                            int32_t apods, int32_t np, uint32_t pos) {
  CandRow w;
  w.acpu = (double)acpu;
  w.amem = (double)amem;
  w.inv_cpu = acpu ? 1.0 / w.acpu : 0.0;
  w.inv_mem = amem ? 1.0 / w.amem : 0.0;
  w.rc = (double)rc;
  w.rm = (double)rm;
  w.zc100 = (double)zc * 100.0;  // exact: < 2^51
  w.zm100 = (double)zm * 100.0;
  w.apods = apods;
  w.np = np;
  w.pos = pos;
  w._pad = 0;
  return w;
}

// grid: x = pod in round.  For every listed candidate of the final record,
// copy the node's S0 row (and label / taint columns) next to the key.
template <bool EXT>
__global__ __launch_bounds__(256) void gather_cand_kernel(RoundArgs a) {
  const uint32_t start = uniform_u32(*a.sstart);
  const uint32_t r = blockIdx.x;
  if (start + r >= a.npods || r >= a.P) return;
  if (a.rep != nullptr && a.rep[r] != r) return;
  const uint64_t *rec = a.frec + (size_t)r * rec_words(a.K);
  const uint32_t nk = ((const ShardRecHdr *)rec)->nkeys;
  for (uint32_t t = threadIdx.x; t < nk; t += blockDim.x) {
    const uint64_t k = rec[REC_HDR_WORDS + t];
    const uint32_t pos = a.slot_pos[0xFFFFFFFFu - (uint32_t)k];
    a.crow[(size_t)r * a.K + t] = cand_row(a.t.acpu[pos], a.t.amem[pos], a.t.rcpu[pos], a.t.rmem[pos], a.t.zcpu[pos],
                                           a.t.zmem[pos], a.t.apods[pos], a.t.npods[pos], pos);
    if (EXT) {
      CandExt x;
      x.w[0] = a.t.hard[pos];
      x.w[1] = a.t.prefer[pos];
#pragma unroll
      for (int q = 0; q < LW; ++q) x.w[2 + q] = a.t.lab[(size_t)q * a.t.npos + pos];
#pragma unroll
      for (int q = 0; q < NNUM; ++q) x.w[2 + LW + q] = (uint64_t)a.t.num[(size_t)q * a.t.npos + pos];
      a.cext[(size_t)r * a.K + t] = x;
    }
  }
}

// ================================================================== patch
// Round k's lists were swept while round k-1 was still resolving, so they miss
// round k-1's commits.  Before resolve k, one block per pod re-evaluates the
// nodes round k-1 modified (the carry) under their live rows: list entries of
// those nodes are dropped, their live keys are inserted in key order where they
// exceed the list bound (truncating at K raises the bound), and the feasible /
// per-plugin failure / normaliser-at-max counts are corrected by their status
// change.  Afterwards a pod's list, bound and counts are exact for the state
// resolve k starts from, so the resolve re-scores only its own commits.
// One thread per carried node and per list entry: 256 threads for K <= 256,
// 512 for longer lists (a 512-thread launch of the EXT variant costs 4x the
// time per round on C4, so it is only used when needed).
constexpr int PHASH = 1024;
static_assert(2 * MAX_P >= MAX_K, "patch thread counts");


// #entries of the descending array v[0..n) that are > x
__device__ __forceinline__ uint32_t count_greater(const uint64_t *v, uint32_t n, uint64_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (v[mid] > x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}


template <bool EXT, int PATCH_THREADS>
__global__ __launch_bounds__(PATCH_THREADS) void patch_kernel(RoundArgs a) {
  static_assert(PATCH_THREADS >= MAX_P, "one thread per carried node");
  constexpr int NW = PATCH_THREADS / WAVE;
  __shared__ uint32_t s_hkey[PHASH];
  __shared__ uint64_t s_k1[MAX_P];    // carried nodes' live keys (0: infeasible)
  __shared__ uint64_t s_ckey[MAX_P];  // those above the bound, descending
  __shared__ uint64_t s_lkey[MAX_K];  // surviving list keys, compacted (descending)
  __shared__ uint32_t s_wl[NW], s_wc[NW];
  __shared__ int32_t s_wd[NW][NFILT + 3];
  __shared__ uint64_t s_wdrop[NW];

  const uint32_t tid = threadIdx.x, lane = tid % WAVE, wid = tid / WAVE;
  const uint32_t start = uniform_u32(*a.act);
  const uint32_t r = blockIdx.x;
  if (a.first || start >= a.npods || uniform_u32(*a.sstart) != start || start + r >= a.npods) return;
  if (a.rep != nullptr && uniform_u32(a.rep[r]) != r) return;
  const uint32_t nc = uniform_u32(*a.carry_in_n);
  if (nc == 0) return;
  const PodDev p = load_pod(a.pods, start + r);
  uint64_t *rec = a.frec + (size_t)r * rec_words(a.K);
  ShardRecHdr *hdr = (ShardRecHdr *)rec;
  const uint64_t bound = hdr->bound;
  const uint32_t nk = hdr->nkeys;
  int64_t tt_max = 0, na_max = 0;
  if (EXT) {
    tt_max = a.norm_max[2 * r];
    na_max = a.norm_max[2 * r + 1];
  }
  for (uint32_t i = tid; i < PHASH; i += PATCH_THREADS) s_hkey[i] = 0;
  __syncthreads();

  // (1) carried node tid: its row at the sweep (rc0 / rm0 / np0) and live.
  // No row is held across the barriers below (aggregates kept live across
  // them were put on the stack): step (3) reads the carry record again.
  int32_t d[NFILT + 3] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t k1 = 0;
  if (tid < nc) {
    const CarryRec &cr = a.carry_in[tid];
    NodeExt ce{};
    if (EXT) ext_from_words(cr.ext, ce);
    const double inv_cpu = cr.acpu ? 1.0 / (double)cr.acpu : 0.0, inv_mem = cr.amem ? 1.0 / (double)cr.amem : 0.0;
    const NodeRegs r1 = make_regs_inv(cr.acpu, cr.amem, cr.rc, cr.rm, cr.zc, cr.zm, cr.apods, cr.np, cr.slot,
                                      inv_cpu, inv_mem);
    NodeRegs r0 = r1;
    r0.free_cpu = (double)(cr.acpu - cr.rc0);
    r0.free_mem = (double)(cr.amem - cr.rm0);
    r0.bits = (r1.bits & ~2u) | ((int64_t)cr.np0 + 1 <= (int64_t)cr.apods ? 2u : 0u);
    const int st0 = filter<EXT>(p, a.clauses, r0, ce);
    const int st1 = filter<EXT>(p, a.clauses, r1, ce);
    if (st1 == ST_FEASIBLE) k1 = pack_key(total_score<EXT>(p, a.clauses, r1, ce, a.w, tt_max, na_max), cr.slot);
    if (st0 != st1) status_delta<EXT>(p, a.clauses, st0, st1, ce, cr.slot, tt_max, na_max, d);
    uint32_t h = rhash(cr.slot);
    while (atomicCAS(&s_hkey[h], 0u, cr.slot + 1) != 0u) h = (h + 1) & (PHASH - 1);
  }
  if (tid < MAX_P) s_k1[tid] = k1;
  if (__ballot(d[0] | d[1] | d[2] | d[3] | d[4] | d[5] | d[6] | d[7]) != 0) {
#pragma unroll
    for (int q = 0; q < NFILT + 3; ++q) d[q] = wave_sum_i32_dpp(d[q]);
  }
  if (lane == 0)
    for (int q = 0; q < NFILT + 3; ++q) s_wd[wid][q] = d[q];
  __syncthreads();

  // (2) list entry tid survives unless its node is carried; compaction keeps key order
  // the entry's row and label words, as named 16-byte pieces (arrays or
  // aggregates live across the barriers below stay on the stack)
  static_assert(sizeof(CandRow) == 80 && sizeof(CandExt) == 64, "patch row pieces");
  uint64_t lk = 0;
  bool keep = false;
  uint4 lr0, lr1, lr2, lr3, lr4, lx0, lx1, lx2, lx3;
  if (tid < nk) {
    lk = rec[REC_HDR_WORDS + tid];
    const uint32_t slot = 0xFFFFFFFFu - (uint32_t)lk;
    uint32_t h = rhash(slot);
    keep = true;
    while (s_hkey[h] != 0) {
      if (s_hkey[h] == slot + 1) { keep = false; break; }
      h = (h + 1) & (PHASH - 1);
    }
    if (keep) {
      const uint4 *sr = (const uint4 *)&a.crow[(size_t)r * a.K + tid];
      lr0 = sr[0], lr1 = sr[1], lr2 = sr[2], lr3 = sr[3], lr4 = sr[4];
      if (EXT) {
        const uint4 *sx = (const uint4 *)&a.cext[(size_t)r * a.K + tid];
        lx0 = sx[0], lx1 = sx[1], lx2 = sx[2], lx3 = sx[3];
      }
    }
  }
  const bool cin = k1 > bound;  // carried keys the bound does not cover must be listed
  const uint64_t kb = __ballot(keep), cb = __ballot(cin);
  const uint64_t lt = (1ull << lane) - 1ull;
  if (lane == 0) {
    s_wl[wid] = (uint32_t)__popcll(kb);
    s_wc[wid] = (uint32_t)__popcll(cb);
  }
  __syncthreads();
  uint32_t li = (uint32_t)__popcll(kb & lt), nsurv = 0, ncl = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    li += (uint32_t)w < wid ? s_wl[w] : 0u;
    nsurv += s_wl[w];
    ncl += s_wc[w];
  }
  uint32_t crank = 0;
  if (cin) {
    for (uint32_t c = 0; c < nc; ++c) crank += s_k1[c] > k1;  // > k1 implies above the bound
    s_ckey[crank] = k1;
  }
  if (keep) s_lkey[li] = lk;
  __syncthreads();

  // (3) merged positions; what falls off the end raises the bound
  uint32_t pos_l = 0xFFFFFFFFu, pos_c = 0xFFFFFFFFu;
  uint64_t drop = 0;
  if (keep) {
    pos_l = li + count_greater(s_ckey, ncl, lk);
    if (pos_l >= a.K) drop = lk;
  }
  if (cin) {
    pos_c = crank + count_greater(s_lkey, nsurv, k1);
    if (pos_c >= a.K) drop = max(drop, k1);
  }
  drop = wave_max_u64_dpp(drop);
  if (lane == 0) s_wdrop[wid] = drop;
  __syncthreads();  // every old key / row of this record has been read: rewrite in place
  if (keep && pos_l < a.K) {
    rec[REC_HDR_WORDS + pos_l] = lk;
    uint4 *dr = (uint4 *)&a.crow[(size_t)r * a.K + pos_l];
    dr[0] = lr0, dr[1] = lr1, dr[2] = lr2, dr[3] = lr3, dr[4] = lr4;
    if (EXT) {
      uint4 *dx = (uint4 *)&a.cext[(size_t)r * a.K + pos_l];
      dx[0] = lx0, dx[1] = lx1, dx[2] = lx2, dx[3] = lx3;
    }
  }
  if (cin && pos_c < a.K) {
    const CarryRec &cr = a.carry_in[tid];
    rec[REC_HDR_WORDS + pos_c] = k1;
    a.crow[(size_t)r * a.K + pos_c] = cand_row(cr.acpu, cr.amem, cr.rc, cr.rm, cr.zc, cr.zm, cr.apods, cr.np, cr.pos);
    if (EXT) {
      uint64_t *dx = a.cext[(size_t)r * a.K + pos_c].w;
#pragma unroll
      for (int q = 0; q < 2 + LW + NNUM; ++q) dx[q] = cr.ext[q];
    }
  }
  if (tid == 0) {
    uint64_t nb = bound;
    int32_t sum[NFILT + 3] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int w = 0; w < NW; ++w) {
      nb = max(nb, s_wdrop[w]);
      for (int q = 0; q < NFILT + 3; ++q) sum[q] += s_wd[w][q];
    }
    hdr->bound = nb;
    hdr->nkeys = min(a.K, nsurv + ncl);
    hdr->feasible -= (uint32_t)sum[0];
    for (int q = 0; q < NFILT; ++q) hdr->fails[q] += (uint32_t)sum[1 + q];
    hdr->tt_cnt -= (uint32_t)sum[6];
    hdr->na_cnt -= (uint32_t)sum[7];
  }
}

// ============================================================ pipeline
// Speculative start of round k's sweep, issued once round k-2 is resolved
// (round k-1 may still be resolving): if round k-1's lists were swept for the
// right pods, assume it resolves all of them; otherwise round k-1 resolves
// nothing and round k restarts at its actual start.
__device__ __forceinline__ void advance_kernel_body(const RoundArgs &a) {
  uint32_t s;
  if (a.first) {
    s = *a.d_start;
    *a.act = s;
  } else {
    const uint32_t ps = *a.prev_sstart, pa = *a.prev_act;
    s = ps == pa ? ps + a.P : pa;
  }
  *a.sstart = s;
  if (s < a.npods) a.counters[2] += min(a.P, a.npods - s);  // pods swept
}

// The round window's classes of identical pods (RoundArgs::cls), one block
// of ADV_THREADS >= P threads after the advance: thread r inserts its class
// into an LDS hash with the lowest r as value, reads back its representative,
// and the representatives are compacted in window order (ballot prefix sums).
constexpr int ADV_THREADS = MAX_P;
constexpr uint32_t DHASH = 2 * MAX_P;
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
__device__ void dedup_round(const RoundArgs &a, uint32_t s) {
  __shared__ uint32_t s_k[DHASH], s_v[DHASH], s_wn[ADV_THREADS / WAVE];
  const uint32_t t = threadIdx.x, lane = t % WAVE, wid = t / WAVE;
  for (uint32_t i = t; i < DHASH; i += ADV_THREADS) {
    s_k[i] = NONE32;
    s_v[i] = NONE32;
  }
  __syncthreads();
  const bool valid = t < a.P && s < a.npods && t < a.npods - s;
  const uint32_t key = valid ? a.cls[s + t] : NONE32;
  uint32_t h = (key * 2654435761u) >> 23;  // 9 bits
  if (valid) {
    for (;;) {
      const uint32_t prev = atomicCAS(&s_k[h], NONE32, key);
      if (prev == NONE32 || prev == key) break;
      h = (h + 1) & (DHASH - 1);
    }
    atomicMin(&s_v[h], t);
  }
  __syncthreads();
  const uint32_t rep = valid ? s_v[h] : t;
  const bool u = valid && rep == t;
  const uint64_t ub = __ballot(u);
  if (lane == 0) s_wn[wid] = (uint32_t)__popcll(ub);
  if (t < (uint32_t)MAX_P) a.rep[t] = rep;
  __syncthreads();
  uint32_t idx = (uint32_t)__popcll(ub & ((1ull << lane) - 1ull)), total = 0;
#pragma unroll
  for (int w = 0; w < ADV_THREADS / WAVE; ++w) {
    idx += (uint32_t)w < wid ? s_wn[w] : 0u;
    total += s_wn[w];
  }
  if (u) a.ulist[idx] = t;
  if (t == 0) {
    *a.nuniq = total;
    // counters[2] counts pods swept (the representatives), [7] the duplicates skipped
    const uint32_t window = s < a.npods ? min(a.P, a.npods - s) : 0u;
    a.counters[2] -= window - total;
    a.counters[7] += window - total;
  }
}

__device__ __forceinline__ void advance_block(const RoundArgs &a) {
  __shared__ uint32_t s_s;
  if (threadIdx.x == 0) {
    advance_kernel_body(a);
    s_s = *a.sstart;
  }
  if (a.rep == nullptr) return;
  __syncthreads();
  dedup_round(a, s_s);
}
__global__ __launch_bounds__(ADV_THREADS) void advance_kernel(RoundArgs a) { advance_block(a); }

// advance + write-back in one dispatch (the main stream's per-round prologue)
__global__ __launch_bounds__(ADV_THREADS) void advance_writeback_kernel(RoundArgs a, NodeTable t, const CarryRec *carry,
                                                                        const uint32_t *n) {
  if (blockIdx.x == 0) advance_block(a);
  const uint32_t cnt = *n;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
    const CarryRec &c = carry[i];
    t.rcpu[c.pos] = c.rc;
    t.rmem[c.pos] = c.rm;
    t.zcpu[c.pos] = c.zc;
    t.zmem[c.pos] = c.zm;
    t.npods[c.pos] = c.np;
  }
}

// Land a resolved round's modified rows in the table (before the sweep that
// must see them; never while a sweep that must not see them runs).
__global__ void writeback_kernel(NodeTable t, const CarryRec *carry, const uint32_t *n) {
  const uint32_t cnt = *n;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += gridDim.x * blockDim.x) {
    const CarryRec &c = carry[i];
    t.rcpu[c.pos] = c.rc;
    t.rmem[c.pos] = c.rm;
    t.zcpu[c.pos] = c.zc;
    t.zmem[c.pos] = c.zm;
    t.npods[c.pos] = c.np;
  }
}

// ============================================================ table updates

// Scatter full rows (upsert) into positions.
__global__ void scatter_rows_kernel(NodeTable t, const uint32_t *pos, const int64_t *core, const uint64_t *ext,
                                    uint32_t n, uint32_t flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = pos[i];
  if (!(flags & 2u)) {  // core row (flags 0: core only, 1: core + ext, 2: ext only)
    const int64_t *c = core + (size_t)i * 8;  // acpu amem apods new
    t.acpu[p] = c[0];
    t.amem[p] = c[1];
    t.apods[p] = (int32_t)c[2];
    if (c[3]) {  // new node or delete: reset requested state
      t.rcpu[p] = 0;
      t.rmem[p] = 0;
      t.zcpu[p] = 0;
      t.zmem[p] = 0;
      t.npods[p] = 0;
    }
  }
  if (flags & 3u) {
    const uint64_t *e = ext + (size_t)i * (2 + LW + NNUM);
    t.hard[p] = e[0];
    t.prefer[p] = e[1];
    for (int k = 0; k < LW; ++k) t.lab[(size_t)k * t.npos + p] = e[2 + k];
    for (int k = 0; k < NNUM; ++k) t.num[(size_t)k * t.npos + p] = (int64_t)e[2 + LW + k];
  }
}

// Pod add/remove events: atomic deltas on the requested state.
__global__ void apply_deltas_kernel(NodeTable t, const uint32_t *pos, const int64_t *delta, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = pos[i];
  const int64_t *d = delta + (size_t)i * 5;
  atomicAdd((unsigned long long *)&t.rcpu[p], (unsigned long long)d[0]);
  atomicAdd((unsigned long long *)&t.rmem[p], (unsigned long long)d[1]);
  atomicAdd((unsigned long long *)&t.zcpu[p], (unsigned long long)d[2]);
  atomicAdd((unsigned long long *)&t.zmem[p], (unsigned long long)d[3]);
  atomicAdd(&t.npods[p], (int32_t)d[4]);
}

__global__ void gather_rows_kernel(NodeTable t, const uint32_t *pos, int64_t *out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = pos[i];
  int64_t *o = out + (size_t)i * 8;
  o[0] = t.acpu[p];
  o[1] = t.amem[p];
  o[2] = t.rcpu[p];
  o[3] = t.rmem[p];
  o[4] = t.zcpu[p];
  o[5] = t.zmem[p];
  o[6] = t.apods[p];
  o[7] = t.npods[p];
}

// Full relabel of one label word column (dictionary growth).
__global__ void scatter_u64_kernel(uint64_t *col, const uint32_t *pos, const uint64_t *val, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) col[pos[i]] = val[i];
}

// ============================================================ score dump
// One pod against every position of every shard: per-plugin scores.
__global__ void dump_max_kernel(DumpArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.nslots) return;
  const uint32_t pos = a.slot_pos[i];
  if (pos == 0xFFFFFFFFu) return;
  NodeRegs r;
  NodeExt e;
  load_core(a.t, pos, i, true, r);
  if (!(r.bits & 1u)) return;
  load_ext(a.t, pos, true, e);
  const PodDev p = a.pods[0];
  if (filter<true>(p, a.clauses, r, e) != ST_FEASIBLE) return;
  if (p.flags & PF_TT) atomicMax(&a.norm_max[0], (uint32_t)taint_raw(p, e));
  if (p.flags & PF_NA) atomicMax(&a.norm_max[1], (uint32_t)preferred_raw(p, a.clauses, e, i));
}

__global__ void dump_scores_kernel(DumpArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.nslots) return;
  const uint32_t pos = a.slot_pos[i];
  int32_t *o = a.out + (size_t)i * 10;
  for (int q = 0; q < 10; ++q) o[q] = 0;
  if (pos == 0xFFFFFFFFu) { o[0] = ST_EMPTY; return; }
  NodeRegs r;
  NodeExt e;
  load_core(a.t, pos, i, true, r);
  if (!(r.bits & 1u)) { o[0] = ST_EMPTY; return; }
  load_ext(a.t, pos, true, e);
  const PodDev p = a.pods[0];
  const int st = filter<true>(p, a.clauses, r, e);
  o[0] = st;
  if (st != ST_FEASIBLE) return;
  const int64_t tt_max = a.norm_max[0], na_max = a.norm_max[1];
  o[1] = (int32_t)score_la(p, r);
  o[2] = (int32_t)score_ba(p, r);
  const int64_t tr = (p.flags & PF_TT) ? taint_raw(p, e) : 0;
  o[3] = (int32_t)tr;
  o[4] = (int32_t)normalize(tr, (p.flags & PF_TT) ? tt_max : 0, true);
  const int64_t nr = (p.flags & PF_NA) ? preferred_raw(p, a.clauses, e, i) : 0;
  o[5] = (int32_t)nr;
  o[6] = (p.flags & PF_HAS_PREF) ? (int32_t)normalize(nr, (p.flags & PF_NA) ? na_max : 0, false) : 0;
  o[7] = 0;
  const int64_t tot = total_score<true>(p, a.clauses, r, e, a.w, tt_max, na_max);
  o[8] = (int32_t)(tot & 0xFFFFFFFF);
  o[9] = (int32_t)(tot >> 32);
}

// ============================================================== launchers

#define KS_CHECK(x)                          \
  do {                                       \
    hipError_t e_ = (x);                     \
    if (e_ != hipSuccess) return e_;         \
  } while (0)

hipError_t launch_norm_check(const RoundArgs &a, hipStream_t st) {
  norm_check_kernel<<<1, MAX_P, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_sweep(const RoundArgs &a, bool ext, uint32_t nblocks, uint32_t ngroups, uint32_t nshards,
                        hipStream_t st) {
  dim3 g(nblocks, ngroups, nshards);
  if (ext) {
    // label words in use (dictionary size): 1, 2 or 4 words per node are read
    const int lwu = a.t.lw <= 1 ? 1 : a.t.lw <= 2 ? 2 : 4;
    if (a.npl == 2) {
      if (lwu == 1) sweep_kernel<2, true, 1><<<g, SWEEP_THREADS, 0, st>>>(a);
      else if (lwu == 2) sweep_kernel<2, true, 2><<<g, SWEEP_THREADS, 0, st>>>(a);
      else sweep_kernel<2, true, 4><<<g, SWEEP_THREADS, 0, st>>>(a);
    } else if (a.npl == 4) {
      if (lwu == 1) sweep_kernel<4, true, 1><<<g, SWEEP_THREADS, 0, st>>>(a);
      else if (lwu == 2) sweep_kernel<4, true, 2><<<g, SWEEP_THREADS, 0, st>>>(a);
      else sweep_kernel<4, true, 4><<<g, SWEEP_THREADS, 0, st>>>(a);
    } else {
      sweep_kernel<8, true, 4><<<g, SWEEP_THREADS, 0, st>>>(a);
    }
  } else {
    if (a.npl == 2) sweep_kernel<2, false><<<g, SWEEP_THREADS, 0, st>>>(a);
    else if (a.npl == 4) sweep_kernel<4, false><<<g, SWEEP_THREADS, 0, st>>>(a);
    else sweep_kernel<8, false><<<g, SWEEP_THREADS, 0, st>>>(a);
  }
  return hipGetLastError();
}

hipError_t launch_merge(const RoundArgs &a, uint32_t nshards, hipStream_t st) {
  merge_kernel<<<dim3(a.P, nshards), MERGE_THREADS, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_merge_shards(const RoundArgs &a, hipStream_t st) {
  merge_shards_kernel<<<dim3(a.P), 256, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_gather_cand(const RoundArgs &a, bool ext, hipStream_t st) {
  if (ext) gather_cand_kernel<true><<<a.P, 256, 0, st>>>(a);
  else gather_cand_kernel<false><<<a.P, 256, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_advance(const RoundArgs &a, hipStream_t st) {
  advance_kernel<<<1, ADV_THREADS, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_advance_writeback(const RoundArgs &a, const CarryRec *carry, const uint32_t *n, hipStream_t st) {
  advance_writeback_kernel<<<2, ADV_THREADS, 0, st>>>(a, a.t, carry, n);
  return hipGetLastError();
}

hipError_t launch_writeback(const NodeTable &t, const CarryRec *carry, const uint32_t *n, hipStream_t st) {
  writeback_kernel<<<2, 256, 0, st>>>(t, carry, n);
  return hipGetLastError();
}

hipError_t launch_patch(const RoundArgs &a, bool ext, hipStream_t st) {
  if (a.K <= (uint32_t)MAX_P) {
    if (ext) patch_kernel<true, MAX_P><<<a.P, MAX_P, 0, st>>>(a);
    else patch_kernel<false, MAX_P><<<a.P, MAX_P, 0, st>>>(a);
  } else {
    if (ext) patch_kernel<true, MAX_K><<<a.P, MAX_K, 0, st>>>(a);
    else patch_kernel<false, MAX_K><<<a.P, MAX_K, 0, st>>>(a);
  }
  return hipGetLastError();
}

hipError_t launch_scatter_rows(const NodeTable &t, const uint32_t *pos, const int64_t *core, const uint64_t *ext,
                               uint32_t n, uint32_t flags, hipStream_t st) {
  if (!n) return hipSuccess;
  scatter_rows_kernel<<<(n + 255) / 256, 256, 0, st>>>(t, pos, core, ext, n, flags);
  return hipGetLastError();
}

hipError_t launch_apply_deltas(const NodeTable &t, const uint32_t *pos, const int64_t *delta, uint32_t n,
                               hipStream_t st) {
  if (!n) return hipSuccess;
  apply_deltas_kernel<<<(n + 255) / 256, 256, 0, st>>>(t, pos, delta, n);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const NodeTable &t, const uint32_t *pos, int64_t *out, uint32_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  gather_rows_kernel<<<(n + 255) / 256, 256, 0, st>>>(t, pos, out, n);
  return hipGetLastError();
}

hipError_t launch_scatter_u64(uint64_t *col, const uint32_t *pos, const uint64_t *val, uint32_t n,
                              hipStream_t st) {
  if (!n) return hipSuccess;
  scatter_u64_kernel<<<(n + 255) / 256, 256, 0, st>>>(col, pos, val, n);
  return hipGetLastError();
}

hipError_t launch_dump(const DumpArgs &a, hipStream_t st) {
  const uint32_t g = (a.nslots + 255) / 256;
  dump_max_kernel<<<g, 256, 0, st>>>(a);
  KS_CHECK(hipGetLastError());
  dump_scores_kernel<<<g, 256, 0, st>>>(a);
  return hipGetLastError();
}

__global__ void stall_kernel(uint32_t usec) {
  if (threadIdx.x == 0) stall_for(usec);
}
hipError_t launch_stall(uint32_t usec, hipStream_t st) {
  stall_kernel<<<1, 64, 0, st>>>(usec);
  return hipGetLastError();
}

}  // namespace ks
