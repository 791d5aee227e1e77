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

__device__ __forceinline__ void ext_from_words(const uint64_t *w, NodeExt &e) {
  e.hard = w[0];
  e.prefer = w[1];
#pragma unroll
  for (int q = 0; q < LW; ++q) e.lab[q] = w[2 + q];
#pragma unroll
  for (int q = 0; q < NNUM; ++q) e.num[q] = (int64_t)w[2 + LW + q];
}

// Status change of one node between the row the counts were taken on (st0)
// and its live row (st1), as count corrections: d[0] feasible lost,
// d[1 + q] first failures gained at plugin q, d[6] / d[7] normaliser-at-max lost.
template <bool EXT>
__device__ __forceinline__ void status_delta(const PodDev &p, const uint64_t *clauses, int st0, int st1,
                                            const NodeExt &e, uint32_t slot, int64_t tt_max, int64_t na_max,
                                            int32_t *d) {
  d[0] += (st0 == ST_FEASIBLE) - (st1 == ST_FEASIBLE);
#pragma unroll
  for (int q = 0; q < NFILT; ++q) d[1 + q] += (st1 == q) - (st0 == q);
  if (EXT && (p.flags & PF_TT)) {
    const int at = taint_raw(p, e) == tt_max;
    d[6] += (st0 == ST_FEASIBLE) * at - (st1 == ST_FEASIBLE) * at;
  }
  if (EXT && (p.flags & PF_NA)) {
    const int at = preferred_raw(p, clauses, e, slot) == na_max;
    d[7] += (st0 == ST_FEASIBLE) * at - (st1 == ST_FEASIBLE) * at;
  }
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

// ================================================================= resolve
// One workgroup walks the round's pods in queue order.
// The patched lists are exact for the round's start state, so pod i's winner is
// the best of (a) its first listed candidate that no pod < i modified (its key
// is unchanged: same row, same normalisation max) and (b) every node a pod < i
// modified (the set M_i), re-scored against its live row.  If neither is
// provably the maximum (every listed candidate modified and the best modified
// key not above the list bound), or a normalising plugin's max may have moved,
// the round ends before pod i and the next sweep restarts there.
//
// Software pipeline, one barrier per pod.  M_{i+1} = M_i + {w_i} and pod i
// changes the state of its winner w_i only, so everything pod i+1 needs except
// w_i's new values is computed while pod i is being decided:
//   list waves  (0-3)  pod i+3's first four listed candidates not in M_i; at
//                      most three of them (w_i .. w_{i+2}) are modified by pod
//                      i+3.  Keys and the chosen rows move global -> LDS by
//                      LDS-DMA (global_load_lds) issued three iterations before
//                      they are read, so the loop never waits on global memory
//                      (the next round's sweep keeps the caches cold)
//   owner waves (4-7)  one node of M_i per thread, in registers: its key for
//                      pod i+1 and its filter-status change since the round
//                      start; per wave the best two (key, node) and the summed
//                      status changes
//   eval wave   (8)    every owner / listed candidate of pod i committed: its
//                      key and status change for pod i+1, speculatively, one
//                      candidate per lane (independent of pod i-1's decision)
//   decider     (9)    pod i from those partials, the last winners' stale
//                      entries replaced by the prev wave's values for w_{i-1}
//   prev wave   (10)   w_{i-1} (state: the eval output for pod i-1) committed
//                      with pod i and evaluated against pod i+1
// Node state is exact binary64 throughout (CandRow), so a re-score is a short
// dependent chain; every role reads its inputs for a pod in one batch of LDS
// loads.
constexpr int RES_LIST_WAVES = 4;
constexpr int RES_OWN_WAVES = 4;
constexpr int RES_EVAL_WAVE = RES_LIST_WAVES + RES_OWN_WAVES;
constexpr int RES_DEC_WAVE = RES_EVAL_WAVE + 1;
constexpr int RES_PREV_WAVE = RES_DEC_WAVE + 1;
constexpr int RES_IDLE = 15;                              // a wave with no role: barriers only
// Hardware wave h of a workgroup runs on SIMD h % 4 (round-robin dispatch onto
// the reserved CU): 16 waves, the decider with one owner wave on its SIMD,
// the eval and prev waves with another, list and owner waves on the last two.
constexpr int RES_HW_WAVES = 16;
__device__ __forceinline__ uint32_t res_role(uint32_t hw) {
  // SIMD 0: eval, prev, owner 2 | 1: decider, owner 3 | 2: list 0, owner 0, list 2 | 3: list 1, owner 1, list 3
  constexpr uint8_t tab[16] = {RES_EVAL_WAVE, RES_DEC_WAVE, 0, 1, RES_PREV_WAVE, RES_IDLE, 4, 5,
                               6,             7,            2, 3, RES_IDLE,      RES_IDLE, RES_IDLE, RES_IDLE};
  return tab[hw & 15];
}
constexpr int RESOLVE_THREADS = RES_HW_WAVES * WAVE;
constexpr int RHASH = 1024;
constexpr int LSEL = 4;                                   // listed candidates kept per list wave
constexpr int LAHEAD = 3;                                 // list waves select pod i + LAHEAD in iteration i
constexpr int KAHEAD = 3;                                 // ... with keys fetched KAHEAD iterations before
constexpr int KSLOTS = 8, RSLOTS = 8;                     // key / row staging slots (by pod mod)
static_assert(LSEL > LAHEAD, "a selection LAHEAD pods ahead must survive the LAHEAD commits before it is used");
static_assert(KSLOTS >= LAHEAD + KAHEAD + 1 && RSLOTS >= LAHEAD + 2, "staging depth (rows live until the owners apply)");
constexpr int NCAND_OWN = 2 * RES_OWN_WAVES;              // lanes [0, 8): owner waves' best two
constexpr int NCAND_LIST = LSEL * RES_LIST_WAVES;         // lanes [8, 24): list waves' first four
constexpr int CAND_PREV = NCAND_OWN + NCAND_LIST;         // candidate 24: the previous pod's winner (prev wave)
constexpr int NCAND = CAND_PREV + 1;
constexpr int DSUM_LANE = 32;                             // decider lanes summing status changes
constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr int ROW_PIECES = sizeof(CandRow) / 16;
constexpr int EXT_PIECES = sizeof(CandExt) / 16;
static_assert(2 * RES_LIST_WAVES * WAVE >= MAX_K && RES_OWN_WAVES * WAVE >= MAX_P, "resolve roles");
// list entries per list wave: 64 (lane l holds entry l) for K <= 256, 128
// (entries l and l + 64) for longer lists -- a resolve_kernel parameter, so
// K <= 256 rounds keep the single-probe loop (the two-entry select costs
// ~15 % of the resolve)
constexpr int LIST_SPAN_1 = WAVE, LIST_SPAN_2 = 2 * WAVE;
static_assert(DSUM_LANE >= NCAND && DSUM_LANE + NFILT + 3 <= WAVE, "decider lanes");



// Wave-uniform copy of an LDS object: every lane reads it (one address: an
// LDS broadcast, no bank conflicts).  Round 3: this replaced a copy read by
// one lane and handed to the SALU by a readfirstlane per dword, which put
// ~25 dependent readfirstlanes on the owner / eval waves' chains (resolve
// 0.287 -> 0.279 ms per round on the 125k-node proxy, profiles/r3/bcast_ab/).
template <class T>
__device__ __forceinline__ T lds_uniform(const T &src) {
  static_assert(sizeof(T) % 4 == 0, "dword object");
  return src;
}

// Resource-only pods (batches without PF_EXT pods: only NodeResourcesFit can
// fail, TaintToleration is the constant 100, NodeAffinity is skipped): the
// resolve's straight-line evaluation of one node, same arithmetic as filter /
// total_score.  A zero request skips its Fit check, encoded as a -inf request.
struct PodQ {
  double rq_c, rq_m;  // Fit: request or -inf
  int32_t wf, wb, cplus;
};
__device__ __forceinline__ PodQ pod_q(const PodDev &p, const Weights &w) {
  PodQ q;
  q.rq_c = ((p.flags & PF_HAS_REQ) && p.req_cpu > 0) ? p.req_cpu_d : -__builtin_inf();
  q.rq_m = ((p.flags & PF_HAS_REQ) && p.req_mem > 0) ? p.req_mem_d : -__builtin_inf();
  q.wf = w.fit;
  q.wb = w.ba;
  q.cplus = w.tt * 100;
  return q;
}
__device__ __forceinline__ bool fit_q(const PodQ &q, const NodeRegs &g) {
  return (g.bits & 2u) && !(q.rq_c > g.free_cpu) && !(q.rq_m > g.free_mem);
}
__device__ __forceinline__ uint64_t key_q(const PodDev &p, const PodQ &q, const NodeRegs &g) {
  const int32_t t = wmul((uint32_t)q.wf, (uint32_t)score_la(p, g)) +
                    wmul((uint32_t)q.wb, (uint32_t)score_ba(p, g)) + q.cplus;
  return pack_key(t, g.slot);
}


template <bool EXT, int LIST_SPAN>
__global__ __launch_bounds__(RESOLVE_THREADS) void resolve_kernel(RoundArgs a) {
  constexpr bool TWO = LIST_SPAN == 2 * WAVE;
  __shared__ PodDev s_pod[MAX_P];
  __shared__ ShardRecHdr s_hdr[MAX_P];
  __shared__ uint32_t s_rep[MAX_P];  // record of each pod (an identical pod's: RoundArgs::rep)
  __shared__ uint32_t s_norm[MAX_P][2];
  __shared__ uint32_t s_hkey[RHASH];  // slots modified this round (+1), linear probing
  __shared__ CandExt s_modx[EXT ? MAX_P : 1];  // label / taint words of the modified nodes
  // owner waves' partials for pod i (written in iteration i-1), by parity of i
  __shared__ RNode s_ocand[2][NCAND_OWN];   // best two nodes per wave
  __shared__ CandExt s_ocandx[EXT ? 2 : 1][EXT ? NCAND_OWN : 1];
  __shared__ uint64_t s_okey[2][NCAND_OWN];  // their keys for pod i, 0 = none
  __shared__ uint32_t s_oidx[2][NCAND_OWN];  // their owner indices
  __shared__ alignas(16) int32_t s_dsum[2][RES_OWN_WAVES][NFILT + 3];
  // list staging (LDS-DMA targets): listed keys by pod mod KSLOTS; the chosen
  // rows by pod mod RSLOTS as [list wave][16-byte piece][candidate]
  __shared__ uint64_t s_keys[KSLOTS][MAX_K];
  __shared__ uint4 s_lrowb[RSLOTS][RES_LIST_WAVES][ROW_PIECES + (EXT ? EXT_PIECES : 0)][LSEL];
  // list waves' candidates for pod i (chosen in iteration i - LAHEAD), by i mod RSLOTS
  __shared__ uint64_t s_lkey[RSLOTS][NCAND_LIST];
  __shared__ uint32_t s_lidx[RSLOTS][NCAND_LIST];  // list index, NONE32 = none
  // eval wave: each candidate of pod i committed, its key / status change for pod i+1 (by parity of i)
  __shared__ RNode s_post[2][NCAND];
  __shared__ CandExt s_postx[EXT ? 2 : 1][EXT ? NCAND : 1];
  __shared__ uint64_t s_ekey[2][NCAND];
  __shared__ alignas(16) int32_t s_edd[2][NCAND][NFILT + 3];
  // decider -> everyone: pod i's commit {valid, candidate lane, joins, owner index}
  __shared__ alignas(16) uint32_t s_pend[2][4];
  // s_done[b]: set by the decider in an iteration of parity b, read by every
  // wave after that iteration's barrier.  Double-buffered: a single word let
  // the decider's next-iteration store (r == nround: immediately after the
  // barrier) overtake a slow wave's read of this iteration, which then left
  // the loop one barrier early
  __shared__ uint32_t s_done[2], s_stop_at;
  // results of the round, written out after the loop (no global stores inside it)
  // per pod: {winning key lo, hi, feasible nodes, status} (one 16-B store by
  // the decider) and the failure counts (lanes of the decider); expanded into
  // DevResults after the loop
  __shared__ uint4 s_resc[MAX_P];
  __shared__ uint32_t s_rfail[MAX_P][NFILT];

  // tid: hardware thread (staging loops); wid / rtid: the wave's role and the
  // thread's index in role order (list entry, owned node)
  const uint32_t tid = threadIdx.x, lane = tid % WAVE;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(res_role(tid / WAVE)), rtid = wid * WAVE + lane;
  // launched after resolve_par_kernel (RoundArgs::rmode): the round is its
  // unless the parallel kernel handed it over
  if (a.rmode != nullptr && uniform_u32(a.rmode[1]) == a.seq) return;
  const uint32_t start = uniform_u32(*a.act);
  // The lists were swept for the pods from *sstart (speculatively); if the
  // previous round stopped early they belong to other pods: resolve nothing.
  if (start >= a.npods || uniform_u32(*a.sstart) != start) {
    if (tid == 0) {
      *a.act_next = start;
      *a.d_start = start;
      *a.carry_out_n = 0;
      if (start < a.npods) {
        a.counters[3] += 1;  // wasted (speculated) round
        mark_pod(a.marks, start, MARK_AFTER_WASTE);  // the next resolved round starts here
      }
      signal_done(a.flag_res, a.seq, a.stall_us);
    }
    return;
  }
  const uint32_t nround = min(a.P, a.npods - start);
  const uint32_t RW = rec_words(a.K);
  const bool is_list = wid < RES_LIST_WAVES;
  const bool is_owner = wid >= RES_LIST_WAVES && wid < RES_EVAL_WAVE;
  const uint32_t ow = wid - RES_LIST_WAVES;         // owner wave
  const uint32_t mj = rtid - RES_LIST_WAVES * WAVE;  // owner thread: owned modified node
  // ---- stage the round
  for (uint32_t i = tid; i < RHASH; i += RESOLVE_THREADS) s_hkey[i] = 0;
  for (uint32_t i = tid; i < nround; i += RESOLVE_THREADS) {
    const uint32_t ri = a.rep != nullptr ? a.rep[i] : i;
    s_rep[i] = ri;
    s_pod[i] = a.pods[start + i];
    s_hdr[i] = *(const ShardRecHdr *)(a.frec + (size_t)ri * RW);
    s_norm[i][0] = a.norm_max[2 * i];
    s_norm[i][1] = a.norm_max[2 * i + 1];
  }
  if (tid < 4) s_pend[1][tid] = 0;  // "pod -1" committed nothing
  if (tid < 2) s_done[tid] = 0;

  // ---- list waves (LDS-DMA pipeline).  Per iteration a list wave issues
  // LIST_DMA global_load_lds instructions (the chosen rows' pieces, one key
  // block) and, before the barrier, waits until those of two iterations ago
  // have landed; every LDS read of a DMA target in this wave is inline asm,
  // which hipcc does not tie to the DMA (it would drain the pipeline).
  constexpr uint32_t LIST_DMA = ROW_PIECES + (EXT ? EXT_PIECES : 0) + 1;
  constexpr int32_t LIST_WAIT = 2 * LIST_DMA;  // vmcnt(N): expcnt / lgkmcnt fields at their max
  static_assert(LIST_WAIT < 64, "vmcnt field");
  const uint32_t lw = wid;
  auto dma_keys = [&](uint32_t pod) {  // keys of list entries [SPAN lw, SPAN lw + SPAN) of pod -> s_keys
    const uint32_t p = min(pod, nround - 1);
    // every wave issues it (list_wait counts LIST_DMA loads per iteration);
    // entries past K: any in-record address (never read back)
    const uint32_t e = LIST_SPAN * lw + 2 * lane;
    const uint64_t *src = a.frec + (size_t)s_rep[p] * RW + REC_HDR_WORDS + (e < a.K ? e : 0u);
    if (TWO || lane < WAVE / 2)
      __builtin_amdgcn_global_load_lds((gvoid_t *)src, (lvoid_t *)&s_keys[pod % KSLOTS][LIST_SPAN * lw], 16, 0, 0);
  };
  auto lds_key = [&](uint32_t slot, uint32_t t) -> uint64_t {
    uint64_t v;
    const uint32_t addr = (uint32_t)(uintptr_t)(lvoid_t *)&s_keys[slot][t];
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
  };
  // pod's first LSEL entries (per list wave) not in the modified-slot hash:
  // keys / indices to s_lkey / s_lidx, rows by DMA
  auto list_select = [&](uint32_t pod) {
    const bool real = pod < nround;
    const uint32_t p = real ? pod : nround - 1;
    const uint32_t nk = s_hdr[p].nkeys;
    // lane l checks entries e0 = 128 lw + l and e1 = e0 + 64 against the
    // modified-slot hash; list order within the wave is e0's 64, then e1's
    const uint32_t e0 = LIST_SPAN * lw + lane, e1 = e0 + WAVE;
    const uint64_t k0 = e0 < a.K ? lds_key(pod % KSLOTS, e0) : 0ull;
    const uint64_t k1 = TWO && e1 < a.K ? lds_key(pod % KSLOTS, e1) : 0ull;
    auto probe = [&](uint64_t k, uint32_t e, bool &unmod, bool &hempty) {
      unmod = hempty = false;
      const uint32_t slot = 0xFFFFFFFFu - (uint32_t)k;
      if (real && k != 0 && e < nk) {
        uint32_t h = rhash(slot);
        unmod = true;
        hempty = s_hkey[h] == 0;
        while (s_hkey[h] != 0) {
          if (s_hkey[h] == slot + 1) { unmod = false; break; }
          h = (h + 1) & (RHASH - 1);
        }
      }
    };
    bool u0, h0, u1 = false, h1 = false;
    probe(k0, e0, u0, h0);
    if (TWO && LIST_SPAN * lw + WAVE < nk) probe(k1, e1, u1, h1);  // wave-uniform: second half only when listed
    const uint64_t ub0 = __ballot(u0), hb0 = __ballot(h0);
    const uint64_t ub1 = TWO ? __ballot(u1) : 0ull, hb1 = TWO ? __ballot(h1) : 0ull;
    const uint32_t n0 = (uint32_t)__popcll(ub0);
    const uint32_t nsel = min(n0 + (TWO ? (uint32_t)__popcll(ub1) : 0u), (uint32_t)LSEL);
    // lane c < LSEL takes the c-th unmodified entry of the wave's span
    const bool second = TWO && lane >= n0;
    uint64_t m = second ? ub1 : ub0;
    const uint32_t skip = second ? lane - n0 : lane;
    for (uint32_t j = 0; j < skip && j < (uint32_t)LSEL; ++j) m &= m - 1;
    const uint32_t tb = m ? (uint32_t)__builtin_ctzll(m) : 0u;
    const uint64_t tk0 = (uint64_t)__shfl((long long)k0, (int)tb, WAVE);
    const uint64_t tk1 = TWO ? (uint64_t)__shfl((long long)k1, (int)tb, WAVE) : 0ull;
    const uint64_t tk = second ? tk1 : tk0;
    const uint32_t te = tb + (second ? (uint32_t)WAVE : 0u);
    const uint64_t hb = second ? hb1 : hb0;
    if (lane < (uint32_t)LSEL) {
      const uint32_t t = LIST_SPAN * lw + te;
      const size_t rb = (size_t)s_rep[p] * a.K;
      const uint4 *row = (const uint4 *)(a.crow + rb + (lane < nsel ? t : 0u));
#pragma unroll
      for (int j = 0; j < ROW_PIECES; ++j)
        __builtin_amdgcn_global_load_lds((gvoid_t *)(row + j), (lvoid_t *)&s_lrowb[pod % RSLOTS][lw][j][0], 16, 0, 0);
      if constexpr (EXT) {
        const uint4 *x = (const uint4 *)(a.cext + rb + (lane < nsel ? t : 0u));
#pragma unroll
        for (int j = 0; j < EXT_PIECES; ++j)
          __builtin_amdgcn_global_load_lds((gvoid_t *)(x + j), (lvoid_t *)&s_lrowb[pod % RSLOTS][lw][ROW_PIECES + j][0],
                                           16, 0, 0);
      }
      if (real) {
        s_lkey[pod % RSLOTS][LSEL * lw + lane] = lane < nsel ? tk : 0ull;
        // bit 16: the entry's home hash bucket was empty when selected
        s_lidx[pod % RSLOTS][LSEL * lw + lane] = lane < nsel ? t | (uint32_t)((hb >> tb) & 1u) << 16 : NONE32;
      }
    }
  };
  auto list_wait = [&]() {  // DMA of two iterations ago landed
    __builtin_amdgcn_s_waitcnt((LIST_WAIT & 0xF) | ((LIST_WAIT >> 4) << 14) | (0x7 << 4) | (0xF << 8));
  };
  __syncthreads();  // staged headers, cleared hash
  if (is_list) {
    // prologue: keys of pods [0, LAHEAD + KAHEAD), then pods [0, LAHEAD) selected (nothing modified yet)
    for (uint32_t p = 0; p < (uint32_t)(LAHEAD + KAHEAD); ++p) dma_keys(p);
    __builtin_amdgcn_s_waitcnt(0);
    for (uint32_t p = 0; p < (uint32_t)LAHEAD; ++p) list_select(p);
    __builtin_amdgcn_s_waitcnt(0);
  }
  __syncthreads();
  if (is_owner && lane == 0) {
    s_okey[0][2 * ow] = s_okey[0][2 * ow + 1] = 0;
    for (int q = 0; q < NFILT + 3; ++q) s_dsum[0][ow][q] = 0;
  }

  // owner thread: the modified node it owns (live state, in registers)
  bool mine = false;
  RNode own{};
  // rank of the owned slot among its wave's owned slots (0 = lowest): owner
  // reductions run on 32-bit keys (score + 1) << 6 | (63 - rank), which order
  // like the packed 64-bit keys within one wave
  uint32_t srank = 0;
  // decider state (wave-uniform): the last three commits, modified count, stop point
  uint32_t pvalid = 0, pcand = 0, pslot = NONE32, p2slot = NONE32, p3slot = NONE32, powner = 0, nmod = 0,
           stop_at = nround;
  // hash buckets the last three pods' joins were inserted at (NONE32: no insert)
  uint32_t pb1 = NONE32, pb2 = NONE32, pb3 = NONE32;
  // the decider is the per-pod critical path, the eval wave next: issue priority
  if (wid == RES_DEC_WAVE) __builtin_amdgcn_s_setprio(3);
  else if (wid == RES_EVAL_WAVE || wid == RES_PREV_WAVE) __builtin_amdgcn_s_setprio(2);
  else if (is_owner) __builtin_amdgcn_s_setprio(3);  // owners: the longest chain per pod
  KS_STAMP_DECL(wid, lane);
  lds_barrier();

  // ROLE: 0 decider, 1 eval / prev, 2 owner, 3 list (one loop per role below)
  auto iteration = [&](uint32_t r, auto role) __attribute__((always_inline)) -> bool {
    constexpr int ROLE = decltype(role)::value;
    const uint32_t buf = r & 1u, nb = buf ^ 1u;
    KS_STAMP_BEGIN();
    if constexpr (ROLE == 0) {
      // ------------------------------------------------------------- decider
      if (r >= nround) {
        if (lane == 0) {
          s_pend[buf][0] = 0;
          s_done[buf] = 1;
        }
      } else {
        const uint32_t b4 = r % RSLOTS;
        // One batch of independent LDS loads.  Lanes 0-7: owner candidates,
        // 8-23: listed candidates, 24: the previous winner committed (its key
        // for this pod); lanes 32-39: the status-change sums per count; lanes
        // 33-37 also their header failure counts.
        const bool is_own = lane < (uint32_t)NCAND_OWN;
        const bool is_lst = lane >= (uint32_t)NCAND_OWN && lane < (uint32_t)CAND_PREV;
        const bool is_prev = lane == (uint32_t)CAND_PREV;
        const uint32_t lo = is_own ? lane : 0u, ll = is_lst ? lane - NCAND_OWN : 0u;
        const uint64_t *kp = is_own ? &s_okey[buf][lo] : is_prev ? &s_ekey[nb][pcand] : &s_lkey[b4][ll];
        const uint32_t *ip = is_own ? &s_oidx[buf][lo] : &s_lidx[b4][ll];
        const uint32_t q = (lane - DSUM_LANE) & 7u;
        const uint64_t rkey = *kp;
        const uint32_t vidx = *ip;
        const uint32_t oslot = s_ocand[buf][lo].slot;
        int32_t vd = s_dsum[buf][0][q] + s_dsum[buf][1][q] + s_dsum[buf][2][q] + s_dsum[buf][3][q] +
                     (pvalid ? s_edd[nb][pcand][q] : 0);
        const ShardRecHdr &hd = s_hdr[r];
        const uint32_t hfail = hd.fails[(lane - DSUM_LANE - 1) % NFILT];
        const uint32_t pflags = uniform_u32(s_pod[r].flags);
        const uint32_t h_feasible = uniform_u32(hd.feasible);
        const uint32_t h_tt = uniform_u32(hd.tt_cnt), h_na = uniform_u32(hd.na_cnt);
        const uint64_t h_bound = ((uint64_t)uniform_u32((uint32_t)(hd.bound >> 32)) << 32) |
                                 uniform_u32((uint32_t)hd.bound);
        KS_STAMP_SPLIT_LGKM(1, 0);
        const uint64_t vkey = (is_prev && !pvalid) ? 0ull : rkey;
        const uint32_t vslot = is_own ? oslot : is_prev ? pslot : 0xFFFFFFFFu - (uint32_t)vkey;
        // entries computed before the last winners' commits are stale: drop them
        const uint64_t mk = ((is_own && vkey && vslot != pslot) || is_prev) ? vkey : 0ull;
        // nonzero only in lanes [0, 8) (owners) and CAND_PREV
        static_assert(NCAND_OWN == 8, "owner candidates fill one 8-lane DPP group");
        const uint64_t bm = max64(readlane64(max8_u64(mk), 0), readlane64(mk, CAND_PREV));
        const bool lok = is_lst && vidx != NONE32 && vslot != pslot && vslot != p2slot && vslot != p3slot;
        const uint64_t lb = __ballot(lok);  // listed candidates are in list order by lane
        const uint32_t ulane = lb ? (uint32_t)__builtin_ctzll(lb) : 0u;
        const uint64_t ku = lb ? readlane64(vkey, (int)ulane) : 0ull;
        const int32_t s0 = __builtin_amdgcn_readlane(vd, DSUM_LANE);
        const uint32_t feasible = h_feasible - (uint32_t)s0;
        KS_STAMP_SPLIT(1, 1);
        int32_t status = 0;
        bool stop = false;
        uint64_t win = 0;
        if (feasible == 0) {
          status = 1;  // KS_POD_UNSCHEDULABLE
        } else if ((pflags & PF_PREF_ERR) && feasible >= 2) {
          status = 2;  // KS_POD_ERROR (NodeAffinity PreScore)
        } else if ((EXT && (pflags & PF_TT) && h_tt - (uint32_t)__builtin_amdgcn_readlane(vd, DSUM_LANE + 6) == 0) ||
                   (EXT && (pflags & PF_NA) && h_na - (uint32_t)__builtin_amdgcn_readlane(vd, DSUM_LANE + 7) == 0)) {
          stop = true;  // a normaliser's max may have moved: re-sweep from this pod
        } else if (lb) {
          win = ku > bm ? ku : bm;
        } else if (bm > h_bound) {
          win = bm;
        } else {
          stop = true;  // candidates exhausted
        }
        if (stop) {
          stop_at = r;
          if (lane == 0) {
            s_pend[buf][0] = 0;
            s_done[buf] = 1;
          }
        } else {
          if (lane == 0) s_resc[r] = make_uint4((uint32_t)win, (uint32_t)(win >> 32), feasible, (uint32_t)status);
          if (lane > (uint32_t)DSUM_LANE && lane <= (uint32_t)DSUM_LANE + NFILT)
            s_rfail[r][lane - DSUM_LANE - 1] = hfail + (uint32_t)vd;
          KS_STAMP_SPLIT(1, 2);
          // commit (AssumePod -> NodeInfo.AddPod): the eval wave holds the
          // committed state of every candidate; record which one won
          uint32_t cand = 0, join = 0, oidx = 0;
          p3slot = p2slot;
          p2slot = pslot;
          if (win) {
            join = (lb && win == ku) ? 1u : 0u;
            cand = join ? ulane : (uint32_t)__builtin_ctzll(__ballot(mk == win));
            const uint32_t wslot = 0xFFFFFFFFu - (uint32_t)win;
            if (join) {
              oidx = nmod++;
              // The home bucket was empty at selection (LAHEAD pods ago); only
              // the last three joins can have filled it since: then a plain
              // store, else probe with compare-and-swap.
              const uint32_t home = rhash(wslot);
              const bool hfree = ((uint32_t)__builtin_amdgcn_readlane((int)vidx, (int)ulane) >> 16 & 1u) &&
                                 home != pb1 && home != pb2 && home != pb3;
              uint32_t h = home;
              if (hfree) {
                if (lane == 0) s_hkey[home] = wslot + 1;
              } else {
                if (lane == 0)
                  while (atomicCAS(&s_hkey[h], 0u, wslot + 1) != 0u) h = (h + 1) & (RHASH - 1);
                h = __builtin_amdgcn_readfirstlane(h);
              }
              pb3 = pb2;
              pb2 = pb1;
              pb1 = h;
            } else {
              oidx = cand == (uint32_t)CAND_PREV ? powner : (uint32_t)__builtin_amdgcn_readlane((int)vidx, (int)cand);
              pb3 = pb2;
              pb2 = pb1;
              pb1 = NONE32;
            }
            pslot = wslot;
            powner = oidx;
          } else {
            pslot = NONE32;
            pb3 = pb2;
            pb2 = pb1;
            pb1 = NONE32;
          }
          pvalid = win ? 1u : 0u;
          pcand = cand;
          if (lane == 0) *(uint4 *)&s_pend[buf][0] = make_uint4(pvalid, cand, join, oidx);
          KS_STAMP_SPLIT(1, 3);
        }
      }
    } else if constexpr (ROLE == 1) {
      // ------------------------------------------------ eval and prev waves
      // every candidate of pod r committed, evaluated against pod r+1: the
      // eval wave takes the owner and listed candidates (one per lane) and
      // never waits for pod r-1's decision; the prev wave's first lane takes
      // the previous winner, whose state is the eval output for pod r-1
      if (r < nround) {
        const bool prevw = wid == RES_PREV_WAVE;
        const uint32_t b4 = r % RSLOTS;
        const uint32_t cl = prevw ? (lane == 0 ? (uint32_t)CAND_PREV : (uint32_t)NCAND)
                                  : (lane < (uint32_t)CAND_PREV ? lane : (uint32_t)NCAND);  // candidate, NCAND = none
        const bool is_own = cl < (uint32_t)NCAND_OWN;
        const bool is_lst = cl >= (uint32_t)NCAND_OWN && cl < (uint32_t)CAND_PREV;
        const bool is_prev = cl == (uint32_t)CAND_PREV;
        const uint32_t lo = is_own ? cl : 0u, c = is_lst ? cl - NCAND_OWN : 0u;
        const uint32_t cw = c / LSEL, ck = c % LSEL;
        // one batch: the candidate's row (owner: published node; listed: DMA
        // pieces) and round-start fields
        RNode pre{};
        CandExt px{};
        uint4 tail = make_uint4(0, 0, 0, 0), tail2 = make_uint4(0, 0, 0, 0);  // owners: rc0, rm0 / np0, slot
        uint64_t lkey = 0;
        uint32_t pv = 0, pc = 0;  // pod r-1's commit (prev wave only)
        bool on = false;
        if (!prevw) {
          const uint4 *rp = is_own ? (const uint4 *)&s_ocand[buf][lo] : &s_lrowb[b4][cw][0][ck];
          const uint32_t rstride = is_own ? 1u : (uint32_t)LSEL;
          uint4 *pp = (uint4 *)&pre;
#pragma unroll
          for (int j = 0; j < ROW_PIECES; ++j) pp[j] = rp[j * rstride];
          if (is_own) {
            tail = rp[ROW_PIECES];
            tail2 = rp[ROW_PIECES + 1];
          }
          if constexpr (EXT) {
            const uint4 *xp = is_own ? (const uint4 *)&s_ocandx[buf][lo] : &s_lrowb[b4][cw][ROW_PIECES][ck];
            uint4 *xo = (uint4 *)&px;
#pragma unroll
            for (int j = 0; j < EXT_PIECES; ++j) xo[j] = xp[j * rstride];
          }
          lkey = s_lkey[b4][c];
          on = is_own ? s_okey[buf][lo] != 0 : is_lst && s_lidx[b4][c] != NONE32;
        } else {
          pv = uniform_u32(s_pend[nb][0]);
          pc = min(uniform_u32(s_pend[nb][1]), (uint32_t)NCAND - 1);
          on = is_prev && pv != 0;
        }
        KS_STAMP_SPLIT_LGKM(2, 0);
        if (is_lst) {
          pre.rc0 = pre.row.rc;
          pre.rm0 = pre.row.rm;
          pre.np0 = pre.row.np;
          pre.slot = 0xFFFFFFFFu - (uint32_t)lkey;
        } else {
          pre.rc0 = __builtin_bit_cast(double, ((uint64_t)tail.y << 32) | tail.x);
          pre.rm0 = __builtin_bit_cast(double, ((uint64_t)tail.w << 32) | tail.z);
          pre.np0 = (int32_t)tail2.x;
          pre.slot = tail2.y;
        }
        pre._pad[0] = pre._pad[1] = 0;
        if (is_prev && pv) {  // the previous winner: its committed node, from the last iteration
          pre = s_post[nb][pc];
          if (EXT) px = s_postx[nb][pc];
        }
        KS_STAMP_SPLIT_LGKM(2, 1);
        RNode post = pre;
        rnode_add(post, lds_uniform(s_pod[r]));
        if (on && cl < (uint32_t)NCAND) {  // the prev wave of the next iteration reads the winner's
          s_post[buf][cl] = post;
          if (EXT) s_postx[buf][cl] = px;
        }
        if constexpr (!EXT) {
          // straight-line for every lane (no branch keeps the pod loads from
          // being hoisted into the candidate batch); stores predicated
          const PodDev p1 = lds_uniform(s_pod[min(r + 1, nround - 1)]);
          const PodQ q1 = pod_q(p1, a.w);
          const NodeRegs g0 = rnode_regs(pre, pre.row.rc, pre.row.rm, pre.row.np);
          const NodeRegs g1 = rnode_regs(post, post.row.rc, post.row.rm, post.row.np);
          const bool f0 = fit_q(q1, g0), f1 = fit_q(q1, g1);
          const uint64_t key = f1 ? key_q(p1, q1, g1) : 0ull;
          if (on && cl < (uint32_t)NCAND && r + 1 < nround) {
            s_ekey[buf][cl] = key;
            // a commit only adds: feasible -> Fit failure is the only change
            const int32_t lost = (f0 && !f1) ? 1 : 0;
            s_edd[buf][cl][0] = lost;
#pragma unroll
            for (int qq = 1; qq < NFILT + 3; ++qq) s_edd[buf][cl][qq] = qq == 1 + KS_PLUGIN_FIT_IDX ? lost : 0;
          }
        } else if (r + 1 < nround) {
          const PodDev p1 = lds_uniform(s_pod[r + 1]);  // every lane
          if (on && cl < (uint32_t)NCAND) {
            int64_t tt_max = 0, na_max = 0;
            if (EXT) {
              tt_max = s_norm[r + 1][0];
              na_max = s_norm[r + 1][1];
            }
            NodeExt e{};
            if (EXT) ext_from_words(px.w, e);
            const NodeRegs g0 = rnode_regs(pre, pre.row.rc, pre.row.rm, pre.row.np);
            const NodeRegs g1 = rnode_regs(post, post.row.rc, post.row.rm, post.row.np);
            const int st0 = filter<EXT>(p1, a.clauses, g0, e);
            const int st1 = filter<EXT>(p1, a.clauses, g1, e);
            uint64_t key = 0;
            if (st1 == ST_FEASIBLE) key = pack_key(total_score<EXT>(p1, a.clauses, g1, e, a.w, tt_max, na_max), post.slot);
            int32_t d[NFILT + 3] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (st0 != st1) status_delta<EXT>(p1, a.clauses, st0, st1, e, post.slot, tt_max, na_max, d);
            s_ekey[buf][cl] = key;
#pragma unroll
            for (int qq = 0; qq < NFILT + 3; ++qq) s_edd[buf][cl][qq] = d[qq];
          }
        }
        KS_STAMP_SPLIT_LGKM(2, 2);
      }
    } else if constexpr (ROLE == 2) {
      // ------------------------------------------------------- owner waves
      if (r >= 1) {  // apply pod r-1's commit: its winner's owner adds the pod
        const uint32_t pv = uniform_u32(s_pend[nb][0]), pc = uniform_u32(s_pend[nb][1]);
        const uint32_t pj = uniform_u32(s_pend[nb][2]), po = uniform_u32(s_pend[nb][3]);
        const PodDev pp = lds_uniform(s_pod[r - 1]);  // every lane (readfirstlane)
        if (pv && pj && po / WAVE == ow) {  // a listed node joins this wave: re-rank
          const uint32_t js = 0xFFFFFFFFu - (uint32_t)s_lkey[(r - 1) % RSLOTS][pc - NCAND_OWN];
          const uint32_t below = (uint32_t)__popcll(__ballot(mine && own.slot < js));
          if (mine && own.slot > js) ++srank;
          if (po == mj) srank = below;
        }
        if (pv && po == mj) {
          if (pj) {  // a listed node joins: its row (DMA-staged for pod r-1, still resident)
            const uint32_t b8 = (r - 1) % RSLOTS, c = pc - NCAND_OWN, cw = c / LSEL, ck = c % LSEL;
            CandRow w;
            uint4 *wp = (uint4 *)&w;
#pragma unroll
            for (int j = 0; j < ROW_PIECES; ++j) wp[j] = s_lrowb[b8][cw][j][ck];
            own = rnode_from_row(w, 0xFFFFFFFFu - (uint32_t)s_lkey[b8][c]);
            if constexpr (EXT) {  // piece by piece into LDS (a punned local goes via scratch)
              uint4 *xp = (uint4 *)&s_modx[mj];
#pragma unroll
              for (int j = 0; j < EXT_PIECES; ++j) xp[j] = s_lrowb[b8][cw][ROW_PIECES + j][ck];
            }
            mine = true;
          }
          rnode_add(own, pp);
        }
      }
      KS_STAMP_SPLIT(3, 0);
      if (r + 1 < nround && __ballot(mine) != 0) {
        uint64_t key = 0;
        int32_t d[NFILT + 3] = {0, 0, 0, 0, 0, 0, 0, 0};
        bool dany = false;
        CandExt ox{};
        if constexpr (!EXT) {
          const PodDev p1 = lds_uniform(s_pod[r + 1]);
          const PodQ q1 = pod_q(p1, a.w);
          const NodeRegs g = rnode_regs(own, own.row.rc, own.row.rm, own.row.np);
          const NodeRegs g0 = rnode_regs(own, own.rc0, own.rm0, own.np0);
          const bool f0 = fit_q(q1, g0), f = fit_q(q1, g);
          key = (mine && f) ? key_q(p1, q1, g) : 0ull;
          dany = mine && f0 && !f;
          // a commit only adds: Fit failures are the only status change
          const int32_t nlost = (int32_t)__popcll(__ballot(dany));
          d[0] = nlost;
          d[1 + KS_PLUGIN_FIT_IDX] = nlost;
        } else {
          const PodDev p1 = lds_uniform(s_pod[r + 1]);
          int64_t tt_max = 0, na_max = 0;
          if (EXT) {
            tt_max = s_norm[r + 1][0];
            na_max = s_norm[r + 1][1];
          }
          NodeExt e{};
          if (EXT) {
            ox = s_modx[mj];
            ext_from_words(ox.w, e);
          }
          const NodeRegs g = rnode_regs(own, own.row.rc, own.row.rm, own.row.np);
          const NodeRegs g0 = rnode_regs(own, own.rc0, own.rm0, own.np0);
          if (mine) {  // p1 above is read by every lane (lds_uniform)
            const int st0 = filter<EXT>(p1, a.clauses, g0, e);
            const int st = filter<EXT>(p1, a.clauses, g, e);
            if (st == ST_FEASIBLE) key = pack_key(total_score<EXT>(p1, a.clauses, g, e, a.w, tt_max, na_max), own.slot);
            if (st0 != st) {
              dany = true;
              status_delta<EXT>(p1, a.clauses, st0, st, e, own.slot, tt_max, na_max, d);
            }
          }
        }
        KS_STAMP_SPLIT(3, 1);
        // total + 1 < 2^24 (weights capped at 10000), rank < 64
        const uint32_t key32 = key ? (uint32_t)(key >> 32) << 6 | (63u - srank) : 0u;
        const uint32_t k1 = wave_max_u32_dpp(key32);
        const uint32_t k2 = wave_max_u32_dpp(key32 == k1 ? 0u : key32);
        KS_STAMP_SPLIT(3, 2);
        // the holders publish their node and packed key for the decider and the eval wave
        if (key32 != 0 && (key32 == k1 || key32 == k2)) {
          const uint32_t c = 2 * ow + (key32 == k1 ? 0u : 1u);
          s_ocand[nb][c] = own;
          if (EXT) s_ocandx[nb][c] = ox;
          s_oidx[nb][c] = mj;
          s_okey[nb][c] = key;
        }
        const bool wdany = __ballot(dany) != 0;
        if (EXT && wdany) {
#pragma unroll
          for (int qq = 0; qq < NFILT + 3; ++qq) d[qq] = wave_sum_i32_dpp(d[qq]);
        }
        if (lane == 0) {
          if (k1 == 0) s_okey[nb][2 * ow] = 0;
          if (k2 == 0) s_okey[nb][2 * ow + 1] = 0;
#pragma unroll
          for (int qq = 0; qq < NFILT + 3; ++qq) s_dsum[nb][ow][qq] = wdany ? d[qq] : 0;
        }
      } else if (r + 1 < nround && lane == 0) {
        s_okey[nb][2 * ow] = s_okey[nb][2 * ow + 1] = 0;
#pragma unroll
        for (int qq = 0; qq < NFILT + 3; ++qq) s_dsum[nb][ow][qq] = 0;
      }
    } else {
      // -------------------------------------------------------- list waves
      list_select(r + LAHEAD);
      KS_STAMP_SPLIT(4, 0);
      dma_keys(r + LAHEAD + KAHEAD);
      KS_STAMP_SPLIT(4, 1);
      list_wait();
      KS_STAMP_SPLIT(4, 2);
    }
    KS_STAMP_PRE_BARRIER();
    lds_barrier();
    KS_STAMP_POST_BARRIER();
    KS_RACE_DELAY(ROLE != 0 && r + 2 >= nround);  // make probe only (ksched_instr.hpp)
    return s_done[buf] != 0;
  };

  // One loop per role (the barrier counts waves, not program locations): each
  // copy of the inlined iteration keeps only its own role's state live, so no
  // wave pays the phi moves of the other roles' registers at the loop latch.
  if (wid == RES_DEC_WAVE) {
    for (uint32_t r = 0;; ++r)
      if (iteration(r, std::integral_constant<int, 0>{})) break;
  } else if (wid == RES_EVAL_WAVE || wid == RES_PREV_WAVE) {
    for (uint32_t r = 0;; ++r)
      if (iteration(r, std::integral_constant<int, 1>{})) break;
  } else if (is_owner) {
    for (uint32_t r = 0;; ++r)
      if (iteration(r, std::integral_constant<int, 2>{})) break;
  } else if (wid == RES_IDLE) {
    for (uint32_t r = 0;; ++r) {
      lds_barrier();
      KS_RACE_DELAY(r + 2 >= nround);
      if (s_done[r & 1u] != 0) break;
    }
  } else {
    for (uint32_t r = 0;; ++r)
      if (iteration(r, std::integral_constant<int, 3>{})) break;
  }
  if (is_list) __builtin_amdgcn_s_waitcnt(0);  // no DMA outlives the block
  // hand the nodes this round modified to the next round's patch and the write-back
  if (is_owner && mine) {
    CandExt ox{};
    if (EXT) ox = s_modx[mj];
    a.carry_out[mj] = rnode_carry(own, ox, EXT);
  }
  KS_STAMP_FLUSH(a.counters, wid);
  if (wid == RES_DEC_WAVE && lane == 0) s_stop_at = stop_at;
  __syncthreads();
  {
    // results of the round: 16 threads per pod, one dword of its DevResult each
    const uint32_t nres = s_stop_at;
    uint32_t *dst = (uint32_t *)((DevResult *)a.results + start);
    constexpr uint32_t RW32 = sizeof(DevResult) / 4;
    for (uint32_t i = tid; i < nres * RW32; i += RESOLVE_THREADS) {
      const uint32_t pr = i / RW32, w = i % RW32;
      const uint4 c = s_resc[pr];
      const uint64_t win = ((uint64_t)c.y << 32) | c.x;
      const int64_t total = win ? (int64_t)(win >> 32) - 1 : 0;
      uint32_t v;
      switch (w) {
        case 0: v = win ? 0xFFFFFFFFu - (uint32_t)win : 0xFFFFFFFFu; break;  // node_index (-1: none)
        case 1: v = c.w; break;                                               // status
        case 2: v = (uint32_t)total; break;                                  // total_score
        case 3: v = (uint32_t)((uint64_t)total >> 32); break;
        case 4: v = c.z; break;                                              // feasible_nodes
        case 5: v = a.evaluated; break;                                      // evaluated_nodes
        case 6: case 7: case 8: case 9: case 10: v = s_rfail[pr][w - 6]; break;  // fail_counts
        case 13: v = s_pod[pr].prefilter_out; break;                         // prefiltered
        case 14: v = (win && c.z == 1) ? 1u : 0u; break;                     // flags
        default: v = 0; break;                                               // spread_fail, ipa_fail, _pad
      }
      dst[i] = v;
    }
  }
  if (wid == RES_DEC_WAVE && lane == 0) {
    *a.carry_out_n = nmod;
    mark_pod(a.marks, start, MARK_ROUND_START);
    *a.act_next = start + stop_at;
    *a.d_start = start + stop_at;
    a.counters[0] += 1;        // rounds
    a.counters[1] += stop_at;  // pods resolved
    if (a.rmode != nullptr && a.rmode[0] > 0) a.rmode[0] -= 1;
  }
  // the streams waiting for this round (write-back, patch) poll the flag:
  // every thread's global stores are ordered before the signal
  __syncthreads();
  if (tid == 0) signal_done(a.flag_res, a.seq, a.stall_us);
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

hipError_t launch_resolve(const RoundArgs &a, bool ext, hipStream_t st) {
  if (a.K <= (uint32_t)(RES_LIST_WAVES * LIST_SPAN_1)) {
    if (ext) resolve_kernel<true, LIST_SPAN_1><<<1, RESOLVE_THREADS, 0, st>>>(a);
    else resolve_kernel<false, LIST_SPAN_1><<<1, RESOLVE_THREADS, 0, st>>>(a);
  } else {
    if (ext) resolve_kernel<true, LIST_SPAN_2><<<1, RESOLVE_THREADS, 0, st>>>(a);
    else resolve_kernel<false, LIST_SPAN_2><<<1, RESOLVE_THREADS, 0, st>>>(a);
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
