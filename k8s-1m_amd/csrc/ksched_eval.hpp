// ksched_eval.hpp — per-(pod, node) Filter and Score arithmetic shared by the
// round kernels (ksched_kernels.hip) and the PodTopologySpread path
// (ksched_spread.hip): node state in exact binary64, label programs, the
// filter chain in default-profile order, LeastAllocated / BalancedAllocation /
// TaintToleration / NodeAffinity scores and the packed selection key.
// Exactness arguments: DESIGN.md §4.
#pragma once

#include <hip/hip_runtime.h>

#include "ksched_dev.hpp"

namespace ks {

// Node resource state held in registers for the whole pod loop.
// Every resource quantity is an integer of magnitude < 2^53, so it is held as an
// exact binary64 and the sums / differences below are exact too: no int64
// arithmetic or int->float conversion per (pod, node) evaluation.  A resource
// with zero allocatable gets inv = 0, which makes both scores' terms for it
// vanish; lashift / bamul then give upstream's weight-sum and fraction-count
// rules without a per-evaluation branch.
struct NodeRegs {
  double free_cpu, free_mem;    // Allocatable - Requested                 (Fit)
  double rcpu, rmem;            // Requested                               (BalancedAllocation)
  double lf100_cpu, lf100_mem;  // (Allocatable - NonZeroRequested) * 100  (LeastAllocated)
  double acpu_d, amem_d;        // Allocatable
  double inv_cpu, inv_mem;      // RN(1 / Allocatable), 0 when Allocatable == 0
  double bamul;                 // 0.5 with two non-zero allocatables, else 0 (std = 0)
  uint32_t slot;
  uint32_t bits;                // 1 valid, 2 pods fit, 4 cpu alloc != 0, 8 mem alloc != 0
  uint32_t lashift;             // 1 with two non-zero allocatables (score / weightSum 2), else 0
};

__device__ __forceinline__ NodeRegs make_regs_inv(int64_t acpu, int64_t amem, int64_t rc, int64_t rm, int64_t zc,
                                                  int64_t zm, int32_t apods, int32_t np, uint32_t slot,
                                                  double inv_cpu, double inv_mem) {
  NodeRegs r;
  r.slot = slot;
  r.free_cpu = (double)(acpu - rc);
  r.free_mem = (double)(amem - rm);
  r.rcpu = (double)rc;
  r.rmem = (double)rm;
  r.lf100_cpu = (double)(acpu - zc) * 100.0;  // exact for a non-negative value (< 2^51)
  r.lf100_mem = (double)(amem - zm) * 100.0;
  r.acpu_d = (double)acpu;
  r.amem_d = (double)amem;
  r.inv_cpu = acpu ? inv_cpu : 0.0;
  r.inv_mem = amem ? inv_mem : 0.0;
  const bool both = acpu && amem;
  r.bamul = both ? 0.5 : 0.0;
  r.lashift = both ? 1u : 0u;
  r.bits = 1u | ((int64_t)np + 1 <= (int64_t)apods ? 2u : 0u) | (acpu ? 4u : 0u) | (amem ? 8u : 0u);
  return r;
}

__device__ __forceinline__ NodeRegs make_regs(int64_t acpu, int64_t amem, int64_t rc, int64_t rm, int64_t zc,
                                              int64_t zm, int32_t apods, int32_t np, uint32_t slot) {
  return make_regs_inv(acpu, amem, rc, rm, zc, zm, apods, np, slot, acpu ? 1.0 / (double)acpu : 0.0,
                       amem ? 1.0 / (double)amem : 0.0);
}

struct NodeExt {
  uint64_t hard, prefer;
  uint64_t lab[LW];
  int64_t num[NNUM];
};

__device__ __forceinline__ void load_core(const NodeTable &t, uint32_t pos, uint32_t slot, bool in_range,
                                          NodeRegs &r) {
  int32_t ap = in_range ? t.apods[pos] : -1;
  if (ap < 0) {  // empty slot: benign finite values, never feasible
    r.free_cpu = r.free_mem = r.rcpu = r.rmem = r.lf100_cpu = r.lf100_mem = 0;
    r.acpu_d = r.amem_d = 1.0;
    r.inv_cpu = r.inv_mem = 0.0;
    r.bamul = 0.0;
    r.lashift = 0;
    r.slot = slot;
    r.bits = 0;
    return;
  }
  r = make_regs(t.acpu[pos], t.amem[pos], t.rcpu[pos], t.rmem[pos], t.zcpu[pos], t.zmem[pos], ap, t.npods[pos], slot);
}

template <int LWU = LW>
__device__ __forceinline__ void load_ext(const NodeTable &t, uint32_t pos, bool valid, NodeExt &e) {
  if (!valid) {
    e.hard = e.prefer = 0;
#pragma unroll
    for (int k = 0; k < LW; ++k) e.lab[k] = 0;
#pragma unroll
    for (int k = 0; k < NNUM; ++k) e.num[k] = 0;
    return;
  }
  e.hard = t.hard[pos];
  e.prefer = t.prefer[pos];
#pragma unroll
  for (int k = 0; k < LW; ++k) e.lab[k] = (k < LWU && k < (int)t.lw) ? t.lab[(size_t)k * t.npos + pos] : 0ull;
#pragma unroll
  for (int k = 0; k < NNUM; ++k) e.num[k] = t.num[(size_t)k * t.npos + pos];
}

// One label-program term (ksched_dev.hpp) against one node: fixed-form mask
// tests, then the rare Gt / Lt and metadata.name entries.
__device__ __forceinline__ bool term_pass(const uint64_t *t, const NodeExt &e, uint32_t slot) {
  const uint64_t w0 = t[0];
  const uint32_t ng = (uint32_t)w0 & 0xFF, nn = ((uint32_t)w0 >> 8) & 0xFF, nm = ((uint32_t)w0 >> 16) & 0xFF;
  uint64_t diff = 0;
#pragma unroll
  for (int k = 0; k < LW; ++k) diff |= (e.lab[k] & t[1 + LW + k]) ^ t[1 + k];
  bool ok = diff == 0;
  const uint64_t *g = t + TERM_HDR_WORDS;
  for (uint32_t i = 0; i < ng; ++i, g += LW) {
    uint64_t any = 0;
#pragma unroll
    for (int k = 0; k < LW; ++k) any |= e.lab[k] & g[k];
    ok &= any != 0;
  }
  for (uint32_t i = 0; i < nn; ++i, g += 2) {
    const int64_t v = (g[0] & 0xFF) ? e.num[1] : e.num[0];
    const int64_t x = (int64_t)g[1];
    ok &= ((g[0] >> 8) & 0xFF) == TO_GT ? v > x : v < x;
  }
  for (uint32_t i = 0; i < nm; ++i, g += 2) {
    const bool eq = (int64_t)slot == (int64_t)g[1];
    ok &= g[0] == TO_NAME_IN ? eq : !eq;
  }
  return ok;
}

// RequiredNodeAffinity.Match: any required term (the nodeSelector is merged
// into each; PF_AFF with no term matches nothing).
__device__ __forceinline__ bool required_match(const PodDev &p, const uint64_t *prog, const NodeExt &e,
                                               uint32_t slot) {
  const uint64_t *t = prog + p.req_off;
  bool any = false;
  for (uint32_t k = 0; k < p.req_len; ++k) {
    any |= term_pass(t, e, slot);
    t += term_words(t[0]);
  }
  return any;
}

// PreferredSchedulingTerms.Score: Σ weight of matching preferred terms.
__device__ __forceinline__ int64_t preferred_raw(const PodDev &p, const uint64_t *prog, const NodeExt &e,
                                                 uint32_t slot) {
  const uint64_t *t = prog + p.pref_off;
  int64_t raw = 0;
  for (uint32_t k = 0; k < p.pref_len; ++k) {
    if (term_pass(t, e, slot)) raw += (int64_t)(uint32_t)(t[0] >> 32);
    t += term_words(t[0]);
  }
  return raw;
}

// NodeAffinity PreFilterResult: the node is one of the named ones (the
// pod's prefilter program lists their slots).
__device__ __forceinline__ bool prefilter_match(const PodDev &p, const uint64_t *prog, uint32_t slot) {
  bool any = false;
  for (uint32_t k = 0; k < p.pre_len; ++k) any |= (uint64_t)slot == prog[p.pre_off + k];
  return any;
}

// Filter chain in default-profile order; returns ST_FEASIBLE, KS_PLUGIN_* or
// ST_PREFILTERED.  NodeAffinity's PreFilter runs before any Filter: a
// conflicting name set fails every node at NodeAffinity, a PreFilterResult
// leaves the nodes outside it unevaluated (schedule_one.go#findNodesThatFitPod).
template <bool EXT>
__device__ __forceinline__ int filter(const PodDev &p, const uint64_t *clauses, const NodeRegs &r,
                                      const NodeExt &e) {
  if (EXT && (p.flags & PF_EXT)) {
    if (p.flags & PF_NA_CONFLICT) return 3;
    if ((p.flags & PF_PREFILTER) && !prefilter_match(p, clauses, r.slot)) return ST_PREFILTERED;
    const uint64_t untol = e.hard & ~p.tol_hard;
    if (untol & UNSCHED_BIT) return 0;                              // NodeUnschedulable
    if (p.name_slot != -1 && (int64_t)r.slot != (int64_t)p.name_slot) return 1;  // NodeName
    if (untol) return 2;                                            // TaintToleration
    if ((p.flags & PF_AFF) && !required_match(p, clauses, e, r.slot)) return 3;  // NodeAffinity
  }
  // NodeResourcesFit (fitsRequest): pod count, then cpu / memory vs Requested.
  bool fail = !(r.bits & 2u);
  if (p.flags & PF_HAS_REQ) {
    fail |= (p.req_cpu > 0) & (p.req_cpu_d > r.free_cpu);
    fail |= (p.req_mem > 0) & (p.req_mem_d > r.free_mem);
  }
  return fail ? 4 : ST_FEASIBLE;
}

// Plugin weight x score (both < 2^24): v_mul_u32_u24, full rate.  Written as
// asm because the compiler turns __umul24 of these operands into
// v_mul_lo_u32, a quarter-rate instruction (two per node in the sweep).
__device__ __forceinline__ uint32_t wmul(uint32_t w, uint32_t x) {
  uint32_t r;
  asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(w), "v"(x));
  return r;
}

// w * x + y, all < 2^24 (v_mad_u32_u24, full rate)
__device__ __forceinline__ uint32_t wmad(uint32_t w, uint32_t x, uint32_t y) {
  uint32_t r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(w), "v"(x), "v"(y));
  return r;
}

// the same with a wave-uniform w read from an SGPR (VOP3 takes one): no
// v_mov of the weight per use where VGPRs are short
__device__ __forceinline__ uint32_t wmad_s(uint32_t w, uint32_t x, uint32_t y) {
  uint32_t r;
  asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "s"(w), "v"(x), "v"(y));
  return r;
}

// leastRequestedScore(requested, capacity) = (capacity - requested) * 100 / capacity
// (int64 truncation; 0 when requested > capacity) from x = max(lf100 - nz100, 0)
// = max(capacity - requested, 0) * 100, exact.  With y = RN(1 / capacity),
// fma(x, y, 2^-45) lies within 1.9e-14 of x / capacity + 2^-45 and the exact
// quotient's fractional part is 0 or in [1/capacity, 1 - 1/capacity]; for
// capacity < 2^44 (ks_nodes_upsert enforces it) 2^-45 is above the error and
// 1/capacity above both, so truncation gives the exact floor: no remainder
// correction.  Proof in DESIGN.md §4; checked by tools/markstein_check.cpp.
constexpr double LA_EPS = 0x1p-45;
// The max with 0 is the conversion's: x = lf100 - nz100 is a multiple of 100,
// so a negative x gives fma <= -100 / capacity + 2^-45 < 0, which
// v_cvt_u32_f64 clamps to 0 (an unsigned conversion of a negative double is
// undefined in C++, hence the instruction itself).
__device__ __forceinline__ int32_t least_requested(double lf100, double pod_nz100, double inv) {
  const double q = __builtin_fma(lf100 - pod_nz100, inv, LA_EPS);  // x >= 0: truncation == floor; inv == 0 -> 0
  uint32_t r;
  asm("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(q));
  return (int32_t)r;
}

__device__ __forceinline__ int32_t score_la(const PodDev &p, const NodeRegs &r) {
  // nodeScore / weightSum: a zero-allocatable resource adds 0 and is not counted
  return (least_requested(r.lf100_cpu, p.nz100_cpu, r.inv_cpu) + least_requested(r.lf100_mem, p.nz100_mem, r.inv_mem)) >>
         r.lashift;
}

// RN(a / b) from y = RN(1 / b): q0 = RN(a y) is within one ulp of a/b, the
// remainder a - b q0 is exact by FMA, and one correction q0 + r y rounds to the
// IEEE quotient (Markstein).  Checked against true division over the operand
// domain in tools/markstein_check.cpp and by every parity test.
__device__ __forceinline__ double div_rn(double a, double b, double y) {
  const double q0 = a * y;
  const double r = __builtin_fma(-b, q0, a);
  return __builtin_fma(r, y, q0);
}

// sc / sm: Requested + the pod's request (the sweep shares them with Fit)
__device__ __forceinline__ int32_t score_ba_sum(double sc, double sm, const NodeRegs &r) {
  // fraction = min(1, requested / allocatable) as an IEEE binary64 quotient
  // (exact numerator); std = |(f0 - f1) / 2| with two fractions, else 0
  const double f0 = fmin(div_rn(sc, r.acpu_d, r.inv_cpu), 1.0);
  const double f1 = fmin(div_rn(sm, r.amem_d, r.inv_mem), 1.0);
  // 1 - std in one FMA: the product |f0 - f1| * bamul (0.5 or 0) is exact,
  // so the FMA rounds the same difference upstream's 1 - std rounds
  const double om = __builtin_fma(-fabs(f0 - f1), r.bamul, 1.0);
  return (int32_t)(om * 100.0);  // in [0, 100]
}

__device__ __forceinline__ int32_t score_ba(const PodDev &p, const NodeRegs &r) {
  return score_ba_sum(r.rcpu + p.req_cpu_d, r.rmem + p.req_mem_d, r);
}

__device__ __forceinline__ int64_t taint_raw(const PodDev &p, const NodeExt &e) {
  return (int64_t)__popcll(e.prefer & ~p.tol_prefer);
}

// DefaultNormalizeScore(100, reverse) for one element.
__device__ __forceinline__ int64_t normalize(int64_t raw, int64_t mx, bool reverse) {
  if (mx == 0) return reverse ? 100 : 0;
  const int64_t s = (int64_t)((uint32_t)(100 * raw) / (uint32_t)mx);  // 0 <= raw <= mx < 2^25
  return reverse ? 100 - s : s;
}

// Plugin scores are in [0, 100] and ks_open caps the weights at 10000, so the
// weighted sum fits 23 bits: 24-bit multiplies, 32-bit adds.
template <bool EXT>
__device__ __forceinline__ int32_t total_score(const PodDev &p, const uint64_t *clauses, const NodeRegs &r,
                                               const NodeExt &e, const Weights &w, int64_t tt_max,
                                               int64_t na_max) {
  int32_t t = (int32_t)wmul((uint32_t)w.fit, (uint32_t)score_la(p, r)) +
              (int32_t)wmul((uint32_t)w.ba, (uint32_t)score_ba(p, r));
  int32_t tt = 100;
  if (EXT && (p.flags & PF_TT)) tt = (int32_t)normalize(taint_raw(p, e), tt_max, true);
  t += w.tt * tt;  // wave-uniform unless TaintToleration is normalised per node
  if (p.flags & PF_HAS_PREF) {
    int32_t na = 0;
    if (EXT && (p.flags & PF_NA)) na = (int32_t)normalize(preferred_raw(p, clauses, e, r.slot), na_max, false);
    t += (int32_t)wmul((uint32_t)w.na, (uint32_t)na);
  }
  return t;  // + w.il * 0 (ImageLocality: nodes report no images)
}

__device__ __forceinline__ uint64_t pack_key(int64_t total, uint32_t slot) {
  return ((uint64_t)(total + 1) << 32) | (uint64_t)(0xFFFFFFFFu - slot);
}

// label / taint words of a node as gathered next to its key (CandExt::w)
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

}  // namespace ks
