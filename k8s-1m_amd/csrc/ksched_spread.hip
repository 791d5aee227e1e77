// ksched_spread.hip — gfx950 kernels of the PodTopologySpread path.
//
// A pod with topology spread constraints depends on counts aggregated over
// whole topology domains (every node of a zone shares its zone's count), so a
// commit changes the score of every node in the committed node's domain: the
// round kernels' premise (a commit changes only its own node) does not hold.
// Such pods are scheduled one at a time, in queue order, by this chain of
// node-parallel passes over the same SoA node table (upstream v1.31.3
// pkg/scheduler/framework/plugins/podtopologyspread, restated in oracle.cpp):
//
//   spread_prep    PreFilter (filtering.go#calPreFilterState) and the
//                  PreScore counts (scoring.go#PreScore): matching bound pods
//                  of every eligible node summed per topology domain
//   spread_min     criticalPaths[0] / TpKeyToDomainsNum per DoNotSchedule
//                  constraint
//   spread_filter  the whole filter chain + PodTopologySpread.Filter; Score
//                  domains of the filtered nodes; normaliser maxima
//   spread_score   Score: Σ cnt·log(size+2) + (maxSkew-1), math.Round; min/max
//   spread_select  total score of every feasible node, NormalizeScore,
//                  packed-key argmax; clears the domain scratch
//   spread_commit  the result and AssumePod (resources, pod count, the bound
//                  pod's selector-class and term-class counts)
//
// InterPodAffinity (interpodaffinity/filtering.go, scoring.go) rides the same
// chain: spread_prep sums each AffDev record's count column per topology
// domain over every node (PreFilter's affinity / anti-affinity /
// existing-anti-affinity counts, PreScore's topologyScore), spread_filter
// checks them (satisfyPodAffinity, satisfyPodAntiAffinity,
// satisfyExistingPodsAntiAffinity) and takes the raw score, spread_select
// normalises it (float64 min-max, as NormalizeScore).
//
// Domain counts are aggregated per block in LDS for low-cardinality keys
// (zones), with global atomics only for high-cardinality ones (hostnames).
#include <hip/hip_runtime.h>

#include "ksched_dev.hpp"
#include "ksched_eval.hpp"
#include "ksched_kernels.hpp"
#include "ksched_util.hpp"

namespace ks {

namespace {

constexpr int SP_THREADS = 1024;  // few fat blocks (at most SPREAD_MAX_BLOCKS): one partial record each
constexpr uint32_t SP_LDS = 4096;     // LDS domain-histogram entries per block
constexpr uint32_t SP_LDS_DOM = 1024; // keys with at most this many domains aggregate in LDS
constexpr uint32_t SP_OFF_NONE = 0xFFFFFFFFu;
constexpr int8_t SST_FEASIBLE = -1, SST_EMPTY = -2, SST_IGNORED = -3;  // per-position status
constexpr int SP_BATCH = 4;           // positions per thread per step of the score / select passes

// The pod's one-pod-path program (ksched_dev.hpp SoloHdr): SpreadDev, XResDev, ImageDev records.
__device__ __forceinline__ const SoloHdr &solo_hdr(const SpreadArgs &a, const PodDev &p) {
  return *reinterpret_cast<const SoloHdr *>(a.clauses + p.solo_off);
}
__device__ __forceinline__ const SpreadDev *spread_recs(const SpreadArgs &a, const PodDev &p) {
  return reinterpret_cast<const SpreadDev *>(&solo_hdr(a, p) + 1);
}
__device__ __forceinline__ uint32_t spread_count(const SpreadArgs &a, const PodDev &p) { return solo_hdr(a, p).n_spread; }
__device__ __forceinline__ const XResDev *xres_recs(const SpreadArgs &a, const PodDev &p) {
  return reinterpret_cast<const XResDev *>(spread_recs(a, p) + solo_hdr(a, p).n_spread);
}
__device__ __forceinline__ const ImageDev *image_recs(const SpreadArgs &a, const PodDev &p) {
  return reinterpret_cast<const ImageDev *>(xres_recs(a, p) + solo_hdr(a, p).n_xres);
}
__device__ __forceinline__ const AffDev *aff_recs(const SpreadArgs &a, const PodDev &p) {
  return reinterpret_cast<const AffDev *>(image_recs(a, p) + solo_hdr(a, p).n_img);
}
// Count column of an InterPodAffinity record at a position.
__device__ __forceinline__ uint32_t aff_count(const SpreadArgs &a, const AffDev &r, uint32_t pos) {
  return ((r.kind & AF_TERM) ? a.tcnt : a.cnt)[(size_t)r.col * a.npos + pos];
}
constexpr uint64_t IPA_BIAS = 1ull << 63;  // signed raw scores as unsigned min / max keys

// interpodaffinity Filter over the prefilter domain counts: every required
// affinity key present and its domain holding a pod that matches all the
// required affinity terms (unless no such pod exists anywhere and the pod
// matches its own terms), no required anti-affinity match in the node's
// domains, no bound pod's required anti-affinity term matching the pod there.
// Domain sum of record r at a position whose domain is d (!= DOM_NONE).
// The filter pass's view of the records at one position: domain sums of the
// low-cardinality records staged in LDS (aoff: segment per record or
// SP_OFF_NONE), the first AF_PF records' domain ids and per-node counts
// loaded with the position's other inputs.
constexpr int AF_PF = 4;
struct AffView {
  const uint32_t *aoff, *lds;
  uint32_t dm[AF_PF], nc[AF_PF];
};
__device__ __forceinline__ uint32_t aff_dom(const SpreadArgs &a, const AffDev *ad, const AffView &v, uint32_t r,
                                            uint32_t pos) {
  if (r >= (uint32_t)AF_PF) return a.dom[(size_t)ad[r].key * a.npos + pos];
  uint32_t d = v.dm[0];
#pragma unroll
  for (int k = 1; k < AF_PF; ++k) d = r == (uint32_t)k ? v.dm[k] : d;
  return d;
}
__device__ __forceinline__ uint32_t aff_sum(const SpreadArgs &a, const AffDev *ad, const AffView &v, uint32_t r,
                                            uint32_t pos, uint32_t d) {
  const AffDev &q = ad[r];
  if (q.kind & AF_NODE) {
    if (r >= (uint32_t)AF_PF) return aff_count(a, q, pos);
    uint32_t c = v.nc[0];
#pragma unroll
    for (int k = 1; k < AF_PF; ++k) c = r == (uint32_t)k ? v.nc[k] : c;
    return c;
  }
  const uint32_t o = v.aoff[r];
  return o != SP_OFF_NONE ? v.lds[o + d] : a.adcnt[(size_t)r * a.dom_cap + d];
}
__device__ __forceinline__ void aff_prefetch(const SpreadArgs &a, const AffDev *ad, uint32_t na, uint32_t pos,
                                             AffView &v) {
#pragma unroll
  for (int r = 0; r < AF_PF; ++r) {
    v.dm[r] = (uint32_t)r < na ? a.dom[(size_t)ad[r].key * a.npos + pos] : DOM_NONE;
    v.nc[r] = (uint32_t)r < na && (ad[r].kind & AF_NODE) ? aff_count(a, ad[r], pos) : 0u;
  }
}

__device__ __forceinline__ bool ipa_fits(const SpreadArgs &a, const AffDev *ad, uint32_t na, const AffView &v,
                                         uint32_t pos, bool first_ok) {
  bool has_req = false, exist = true;
  for (uint32_t r = 0; r < na; ++r) {
    const uint32_t kind = ad[r].kind & AF_KIND;
    if (kind > AF_EXIST_ANTI) continue;
    const uint32_t d = aff_dom(a, ad, v, r, pos);
    if (kind == AF_REQ_AFF) {
      has_req = true;
      if (d == DOM_NONE) return false;  // all topology labels must exist on the node
      if (!aff_sum(a, ad, v, r, pos, d)) exist = false;
    } else if (d != DOM_NONE && aff_sum(a, ad, v, r, pos, d)) {
      return false;
    }
  }
  return !has_req || exist || first_ok;
}

// interpodaffinity Score: Σ topologyScore[key][node's value].
__device__ __forceinline__ int64_t ipa_raw_score(const SpreadArgs &a, const AffDev *ad, uint32_t na, const AffView &v,
                                                 uint32_t pos) {
  int64_t raw = 0;
  for (uint32_t r = 0; r < na; ++r) {
    if ((ad[r].kind & AF_KIND) != AF_SCORE) continue;
    const uint32_t d = aff_dom(a, ad, v, r, pos);
    if (d != DOM_NONE) raw += (int64_t)ad[r].weight * (int64_t)aff_sum(a, ad, v, r, pos, d);
  }
  return raw;
}

// The pod's program staged in LDS by the node-parallel passes: read in every
// node iteration, records in global memory would be re-fetched after each of
// the iteration's stores (the compiler cannot rule out aliasing).
struct SoloLds {
  SoloHdr h;
  SpreadDev sd[MAX_SPREAD];
  XResDev xr[MAX_XRES];
  ImageDev img[MAX_IMG];
  AffDev ad[MAX_AFF];
};
__device__ __forceinline__ void stage_solo(const SpreadArgs &a, const PodDev &p, SoloLds &s) {
  const SoloHdr &h = solo_hdr(a, p);
  const uint32_t t = threadIdx.x;
  if (t == 0) s.h = h;
  if (t < h.n_spread) s.sd[t] = spread_recs(a, p)[t];
  if (t < h.n_xres) s.xr[t] = xres_recs(a, p)[t];
  if (t < h.n_img) s.img[t] = image_recs(a, p)[t];
  if (t < h.n_aff) s.ad[t] = aff_recs(a, p)[t];
}

// imagelocality#calculatePriority over sumImageScores of the node (label bits
// of the "image present" keys); 0 without present images.
__device__ __forceinline__ int64_t image_score(const SoloLds &sl, const NodeExt &e) {
  const SoloHdr &h = sl.h;
  if (!h.n_img) return 0;
  const ImageDev *g = sl.img;
  int64_t sum = 0;
  for (uint32_t k = 0; k < h.n_img; ++k) {
    // the label word by a select chain: a dynamic index would put e.lab in scratch
    const uint32_t wi = g[k].bit >> 6;
    uint64_t w = 0;
#pragma unroll
    for (int q = 0; q < LW; ++q) w = (uint32_t)q == wi ? e.lab[q] : w;
    if ((w >> (g[k].bit & 63)) & 1ull) sum += g[k].scaled;
  }
  const int64_t mb = 1024 * 1024, min_t = 23 * mb, max_t = 1000 * mb * (int64_t)h.n_containers;
  sum = sum < min_t ? min_t : (sum > max_t ? max_t : sum);
  return 100 * (sum - min_t) / (max_t - min_t);
}

// Go math.Log (log.go, fdlibm e_log.c; the amd64 assembly performs the same
// operations) for a finite x >= 2, one rounding per operation.
__device__ double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  // Frexp: x = f1 * 2^ki, f1 in [0.5, 1)
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  int ki = (int)((b >> 52) & 0x7FF) - 1022;
  double f1 = __longlong_as_double((long long)((b & 0x800FFFFFFFFFFFFFull) | (1022ull << 52)));
  if (f1 < 0.70710678118654752440) {  // Sqrt2 / 2
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1;
  const double k = (double)ki;
  const double s = f / (2 + f);
  const double s2 = s * s;
  const double s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2;
  const double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o);
    v = w > v ? w : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o);
    v = w < v ? w : v;
  }
  return v;
}

// LDS segments of the low-cardinality constraints (thread 0; caller syncs);
// with `aoff`, then of the InterPodAffinity records the prep pass sums.
__device__ void lds_segments(const SpreadArgs &a, const SpreadDev *sd, uint32_t n, uint32_t *off,
                             const AffDev *ad = nullptr, uint32_t na = 0, uint32_t *aoff = nullptr) {
  uint32_t o = 0;
  for (uint32_t c = 0; c < n; ++c) {
    const uint32_t nd = a.ndom[sd[c].key];
    const bool small = nd <= SP_LDS_DOM && o + nd <= SP_LDS;
    off[c] = small ? o : SP_OFF_NONE;
    if (small) o += nd;
  }
  for (uint32_t r = 0; r < na; ++r) {
    const uint32_t nd = a.ndom[ad[r].key];
    const bool small = (ad[r].kind & AF_KIND) != AF_OWN && !(ad[r].kind & AF_NODE) && nd <= SP_LDS_DOM &&
                       o + nd <= SP_LDS;
    aoff[r] = small ? o : SP_OFF_NONE;
    if (small) o += nd;
  }
}

__device__ __forceinline__ uint32_t grid_threads() { return gridDim.x * blockDim.x; }

// A position's inputs of the node passes, every load issued before any branch:
// the passes visit each position once, so the slot -> pod-count -> resource-row
// chain of load_core (three dependent round trips through the memory system)
// becomes one.  dm / kc: domain ids and selector-class counts of the pod's
// first SP_PF constraints (kc only where `want_cnt`).
constexpr int SP_PF = 4;
struct PosIn {
  uint32_t slot;
  int32_t ap, np;
  int64_t acpu, amem, rc, rm, zc, zm;
  uint32_t dm[SP_PF], kc[SP_PF];
};
__device__ __forceinline__ void load_pos(const SpreadArgs &a, const SpreadDev *sd, uint32_t n, uint32_t want_cnt,
                                         uint32_t pos, bool core, PosIn &v) {
  v.slot = a.pos_slot[pos];
  v.ap = a.t.apods[pos];
  if (core) {
    v.np = a.t.npods[pos];
    v.acpu = a.t.acpu[pos];
    v.amem = a.t.amem[pos];
    v.rc = a.t.rcpu[pos];
    v.rm = a.t.rmem[pos];
    v.zc = a.t.zcpu[pos];
    v.zm = a.t.zmem[pos];
  }
#pragma unroll
  for (int c = 0; c < SP_PF; ++c) {
    v.dm[c] = (uint32_t)c < n ? a.dom[(size_t)sd[c].key * a.npos + pos] : DOM_NONE;
    v.kc[c] = (uint32_t)c < n && ((want_cnt >> c) & 1u) ? a.cnt[(size_t)sd[c].cls * a.npos + pos] : 0u;
  }
  // the values are needed before the first branch: no load sinks below it
  asm volatile("" ::"v"(v.slot), "v"(v.ap), "v"(v.dm[0]), "v"(v.dm[1]), "v"(v.dm[2]), "v"(v.dm[3]), "v"(v.kc[0]),
               "v"(v.kc[1]), "v"(v.kc[2]), "v"(v.kc[3]));
  if (core) asm volatile("" ::"v"(v.np), "v"(v.acpu), "v"(v.amem), "v"(v.rc), "v"(v.rm), "v"(v.zc), "v"(v.zm));
}
// Domain id of constraint c at the position (prefetched for c < SP_PF).
__device__ __forceinline__ uint32_t pos_dom(const SpreadArgs &a, const SpreadDev *sd, const PosIn &v, uint32_t c,
                                            uint32_t pos) {
  if (c >= (uint32_t)SP_PF) return a.dom[(size_t)sd[c].key * a.npos + pos];
  uint32_t d = v.dm[0];
#pragma unroll
  for (int k = 1; k < SP_PF; ++k) d = c == (uint32_t)k ? v.dm[k] : d;
  return d;
}
// Selector-class count of constraint c at the position (prefetched where want_cnt).
__device__ __forceinline__ uint32_t pos_cnt(const SpreadArgs &a, const SpreadDev *sd, const PosIn &v, uint32_t c,
                                            uint32_t pos) {
  if (c >= (uint32_t)SP_PF) return a.cnt[(size_t)sd[c].cls * a.npos + pos];
  uint32_t k = v.kc[0];
#pragma unroll
  for (int q = 1; q < SP_PF; ++q) k = c == (uint32_t)q ? v.kc[q] : k;
  return k;
}
__device__ __forceinline__ void pos_regs(const SpreadArgs &a, uint32_t pos, const PosIn &v, NodeRegs &r) {
  if (v.ap < 0) load_core(a.t, pos, v.slot, false, r);  // empty slot: load_core's benign values, no loads
  else r = make_regs(v.acpu, v.amem, v.rc, v.rm, v.zc, v.zm, v.ap, v.np, v.slot);
}

// Totals of the accumulator copies (ACC_SHARDS) written by the previous passes.
struct Totals {
  uint32_t fail[NFILT + 2];
  uint32_t feasible, ignored, tt_max, na_max;
  uint64_t pts_min, pts_max, ipa_min, ipa_max, best;
};
__device__ __forceinline__ Totals acc_totals(const SpreadAcc *acc) {
  Totals t{};
  t.pts_min = t.ipa_min = ~0ull;
  for (int k = 0; k < ACC_SHARDS; ++k) {
    const SpreadAccShard &q = acc->sh[k];
    for (int f = 0; f < NFILT + 2; ++f) t.fail[f] += q.fail[f];
    t.ipa_min = min(t.ipa_min, q.ipa_min);
    t.ipa_max = max(t.ipa_max, q.ipa_max);
    t.feasible += q.feasible;
    t.ignored += q.ignored;
    t.tt_max = max(t.tt_max, q.tt_max);
    t.na_max = max(t.na_max, q.na_max);
    t.pts_min = min(t.pts_min, q.pts_min);
    t.pts_max = max(t.pts_max, q.pts_max);
    t.best = max(t.best, q.best);
  }
  return t;
}
__device__ __forceinline__ SpreadAccShard &acc_shard(const SpreadArgs &a) { return a.acc->sh[blockIdx.x % ACC_SHARDS]; }

}  // namespace

// ------------------------------------------------------------------ prep
// Per DoNotSchedule constraint c: dcnt[c][d] = matching pods on the eligible
// nodes of domain d (the node has every DoNotSchedule key and passes the
// constraint's inclusion policies), dflag[c][d] bit 0 = d has an eligible
// node.  (The ScheduleAnyway counts are taken by the filter pass, which
// visits every node anyway.)  Launched only for pods with DoNotSchedule
// constraints.  InterPodAffinity: adcnt[r][d] = Σ count column of record r
// over every node of domain d (any node: upstream's PreFilter / PreScore walk
// all nodes), aff_any / score_any = some affinityCounts / topologyScore entry.
__global__ __launch_bounds__(SP_THREADS) void spread_prep_kernel(SpreadArgs a) {
  __shared__ uint32_t s_h[SP_LDS];
  __shared__ uint32_t s_off[MAX_SPREAD];
  __shared__ uint32_t s_aoff[MAX_AFF];
  __shared__ SoloLds s_solo;
  const PodDev p = a.pods[a.pod];
  stage_solo(a, p, s_solo);
  for (uint32_t i = threadIdx.x; i < SP_LDS; i += SP_THREADS) s_h[i] = 0;
  __syncthreads();
  const SpreadDev *sd = s_solo.sd;
  const uint32_t n = s_solo.h.n_spread;
  const AffDev *ad = s_solo.ad;
  const uint32_t na = s_solo.h.n_aff;
  if (threadIdx.x == 0) lds_segments(a, sd, n, s_off, ad, na, s_aoff);
  __syncthreads();
  bool aff_needed = false, taint_needed = false;
  for (uint32_t c = 0; c < n; ++c) {
    if (sd[c].flags & SP_SCORE) continue;
    aff_needed |= (sd[c].flags & SP_AFF) && (p.flags & PF_AFF);
    taint_needed |= (sd[c].flags & SP_TAINT) != 0;
  }
  uint32_t want_cnt = 0;  // DoNotSchedule counts this pass takes per node
  for (uint32_t c = 0; c < n && c < (uint32_t)SP_PF; ++c)
    if (!(sd[c].flags & SP_SCORE) && sd[c].cls != CLS_NONE) want_cnt |= 1u << c;
  bool any_aff = false, any_score = false;
  for (uint32_t pos = blockIdx.x * SP_THREADS + threadIdx.x; pos < a.npos; pos += grid_threads()) {
    // the first AF_PF summed records' counts and domain ids, loaded with the
    // position's other inputs
    uint32_t pv[AF_PF], pd[AF_PF];
#pragma unroll
    for (int r = 0; r < AF_PF; ++r) {
      const bool summed = (uint32_t)r < na && (ad[r].kind & AF_KIND) != AF_OWN && !(ad[r].kind & AF_NODE);
      pv[r] = summed ? aff_count(a, ad[r], pos) : 0u;
      pd[r] = summed ? a.dom[(size_t)ad[r].key * a.npos + pos] : DOM_NONE;
    }
    PosIn in;
    load_pos(a, sd, n, want_cnt, pos, false, in);
    const uint32_t slot = in.slot;
    if (slot == SLOT_NONE || in.ap < 0) continue;
    for (uint32_t r = 0; r < na; ++r) {
      const AffDev &q = ad[r];
      const uint32_t kind = q.kind & AF_KIND;
      if (kind == AF_OWN || (q.kind & AF_NODE)) continue;  // per-node records: read in place
      uint32_t v = pv[0], d = pd[0];
#pragma unroll
      for (int k = 1; k < AF_PF; ++k) {
        v = r == (uint32_t)k ? pv[k] : v;
        d = r == (uint32_t)k ? pd[k] : d;
      }
      if (r >= (uint32_t)AF_PF) v = aff_count(a, q, pos);
      if (!v) continue;
      if (r >= (uint32_t)AF_PF) d = a.dom[(size_t)q.key * a.npos + pos];
      if (d == DOM_NONE) continue;  // no topology pair for this node
      any_aff |= kind == AF_REQ_AFF;
      any_score |= kind == AF_SCORE;
      if (s_aoff[r] != SP_OFF_NONE) atomicAdd(&s_h[s_aoff[r] + d], v);
      else atomicAdd(&a.adcnt[(size_t)r * a.dom_cap + d], v);
    }
    NodeExt e;
    if (aff_needed || taint_needed) load_ext(a.t, pos, true, e);
    const bool aff_ok = !aff_needed || required_match(p, a.clauses, e, slot);
    const bool taint_ok = !taint_needed || (e.hard & ~p.tol_hard & ~UNSCHED_BIT) == 0;
    bool all_f = true;
    for (uint32_t c = 0; c < n; ++c)
      if (!(sd[c].flags & SP_SCORE) && pos_dom(a, sd, in, c, pos) == DOM_NONE) all_f = false;
    if (!all_f) continue;
    for (uint32_t c = 0; c < n; ++c) {
      const SpreadDev &s = sd[c];
      if ((s.flags & SP_SCORE) || ((s.flags & SP_AFF) && !aff_ok) || ((s.flags & SP_TAINT) && !taint_ok)) continue;
      const uint32_t d = pos_dom(a, sd, in, c, pos);
      const uint32_t k = s.cls == CLS_NONE ? 0u : pos_cnt(a, sd, in, c, pos);
      if (s_off[c] != SP_OFF_NONE) {
        const uint32_t e = s_off[c] + d;
        if (k) atomicAdd(&s_h[e], k);
        if (!(s_h[e] >> 31)) atomicOr(&s_h[e], 0x80000000u);
      } else {
        if (k) atomicAdd(&a.dcnt[(size_t)c * a.dom_cap + d], k);
        if (!(a.dflag[(size_t)c * a.dom_cap + d] & 1u)) atomicOr(&a.dflag[(size_t)c * a.dom_cap + d], 1u);
      }
    }
  }
  const int blk_aff = __syncthreads_or(any_aff ? 1 : 0);
  const int blk_score = __syncthreads_or(any_score ? 1 : 0);
  if (threadIdx.x == 0) {
    if (blk_aff) atomicOr(&a.acc->aff_any, 1u);
    if (blk_score) atomicOr(&a.acc->score_any, 1u);
  }
  for (uint32_t c = 0; c < n; ++c) {
    if (s_off[c] == SP_OFF_NONE) continue;
    for (uint32_t d = threadIdx.x; d < a.ndom[sd[c].key]; d += SP_THREADS) {
      const uint32_t v = s_h[s_off[c] + d];
      if (v & 0x7FFFFFFFu) atomicAdd(&a.dcnt[(size_t)c * a.dom_cap + d], v & 0x7FFFFFFFu);
      if (v >> 31) atomicOr(&a.dflag[(size_t)c * a.dom_cap + d], 1u);
    }
  }
  for (uint32_t r = 0; r < na; ++r) {
    if (s_aoff[r] == SP_OFF_NONE) continue;
    for (uint32_t d = threadIdx.x; d < a.ndom[ad[r].key]; d += SP_THREADS) {
      const uint32_t v = s_h[s_aoff[r] + d];
      if (v) atomicAdd(&a.adcnt[(size_t)r * a.dom_cap + d], v);
    }
  }
}

// ------------------------------------------------------------------- min
// criticalPaths[0].MatchNum (min over the eligible domains) and the number of
// eligible domains of every DoNotSchedule constraint.
__global__ __launch_bounds__(SP_THREADS) void spread_min_kernel(SpreadArgs a) {
  __shared__ uint32_t s_r[SP_THREADS / WAVE][2];
  const PodDev p = a.pods[a.pod];
  const SpreadDev *sd = spread_recs(a, p);
  const uint32_t n = spread_count(a, p);
  const uint32_t lane = threadIdx.x % WAVE, wid = threadIdx.x / WAVE;
  for (uint32_t c = 0; c < n; ++c) {
    if (sd[c].flags & SP_SCORE) continue;
    uint32_t mn = 0xFFFFFFFFu, cnt = 0;
    for (uint32_t d = blockIdx.x * SP_THREADS + threadIdx.x; d < a.ndom[sd[c].key]; d += grid_threads()) {
      if (!(a.dflag[(size_t)c * a.dom_cap + d] & 1u)) continue;
      mn = min(mn, a.dcnt[(size_t)c * a.dom_cap + d]);
      ++cnt;
    }
    mn = wave_min(mn);
    cnt = wave_sum(cnt);
    if (lane == 0) {
      s_r[wid][0] = mn;
      s_r[wid][1] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < SP_THREADS / WAVE; ++w) {
        mn = min(mn, s_r[w][0]);
        cnt += s_r[w][1];
      }
      if (cnt) {
        atomicMin(&a.acc->min_match[c], mn);
        atomicAdd(&a.acc->ndomains[c], cnt);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- filter
// Filter chain in default-profile order, PodTopologySpread last
// (filtering.go#Filter: node without the key -> UnschedulableAndUnresolvable;
// matchNum + selfMatch - minMatchNum > maxSkew -> Unschedulable).  Every
// node: PreScore's ScheduleAnyway counts (dcnt over the nodes PreScore
// counts: requireAllTopologies, inclusion policies; a node lacking the key
// belongs to the "" domain, id 0, when it is not required).  Feasible nodes:
// normaliser maxima, PreScore's ignored nodes, the Score domains of the rest
// (topoSize), and the node's normalisation-free score parts packed for the
// select pass (Σ weight x LeastAllocated / BalancedAllocation, raw
// TaintToleration, raw NodeAffinity), so that it reads 8 bytes per node
// instead of the resource and label rows.
__device__ __forceinline__ uint64_t pack_part(uint32_t base, uint32_t tt_raw, uint32_t na_raw) {
  return (uint64_t)base | ((uint64_t)(tt_raw & 0xFFu) << 32) | ((uint64_t)(na_raw & 0xFFFFFFu) << 40);
}

// Block-reduction slots of the filter pass: first failures per plugin, then
// feasible / ignored counts and the normaliser maxima.
constexpr int RF = NFILT + 2, R_FEAS = RF, R_IGN = RF + 1, R_TT = RF + 2, R_NA = RF + 3, R_N = RF + 4;

// AFF: the pod has InterPodAffinity records (SPL_AFF); the variant without
// them keeps their prefetched values out of the registers of spread pods.
// PROBE: the percentageOfNodesToScore probe pass (win_mode 1) -- the filter
// chain only; as a template parameter the score work compiles away there
template <bool AFF, bool PROBE = false>
__global__ __launch_bounds__(SP_THREADS) void spread_filter_kernel(SpreadArgs a) {
  __shared__ uint32_t s_seen[SP_LDS / 32];
  __shared__ uint32_t s_h[SP_LDS];
  __shared__ uint32_t s_off[MAX_SPREAD];
  __shared__ uint32_t s_aoff[MAX_AFF];
  __shared__ uint32_t s_minm[MAX_SPREAD];
  __shared__ uint32_t s_red[SP_THREADS / WAVE][R_N];
  __shared__ uint64_t s_r64[SP_THREADS / WAVE][2];
  __shared__ SoloLds s_solo;
  const PodDev p = a.pods[a.pod];
  stage_solo(a, p, s_solo);
  for (uint32_t i = threadIdx.x; i < SP_LDS / 32; i += SP_THREADS) s_seen[i] = 0;
  for (uint32_t i = threadIdx.x; i < SP_LDS; i += SP_THREADS) s_h[i] = 0;
  __syncthreads();
  const SpreadDev *sd = s_solo.sd;
  const uint32_t n = s_solo.h.n_spread;
  if (threadIdx.x == 0) lds_segments(a, sd, n, s_off, s_solo.ad, AFF ? s_solo.h.n_aff : 0u, s_aoff);
  __syncthreads();
  // InterPodAffinity domain sums of the low-cardinality records (the prep
  // pass's), read per node by the checks and the raw score
  for (uint32_t r = 0; r < (AFF ? s_solo.h.n_aff : 0u); ++r) {
    if (s_aoff[r] == SP_OFF_NONE) continue;
    for (uint32_t d = threadIdx.x; d < a.ndom[s_solo.ad[r].key]; d += SP_THREADS)
      s_h[s_aoff[r] + d] = a.adcnt[(size_t)r * a.dom_cap + d];
  }
  // DoNotSchedule constraints: the prep pass's domain counts (low-cardinality
  // keys: into their s_h segments, which only ScheduleAnyway constraints
  // accumulate into) and minMatchNum, read per node by the skew check
  for (uint32_t c = 0; c < n; ++c) {
    if ((sd[c].flags & SP_SCORE) || s_off[c] == SP_OFF_NONE) continue;
    for (uint32_t d = threadIdx.x; d < a.ndom[sd[c].key]; d += SP_THREADS)
      s_h[s_off[c] + d] = a.dcnt[(size_t)c * a.dom_cap + d];
  }
  if (threadIdx.x < n && !(sd[threadIdx.x].flags & SP_SCORE)) {
    const uint32_t c = threadIdx.x;
    s_minm[c] = a.acc->ndomains[c] < (uint32_t)sd[c].min_domains ? 0u : a.acc->min_match[c];
  }
  uint32_t want_cnt = 0;  // ScheduleAnyway counts this pass takes per node
  for (uint32_t c = 0; c < n && c < (uint32_t)SP_PF; ++c)
    if ((sd[c].flags & (SP_SCORE | SP_HOST)) == SP_SCORE && sd[c].cls != CLS_NONE) want_cnt |= 1u << c;
  __syncthreads();
  const uint32_t n_xres = s_solo.h.n_xres;
  const AffDev *ad = s_solo.ad;
  const uint32_t na = AFF ? s_solo.h.n_aff : 0u;
  bool ipa_filter = false;
  for (uint32_t r = 0; r < na; ++r) ipa_filter |= (ad[r].kind & AF_KIND) <= AF_EXIST_ANTI;
  const bool ipa_first_ok = !a.acc->aff_any && (s_solo.h.aff_flags & AFF_SELF);
  bool ipa_score = false, node_score = false;  // topologyScore records; per-node ones
  for (uint32_t r = 0; r < na; ++r)
    if ((ad[r].kind & AF_KIND) == AF_SCORE) {
      ipa_score = true;
      node_score |= (ad[r].kind & AF_NODE) != 0;
    }
  bool score_any = false;  // topologyScore entries of the per-node records
  bool any_s = false, aff_needed = false, taint_needed = false;
  for (uint32_t c = 0; c < n; ++c) {
    if (!(sd[c].flags & SP_SCORE)) continue;
    any_s |= !(sd[c].flags & SP_HOST);
    aff_needed |= (sd[c].flags & SP_AFF) != 0;
    taint_needed |= (sd[c].flags & SP_TAINT) != 0;
  }
  const bool allkeys = p.flags & PF_SPREAD_ALLKEYS;
  // label / taint columns (64 B per node) only for pods that read them: the
  // EXT filter chain and normalising plugins, the spread policies' node
  // affinity / taint checks, ImageLocality's "image present" bits
  const bool need_ext = (p.flags & PF_EXT) || aff_needed || taint_needed || s_solo.h.n_img != 0;
  const uint32_t lane = threadIdx.x % WAVE, wid = threadIdx.x / WAVE;
  uint32_t fails[RF] = {0, 0, 0, 0, 0, 0, 0};
  uint32_t feasible = 0, ignored = 0, tt_max = 0, na_max = 0;
  uint64_t ipa_mn = ~0ull, ipa_mx = 0;
  // percentageOfNodesToScore < 100: the probe pass (filter only, win_st) or
  // the pass over the window spread_window_kernel found
  constexpr bool probe = PROBE;  // (the launcher passes win_mode 1 exactly to this instantiation)
  const bool windowed = !PROBE && a.win_mode == 2;
  const uint32_t w_s0 = windowed ? a.win[1] : 0u, w_x = windowed ? a.win[2] : 0u;
  const bool w_all = !windowed || a.win[3] != 0;
  // the window pass of a pod that reads nothing from the nodes outside the
  // window (no PreScore counts, no per-node topologyScore records) skips them
  // before loading their rows
  const bool w_skip = windowed && !w_all && !any_s && !node_score;
  for (uint32_t pos = blockIdx.x * SP_THREADS + threadIdx.x; pos < a.npos; pos += grid_threads()) {
    if (w_skip) {
      const uint32_t sl = a.pos_slot[pos];
      if (sl != SLOT_NONE && !(w_s0 < w_x ? sl >= w_s0 && sl < w_x : sl >= w_s0 || sl < w_x)) {
        a.st[pos] = SST_EMPTY;
        continue;
      }
    }
    PosIn in;
    AffView av{s_aoff, s_h, {}, {}};
    if (AFF) aff_prefetch(a, ad, na, pos, av);
    load_pos(a, sd, n, want_cnt, pos, true, in);
    const uint32_t slot = in.slot;
    if (slot == SLOT_NONE) continue;
    NodeRegs r;
    pos_regs(a, pos, in, r);
    if (!(r.bits & 1u)) {
      a.st[pos] = SST_EMPTY;
      if (probe) a.win_st[slot] = 0;
      continue;
    }
    if (node_score && !probe)
      for (uint32_t q = 0; q < na; ++q)
        if ((ad[q].kind & (AF_KIND | AF_NODE)) == (AF_SCORE | AF_NODE) && aff_dom(a, ad, av, q, pos) != DOM_NONE &&
            aff_sum(a, ad, av, q, pos, 0))
          score_any = true;
    NodeExt e{};
    if (need_ext) load_ext(a.t, pos, true, e);
    bool all_s = true;
    for (uint32_t c = 0; c < n; ++c)
      if ((sd[c].flags & SP_SCORE) && pos_dom(a, sd, in, c, pos) == DOM_NONE) all_s = false;
    if (any_s && (!allkeys || all_s) && !probe) {
      // PreScore counts (scoring.go#PreScore processAllNode) of this node
      const bool aff_ok = !aff_needed || !(p.flags & PF_AFF) || required_match(p, a.clauses, e, slot);
      const bool taint_ok = !taint_needed || (e.hard & ~p.tol_hard & ~UNSCHED_BIT) == 0;
      for (uint32_t c = 0; c < n; ++c) {
        const SpreadDev &q = sd[c];
        if (!(q.flags & SP_SCORE) || (q.flags & SP_HOST) || ((q.flags & SP_AFF) && !aff_ok) ||
            ((q.flags & SP_TAINT) && !taint_ok))
          continue;
        uint32_t d = pos_dom(a, sd, in, c, pos);
        if (d == DOM_NONE) d = 0;
        const uint32_t k = q.cls == CLS_NONE ? 0u : pos_cnt(a, sd, in, c, pos);
        if (!k) continue;
        if (s_off[c] != SP_OFF_NONE) atomicAdd(&s_h[s_off[c] + d], k);
        else atomicAdd(&a.dcnt[(size_t)c * a.dom_cap + d], k);
      }
    }
    // percentageOfNodesToScore < 100: a node outside the visited window is
    // neither filtered nor counted (its PreScore counts above are: upstream's
    // PreScore walks every node)
    if (windowed && !(w_all || (w_s0 < w_x ? slot >= w_s0 && slot < w_x : slot >= w_s0 || slot < w_x))) {
      a.st[pos] = SST_EMPTY;
      continue;
    }
    int s = filter<true>(p, a.clauses, r, e);
    if (s == ST_FEASIBLE) {
      // NodeResourcesFit (fitsRequest) for ephemeral-storage / scalar resources
      const XResDev *xr = s_solo.xr;
      for (uint32_t k = 0; k < n_xres; ++k) {
        const size_t ix = (size_t)xr[k].col * a.npos + pos;
        if (xr[k].req > a.xalloc[ix] - a.xreq[ix]) s = 4;  // KS_PLUGIN_NODE_RESOURCES_FIT
      }
    }
    if (s == ST_FEASIBLE) {
      for (uint32_t c = 0; c < n; ++c) {
        const SpreadDev &q = sd[c];
        if (q.flags & SP_SCORE) continue;
        const uint32_t d = pos_dom(a, sd, in, c, pos);
        if (d == DOM_NONE) {
          s = PLUGIN_SPREAD;  // ErrReasonNodeLabelNotMatch
          break;
        }
        const uint32_t dc = s_off[c] != SP_OFF_NONE ? s_h[s_off[c] + d] : a.dcnt[(size_t)c * a.dom_cap + d];
        const int64_t skew = (int64_t)dc + ((q.flags & SP_SELF) ? 1 : 0) - (int64_t)s_minm[c];
        if (skew > (int64_t)q.max_skew) {
          s = PLUGIN_SPREAD;  // ErrReasonConstraintsNotMatch
          break;
        }
      }
    }
    if (s == ST_FEASIBLE && ipa_filter && !ipa_fits(a, ad, na, av, pos, ipa_first_ok)) s = PLUGIN_IPA;
    if (probe) {  // the node list (PreFilterResult nodes) and the feasible nodes, by slot
      a.win_st[slot] = (uint8_t)((s != ST_PREFILTERED ? 1u : 0u) | (s == ST_FEASIBLE ? 2u : 0u));
      continue;
    }
    int8_t out = (int8_t)s;
    if (s == ST_FEASIBLE) {
      ++feasible;
      const uint32_t tr = (p.flags & PF_TT) ? (uint32_t)taint_raw(p, e) : 0u;
      const uint32_t nr = (p.flags & PF_NA) ? (uint32_t)preferred_raw(p, a.clauses, e, slot) : 0u;
      tt_max = max(tt_max, tr);
      na_max = max(na_max, nr);
      a.part[pos] = pack_part((uint32_t)a.w.fit * (uint32_t)score_la(p, r) + (uint32_t)a.w.ba * (uint32_t)score_ba(p, r) +
                                  (uint32_t)a.w.il * (uint32_t)image_score(s_solo, e),
                              tr, nr);
      if (ipa_score) {
        const int64_t raw = ipa_raw_score(a, ad, na, av, pos);
        a.ipa_raw[pos] = raw;
        const uint64_t k = (uint64_t)raw + IPA_BIAS;
        ipa_mn = min(ipa_mn, k);
        ipa_mx = max(ipa_mx, k);
      }
      // PreScore (initPreScoreState): with requireAllTopologies a node lacking
      // a ScheduleAnyway key is ignored; the others' domains make topoSize
      if (allkeys && !all_s) {
        ++ignored;
        out = SST_IGNORED;
      } else {
        for (uint32_t c = 0; c < n; ++c) {
          const SpreadDev &q = sd[c];
          if (!(q.flags & SP_SCORE) || (q.flags & SP_HOST)) continue;
          uint32_t d = pos_dom(a, sd, in, c, pos);
          if (d == DOM_NONE) d = 0;
          if (s_off[c] != SP_OFF_NONE) {
            const uint32_t bit = s_off[c] + d, m = 1u << (bit & 31);
            if ((s_seen[bit >> 5] & m) || (atomicOr(&s_seen[bit >> 5], m) & m)) continue;
          } else if (a.dflag[(size_t)c * a.dom_cap + d] & 2u) {
            continue;
          }
          if (!(atomicOr(&a.dflag[(size_t)c * a.dom_cap + d], 2u) & 2u)) atomicAdd(&a.acc->topo_size[c], 1u);
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < RF; ++q) fails[q] += s == q ? 1u : 0u;  // ST_PREFILTERED: no plugin
    }
    a.st[pos] = out;
  }
  if (probe) return;  // (uniform: no barrier below is skipped by part of the block)
  // block reduction: counts, maxima
  uint32_t v[R_N];
#pragma unroll
  for (int q = 0; q < RF; ++q) v[q] = wave_sum(fails[q]);
  v[R_FEAS] = wave_sum(feasible);
  v[R_IGN] = wave_sum(ignored);
  v[R_TT] = wave_max(tt_max);
  v[R_NA] = wave_max(na_max);
  ipa_mn = wave_min64(ipa_mn);
  ipa_mx = wave_max64(ipa_mx);
  if (__syncthreads_or(score_any ? 1 : 0) && threadIdx.x == 0) atomicOr(&a.acc->score_any, 1u);
  if (lane == 0) {
#pragma unroll
    for (int q = 0; q < R_N; ++q) s_red[wid][q] = v[q];
    s_r64[wid][0] = ipa_mn;
    s_r64[wid][1] = ipa_mx;
  }
  __syncthreads();
  // flush the block's ScheduleAnyway domain counts
  for (uint32_t c = 0; c < n; ++c) {
    if (s_off[c] == SP_OFF_NONE || !(sd[c].flags & SP_SCORE)) continue;
    for (uint32_t d = threadIdx.x; d < a.ndom[sd[c].key]; d += SP_THREADS) {
      const uint32_t v = s_h[s_off[c] + d];
      if (v) atomicAdd(&a.dcnt[(size_t)c * a.dom_cap + d], v);
    }
  }
  if (threadIdx.x < R_N) {
    const int q = threadIdx.x;
    uint32_t t = s_red[0][q];
    for (int w = 1; w < SP_THREADS / WAVE; ++w) t = q >= R_TT ? max(t, s_red[w][q]) : t + s_red[w][q];
    SpreadAccShard &bp = acc_shard(a);
    if (t) {
      if (q < RF) atomicAdd(&bp.fail[q], t);
      else if (q == R_FEAS) atomicAdd(&bp.feasible, t);
      else if (q == R_IGN) atomicAdd(&bp.ignored, t);
      else if (q == R_TT) atomicMax(&bp.tt_max, t);
      else atomicMax(&bp.na_max, t);
    }
  } else if (threadIdx.x == R_N && ipa_score) {
    uint64_t mn = s_r64[0][0], mx = s_r64[0][1];
    for (int w = 1; w < SP_THREADS / WAVE; ++w) {
      mn = min(mn, s_r64[w][0]);
      mx = max(mx, s_r64[w][1]);
    }
    SpreadAccShard &bp = acc_shard(a);
    if (mn != ~0ull) atomicMin((unsigned long long *)&bp.ipa_min, (unsigned long long)mn);
    if (mx) atomicMax((unsigned long long *)&bp.ipa_max, (unsigned long long)mx);
  }
}

// ----------------------------------------------------------------- score
// scoring.go#Score: Σ over the ScheduleAnyway constraints whose key the node
// has of float64(cnt) * log(size + 2) + float64(maxSkew - 1), rounded
// (math.Round); cnt = matching pods of the node's domain (of the node itself
// for kubernetes.io/hostname); size = Score domains (filtered nodes minus
// ignored ones for hostname).
__global__ __launch_bounds__(SP_THREADS) void spread_score_kernel(SpreadArgs a) {
  __shared__ double s_w[MAX_SPREAD];
  __shared__ uint64_t s_r[SP_THREADS / WAVE][2];
  __shared__ SpreadDev s_sd[MAX_SPREAD];
  const PodDev p = a.pods[a.pod];
  const uint32_t n = spread_count(a, p);
  if (threadIdx.x < n) s_sd[threadIdx.x] = spread_recs(a, p)[threadIdx.x];
  const SpreadDev *sd = s_sd;
  __syncthreads();
  if (threadIdx.x < n) {
    const Totals tot = acc_totals(a.acc);
    const SpreadDev &q = sd[threadIdx.x];
    const uint32_t sz = (q.flags & SP_HOST) ? tot.feasible - tot.ignored : a.acc->topo_size[threadIdx.x];
    s_w[threadIdx.x] = go_log((double)sz + 2.0);  // topologyNormalizingWeight
  }
  __syncthreads();
  uint64_t mn = ~0ull, mx = 0;
  // SP_BATCH positions per thread per step (spans of SP_THREADS, coalesced):
  // their loads are issued together, not one dependent chain per position
  for (uint32_t base = blockIdx.x * SP_THREADS * SP_BATCH + threadIdx.x; base < a.npos;
       base += grid_threads() * SP_BATCH) {
    bool on[SP_BATCH];
#pragma unroll
    for (int u = 0; u < SP_BATCH; ++u) {
      const uint32_t pos = base + u * SP_THREADS;
      on[u] = pos < a.npos && a.st[pos] == SST_FEASIBLE;
    }
    double score[SP_BATCH];
#pragma unroll
    for (int u = 0; u < SP_BATCH; ++u) score[u] = 0;
    for (uint32_t c = 0; c < n; ++c) {
      const SpreadDev &q = sd[c];
      if (!(q.flags & SP_SCORE)) continue;
      uint32_t d[SP_BATCH], cnt[SP_BATCH];
#pragma unroll
      for (int u = 0; u < SP_BATCH; ++u) d[u] = on[u] ? a.dom[(size_t)q.key * a.npos + base + u * SP_THREADS] : DOM_NONE;
#pragma unroll
      for (int u = 0; u < SP_BATCH; ++u) {
        cnt[u] = 0;
        if (d[u] == DOM_NONE) continue;  // the node lacks the key: no term
        if (q.flags & SP_HOST) cnt[u] = q.cls == CLS_NONE ? 0u : a.cnt[(size_t)q.cls * a.npos + base + u * SP_THREADS];
        else cnt[u] = a.dcnt[(size_t)c * a.dom_cap + d[u]];
      }
#pragma unroll
      for (int u = 0; u < SP_BATCH; ++u)
        if (d[u] != DOM_NONE) score[u] += (double)cnt[u] * s_w[c] + (double)(q.max_skew - 1);  // scoreForCount
    }
#pragma unroll
    for (int u = 0; u < SP_BATCH; ++u) {
      if (!on[u]) continue;
      const int64_t raw = (int64_t)round(score[u]);
      a.raw[base + u * SP_THREADS] = raw;
      mn = min(mn, (uint64_t)raw);
      mx = max(mx, (uint64_t)raw);
    }
  }
  mn = wave_min64(mn);
  mx = wave_max64(mx);
  const uint32_t lane = threadIdx.x % WAVE, wid = threadIdx.x / WAVE;
  if (lane == 0) {
    s_r[wid][0] = mn;
    s_r[wid][1] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < SP_THREADS / WAVE; ++w) {
      mn = min(mn, s_r[w][0]);
      mx = max(mx, s_r[w][1]);
    }
    if (mn != ~0ull) atomicMin((unsigned long long *)&acc_shard(a).pts_min, (unsigned long long)mn);
    if (mx) atomicMax((unsigned long long *)&acc_shard(a).pts_max, (unsigned long long)mx);
  }
}

// ---------------------------------------------------------------- window
// percentageOfNodesToScore < 100 (schedule_one.go#numFeasibleNodesToFind,
// findNodesThatFitPod, findNodesThatPassFilters; restated sequentially as
// oracle.cpp window()).  The probe filter pass has written
// every slot's byte: bit 0 the node is in the list (present, not excluded by
// a NodeAffinity PreFilterResult), bit 1 it passes every filter.  Visiting
// starts at the list node of rank nextStartNodeIndex % len(list) and goes
// round the list in slot order; it stops at the (k+1)-th feasible node, k =
// numFeasibleNodesToFind(pct, len(list)): the window is the nodes before it,
// k feasible ones and the infeasible ones among them (fewer than k + 1
// feasible: every node).  nextStartNodeIndex += processed, modulo the present
// nodes.  One workgroup: per-thread counts over a contiguous slot range, a
// block scan, then the two threads whose ranges hold the start rank and the
// stopping rank walk them.
constexpr int WIN_THREADS = 1024;
// slots per count of spread_wcount_kernel (one walk step of the window);
// ksched_host.cpp sizes win[] with the same value (WIN_CHUNK_SLOTS)
constexpr uint32_t WIN_CHUNK = 1024;

__device__ __forceinline__ int64_t num_feasible_to_find(int32_t pct, int64_t n) {
  if (n < 100) return n;  // minFeasibleNodesToFind
  int64_t q = pct;
  if (q == 0) q = max<int64_t>(50 - n / 125, 5);  // adaptive, minFeasibleNodesPercentageToFind
  const int64_t k = n * q / 100;
  return k < 100 ? 100 : k;
}

__device__ __forceinline__ uint32_t byte_bits(uint32_t w, uint32_t bit) {
  return (uint32_t)__popc(w & (0x01010101u << bit));
}

// Exclusive block prefix sums of two counts, and their block totals (every
// thread); sx / sy: WIN_THREADS / WAVE words of LDS each.  Ends with a barrier
// after its last LDS read, so the next call may reuse them.
__device__ __forceinline__ void block_scan2(uint32_t x, uint32_t y, uint32_t &ex, uint32_t &ey, uint32_t &tx,
                                            uint32_t &ty, uint32_t *sx, uint32_t *sy) {
  const uint32_t lane = threadIdx.x % WAVE, wid = threadIdx.x / WAVE;
  uint32_t ix = x, iy = y;
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    const uint32_t u = __shfl_up(ix, o), v = __shfl_up(iy, o);
    if (lane >= (uint32_t)o) {
      ix += u;
      iy += v;
    }
  }
  if (lane == WAVE - 1) {
    sx[wid] = ix;
    sy[wid] = iy;
  }
  __syncthreads();
  ex = ix - x;
  ey = iy - y;
  tx = ty = 0;
  for (uint32_t w = 0; w < WIN_THREADS / WAVE; ++w) {
    const uint32_t u = sx[w], v = sy[w];
    if (w < wid) {
      ex += u;
      ey += v;
    }
    tx += u;
    ty += v;
  }
  __syncthreads();
}

// The list / feasible counts of every WIN_CHUNK-slot chunk of win_st, into
// win[WIN_WORDS + 2 c] / [WIN_WORDS + 2 c + 1]: 16 bytes per thread.
__global__ __launch_bounds__(WIN_CHUNK / 16) void spread_wcount_kernel(SpreadArgs a) {
  __shared__ uint32_t s_c[WIN_CHUNK / 16 / WAVE][2];
  const uint32_t ns = a.nslots, j = blockIdx.x * WIN_CHUNK + threadIdx.x * 16;
  uint32_t cl = 0, cf = 0;
  if (j + 16 <= ns) {
    const uint4 v = *reinterpret_cast<const uint4 *>(a.win_st + j);
    cl = byte_bits(v.x, 0) + byte_bits(v.y, 0) + byte_bits(v.z, 0) + byte_bits(v.w, 0);
    cf = byte_bits(v.x, 1) + byte_bits(v.y, 1) + byte_bits(v.z, 1) + byte_bits(v.w, 1);
  } else {
    for (uint32_t i = j; i < ns && i < j + 16; ++i) {
      cl += a.win_st[i] & 1u;
      cf += (a.win_st[i] >> 1) & 1u;
    }
  }
  cl = wave_sum(cl);
  cf = wave_sum(cf);
  if (threadIdx.x % WAVE == 0) {
    s_c[threadIdx.x / WAVE][0] = cl;
    s_c[threadIdx.x / WAVE][1] = cf;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint32_t v = 0;
    for (int w = 0; w < WIN_CHUNK / 16 / WAVE; ++w) v += s_c[w][threadIdx.x];
    a.win[WIN_WORDS + 2 * blockIdx.x + threadIdx.x] = v;
  }
}

__global__ __launch_bounds__(WIN_THREADS) void spread_window_kernel(SpreadArgs a) {
  __shared__ uint32_t s_sx[WIN_THREADS / WAVE], s_sy[WIN_THREADS / WAVE];
  __shared__ uint32_t s_x[8];
  const uint32_t t = threadIdx.x;
  const uint32_t ns = a.nslots, nch = (ns + WIN_CHUNK - 1) / WIN_CHUNK;
  const uint32_t cpt = (nch + WIN_THREADS - 1) / WIN_THREADS;  // chunks per thread
  const uint32_t c_lo = min(nch, t * cpt), c_hi = min(nch, c_lo + cpt);
  const uint32_t *cc = a.win + WIN_WORDS;
  uint32_t cl = 0, cf = 0;  // list / feasible nodes of the thread's chunks
  for (uint32_t c = c_lo; c < c_hi; ++c) {
    cl += cc[2 * c];
    cf += cc[2 * c + 1];
  }
  uint32_t pl, pf, nl, nf;
  block_scan2(cl, cf, pl, pf, nl, nf, s_sx, s_sy);
  const int64_t k = num_feasible_to_find(a.pct, (int64_t)nl);
  const uint32_t next = a.win[0];
  const bool all = (int64_t)nf <= k;  // block-uniform
  uint32_t s0 = 0, x = 0, processed = nl;
  const uint8_t *b = a.win_st;
  // The slot of the node of rank `want` among the nodes whose bit `bit` is
  // set (and the other bit's count before it): the one thread whose chunks
  // hold it finds the chunk, then the whole workgroup walks that chunk, a
  // byte per thread per step, with block scans.
  auto find = [&](uint32_t want, uint32_t bit, uint32_t *out) {
    const uint32_t p_mine = bit ? pf : pl, c_mine = bit ? cf : cl;
    if (want >= p_mine && want < p_mine + c_mine) {
      uint32_t al = pl, af = pf, c = c_lo;
      for (; c + 1 < c_hi; ++c) {
        const uint32_t nl_c = cc[2 * c], nf_c = cc[2 * c + 1];
        if ((bit ? af + nf_c : al + nl_c) > want) break;
        al += nl_c;
        af += nf_c;
      }
      s_x[4] = c;
      s_x[5] = al;
      s_x[6] = af;
    }
    __syncthreads();
    const uint32_t base = s_x[4] * WIN_CHUNK, end = min(ns, base + WIN_CHUNK);
    uint32_t al = s_x[5], af = s_x[6];  // counts before the step
    for (uint32_t off = base; off < end; off += WIN_THREADS) {
      const uint32_t j = off + t;
      const uint32_t v = j < end ? b[j] : 0u;
      uint32_t el, ef, tl, tf;
      block_scan2(v & 1u, (v >> 1) & 1u, el, ef, tl, tf, s_sx, s_sy);
      const uint32_t r = bit ? af + ef : al + el;
      if (((v >> bit) & 1u) && r == want) {
        out[0] = j;
        out[1] = bit ? al + el : af + ef;  // the other count before the node
      }
      al += tl;
      af += tf;
    }
    __syncthreads();
  };
  if (!all) {
    const uint32_t s = next % nl;
    find(s, 0, s_x);  // the start node: its slot, the feasible nodes before it
    s0 = s_x[0];
    const uint32_t f0 = s_x[1], after = nf - f0;  // feasible nodes at or after the start slot
    // slot-order rank of the (k+1)-th feasible node in list order
    const uint32_t target = (int64_t)after >= k + 1 ? f0 + (uint32_t)k : (uint32_t)k - after;
    find(target, 1, s_x + 2);  // the stopping node: its slot, its list rank
    x = s_x[2];
    processed = (s_x[3] + nl - s) % nl;
  }
  if (t == 0) {
    a.win[1] = s0;
    a.win[2] = x;
    a.win[3] = all ? 1u : 0u;
    if (a.evaluated) a.win[0] = (uint32_t)(((uint64_t)next + processed) % a.evaluated);  // % len(allNodes)
  }
}

// ---------------------------------------------------------------- select
// TotalScore of every feasible node (PodTopologySpread NormalizeScore:
// ignored -> 0, max 0 -> 100, else 100 (max + min - s) / max), the packed-key
// argmax; ks_plugin_scores writes the per-node plugin scores instead.  The
// domain scratch is cleared for the next pod (its last reader was the score
// pass).
__global__ __launch_bounds__(SP_THREADS) void spread_select_kernel(SpreadArgs a) {
  __shared__ uint64_t s_r[SP_THREADS / WAVE];
  __shared__ SoloLds s_solo;
  const PodDev p = a.pods[a.pod];
  stage_solo(a, p, s_solo);
  __syncthreads();
  const SpreadDev *sd = s_solo.sd;
  const uint32_t n = s_solo.h.n_spread;
  bool has_score = false;
  for (uint32_t c = 0; c < n; ++c) has_score |= (sd[c].flags & SP_SCORE) != 0;
  const Totals tot = acc_totals(a.acc);
  const int64_t tt_max = tot.tt_max, na_max = tot.na_max;
  const int64_t pmin = (int64_t)tot.pts_min, pmax = (int64_t)tot.pts_max;
  const bool ipa_on = a.acc->score_any != 0;
  const int64_t imin = (int64_t)(tot.ipa_min - IPA_BIAS), idiff = (int64_t)(tot.ipa_max - tot.ipa_min);
  uint64_t best = 0;
  // one feasible (or ignored) position: its total score, the packed key
  auto select_one = [&](uint32_t pos, int8_t s, uint32_t slot, uint64_t pk, int64_t raw_in, int64_t ipa_in) {
    int64_t raw = 0, norm = 0;
    if (has_score && s != SST_IGNORED) {
      raw = raw_in;
      norm = pmax == 0 ? 100 : 100 * (pmax + pmin - raw) / pmax;
    }
    // total_score<true> from the packed parts (same terms, same order)
    int64_t total = (int64_t)(uint32_t)pk;
    int64_t tt = 100;
    if (p.flags & PF_TT) tt = normalize((int64_t)((pk >> 32) & 0xFF), tt_max, true);
    total += (int64_t)a.w.tt * tt;
    if (p.flags & PF_HAS_PREF) {
      int64_t na = 0;
      if (p.flags & PF_NA) na = normalize((int64_t)(pk >> 40), na_max, false);
      total += (int64_t)a.w.na * na;
    }
    if (has_score) total += (int64_t)a.w_pts * norm;
    // InterPodAffinity NormalizeScore: int64(MaxNodeScore * float64(s - min) / float64(max - min))
    int64_t ipa_raw = 0, ipa = 0;
    if (ipa_on) {
      ipa_raw = ipa_in;
      if (idiff > 0) ipa = (int64_t)(100.0 * ((double)(ipa_raw - imin) / (double)idiff));
    }
    total += (int64_t)a.w_ipa * ipa;
    if (a.dump) {
      NodeRegs r;
      load_core(a.t, pos, slot, true, r);
      NodeExt e;
      load_ext(a.t, pos, true, e);
      int32_t *o = a.dump + (size_t)slot * SPREAD_DUMP_WORDS;
      o[0] = ST_FEASIBLE;
      o[1] = score_la(p, r);
      o[2] = score_ba(p, r);
      const int64_t tr = (p.flags & PF_TT) ? taint_raw(p, e) : 0;
      o[3] = (int32_t)tr;
      o[4] = (int32_t)normalize(tr, (p.flags & PF_TT) ? tt_max : 0, true);
      const int64_t nr = (p.flags & PF_NA) ? preferred_raw(p, a.clauses, e, slot) : 0;
      o[5] = (int32_t)nr;
      o[6] = (p.flags & PF_HAS_PREF) ? (int32_t)normalize(nr, (p.flags & PF_NA) ? na_max : 0, false) : 0;
      o[7] = (int32_t)image_score(s_solo, e);
      o[8] = (int32_t)raw;
      o[9] = (int32_t)norm;
      o[10] = (int32_t)(total & 0xFFFFFFFF);
      o[11] = (int32_t)(total >> 32);
      o[12] = (int32_t)ipa_raw;
      o[13] = (int32_t)ipa;
    }
    const uint64_t k = pack_key(total, slot);
    best = k > best ? k : best;
  };
  // SP_BATCH positions per thread per step (spans of SP_THREADS, coalesced):
  // their loads are issued together, not one dependent chain per position
  for (uint32_t base = blockIdx.x * SP_THREADS * SP_BATCH + threadIdx.x; base < a.npos;
       base += grid_threads() * SP_BATCH) {
    int8_t sv[SP_BATCH];
    uint32_t slv[SP_BATCH];
    uint64_t pkv[SP_BATCH];
    int64_t rawv[SP_BATCH], iprv[SP_BATCH];
#pragma unroll
    for (int u = 0; u < SP_BATCH; ++u) {
      const uint32_t pos = base + u * SP_THREADS;
      sv[u] = pos < a.npos ? a.st[pos] : SST_EMPTY;
      slv[u] = pos < a.npos ? a.pos_slot[pos] : SLOT_NONE;
    }
#pragma unroll
    for (int u = 0; u < SP_BATCH; ++u) {
      const uint32_t pos = base + u * SP_THREADS;
      const bool f = sv[u] == SST_FEASIBLE || sv[u] == SST_IGNORED;
      pkv[u] = f ? a.part[pos] : 0ull;
      rawv[u] = f && has_score && sv[u] == SST_FEASIBLE ? a.raw[pos] : 0;
      iprv[u] = f && ipa_on ? a.ipa_raw[pos] : 0;
    }
#pragma unroll
    for (int u = 0; u < SP_BATCH; ++u) {
      const int8_t s = sv[u];
      if (s == SST_FEASIBLE || s == SST_IGNORED) {
        select_one(base + u * SP_THREADS, s, slv[u], pkv[u], rawv[u], iprv[u]);
      } else if (a.dump && slv[u] != SLOT_NONE) {
        int32_t *o = a.dump + (size_t)slv[u] * SPREAD_DUMP_WORDS;
        for (int q = 0; q < SPREAD_DUMP_WORDS; ++q) o[q] = 0;
        o[0] = s == SST_EMPTY ? ST_EMPTY : s;
      }
    }
  }
  best = wave_max64(best);
  if (threadIdx.x % WAVE == 0) s_r[threadIdx.x / WAVE] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < SP_THREADS / WAVE; ++w) best = s_r[w] > best ? s_r[w] : best;
    if (best) atomicMax((unsigned long long *)&acc_shard(a).best, (unsigned long long)best);
  }
  // clear the domain scratch of this pod's constraints (a ScheduleAnyway
  // kubernetes.io/hostname constraint counts per node and never used it)
  for (uint32_t c = 0; c < n; ++c)
    if ((sd[c].flags & (SP_SCORE | SP_HOST)) != (SP_SCORE | SP_HOST))
    for (uint32_t d = blockIdx.x * SP_THREADS + threadIdx.x; d < a.ndom[sd[c].key]; d += grid_threads()) {
      a.dcnt[(size_t)c * a.dom_cap + d] = 0;
      a.dflag[(size_t)c * a.dom_cap + d] = 0;
    }
  const AffDev *ad = s_solo.ad;
  for (uint32_t r = 0; r < s_solo.h.n_aff; ++r)
    if ((ad[r].kind & AF_KIND) != AF_OWN && !(ad[r].kind & AF_NODE))
      for (uint32_t d = blockIdx.x * SP_THREADS + threadIdx.x; d < a.ndom[ad[r].key]; d += grid_threads())
        a.adcnt[(size_t)r * a.dom_cap + d] = 0;
}

// ---------------------------------------------------------------- commit
// One thread: the pod's result (ScheduleResult / FitError / Error as the round
// kernels report them), AssumePod on the winner (Requested, NonZeroRequested,
// pod count, and +1 in every selector-class column the pod matches), and the
// accumulators reset for the next pod.
__global__ void spread_commit_kernel(SpreadArgs a) {
  if (threadIdx.x != 0) return;
  const Totals tot = acc_totals(a.acc);
  const PodDev p = a.pods[a.pod];
  SpreadAcc &acc = *a.acc;
  DevResult r;
  r.node_index = -1;
  r.status = 1;  // KS_POD_UNSCHEDULABLE
  r.total_score = 0;
  r.feasible_nodes = tot.feasible;
  r.evaluated_nodes = a.evaluated;
  if (a.win_mode) {  // the visited nodes and the PreFilterResult's exclusions
    uint32_t v = tot.feasible + p.prefilter_out;
    for (int q = 0; q < NFILT + 2; ++q) v += tot.fail[q];
    r.evaluated_nodes = v;
  }
  for (int q = 0; q < NFILT; ++q) r.fail_counts[q] = tot.fail[q];
  r.spread_fail = tot.fail[PLUGIN_SPREAD];
  r.ipa_fail = tot.fail[PLUGIN_IPA];
  r._pad = 0;
  r.prefiltered = p.prefilter_out;
  r.flags = 0;
  if (tot.feasible > 0) {
    if ((p.flags & PF_PREF_ERR) && tot.feasible >= 2) {
      r.status = 2;  // KS_POD_ERROR (NodeAffinity PreScore)
    } else if (tot.best == 0) {
      r.status = 2;  // no key although a node passed the filters: never expected, never committed
    } else {
      const uint64_t win = tot.best;
      const uint32_t slot = 0xFFFFFFFFu - (uint32_t)win;
      r.node_index = (int32_t)slot;
      r.status = 0;
      r.total_score = (int64_t)(win >> 32) - 1;
      r.flags = tot.feasible == 1 ? 1u : 0u;  // KS_RESULT_SINGLE_FEASIBLE
      if (!a.no_commit) {
        const uint32_t pos = a.slot_pos[slot];
        a.t.rcpu[pos] += p.req_cpu;
        a.t.rmem[pos] += p.req_mem;
        a.t.zcpu[pos] += p.nz_cpu;
        a.t.zmem[pos] += p.nz_mem;
        a.t.npods[pos] += 1;
        const XResDev *xr = xres_recs(a, p);
        for (uint32_t k = 0; k < solo_hdr(a, p).n_xres; ++k) a.xreq[(size_t)xr[k].col * a.npos + pos] += xr[k].req;
        for (int w = 0; w < CMASK_WORDS; ++w) {
          uint64_t m = a.cmask[(size_t)a.pod * CMASK_WORDS + w];
          while (m) {
            const uint32_t cls = 64 * w + (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            a.cnt[(size_t)cls * a.npos + pos] += 1;
          }
        }
        const AffDev *ad = aff_recs(a, p);
        for (uint32_t k = 0; k < solo_hdr(a, p).n_aff; ++k)
          if ((ad[k].kind & AF_KIND) == AF_OWN) a.tcnt[(size_t)ad[k].col * a.npos + pos] += (uint32_t)ad[k].weight;
        a.counters[1] += 1;  // pods resolved
      }
    }
  } else if (!a.no_commit) {
    a.counters[1] += 1;
  }
  if (!a.no_commit) a.results[a.pod] = r;
  for (int c = 0; c < MAX_SPREAD; ++c) {
    acc.min_match[c] = 0xFFFFFFFFu;
    acc.ndomains[c] = 0;
    acc.topo_size[c] = 0;
  }
  acc.aff_any = acc.score_any = 0;
  for (int k = 0; k < ACC_SHARDS; ++k) {
    SpreadAccShard &q = acc.sh[k];
    for (int f = 0; f < NFILT + 2; ++f) q.fail[f] = 0;
    q.feasible = q.ignored = q.tt_max = q.na_max = 0;
    q.pts_min = q.ipa_min = ~0ull;
    q.pts_max = q.ipa_max = 0;
    q.best = 0;
  }
}

// ----------------------------------------------------------- replica runs
//  Consecutive identical pods whose constraints are all
// ScheduleAnyway -- deployment replicas under the system default constraints
// (podtopologyspread systemDefaultConstraints: hostname maxSkew 3, zone
// maxSkew 5) -- see one Filter result until a commit makes a node infeasible,
// and with it the same normaliser maxima and Score domain sizes.  A feasible
// node's TotalScore is then S + w x NormalizeScore(raw): S (LeastAllocated,
// BalancedAllocation, normalised TaintToleration / NodeAffinity) changes only
// when a pod of the run takes the node, and raw depends on the node only
// through its group (its domain of the other key, its own hostname count).
// One filter pass, the sort keys, a radix sort by (group, S descending, slot
// ascending) and the group starts; then one workgroup walks the pods.  Each
// pod's candidates are every group's first untaken node (the group's best:
// same raw, highest S, lowest slot) and every node the run has taken,
// re-scored after each commit; min / max raw over the non-ignored ones, the
// packed-key argmax as spread_select, AssumePod as spread_commit.  The run
// ends before a pod whose Filter result would differ (a taken node no longer
// fits) and after RUN_TOUCHED taken nodes; the host starts the next run there.
//
// DoNotSchedule on the other key (round 6): the Filter result
// then also depends on the domain counts -- a domain is blocked while its
// count + self - minMatch > maxSkew -- and every commit moves one domain's
// count, and with it perhaps the global minimum.  Blocking depends on the
// node only through its domain, i.e. its group: the run takes the nodes the
// skew check alone rejected as candidates too, blocks and unblocks whole
// domains as counts and the minimum move, and derives each pod's feasible
// count, PodTopologySpread failures and hostname Score weight
// (log(filtered - ignored + 2)) from the blocked nodes.  Runs of pods with a
// normalised TaintToleration / NodeAffinity score (maxima over the feasible
// nodes) or ignored nodes are not taken (the chain schedules them).

// ReplicaArgs::ctl word 4: candidates the skew check alone rejected
// (DoNotSchedule runs; the sorted keys hold feasible + these)
constexpr uint32_t RUN_CTL_SKEW = 4;
// DoNotSchedule runs track the domains' counts as offsets from the minimum
// at the run's start: a run whose minimum or blocking threshold would move
// past RUN_HIST offsets ends there (RUN_FULL)
constexpr uint32_t RUN_HIST = 512;

struct RunCons {
  uint32_t cz, ch;  // constraint of the other key, of kubernetes.io/hostname (MAX_SPREAD: none)
};
__device__ __forceinline__ RunCons run_cons(const SpreadDev *sd, uint32_t n) {
  RunCons k{(uint32_t)MAX_SPREAD, (uint32_t)MAX_SPREAD};
  for (uint32_t c = 0; c < n; ++c) {
    if (sd[c].flags & SP_HOST) k.ch = c;
    else k.cz = c;
  }
  return k;
}

// spread_select's TotalScore of a feasible node without its PodTopologySpread
// term (same terms, same integer arithmetic)
__device__ __forceinline__ uint32_t run_static(const PodDev &p, const Weights &w, uint64_t pk, int64_t tt_max,
                                               int64_t na_max) {
  int64_t total = (int64_t)(uint32_t)pk;
  int64_t tt = 100;
  if (p.flags & PF_TT) tt = normalize((int64_t)((pk >> 32) & 0xFF), tt_max, true);
  total += (int64_t)w.tt * tt;
  if (p.flags & PF_HAS_PREF) {
    int64_t na = 0;
    if (p.flags & PF_NA) na = normalize((int64_t)(pk >> 40), na_max, false);
    total += (int64_t)w.na * na;
  }
  return (uint32_t)total;
}

// Sort key of every position (~0: not feasible) after the run's filter pass.
__global__ __launch_bounds__(SP_THREADS) void replica_keys_kernel(SpreadArgs a, ReplicaArgs r) {
  __shared__ SpreadDev s_sd[MAX_SPREAD];
  __shared__ uint32_t s_max[2];
  const PodDev p = a.pods[a.pod];
  const uint32_t n = spread_count(a, p);
  if (threadIdx.x < n) s_sd[threadIdx.x] = spread_recs(a, p)[threadIdx.x];
  if (threadIdx.x == 0) {
    const Totals t = acc_totals(a.acc);
    s_max[0] = t.tt_max;
    s_max[1] = t.na_max;
  }
  __syncthreads();
  const RunCons k = run_cons(s_sd, n);
  const int64_t tt_max = s_max[0], na_max = s_max[1];
  // DoNotSchedule on the other key: nodes that failed only its skew check are
  // candidates too (they become feasible when the minimum moves); their
  // packed score parts (the filter pass writes them for feasible nodes only)
  // are computed here: no TaintToleration / NodeAffinity normalisation and no
  // image records in such runs
  const bool dns = k.cz < (uint32_t)MAX_SPREAD && !(s_sd[k.cz].flags & SP_SCORE);
  bool ovf = false, refuse = false;
  uint32_t nskew = 0;
  for (uint32_t pos = blockIdx.x * SP_THREADS + threadIdx.x; pos < a.npos; pos += grid_threads()) {
    const int8_t s = a.st[pos];
    const uint32_t slot = a.pos_slot[pos];
    uint64_t key = ~0ull;
    const bool skew = dns && s == PLUGIN_SPREAD && slot != SLOT_NONE &&
                      a.dom[(size_t)s_sd[k.cz].key * a.npos + pos] != DOM_NONE;
    if (skew) {
      NodeRegs g;
      load_core(a.t, pos, slot, true, g);
      a.part[pos] = pack_part((uint32_t)a.w.fit * (uint32_t)score_la(p, g) + (uint32_t)a.w.ba * (uint32_t)score_ba(p, g),
                              0u, 0u);
      ++nskew;
    }
    if (dns && s == SST_IGNORED) refuse = true;  // an ignored node has no domain in its group code
    if ((s == SST_FEASIBLE || s == SST_IGNORED || skew) && slot != SLOT_NONE) {
      const uint32_t S = run_static(p, a.w, a.part[pos], tt_max, na_max);
      uint32_t code = RK_IGN;
      if (s != SST_IGNORED) {
        uint32_t dz = 0, hk = 0;
        if (k.cz < (uint32_t)MAX_SPREAD) {
          const uint32_t d = a.dom[(size_t)s_sd[k.cz].key * a.npos + pos];
          dz = d == DOM_NONE ? RK_DZ_NONE : d;
        }
        if (k.ch < (uint32_t)MAX_SPREAD) {
          const SpreadDev &q = s_sd[k.ch];
          if (a.dom[(size_t)q.key * a.npos + pos] == DOM_NONE) {
            hk = RK_HK_NONE;
          } else if (q.cls != CLS_NONE) {
            hk = a.cnt[(size_t)q.cls * a.npos + pos];
            if (hk >= RK_HK_NONE) {
              ovf = true;
              hk = RK_HK_NONE - 1;
            }
          }
        }
        code = dz << 8 | hk;
      }
      key = (uint64_t)code << r.s_bits | (uint64_t)(((1u << r.s_bits) - 1) - S);
    }
    // indexed by slot: the (stable) radix sort keeps equal keys in slot order,
    // upstream's tie-break, without the slot in the key
    if (slot != SLOT_NONE) {
      r.keys[slot] = key;
      r.val[slot] = (uint64_t)slot << 32 | pos;
    }
  }
  if (__syncthreads_or((ovf || refuse) ? 1 : 0) && threadIdx.x == 0) atomicOr(&r.ctl[1], 1u);
  if (dns) {
    nskew = wave_sum(nskew);
    if (threadIdx.x % WAVE == 0 && nskew) atomicAdd(&r.ctl[RUN_CTL_SKEW], nskew);
  }
}

// First sorted index of every group (feasible keys sort first).
__global__ __launch_bounds__(SP_THREADS) void replica_groups_kernel(SpreadArgs a, ReplicaArgs r) {
  __shared__ uint32_t s_f;
  if (threadIdx.x == 0) s_f = acc_totals(a.acc).feasible + r.ctl[RUN_CTL_SKEW];  // candidates
  __syncthreads();
  const uint32_t f = s_f;
  for (uint32_t i = blockIdx.x * SP_THREADS + threadIdx.x; i < f; i += grid_threads()) {
    const uint64_t g = r.sorted[i] >> r.s_bits;
    if (i == 0 || (r.sorted[i - 1] >> r.s_bits) != g) {
      const uint32_t q = atomicAdd(&r.ctl[0], 1u);
      if (q < RUN_GROUPS) r.gstart[q] = i;
    }
  }
}

// 512 threads: 256 VGPRs per lane, so the prefetched rows need no scratch
// (a spill reload waits for every outstanding load, store and atomic)
constexpr int RUN_THREADS = 512;  // thread g owns group g, thread t the run's t-th taken node
static_assert(RUN_GROUPS == (uint32_t)RUN_THREADS && RUN_TOUCHED == (uint32_t)RUN_THREADS, "one group / node per thread");

// Workgroup barrier for LDS hand-offs only (__syncthreads() also waits for the
// group owners' prefetches of their next nodes' rows)
__device__ __forceinline__ void run_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// floor(a / b) for a < 2^31, 0 < b < 2^24 and a quotient below 2^7 (the
// normalised PodTopologySpread score: a = 100 (max + min - raw), b = max, raw
// in [min, max]), with inv = RN(1 / b): the product is within one of it and
// the corrections' products stay below 2^31
__device__ __forceinline__ uint32_t run_div32(uint32_t a, uint32_t b, double inv) {
  uint32_t q = (uint32_t)((double)a * inv);
  q -= q * b > a ? 1u : 0u;
  q += (q + 1) * b <= a ? 1u : 0u;
  return q;
}
// raws of a run stay below this (checked at its start): 32-bit min / max and
// normalisation
constexpr double RUN_RAW_LIMIT = 16777216.0;  // 2^24

// A node's row as the run kernel carries it
struct RunRow {
  int64_t ac, am, rc, rm, zc, zm;
  uint64_t pk;  // the filter pass's packed score parts (raw TaintToleration / NodeAffinity)
  int32_t ap, np;
};
__device__ __forceinline__ RunRow run_row(const SpreadArgs &a, uint32_t pos) {
  RunRow w;
  w.ac = a.t.acpu[pos];
  w.am = a.t.amem[pos];
  w.rc = a.t.rcpu[pos];
  w.rm = a.t.rmem[pos];
  w.zc = a.t.zcpu[pos];
  w.zm = a.t.zmem[pos];
  w.pk = a.part[pos];
  w.ap = a.t.apods[pos];
  w.np = a.t.npods[pos];
  return w;
}

// DNS: the run's other-key constraint is DoNotSchedule (a template
// parameter: the ScheduleAnyway runs compile without the blocking code,
// which costs them registers and ~1k cycles per pod)
template <bool DNS>
__global__ __launch_bounds__(RUN_THREADS) void replica_run_kernel(SpreadArgs a, ReplicaArgs r) {
  __shared__ SpreadDev s_sd[MAX_SPREAD];
  __shared__ Totals s_tot;
  __shared__ uint32_t s_dz[RK_DZ_NONE];     // live PreScore counts of the other key's domains
  __shared__ uint32_t s_gs[RUN_GROUPS];     // group starts, ascending
  __shared__ uint32_t s_mn[RUN_THREADS / WAVE], s_mx[RUN_THREADS / WAVE];
  __shared__ uint64_t s_bk[RUN_THREADS / WAVE];
  __shared__ uint32_t s_dzmax;  // the largest live domain count at the start
  __shared__ uint64_t s_bk2[RUN_THREADS / WAVE];  // the argmax again when min / max raw moved
  __shared__ uint32_t s_cls[MAX_CLASSES];   // selector classes the pods match (commit: +1 each)
  // 0 groups, 1 refused, 2 classes, 3 RunStop, 4 taken nodes, 5-7 a head that joined them: slot,
  // position, group code, 8 the domain whose count the last commit raised (RK_DZ_NONE: none),
  // 9-10 the head's static terms and S after its commit, DoNotSchedule runs: 11 the minimum's
  // offset, 12 candidate nodes in blocked domains
  __shared__ uint32_t s_ctl[13];
  // DoNotSchedule runs: candidate nodes per domain; per offset above the
  // start's minimum, eligible domains and their candidate nodes
  __shared__ uint32_t s_nodes[RK_DZ_NONE];
  __shared__ uint32_t s_hist[RUN_HIST], s_nhist[RUN_HIST];
  const uint32_t tid = threadIdx.x, lane = tid % WAVE, wid = tid / WAVE;
  const PodDev p = a.pods[a.pod];  // every pod of the run is identical (host-checked)
  const uint32_t n = spread_count(a, p);
  if (tid < n) s_sd[tid] = spread_recs(a, p)[tid];
  if (tid == 0) {
    s_tot = acc_totals(a.acc);
    const uint32_t g = r.ctl[0];
    s_ctl[0] = min(g, RUN_GROUPS);
    s_ctl[1] = g > RUN_GROUPS || r.ctl[1] ? 1u : 0u;
    uint32_t m = 0;
    for (int w = 0; w < CMASK_WORDS; ++w) {
      uint64_t b = a.cmask[(size_t)a.pod * CMASK_WORDS + w];
      while (b) {
        s_cls[m++] = 64 * w + (uint32_t)__builtin_ctzll(b);
        b &= b - 1;
      }
    }
    s_ctl[2] = m;
    s_ctl[3] = RUN_END;
    s_ctl[4] = 0;
    s_ctl[8] = RK_DZ_NONE;
    s_dzmax = 0;
  }
  __syncthreads();
  const RunCons k = run_cons(s_sd, n);
  const uint32_t G = s_ctl[0], F = s_tot.feasible;
  const uint32_t ndz = k.cz < (uint32_t)MAX_SPREAD ? a.ndom[s_sd[k.cz].key] : 0u;
  // DoNotSchedule on the other key: blocked while count + self - minMatch > maxSkew
  constexpr bool dns = DNS;
  const bool dns_prog = k.cz < (uint32_t)MAX_SPREAD && !(s_sd[k.cz].flags & SP_SCORE);  // must equal DNS
  const uint32_t C = F + (dns ? r.ctl[RUN_CTL_SKEW] : 0u);  // candidates (sorted keys)
  const bool m_fixed = dns && a.acc->ndomains[k.cz] < (uint32_t)s_sd[k.cz].min_domains;  // minMatch 0
  const uint32_t m0 = dns && !m_fixed ? a.acc->min_match[k.cz] : 0u;
  const uint32_t d_skew = dns ? (uint32_t)s_sd[k.cz].max_skew : 0u, d_self = dns && (s_sd[k.cz].flags & SP_SELF) ? 1u : 0u;
  for (uint32_t d = tid; d < ndz; d += RUN_THREADS) {
    const uint32_t v = a.dcnt[(size_t)k.cz * a.dom_cap + d];
    s_dz[d] = v;
    if (v) atomicMax(&s_dzmax, v);
  }
  s_gs[tid] = tid < G ? r.gstart[tid] : 0xFFFFFFFFu;
  // bitonic sort of the group starts
  for (uint32_t size = 2; size <= RUN_GROUPS; size <<= 1)
    for (uint32_t stride = size / 2; stride > 0; stride >>= 1) {
      __syncthreads();
      const uint32_t j = tid ^ stride;
      if (j > tid) {
        const uint32_t x = s_gs[tid], y = s_gs[j];
        if ((x > y) == ((tid & size) == 0)) {
          s_gs[tid] = y;
          s_gs[j] = x;
        }
      }
    }
  __syncthreads();
  auto cls_in = [&](uint32_t cls) {
    if (cls == CLS_NONE) return false;
    return ((a.cmask[(size_t)a.pod * CMASK_WORDS + cls / 64] >> (cls % 64)) & 1ull) != 0;
  };
  const bool inc_h = k.ch < (uint32_t)MAX_SPREAD && cls_in(s_sd[k.ch].cls);
  const bool inc_z = k.cz < (uint32_t)MAX_SPREAD && cls_in(s_sd[k.cz].cls);
  // topologyNormalizingWeight per constraint (spread_score); the hostname
  // one, log(filtered - ignored + 2), moves with the feasible count in
  // DoNotSchedule runs (re-taken per pod there)
  double w_h = k.ch < (uint32_t)MAX_SPREAD ? go_log((double)(F - s_tot.ignored) + 2.0) : 0.0;
  const double w_z = k.cz < (uint32_t)MAX_SPREAD ? go_log((double)a.acc->topo_size[k.cz] + 2.0) : 0.0;
  // raw Score of a group code (spread_score: the constraints in their order,
  // each adding cnt x weight + (maxSkew - 1), math.Round); at most one of
  // each kind, so the order is one flag
  const bool host_first = k.ch < k.cz;
  const double ms_h = k.ch < (uint32_t)MAX_SPREAD ? (double)(s_sd[k.ch].max_skew - 1) : 0.0;
  const double ms_z = k.cz < (uint32_t)MAX_SPREAD ? (double)(s_sd[k.cz].max_skew - 1) : 0.0;
  auto raw_of = [&](uint32_t code) -> uint32_t {
    const uint32_t dz = (code >> 8) & RK_DZ_NONE, hk = code & RK_HK_NONE;
    const bool th = k.ch < (uint32_t)MAX_SPREAD && hk != RK_HK_NONE;
    const bool tz = k.cz < (uint32_t)MAX_SPREAD && !dns && dz != RK_DZ_NONE;  // DoNotSchedule: no Score term
    const double xh = (double)hk * w_h + ms_h;
    const double xz = tz ? (double)s_dz[dz] * w_z + ms_z : 0.0;
    double s = 0;
    if (host_first) {
      if (th) s += xh;
      if (tz) s += xz;
    } else {
      if (tz) s += xz;
      if (th) s += xh;
    }
    return (uint32_t)round(s);  // < RUN_RAW_LIMIT (checked below)
  };
  // Every raw of the run is below RUN_RAW_LIMIT: at most 254 own pods per
  // node and a domain count at most the largest at the start plus one per
  // pod of the run.  Otherwise the run is refused (the per-pod chain takes
  // the pods).
  const double w_h_max = dns && k.ch < (uint32_t)MAX_SPREAD ? go_log((double)(C - s_tot.ignored) + 2.0) : w_h;
  const double raw_bound =
      (k.ch < (uint32_t)MAX_SPREAD ? 254.0 * w_h_max + ms_h : 0.0) +
      (k.cz < (uint32_t)MAX_SPREAD && !dns ? ((double)s_dzmax + (double)(r.end - a.pod)) * w_z + ms_z : 0.0);
  const bool raw_narrow = raw_bound + 1.0 < RUN_RAW_LIMIT;
  // no ScheduleAnyway constraint (DoNotSchedule only): PreScore skips, no Score term
  const int64_t w_pts = dns && k.ch >= (uint32_t)MAX_SPREAD ? 0 : (int64_t)a.w_pts;
  // group tid: its first untaken sorted index (head), the head's key, position
  // and row (prefetched), the next key and position
  const bool g_on = tid < G;
  uint32_t g_i = g_on ? s_gs[tid] : 0u;
  const uint32_t g_end = tid + 1 < G ? s_gs[tid + 1] : C;
  // (head: key, slot << 32 | position, row; next: key, value).  The argmax
  // reads only the head's key and value, which change by register moves at a
  // win.  Every thread reloads its head's row and its next key / value at the
  // end of every pod, at clamped indices, with no branch (a load under a
  // branch leaves a phi copy at the join that waits for it); only a winner
  // reads them, a pod later.  A head is untaken: no commit of the run writes
  // its row.
  const uint32_t g_last = g_on ? g_end - 1 : 0u;
  uint64_t g_key = r.sorted[g_on ? g_i : 0u];
  uint64_t g_val = r.sval[g_on ? g_i : 0u];
  uint64_t g_nkey = r.sorted[min(g_i + 1, g_last)];
  uint64_t g_nval = r.sval[min(g_i + 1, g_last)];
  RunRow g_row = run_row(a, (uint32_t)g_val);
  const uint32_t smask = (1u << r.s_bits) - 1;
  const uint32_t g_code = (uint32_t)(g_key >> r.s_bits) & 0xFFFFFu;
  // raw Score of the group (kept; recomputed when its domain's count moves)
  uint32_t graw = g_on && !(g_code & RK_IGN) ? raw_of(g_code) : 0u;
  // taken node tid: slot, position, group code (live), S, static tt / na part,
  // row, RN(1 / Allocatable) of cpu and memory, raw Score (kept as graw)
  bool t_on = false, t_dirty = false;
  uint32_t t_slot = 0, t_pos = 0, t_code = 0, t_S = 0, t_stat = 0;
  uint32_t traw = 0;
  __shared__ RunRow s_trow[RUN_TOUCHED];  // taken node t's row (its owner's; the winning head writes it)
  __shared__ double s_tinv[RUN_TOUCHED][2];  // its RN(1 / Allocatable) of cpu and memory
  // DoNotSchedule runs: candidate nodes per domain, the domains' offsets
  // above the minimum, the candidates in blocked domains at the start -- which
  // must be exactly the ones the filter pass's skew check rejected
  bool dns_bad = false;
  if (dns) {
    for (uint32_t d = tid; d < ndz; d += RUN_THREADS) s_nodes[d] = 0;
    for (uint32_t i = tid; i < RUN_HIST; i += RUN_THREADS) s_hist[i] = s_nhist[i] = 0;
    if (tid == 0) s_ctl[11] = s_ctl[12] = 0;
    __syncthreads();
    if (g_on && !(g_code & RK_IGN)) atomicAdd(&s_nodes[(g_code >> 8) & RK_DZ_NONE], g_end - g_i);
    __syncthreads();
    const uint32_t thr0 = m0 + d_skew - d_self;
    bool bad = false;
    for (uint32_t d = tid; d < ndz; d += RUN_THREADS) {
      const bool elig = a.dflag[(size_t)k.cz * a.dom_cap + d] & 1u;
      const uint32_t v = s_dz[d], nd = s_nodes[d];
      if (nd && !elig) bad = true;  // (a feasible node is eligible under either policy)
      if (elig && !m_fixed && v - m0 < RUN_HIST) {
        atomicAdd(&s_hist[v - m0], 1u);
        if (nd) atomicAdd(&s_nhist[v - m0], nd);
      }
      if (nd && v > thr0) atomicAdd(&s_ctl[12], nd);
    }
    dns_bad = __syncthreads_or(bad ? 1 : 0) != 0 || s_ctl[12] != r.ctl[RUN_CTL_SKEW];
  }
  const uint32_t dns_fail0 = dns ? s_tot.fail[PLUGIN_SPREAD] - r.ctl[RUN_CTL_SKEW] : 0u;  // PodTopologySpread
                                                                                        // failures besides the skew
  uint32_t T = 0, next = a.pod, stop = RUN_END;
  if (s_ctl[1] || !raw_narrow || dns_bad || dns_prog != DNS) {
    stop = RUN_REFUSED;
  } else if (F == 0) {
    // no feasible node: every pod of the run gets the same FitError, nothing is committed
    for (uint32_t pod = a.pod + tid; pod < r.end; pod += RUN_THREADS) {
      DevResult res;
      res.node_index = -1;
      res.status = 1;  // KS_POD_UNSCHEDULABLE
      res.total_score = 0;
      res.feasible_nodes = 0;
      res.evaluated_nodes = a.evaluated;
      for (int q = 0; q < NFILT; ++q) res.fail_counts[q] = s_tot.fail[q];
      res.spread_fail = s_tot.fail[PLUGIN_SPREAD];
      res.ipa_fail = s_tot.fail[PLUGIN_IPA];
      res._pad = 0;
      res.prefiltered = p.prefilter_out;
      res.flags = 0;
      a.results[pod] = res;
    }
    if (tid == 0) a.counters[1] += r.end - a.pod;
    next = r.end;
  } else {
    uint64_t ph[3] = {0, 0, 0}, t0 = r.prof ? __builtin_readcyclecounter() : 0;  // phase clocks (thread 0)
    auto clock = [&](int q) {
      if (r.prof && tid == 0) {
        const uint64_t t1 = __builtin_readcyclecounter();
        ph[q] += t1 - t0;
        t0 = t1;
      }
    };
    // min / max raw of the previous pod: this pod's keys are taken with them
    // and reduced together with this pod's min / max; only when those moved
    // (a domain's count or a taken node's hostname count raised the least or
    // the greatest raw, or a group ran out) are the keys taken again
    uint32_t q_mn = ~0u, q_mx = 0;
    double q_pinv = 0.0;  // RN(1 / q_mx)
    bool q_ok = false;  // no previous pod yet
    // the run's constant result fields and selector classes, in registers
    DevResult res_tpl;
    res_tpl.node_index = -1;
    res_tpl.status = 0;
    res_tpl.total_score = 0;
    res_tpl.feasible_nodes = F;
    res_tpl.evaluated_nodes = a.evaluated;
    for (int q = 0; q < NFILT; ++q) res_tpl.fail_counts[q] = s_tot.fail[q];
    res_tpl.spread_fail = s_tot.fail[PLUGIN_SPREAD];
    res_tpl.ipa_fail = s_tot.fail[PLUGIN_IPA];
    res_tpl._pad = 0;
    res_tpl.prefiltered = p.prefilter_out;
    res_tpl.flags = F == 1 ? 1u : 0u;  // KS_RESULT_SINGLE_FEASIBLE
    const uint32_t ncls = s_ctl[2], cls0 = ncls > 0 ? s_cls[0] : 0u, cls1 = ncls > 1 ? s_cls[1] : 0u;
    uint32_t q_F = F;  // DoNotSchedule runs: the feasible count w_h was taken with
    for (uint32_t pod = a.pod; pod < r.end; ++pod) {
      // DoNotSchedule runs: this pod's blocking threshold (a domain whose
      // count exceeds it fails the skew check), feasible count and hostname
      // Score weight (every raw moves with it)
      uint32_t thr = 0, n_blk = 0, Fp = F;
      bool redo = false;
      if (dns) {
        thr = (m_fixed ? 0u : m0 + s_ctl[11]) + d_skew - d_self;
        n_blk = s_ctl[12];
        Fp = C - n_blk;
        if (Fp == 0) {  // every candidate blocked: the chain reports it (never the run's first pod)
          stop = RUN_FIT;
          break;
        }
        if (Fp != q_F) {
          q_F = Fp;
          if (k.ch < (uint32_t)MAX_SPREAD) {
            w_h = go_log((double)(Fp - s_tot.ignored) + 2.0);
            redo = true;
          }
        }
      }
      // raw Scores the last commit moved; min / max raw over the non-ignored
      // feasible nodes
      const uint32_t chg = s_ctl[8];
      const bool g_live = g_on && g_i < g_end && !(dns && s_dz[(g_code >> 8) & RK_DZ_NONE] > thr);
      const bool t_live = t_on && !(dns && s_dz[(t_code >> 8) & RK_DZ_NONE] > thr);
      uint32_t mn = ~0u, mx = 0;
      if (g_on && !(g_code & RK_IGN) && (redo || ((g_code >> 8) & RK_DZ_NONE) == chg)) graw = raw_of(g_code);
      if (g_live && !(g_code & RK_IGN)) {
        mn = min(mn, graw);
        mx = max(mx, graw);
      }
      if (t_on && !(t_code & RK_IGN)) {
        if (t_dirty || redo || ((t_code >> 8) & RK_DZ_NONE) == chg) traw = raw_of(t_code);
        t_dirty = false;
      }
      if (t_live && !(t_code & RK_IGN)) {
        mn = min(mn, traw);
        mx = max(mx, traw);
      }
      // the candidates' packed keys under min / max raw (pmin, pmax)
      uint64_t gk = 0, tk = 0;
      auto keys = [&](uint32_t pmin, uint32_t pmax, double pinv) {
        auto total_of = [&](uint32_t S, uint32_t code, uint32_t raw) -> int64_t {
          uint32_t norm = 0;  // PodTopologySpread NormalizeScore: ignored -> 0, max 0 -> 100
          if (!(code & RK_IGN)) norm = pmax == 0 ? 100u : run_div32(100u * (pmax + pmin - raw), pmax, pinv);
          return (int64_t)S + w_pts * (int64_t)norm;
        };
        gk = g_live ? pack_key(total_of(smask - (uint32_t)(g_key & smask), g_code, graw), (uint32_t)(g_val >> 32)) : 0ull;
        tk = t_live ? pack_key(total_of(t_S, t_code, traw), t_slot) : 0ull;
      };
      // this pod's min / max raw and, with the previous pod's, the argmax: one barrier
      if (q_ok) keys(q_mn, q_mx, q_pinv);
      mn = ~wave_max_u32_dpp(~mn);
      mx = wave_max_u32_dpp(mx);
      uint64_t b = wave_max_u64_dpp(gk > tk ? gk : tk);
      if (lane == 0) {
        s_mn[wid] = mn;
        s_mx[wid] = mx;
        s_bk[wid] = b;
      }
      run_barrier();
      for (int w = 0; w < RUN_THREADS / WAVE; ++w) {
        mn = min(mn, s_mn[w]);
        mx = max(mx, s_mx[w]);
        b = s_bk[w] > b ? s_bk[w] : b;
      }
      clock(0);
      if (!q_ok || mn != q_mn || mx != q_mx) {  // (workgroup-uniform)
        if (!q_ok || mx != q_mx) q_pinv = mx ? 1.0 / (double)mx : 0.0;
        keys(mn, mx, q_pinv);
        b = wave_max_u64_dpp(gk > tk ? gk : tk);
        if (lane == 0) s_bk2[wid] = b;
        run_barrier();
        for (int w = 0; w < RUN_THREADS / WAVE; ++w) b = s_bk2[w] > b ? s_bk2[w] : b;
      }
      q_mn = mn;
      q_mx = mx;
      q_ok = true;
      clock(1);
      // The winner commits (AssumePod as spread_commit): a group's head from
      // its row in registers (the node joins the taken nodes as node T: its
      // state goes to LDS and thread T adopts it after the barrier, the group's
      // next node becomes the head), or a taken node, by its owner.
      const bool gwin = g_live && gk == b, twin = !gwin && t_live && tk == b;
      if (gwin || twin) {
        RunRow w;
        uint32_t slot, pos, code, stat;
        double ic, im;
        if (gwin) {
          w = g_row;
          slot = (uint32_t)(g_val >> 32);
          pos = (uint32_t)g_val;
          code = g_code;
          // S less its LeastAllocated / BalancedAllocation part (the packed
          // low word): the normalised TaintToleration / NodeAffinity terms
          stat = (smask - (uint32_t)(g_key & smask)) - (uint32_t)w.pk;
          ic = w.ac ? 1.0 / (double)w.ac : 0.0;  // as make_regs
          im = w.am ? 1.0 / (double)w.am : 0.0;
        } else {
          w = s_trow[tid];
          slot = t_slot;
          pos = t_pos;
          code = t_code;
          stat = t_stat;
          ic = s_tinv[tid][0];
          im = s_tinv[tid][1];
        }
        // Requested, NonZeroRequested, pod count
        w.rc += p.req_cpu;
        w.rm += p.req_mem;
        w.zc += p.nz_cpu;
        w.zm += p.nz_mem;
        w.np += 1;
        // the next pod's view of the node first (its S and Fit: the long
        // binary64 chain), then the stores nothing in the run reads
        const NodeRegs g = make_regs_inv(w.ac, w.am, w.rc, w.rm, w.zc, w.zm, w.ap, w.np, slot, ic, im);
        const uint32_t S = (uint32_t)a.w.fit * (uint32_t)score_la(p, g) + (uint32_t)a.w.ba * (uint32_t)score_ba(p, g) + stat;
        const bool fit_lost = filter<false>(p, a.clauses, g, NodeExt{}) != ST_FEASIBLE;
        // own hostname count, its domain's count
        if (inc_h && (code & RK_HK_NONE) != RK_HK_NONE) {
          code += 1;
          if ((code & RK_HK_NONE) == RK_HK_NONE) s_ctl[3] = RUN_FULL;  // beyond the key's range
        }
        uint32_t moved = RK_DZ_NONE;
        if (inc_z && !(code & RK_IGN)) {
          const uint32_t dz = (code >> 8) & RK_DZ_NONE;
          moved = dz == RK_DZ_NONE ? 0u : dz;  // PreScore counts a node lacking the key in ""
          if (!dns) {
            atomicAdd(&s_dz[moved], 1u);  // (no returned value: no LDS round trip)
          } else {
            // the domain's count (filtering.go: matching pods on eligible
            // nodes), its offset above the start's minimum, the blocked
            // candidates: the domain reaches the threshold + 1, or the last
            // domain at the minimum moves up and the threshold with it
            const uint32_t old = s_dz[moved], nd = s_nodes[moved];
            s_dz[moved] = old + 1;
            uint32_t blk = s_ctl[12], moff = s_ctl[11];
            if (old == thr) blk += nd;
            if (!m_fixed) {
              const uint32_t off = old - m0;
              if (off + 1 >= RUN_HIST) {
                s_ctl[3] = RUN_FULL;
              } else {
                s_hist[off] -= 1;
                s_hist[off + 1] += 1;
                s_nhist[off] -= nd;
                s_nhist[off + 1] += nd;
                if (off == moff && s_hist[off] == 0) {
                  ++moff;
                  const uint32_t toff = moff + d_skew - d_self;  // the new threshold, as an offset
                  if (toff >= RUN_HIST) s_ctl[3] = RUN_FULL;
                  else blk -= s_nhist[toff];  // domains at the new threshold: no longer over the skew
                }
              }
            }
            s_ctl[11] = moff;
            s_ctl[12] = blk;
          }
        }
        s_ctl[8] = moved;
        if (fit_lost) s_ctl[3] = RUN_FIT;  // (after RUN_FULL: a Fit loss wins, as before)
        a.t.rcpu[pos] = w.rc;
        a.t.rmem[pos] = w.rm;
        a.t.zcpu[pos] = w.zc;
        a.t.zmem[pos] = w.zm;
        a.t.npods[pos] = w.np;
        // class columns: no returned value, the atomics leave without a round trip
        for (uint32_t q = 0; q < ncls; ++q)
          atomicAdd(&a.cnt[(size_t)(q < 2 ? (q ? cls1 : cls0) : s_cls[q]) * a.npos + pos], 1u);
        DevResult res = res_tpl;
        res.node_index = (int32_t)slot;
        res.total_score = (int64_t)(b >> 32) - 1;
        if (dns) {
          res.feasible_nodes = Fp;
          res.spread_fail = dns_fail0 + n_blk;
          res.flags = Fp == 1 ? 1u : 0u;  // KS_RESULT_SINGLE_FEASIBLE
        }
        a.results[pod] = res;
        const uint32_t j = gwin ? T : tid;
        s_trow[j] = w;
        if (gwin) {
          s_tinv[j][0] = ic;
          s_tinv[j][1] = im;
          s_ctl[5] = slot;
          s_ctl[6] = pos;
          s_ctl[7] = code;
          s_ctl[9] = stat;
          s_ctl[10] = S;
          s_ctl[4] = T + 1;  // taken nodes
          ++g_i;
          g_key = g_nkey;
          g_val = g_nval;
        } else {
          t_code = code;
          t_S = S;
          t_dirty = true;
        }
      }
      g_row = run_row(a, (uint32_t)g_val);
      g_nkey = r.sorted[min(g_i + 1, g_last)];
      g_nval = r.sval[min(g_i + 1, g_last)];
      run_barrier();
      clock(2);  // the commit: the winner's chain, seen as thread 0's wait here
      if (s_ctl[4] != T) {  // a head joined the taken nodes: thread T owns it
        if (tid == T) {
          t_on = t_dirty = true;
          t_slot = s_ctl[5];
          t_pos = s_ctl[6];
          t_code = s_ctl[7];
          t_stat = s_ctl[9];
          t_S = s_ctl[10];
        }
        ++T;
      }
      next = pod + 1;
      stop = s_ctl[3];
      if (stop == RUN_END && T == RUN_TOUCHED && next < r.end) stop = RUN_FULL;
      if (stop != RUN_END) break;
    }
    if (r.prof && tid == 0) {
      for (int q = 0; q < 3; ++q) r.prof[q] += ph[q];
      r.prof[3] += next - a.pod;
    }
  }
  if (tid == 0) {
    r.ctl[2] = next;
    r.ctl[3] = stop;
    if (F != 0) a.counters[1] += next - a.pod;  // pods resolved (F == 0: counted above)
  }
  // clear the domain scratch of the other key (spread_select's clearing)
  for (uint32_t d = tid; d < ndz; d += RUN_THREADS) {
    a.dcnt[(size_t)k.cz * a.dom_cap + d] = 0;
    a.dflag[(size_t)k.cz * a.dom_cap + d] = 0;
  }
}

// Selector-class counts of the pods a round-kernel segment [lo, hi) bound.
__global__ void class_commit_kernel(const DevResult *res, const uint64_t *cmask, const uint32_t *slot_pos,
                                    uint32_t *cnt, uint32_t npos, uint32_t lo, uint32_t hi) {
  const uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= hi) return;
  if (res[i].status != 0) return;
  const uint32_t pos = slot_pos[res[i].node_index];
  for (int w = 0; w < CMASK_WORDS; ++w) {
    uint64_t m = cmask[(size_t)i * CMASK_WORDS + w];
    while (m) {
      const uint32_t cls = 64 * w + (uint32_t)__builtin_ctzll(m);
      m &= m - 1;
      atomicAdd(&cnt[(size_t)cls * npos + pos], 1u);
    }
  }
}

// col[idx[i]] = val[i] / col[idx[i]] += delta[i] (domain and class columns).
__global__ void scatter_u32_kernel(uint32_t *col, const uint64_t *idx, const uint32_t *val, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) col[idx[i]] = val[i];
}
__global__ void add_u32_kernel(uint32_t *col, const uint64_t *idx, const int32_t *delta, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&col[idx[i]], (uint32_t)delta[i]);
}
// dst[i] = max(dst[i], src[i]) (the in-process communicator's all-reduce(max))
__global__ void umax_u32_kernel(uint32_t *dst, const uint32_t *src, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = max(dst[i], src[i]);
}
__global__ void scatter_i64_kernel(int64_t *col, const uint64_t *idx, const int64_t *val, uint32_t n, uint32_t add) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (add) atomicAdd((unsigned long long *)&col[idx[i]], (unsigned long long)val[i]);
  else col[idx[i]] = val[i];
}

// ------------------------------------------------------------- launchers

hipError_t launch_spread_pod(const SpreadArgs &args, uint32_t passes, hipStream_t st) {
  // node passes: at most SPREAD_MAX_BLOCKS blocks (248 measured no better)
  const uint32_t blocks =
      std::max<uint32_t>(1, std::min<uint32_t>((args.npos + SP_THREADS - 1) / SP_THREADS, (uint32_t)SPREAD_MAX_BLOCKS));
  const SpreadArgs &a = args;
  if (passes & SPL_PREP) spread_prep_kernel<<<blocks, SP_THREADS, 0, st>>>(a);
  if (passes & SPL_MIN) spread_min_kernel<<<blocks, SP_THREADS, 0, st>>>(a);
  if (a.win_mode) {  // percentageOfNodesToScore < 100: probe, window, then the pass over the window
    SpreadArgs pr = a;
    pr.win_mode = 1;
    // (the probe instantiation holds half the VGPRs: two workgroups per CU)
    const uint32_t pblocks = std::max<uint32_t>(
        1, std::min<uint32_t>((a.npos + SP_THREADS - 1) / SP_THREADS, 2u * (uint32_t)SPREAD_MAX_BLOCKS));
    if (passes & SPL_AFF) spread_filter_kernel<true, true><<<pblocks, SP_THREADS, 0, st>>>(pr);
    else spread_filter_kernel<false, true><<<pblocks, SP_THREADS, 0, st>>>(pr);
    spread_wcount_kernel<<<(a.nslots + WIN_CHUNK - 1) / WIN_CHUNK, WIN_CHUNK / 16, 0, st>>>(a);
    spread_window_kernel<<<1, WIN_THREADS, 0, st>>>(a);
  }
  if (passes & SPL_AFF) spread_filter_kernel<true><<<blocks, SP_THREADS, 0, st>>>(a);
  else spread_filter_kernel<false><<<blocks, SP_THREADS, 0, st>>>(a);
  if (passes & SPL_SCORE) spread_score_kernel<<<blocks, SP_THREADS, 0, st>>>(a);
  spread_select_kernel<<<blocks, SP_THREADS, 0, st>>>(a);
  spread_commit_kernel<<<1, WAVE, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_spread_reset(const SpreadArgs &a, hipStream_t st) {
  SpreadArgs z = a;
  z.no_commit = 1;  // reset only: no result, no commit
  spread_commit_kernel<<<1, WAVE, 0, st>>>(z);
  return hipGetLastError();
}

hipError_t launch_replica_run(const SpreadArgs &a, const ReplicaArgs &r, void *sort_tmp, size_t sort_tmp_bytes,
                              uint32_t passes, hipStream_t st) {
  const uint32_t blocks =
      std::max<uint32_t>(1, std::min<uint32_t>((a.npos + SP_THREADS - 1) / SP_THREADS, (uint32_t)SPREAD_MAX_BLOCKS));
  hipError_t e = hipMemsetAsync(r.ctl, 0, RUN_CTL_WORDS * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  // a DoNotSchedule constraint: its domain counts and minimum first, as the chain
  if (passes & SPL_PREP) spread_prep_kernel<<<blocks, SP_THREADS, 0, st>>>(a);
  if (passes & SPL_MIN) spread_min_kernel<<<blocks, SP_THREADS, 0, st>>>(a);
  spread_filter_kernel<false><<<blocks, SP_THREADS, 0, st>>>(a);
  replica_keys_kernel<<<blocks, SP_THREADS, 0, st>>>(a, r);
  size_t bytes = sort_tmp_bytes;
  if ((e = launch_sort_pairs(r.keys, r.sorted, r.val, r.sval, r.nslots, 20 + r.s_bits, sort_tmp, &bytes, st)) !=
      hipSuccess)
    return e;
  replica_groups_kernel<<<blocks, SP_THREADS, 0, st>>>(a, r);
  if (passes & SPL_MIN) replica_run_kernel<true><<<1, RUN_THREADS, 0, st>>>(a, r);  // DoNotSchedule (SPL_MIN)
  else replica_run_kernel<false><<<1, RUN_THREADS, 0, st>>>(a, r);
  return launch_spread_reset(a, st);
}

hipError_t launch_class_commit(const DevResult *res, const uint64_t *cmask, const uint32_t *slot_pos, uint32_t *cnt,
                               uint32_t npos, uint32_t lo, uint32_t hi, hipStream_t st) {
  if (hi <= lo) return hipSuccess;
  class_commit_kernel<<<(hi - lo + 255) / 256, 256, 0, st>>>(res, cmask, slot_pos, cnt, npos, lo, hi);
  return hipGetLastError();
}

hipError_t launch_scatter_u32(uint32_t *col, const uint64_t *idx, const uint32_t *val, uint32_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  scatter_u32_kernel<<<(n + 255) / 256, 256, 0, st>>>(col, idx, val, n);
  return hipGetLastError();
}

hipError_t launch_scatter_i64(int64_t *col, const uint64_t *idx, const int64_t *val, uint32_t n, bool add,
                              hipStream_t st) {
  if (!n) return hipSuccess;
  scatter_i64_kernel<<<(n + 255) / 256, 256, 0, st>>>(col, idx, val, n, add ? 1u : 0u);
  return hipGetLastError();
}

hipError_t launch_add_u32(uint32_t *col, const uint64_t *idx, const int32_t *delta, uint32_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  add_u32_kernel<<<(n + 255) / 256, 256, 0, st>>>(col, idx, delta, n);
  return hipGetLastError();
}

hipError_t launch_umax_u32(uint32_t *dst, const uint32_t *src, uint32_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  umax_u32_kernel<<<(n + 255) / 256, 256, 0, st>>>(dst, src, n);
  return hipGetLastError();
}

}  // namespace ks
