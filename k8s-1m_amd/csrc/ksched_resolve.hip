// ksched_resolve.hip — the round's in-order commit as a parallel proposal /
// verify over chunks of the window (resource-only and label / taint rounds;
// DESIGN.md §5.6).
//
// Sequential semantics (the serial resolve_kernel in
// ksched_kernels.hip): pod j's winner is the best of (a) its first listed
// candidate that no earlier pod of the round took and (b) every node an
// earlier pod took, re-scored against its state after those commits; the
// round stops at j when neither is provably the maximum.  The serial kernel
// walks the pods one barrier each (~1.2 us per pod).  Here the round is
// resolved in passes over chunks of up to PCH pods:
//
//   fixed prefix [0, f)   exact, committed.  Its modified nodes are held in
//                         LDS with their live rows (M); for every later pod j
//                         Rpre[j] = max over M of j's key on the live row and
//                         dl[j] = feasible nodes j lost to those commits are
//                         maintained incrementally as pods are fixed
//   A   (all waves)       each chunk pod gathers its first PNC listed entries
//                         that are not in M and score above Rpre[j]
//   B1  (one wave)        proposals: the serial greedy "first entry no
//                         earlier pod takes, else Rpre's node" -- computed as
//                         deferred acceptance with the pod index as priority,
//                         which reaches the serial-dictatorship matching
//   B2  (all waves)       exact decisions given the proposals: every node
//                         taken by an earlier chunk pod is re-scored for every
//                         later chunk pod (pairs in parallel), feasible counts
//                         corrected; the first pod whose exact decision
//                         differs from its proposal is fixed with the exact one
//   C   (all waves)       commit the verified pods, extend M, update Rpre / dl
//                         of every pod after them (pairs in parallel)
//
// Proposals differ from the exact decision only where a chunk pod re-takes a
// node an earlier pod of the same chunk took (Rpre covers every node of the
// fixed prefix exactly), so a C3 round of 256 pods takes 6-12 passes
// (tools/jacobi_sim.cpp).  Rounds whose pods pile onto the same nodes (kwok
// clusters of identical nodes) would take many passes: under RESOLVE_AUTO such
// a round is handed whole to the serial kernel (pass cap / too few pods per
// pass), and so are the following rounds, a stretch that doubles per
// consecutive hand-over (RoundArgs::rmode).
//
// Arithmetic is the serial kernel's (exact binary64 rows, one-FMA
// LeastAllocated, Markstein BalancedAllocation; ksched_eval.hpp), and the
// outputs are the same: results of the resolved pods, the modified nodes'
// carry records, the next round's start, the completion signal.
#include <hip/hip_runtime.h>

#include "ksched_dev.hpp"
#include "ksched_eval.hpp"
#include "ksched_kernels.hpp"
#include "ksched_resolve_serial.hpp"
#include "ksched_util.hpp"

namespace ks {

constexpr int PR_THREADS = 1024;
constexpr int PR_NW = PR_THREADS / WAVE;
constexpr int PCH = 64;     // pods per chunk: one deferred-acceptance lane each
constexpr int PNC = 16;     // candidates gathered per chunk pod (resource-only rounds)
constexpr int PMH = 1024;   // modified-slot hash (rhash: 10 bits), M <= MAX_P nodes
constexpr int PNR = 4;      // candidates per chunk pod whose rows are prefetched (LDS-DMA)
constexpr int PGH_BITS = 7, PGH = 1 << PGH_BITS;  // chunk slot-group hash (<= PCH slots)
constexpr uint32_t PNONE = 0xFFFFFFFFu;
constexpr uint32_t PSRC_M = 0x10000u;  // proposal source: Rpre's node (M index in the low bits)
static_assert(PCH == WAVE, "B1 runs one chunk pod per lane of one wave");

// decision codes (proposal and exact)
constexpr uint32_t PAR_RATE_PASSES = 4, PAR_MAX_BACKOFF = 16, PAR_MAX_STRETCH = 256;
enum : uint32_t { PD_NODE = 0, PD_UNSCHED = 1, PD_ERROR = 2, PD_STOP = 3, PD_INCOMPLETE = 4 };

// Resource-only pod as the commit evaluates it: Fit thresholds (request, or
// -inf when Fit does not check the resource), requests, non-zero requests x 100
struct PQ {
  double rqc, rqm, rc, rm, zc, zm;
};

__device__ __forceinline__ PQ make_pq(const PodDev &p) {
  PQ q;
  q.rqc = ((p.flags & PF_HAS_REQ) && p.req_cpu > 0) ? p.req_cpu_d : -__builtin_inf();
  q.rqm = ((p.flags & PF_HAS_REQ) && p.req_mem > 0) ? p.req_mem_d : -__builtin_inf();
  q.rc = p.req_cpu_d;
  q.rm = p.req_mem_d;
  q.zc = p.nz100_cpu;
  q.zm = p.nz100_mem;
  return q;
}

// NodeResourcesFit of a resource-only pod on row r with Requested (rc, rm)
// and np pods: the serial kernel's fit_q on rnode_regs
__device__ __forceinline__ bool pq_fit(const PQ &q, const CandRow &r, double rc, double rm, int32_t np) {
  return np + 1 <= r.apods && !(q.rqc > r.acpu - rc) && !(q.rqm > r.amem - rm);
}

// Label / taint pods (EXT rounds): the part of the pod the resource-free
// filters and scores read.  Labels, taints and the normaliser maxima do not
// change within a round, so a node's status before NodeResourcesFit and its
// normalised TaintToleration / NodeAffinity scores are fixed for the round.
struct alignas(16) PX {
  uint64_t tol_hard, tol_prefer;
  uint32_t flags;
  int32_t name_slot;
  uint32_t req_off, req_len, pref_off, pref_len, pre_off, pre_len;
  uint32_t tt_max, na_max;  // the measured maxima (norm_check) the sweep scored with
  uint32_t _pad[2];
};
static_assert(sizeof(PX) == 64, "PX layout");

__device__ __forceinline__ PX make_px(const PodDev &p, uint32_t tt_max, uint32_t na_max) {
  PX x;
  x.tol_hard = p.tol_hard;
  x.tol_prefer = p.tol_prefer;
  x.flags = p.flags;
  x.name_slot = p.name_slot;
  x.req_off = p.req_off;
  x.req_len = p.req_len;
  x.pref_off = p.pref_off;
  x.pref_len = p.pref_len;
  x.pre_off = p.pre_off;
  x.pre_len = p.pre_len;
  x.tt_max = tt_max;
  x.na_max = na_max;
  x._pad[0] = x._pad[1] = 0;
  return x;
}

// The resource-free part of an EXT pod on a node: st = the first failing
// filter before NodeResourcesFit (filter<true>'s order), ST_FEASIBLE if none;
// ss = w_tt x TaintToleration + w_na x NodeAffinity as total_score<true>
// adds them; at = bit 0 / 1: the node's raw TaintToleration / NodeAffinity
// score is the pod's max (the node counts in ShardRecHdr::tt_cnt / na_cnt
// while it is feasible).
struct XS {
  int32_t st;
  int32_t ss;
  uint32_t at;
};
__device__ __forceinline__ XS px_static(const PX &x, const uint64_t *clauses, const CandExt &cx, uint32_t slot,
                                        const Weights &w) {
  PodDev p;  // the fields the label programs read
  p.flags = x.flags;
  p.tol_prefer = x.tol_prefer;
  p.req_off = x.req_off;
  p.req_len = x.req_len;
  p.pref_off = x.pref_off;
  p.pref_len = x.pref_len;
  p.pre_off = x.pre_off;
  p.pre_len = x.pre_len;
  NodeExt e;
  e.hard = cx.w[0];
  e.prefer = cx.w[1];
#pragma unroll
  for (int k = 0; k < LW; ++k) e.lab[k] = cx.w[2 + k];
#pragma unroll
  for (int k = 0; k < NNUM; ++k) e.num[k] = (int64_t)cx.w[2 + LW + k];
  XS r;
  r.st = ST_FEASIBLE;
  r.ss = w.tt * 100;
  r.at = 0;
  if (x.flags & PF_EXT) {
    const uint64_t untol = e.hard & ~x.tol_hard;
    if (x.flags & PF_NA_CONFLICT) r.st = 3;
    else if ((x.flags & PF_PREFILTER) && !prefilter_match(p, clauses, slot)) r.st = ST_PREFILTERED;
    else if (untol & UNSCHED_BIT) r.st = 0;                                          // NodeUnschedulable
    else if (x.name_slot != -1 && (int64_t)slot != (int64_t)x.name_slot) r.st = 1;  // NodeName
    else if (untol) r.st = 2;                                                        // TaintToleration
    else if ((x.flags & PF_AFF) && !required_match(p, clauses, e, slot)) r.st = 3;   // NodeAffinity
  }
  if (r.st != ST_FEASIBLE) return r;
  if (x.flags & PF_TT) {
    const int64_t raw = taint_raw(p, e);
    r.ss = w.tt * (int32_t)normalize(raw, x.tt_max, true);
    r.at |= raw == (int64_t)x.tt_max ? 1u : 0u;
  }
  if (x.flags & PF_HAS_PREF) {
    int32_t na = 0;
    if (x.flags & PF_NA) {
      const int64_t raw = preferred_raw(p, clauses, e, slot);
      na = (int32_t)normalize(raw, x.na_max, false);
      r.at |= raw == (int64_t)x.na_max ? 2u : 0u;
    }
    r.ss += (int32_t)wmul((uint32_t)w.na, (uint32_t)na);
  }
  return r;
}

// packed key of the pod on the row's live state (0: infeasible): key_q on
// rnode_regs, with the resource-free score part ss (w_tt x 100 for a
// resource-only pod)
__device__ __forceinline__ uint64_t pq_key_ss(const PQ &q, const CandRow &r, uint32_t slot, const Weights &w,
                                              int32_t ss) {
  if (!pq_fit(q, r, r.rc, r.rm, r.np)) return 0;
  NodeRegs g;
  g.free_cpu = r.acpu - r.rc;
  g.free_mem = r.amem - r.rm;
  g.rcpu = r.rc;
  g.rmem = r.rm;
  g.lf100_cpu = r.acpu * 100.0 - r.zc100;
  g.lf100_mem = r.amem * 100.0 - r.zm100;
  g.acpu_d = r.acpu;
  g.amem_d = r.amem;
  g.inv_cpu = r.inv_cpu;
  g.inv_mem = r.inv_mem;
  const bool ac = r.acpu != 0.0, am = r.amem != 0.0;
  g.bamul = (ac && am) ? 0.5 : 0.0;
  g.lashift = (ac && am) ? 1u : 0u;
  g.slot = slot;
  const int32_t la = (least_requested(g.lf100_cpu, q.zc, g.inv_cpu) + least_requested(g.lf100_mem, q.zm, g.inv_mem)) >>
                     g.lashift;
  const int32_t ba = score_ba_sum(g.rcpu + q.rc, g.rmem + q.rm, g);
  const int32_t t = (int32_t)wmul((uint32_t)w.fit, (uint32_t)la) + (int32_t)wmul((uint32_t)w.ba, (uint32_t)ba) + ss;
  return pack_key(t, slot);
}
__device__ __forceinline__ uint64_t pq_key(const PQ &q, const CandRow &r, uint32_t slot, const Weights &w) {
  return pq_key_ss(q, r, slot, w, w.tt * 100);
}

// One (pod, node) pair of a round: the key on the node's live row and the
// status change since `rc0 / rm0 / np0` (the row the pod's counts were taken
// on): lost = 1 when the node was feasible there and is not now (only
// NodeResourcesFit can change), `at` the normaliser-at-max bits it takes
// with it (EXT).  Resource-only pods: every filter but Fit passes.
struct PairEval {
  uint64_t key;
  int32_t lost;
  uint32_t at_lost;
};
template <bool EXT>
__device__ __forceinline__ PairEval pair_eval(const PQ &q, const PX *px, const uint64_t *clauses, const CandRow &r,
                                              const CandExt *cx, uint32_t slot, double rc0, double rm0, int32_t np0,
                                              const Weights &w) {
  PairEval v;
  int32_t ss = w.tt * 100;
  uint32_t at = 0;
  if constexpr (EXT) {
    const XS xs = px_static(*px, clauses, *cx, slot, w);
    if (xs.st != ST_FEASIBLE) {
      v.key = 0;
      v.lost = 0;
      v.at_lost = 0;
      return v;
    }
    ss = xs.ss;
    at = xs.at;
  }
  v.key = pq_key_ss(q, r, slot, w, ss);
  v.lost = (pq_fit(q, r, rc0, rm0, np0) ? 1 : 0) - (v.key != 0 ? 1 : 0);
  v.at_lost = v.lost ? at : 0u;
  return v;
}

__device__ __forceinline__ void pq_add(CandRow &r, const PQ &q) {  // NodeInfo.AddPod: exact binary64 sums
  r.rc += q.rc;
  r.rm += q.rm;
  r.zc100 += q.zc;
  r.zm100 += q.zm;
  r.np += 1;
}

// Phase clock of the parallel commit (ks_debug_set_profile): thread 0 reads
// s_memtime after each barrier and charges the interval to a phase, in LDS
// (no registers held across the kernel).
struct PhaseClock {
  uint64_t *out, *acc;  // out: wave-uniform (wave 0 only), null when off
  uint64_t t;
  bool lead;            // thread 0: adds the sums to `out`
  __device__ __forceinline__ void tick(int phase) {
    if (out == nullptr) return;
    const uint64_t now = __builtin_amdgcn_s_memtime();
    if (phase >= 0) acc[phase] += now - t;  // every lane of wave 0 stores the same sum
    t = now;
  }
  __device__ __forceinline__ void flush() {
    if (out == nullptr || !lead) return;
    acc[9] = 1;
    for (int i = 0; i < 16; ++i) atomicAdd((unsigned long long *)&out[i], (unsigned long long)acc[i]);
  }
};

__device__ __forceinline__ uint32_t key_slot(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }
template <int BITS>
__device__ __forceinline__ uint32_t dhash(uint32_t x) { return (x * 2654435761u) >> (32 - BITS); }

// EXT rounds carry each M node's and each proposal's label / taint words and
// each pod's PX beside the resource rows; to stay within the CU's LDS they
// gather PNC_EXT candidates per chunk pod (claims hash halved accordingly)
// and prefetch the rows of the first PNR_EXT, and have no one-step path
// (label / taint batches keep one record per pod: no identical-pod classes).
constexpr int PNC_EXT = 8, PNR_EXT = 2;

// The parallel commit's LDS, a member of the resolve kernel's LDS union
template <bool EXT>
struct ParLds {
  static constexpr int NC = EXT ? PNC_EXT : PNC;      // candidates gathered per chunk pod
  static constexpr int NR = EXT ? PNR_EXT : PNR;      // ... whose rows are prefetched
  static constexpr int DH_BITS = EXT ? 10 : 11;
  static constexpr int DH = 1 << DH_BITS;             // chunk claim hash (<= PCH * NC + PCH slots)
  static constexpr int XP = EXT ? 1 : 0;              // EXT-only arrays: full size, else one element
  static constexpr int FP = EXT ? 0 : 1;              // one-step-path arrays (resource-only rounds)
  // ---- per pod of the round
  PQ s_q[MAX_P];
  PX s_px[XP ? MAX_P : 1];          // EXT: labels / taints / normaliser maxima
  uint32_t s_dn[XP ? MAX_P : 1];    // EXT: normaliser-at-max nodes lost to the fixed prefix (tt | na << 16)
  uint32_t s_fl[MAX_P];
  ShardRecHdr s_hdr[MAX_P];
  uint32_t s_rep[MAX_P];
  uint64_t s_rk[MAX_P];     // Rpre: best key over the fixed prefix's modified nodes (0: none feasible)
  int32_t s_dl[MAX_P];      // feasible nodes lost (Fit) to the fixed prefix's commits
  uint32_t s_dirty[MAX_P];  // Rpre's node was re-taken: recompute before use
  uint32_t s_lptr[MAX_P];   // list entries before it are all in M
  uint4 s_resc[MAX_P];      // result: {win lo, win hi, feasible, status}
  int32_t s_rdl[MAX_P];     // result: Fit failures gained
  uint32_t s_pfo[MAX_P];    // result: PodDev::prefilter_out (staged: no global read in the epilogue)
  // ---- fixed modified nodes (M): live row, round-start Requested / pod count, slot
  RNode s_m[MAX_P];
  CandExt s_mx[XP ? MAX_P : 1];   // EXT: their label / taint words
  uint32_t s_mh[PMH], s_mi[PMH];  // slot + 1 -> M index
  // ---- chunk
  uint64_t s_ck[PCH][NC];  // gathered candidates: keys ...
  uint16_t s_ce[PCH][NC];  // ... and list entries
  uint4 s_crow[PCH][ROW_PIECES][NR];  // the first NR candidates' rows (LDS-DMA)
  uint4 s_crowx[XP ? PCH : 1][EXT_PIECES][NR];  // EXT: ... and their label / taint words
  uint32_t s_cnc[PCH], s_cmore[PCH], s_cpst[PCH];
  uint32_t s_dh[DH], s_do[DH];    // claims: slot + 1 -> lowest claiming chunk pod
  uint32_t s_gh[PGH];             // chunk slot groups: slot + 1 ...
  uint64_t s_gm[PGH];             // ... -> lanes
  uint64_t s_pk[PCH];    // proposal key
  uint32_t s_ps[PCH];    // proposal slot (PNONE: none)
  uint32_t s_pnx[PCH];   // next chunk pod proposing the same slot (PNONE)
  uint32_t s_pfst[PCH];  // first chunk pod proposing its slot
  RNode s_prow[PCH];     // proposed node's state at the chunk start
  CandExt s_prowx[XP ? PCH : 1];  // EXT: its label / taint words
  uint64_t s_ik[PCH];    // best key over nodes taken earlier in the chunk
  int32_t s_idl[PCH];    // feasible nodes lost to them
  uint32_t s_idn[XP ? PCH : 1];   // EXT: normaliser-at-max nodes lost to them
  uint32_t s_cdm[PCH];   // distinct nodes committed by the fixed pods: M index,
  double s_cdp[PCH][2];  // Requested before this chunk's commits,
  int32_t s_cdn[PCH];    // pod count before,
  uint32_t s_cdr[PCH];   // node was in M before the chunk
  // control: [0] f, [1] stopped, [2] cut, [4] distinct nodes, [5] |M|, [6] passes
  uint32_t s_ctl[8];
  // a round of identical request-less pods in one step (identical_round below)
  uint64_t s_ek[FP ? PR_THREADS : 1];  // entries: node key after k of the round's pods
  uint32_t s_ex[FP ? PR_THREADS : 1];  //   list index << 16 | k << 1 | Fit lost by taking it
  uint32_t s_tx[FP ? MAX_K : 1];       // pods each listed node takes
  uint32_t s_ic[4];           // [0] entries, [1] not applicable, [2] modified nodes
  uint32_t s_wt[PR_NW];       // per-wave counts (prefix sums)
  uint64_t s_clk[16];  // phase clock (ks_debug_set_profile)
};

// The resolve kernel's LDS: one buffer that the parallel commit's and the
// serial commit's layouts overlay (each fits the CU's 160 KB on its own, not
// both).  Accessed through a namespace-scope symbol, so that the commits'
// lambdas read their arrays without capturing a pointer to them.
constexpr size_t cmax(size_t x, size_t y) { return x > y ? x : y; }
constexpr size_t RES_LDS_BYTES =
    cmax(cmax(sizeof(ParLds<true>), sizeof(ParLds<false>)),
         cmax(cmax(sizeof(SerialLds<true, LIST_SPAN_1>), sizeof(SerialLds<true, LIST_SPAN_2>)),
              cmax(sizeof(SerialLds<false, LIST_SPAN_1>), sizeof(SerialLds<false, LIST_SPAN_2>))));
alignas(16) __shared__ uint8_t g_res_lds[RES_LDS_BYTES];
template <bool EXT>
__device__ __forceinline__ ParLds<EXT> *par_lds() {
  return reinterpret_cast<ParLds<EXT> *>(g_res_lds);
}
template <bool EXT, int LIST_SPAN>
__device__ __forceinline__ SerialLds<EXT, LIST_SPAN> *ser_lds() {
  return reinterpret_cast<SerialLds<EXT, LIST_SPAN> *>(g_res_lds);
}

// Returns true when it resolved the round (or found it wasted); false when
// the serial commit must take it (RESOLVE_SERIAL, a serial stretch of
// RESOLVE_AUTO, or a hand-over from this round)
template <bool EXT>
__device__ __forceinline__ bool resolve_parallel(const RoundArgs &a) {
  constexpr int NC = EXT ? PNC_EXT : PNC;      // candidates gathered per chunk pod
  constexpr int NR = EXT ? PNR_EXT : PNR;      // ... whose rows are prefetched
  constexpr int DH_BITS = EXT ? 10 : 11;
  constexpr int DH = 1 << DH_BITS;             // chunk claim hash (<= PCH * NC + PCH slots)
  static_assert(DH >= PCH * NC + PCH, "claims hash: every slot a chunk can claim");
#define s_q (par_lds<EXT>()->s_q)
#define s_px (par_lds<EXT>()->s_px)
#define s_dn (par_lds<EXT>()->s_dn)
#define s_fl (par_lds<EXT>()->s_fl)
#define s_hdr (par_lds<EXT>()->s_hdr)
#define s_rep (par_lds<EXT>()->s_rep)
#define s_rk (par_lds<EXT>()->s_rk)
#define s_dl (par_lds<EXT>()->s_dl)
#define s_dirty (par_lds<EXT>()->s_dirty)
#define s_lptr (par_lds<EXT>()->s_lptr)
#define s_resc (par_lds<EXT>()->s_resc)
#define s_rdl (par_lds<EXT>()->s_rdl)
#define s_pfo (par_lds<EXT>()->s_pfo)
#define s_m (par_lds<EXT>()->s_m)
#define s_mx (par_lds<EXT>()->s_mx)
#define s_mh (par_lds<EXT>()->s_mh)
#define s_mi (par_lds<EXT>()->s_mi)
#define s_ck (par_lds<EXT>()->s_ck)
#define s_ce (par_lds<EXT>()->s_ce)
#define s_crow (par_lds<EXT>()->s_crow)
#define s_crowx (par_lds<EXT>()->s_crowx)
#define s_cnc (par_lds<EXT>()->s_cnc)
#define s_cmore (par_lds<EXT>()->s_cmore)
#define s_cpst (par_lds<EXT>()->s_cpst)
#define s_dh (par_lds<EXT>()->s_dh)
#define s_do (par_lds<EXT>()->s_do)
#define s_gh (par_lds<EXT>()->s_gh)
#define s_gm (par_lds<EXT>()->s_gm)
#define s_pk (par_lds<EXT>()->s_pk)
#define s_ps (par_lds<EXT>()->s_ps)
#define s_pnx (par_lds<EXT>()->s_pnx)
#define s_pfst (par_lds<EXT>()->s_pfst)
#define s_prow (par_lds<EXT>()->s_prow)
#define s_prowx (par_lds<EXT>()->s_prowx)
#define s_ik (par_lds<EXT>()->s_ik)
#define s_idl (par_lds<EXT>()->s_idl)
#define s_idn (par_lds<EXT>()->s_idn)
#define s_cdm (par_lds<EXT>()->s_cdm)
#define s_cdp (par_lds<EXT>()->s_cdp)
#define s_cdn (par_lds<EXT>()->s_cdn)
#define s_cdr (par_lds<EXT>()->s_cdr)
#define s_ctl (par_lds<EXT>()->s_ctl)
#define s_ek (par_lds<EXT>()->s_ek)
#define s_ex (par_lds<EXT>()->s_ex)
#define s_tx (par_lds<EXT>()->s_tx)
#define s_ic (par_lds<EXT>()->s_ic)
#define s_wt (par_lds<EXT>()->s_wt)
#define s_clk (par_lds<EXT>()->s_clk)

  // tid / lane are re-materialised at each pass (see the pass loop)
  uint32_t tid = threadIdx.x, lane = tid % WAVE;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  if (a.serial_only) return false;                                         // RESOLVE_SERIAL
  if (a.rmode != nullptr && uniform_u32(a.rmode[0]) != 0) return false;  // a serial stretch (AUTO)
  const uint32_t start = uniform_u32(*a.act);
  if (start >= a.npods || uniform_u32(*a.sstart) != start) {  // the lists belong to other pods
    if (tid == 0) {
      *a.act_next = start;
      *a.d_start = start;
      *a.carry_out_n = 0;
      if (start < a.npods) {
        a.counters[3] += 1;
        mark_pod(a.marks, start, MARK_AFTER_WASTE);
      }
      if (a.rmode != nullptr) a.rmode[1] = a.seq;
      signal_done(a.flag_res, a.seq, a.stall_us);
    }
    return true;
  }
  const uint32_t n = min(a.P, a.npods - start);
  const uint32_t RW = rec_words(a.K);
  // lanes below this one (recomputed where used: a 64-bit value held across
  // the kernel costs two of the 128 VGPRs)
#define lt_mask ((1ull << lane) - 1ull)
  // phases: 0 stage, 1 gather barrier, 2 proposals, 3 wave 0's row DMA issue, 4 chunk pairs, 5 wave 0's
  // DMA wait, 6 decide + commit, 7 Rpre updates, 8 epilogue, [9] rounds, [10] dirty recomputes, [11] extra
  // windows, 12 wave 0's wait for the prefetched windows, 13 its scalar state + probes, 14 its window scans
  if (tid < 16) s_clk[tid] = 0;
  PhaseClock clk{wid == 0 ? a.prof : nullptr, s_clk, 0, tid == 0};
  clk.tick(-1);

  auto mh_find = [&](uint32_t slot) -> uint32_t {
    uint32_t h = rhash(slot);
    for (;;) {
      const uint32_t v = s_mh[h];
      if (v == 0) return PNONE;
      if (v == slot + 1) return s_mi[h];
      h = (h + 1) & (PMH - 1);
    }
  };
  auto dh_insert = [&](uint32_t slot) -> uint32_t {
    uint32_t h = dhash<DH_BITS>(slot);
    for (;;) {
      const uint32_t old = atomicCAS(&s_dh[h], 0u, slot + 1);
      if (old == 0 || old == slot + 1) return h;
      h = (h + 1) & (DH - 1);
    }
  };
  auto dh_owner = [&](uint32_t slot) -> uint32_t {
    uint32_t h = dhash<DH_BITS>(slot);
    for (;;) {
      const uint32_t v = s_dh[h];
      if (v == 0) return PNONE;
      if (v == slot + 1) return s_do[h];
      h = (h + 1) & (DH - 1);
    }
  };
  // wave 0: lanes of the chunk grouped by slot (s_gh / s_gm cleared by the caller)
  auto group_of = [&](uint32_t slot, bool in) -> uint64_t {
    uint32_t h = PNONE;
    if (in) {
      h = (slot * 2654435761u) >> (32 - PGH_BITS);
      for (;;) {
        const uint32_t old = atomicCAS(&s_gh[h], 0u, slot + 1);
        if (old == 0 || old == slot + 1) break;
        h = (h + 1) & (PGH - 1);
      }
      atomicOr((unsigned long long *)&s_gm[h], (unsigned long long)(1ull << lane));
    }
    return in ? s_gm[h] : 0ull;
  };
  // s_prow[dst] <- a gathered candidate's node at the round start (its S0 row:
  // live state = round-start state), copied piece by piece
  auto prow_from_cand = [&](uint32_t dst, uint32_t c, uint32_t j, uint32_t cand, uint32_t slot) {
    uint4 *d = (uint4 *)&s_prow[dst];
    if (cand < (uint32_t)NR) {
#pragma unroll
      for (int q = 0; q < ROW_PIECES; ++q) d[q] = s_crow[c][q][cand];
      if constexpr (EXT) {
        uint4 *dx = (uint4 *)&s_prowx[dst];
#pragma unroll
        for (int q = 0; q < EXT_PIECES; ++q) dx[q] = s_crowx[c][q][cand];
      }
    } else {  // beyond the prefetched rows: one global round trip
      const size_t e = (size_t)s_rep[j] * a.K + s_ce[c][cand];
      const uint4 *g = (const uint4 *)(a.crow + e);
#pragma unroll
      for (int q = 0; q < ROW_PIECES; ++q) d[q] = g[q];
      if constexpr (EXT) {
        const uint4 *gx = (const uint4 *)(a.cext + e);
        uint4 *dx = (uint4 *)&s_prowx[dst];
#pragma unroll
        for (int q = 0; q < EXT_PIECES; ++q) dx[q] = gx[q];
      }
    }
    RNode &x = s_prow[dst];
    x.rc0 = x.row.rc;
    x.rm0 = x.row.rm;
    x.np0 = x.row.np;
    x.slot = slot;
    x._pad[0] = x._pad[1] = 0;
  };

  // EXT: a normalising plugin's count of feasible nodes at its max has
  // dropped to 0 (dn: at-max nodes lost, TaintToleration | NodeAffinity << 16):
  // the max may have moved, the round stops before the pod (the serial
  // kernel's rule)
  auto norm_stop = [&](uint32_t j, uint32_t dn) -> bool {
    if constexpr (!EXT) {
      return false;
    } else {
      const uint32_t fl = s_fl[j];
      const ShardRecHdr &h = s_hdr[j];
      return ((fl & PF_TT) && h.tt_cnt - (dn & 0xFFFFu) == 0) || ((fl & PF_NA) && h.na_cnt - (dn >> 16) == 0);
    }
  };

  // ---- stage the round
  for (uint32_t i = tid; i < n; i += PR_THREADS) {
    const uint32_t ri = a.rep != nullptr ? a.rep[i] : i;
    const PodDev p = a.pods[start + i];
    s_rep[i] = ri;
    s_q[i] = make_pq(p);
    s_fl[i] = p.flags;
    s_pfo[i] = p.prefilter_out;
    s_hdr[i] = *(const ShardRecHdr *)(a.frec + (size_t)ri * RW);
    s_rk[i] = 0;
    s_dl[i] = 0;
    s_dirty[i] = 0;
    s_lptr[i] = 0;
    if constexpr (EXT) {
      s_px[i] = make_px(p, a.norm_max[2 * i], a.norm_max[2 * i + 1]);
      s_dn[i] = 0;
    }
  }
  for (uint32_t i = tid; i < PMH; i += PR_THREADS) s_mh[i] = 0;
  if (tid < 8) s_ctl[tid] = 0;
  __syncthreads();
  clk.tick(0);

  // Each wave gathers chunk pods wid + PR_NW t; their first list windows are
  // loaded ahead into registers (here for the first chunk, then during the
  // previous pass's Rpre updates), so a pass starts on resident keys.
  constexpr int PPW = PCH / PR_NW;
  uint64_t kw0 = 0, kw1 = 0, kw2 = 0, kw3 = 0;
  static_assert(PPW == 4, "four chunk pods per wave");
  auto load_windows = [&](uint32_t f, uint32_t cn) {
    auto ld = [&](uint32_t c) -> uint64_t {
      if (c >= cn) return 0ull;
      const uint32_t j = f + c, e = s_lptr[j] + lane;
      return e < s_hdr[j].nkeys ? a.frec[(size_t)s_rep[j] * RW + REC_HDR_WORDS + e] : 0ull;
    };
    kw0 = ld(wid);
    kw1 = ld(wid + PR_NW);
    kw2 = ld(wid + 2 * PR_NW);
    kw3 = ld(wid + 3 * PR_NW);
  };
  // ---- a round whose pods are all one identical pod (kwok's busybox pods, a
  // deployment's replicas): when node x's key after k of these pods,
  // key_x(k), is non-increasing in k for every listed node, the sequential
  // greedy gives pod j the j-th largest entry of {key_x(k)} in (key desc,
  // k asc) order (ties are within one node: the key carries the slot), and
  // only entries at or above the n-th listed key can be among the first n
  // (or, with a shorter list, above the bound: the round stops where they
  // run out).  Request-less pods never change Requested, so
  // BalancedAllocation is constant and LeastAllocated only falls: always
  // non-increasing.  With requests BalancedAllocation can rise, so every
  // node's sequence is checked to its end (no fit, or n pods) and any rise
  // sends the round to the passes.  One step instead of a pass per one or
  // two pods.
  bool fast = false;
  if constexpr (!EXT) {
    if (tid < 4) s_ic[tid] = 0;
    __syncthreads();
    const PQ q0 = s_q[0];
    const ShardRecHdr &h0 = s_hdr[0];
    if (tid < n && s_rep[tid] != s_rep[0]) s_ic[1] = 1;  // more than one pod class
    if (tid == 0 && (n < 2 || a.rep == nullptr || h0.feasible == 0 || (s_fl[0] & PF_PREF_ERR) || h0.nkeys == 0))
      s_ic[1] = 1;
    const bool check_all = q0.rc != 0.0 || q0.rm != 0.0;  // requests: BalancedAllocation moves
    __syncthreads();
    if (s_ic[1] == 0) {
      const uint32_t nk = min(h0.nkeys, (uint32_t)MAX_K);
      const uint64_t *keys0 = a.frec + (size_t)s_rep[0] * RW + REC_HDR_WORDS;
      const uint64_t thr = nk >= n ? keys0[n - 1] : h0.bound + 1;
      if (tid < nk) {
        CandRow r = a.crow[(size_t)s_rep[0] * a.K + tid];
        const uint32_t slot = key_slot(keys0[tid]);
        uint64_t prev = ~0ull;
        for (uint32_t k = 0; k < n; ++k) {
          const uint64_t key = pq_key(q0, r, slot, a.w);
          if (key > prev) {  // not non-increasing: the general passes
            s_ic[1] = 1;
            break;
          }
          if (key == 0 || (key < thr && !check_all)) break;
          prev = key;
          pq_add(r, q0);
          if (key < thr) continue;  // checked for monotonicity only
          const bool lost = !pq_fit(q0, r, r.rc, r.rm, r.np);  // the next identical pod no longer fits
          const uint32_t e = atomicAdd(&s_ic[0], 1u);
          if (e < (uint32_t)PR_THREADS) {
            s_ek[e] = key;
            s_ex[e] = tid << 16 | k << 1 | (lost ? 1u : 0u);
          }
        }
      }
      if (tid < MAX_K) s_tx[tid] = 0;
      __syncthreads();
      const uint32_t ne = s_ic[0];
      if (s_ic[1] == 0 && ne <= (uint32_t)PR_THREADS) {
        // bitonic sort of the entries, padded to a power of two: key desc, then k asc
        uint32_t p2 = 1;
        while (p2 < ne) p2 <<= 1;
        if (tid >= ne && tid < p2) {
          s_ek[tid] = 0;
          s_ex[tid] = 0xFFFFFFFFu;
        }
        __syncthreads();
        auto before = [](uint64_t ka, uint32_t xa, uint64_t kb, uint32_t xb) {
          return ka > kb || (ka == kb && xa < xb);
        };
        for (uint32_t size = 2; size <= p2; size <<= 1) {
          for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            const uint32_t i = tid, j = tid ^ stride;
            if (j > i && j < p2) {
              const uint64_t ki = s_ek[i], kj = s_ek[j];
              const uint32_t xi = s_ex[i], xj = s_ex[j];
              const bool up = (i & size) == 0;
              if (up ? before(kj, xj, ki, xi) : before(ki, xi, kj, xj)) {
                s_ek[i] = kj;
                s_ek[j] = ki;
                s_ex[i] = xj;
                s_ex[j] = xi;
              }
            }
            __syncthreads();
          }
        }
        // pod j takes entry j; its feasible count = the round start's minus the
        // nodes earlier pods filled (exclusive prefix sum of the lost flags)
        const uint32_t nres = min(n, ne);
        const bool in = tid < nres;
        const uint32_t x = in ? s_ex[tid] : 0u;
        const uint64_t bm = __ballot(in && (x & 1u));
        if (lane == 0) s_wt[wid] = (uint32_t)__popcll(bm);
        if (in) atomicAdd(&s_tx[x >> 16], 1u);
        __syncthreads();
        uint32_t dl = (uint32_t)__popcll(bm & lt_mask);
        for (uint32_t w = 0; w < wid; ++w) dl += s_wt[w];
        if (in) {
          const uint64_t key = s_ek[tid];
          const uint32_t feas = h0.feasible - dl;  // >= 1: pod tid has a feasible node, the entry's
          s_resc[tid] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), feas, 0u);
          s_rdl[tid] = (int32_t)dl;
        }
        // the nodes taken: their rows after the round, for the carry / write-back
        if (tid < nk && s_tx[tid] > 0) {
          const uint32_t mi = atomicAdd(&s_ic[2], 1u);
          const CandRow r0 = a.crow[(size_t)s_rep[0] * a.K + tid];
          RNode &m = s_m[mi];
          m.row = r0;
          for (uint32_t k = 0; k < s_tx[tid]; ++k) pq_add(m.row, q0);
          m.rc0 = r0.rc;
          m.rm0 = r0.rm;
          m.np0 = r0.np;
          m.slot = key_slot(keys0[tid]);
          m._pad[0] = m._pad[1] = 0;
        }
        __syncthreads();
        if (tid == 0) {
          s_ctl[0] = nres;
          s_ctl[1] = nres < n ? 1u : 0u;  // the list ran out: the round stops there
          s_ctl[5] = s_ic[2];
          s_ctl[6] = 1;
        }
        fast = true;
      }
    }
    __syncthreads();
  }
  if (!fast) load_windows(0, min((uint32_t)PCH, n));

  // Under RESOLVE_AUTO a round that runs past par_max_passes passes, or whose
  // pace after PAR_RATE_PASSES passes projects more than that many for its n
  // pods (passes * n > par_max_passes * fixed), is handed whole to the
  // serial kernel, with the following rounds.
  const uint32_t pass_cap = a.rmode != nullptr ? a.par_max_passes : (uint32_t)MAX_P + 1;
  bool bailed = false;
  for (uint32_t guard = 0; guard <= MAX_P; ++guard) {
    // Opaque per pass: otherwise the compiler hoists every lane-derived LDS
    // address out of the pass loop, which at the 128-VGPR cap of a
    // 1024-thread block spills them to scratch.
    asm volatile("" : "+v"(tid), "+v"(lane));
    const uint32_t f = s_ctl[0];
    if (f >= n || s_ctl[1] != 0) break;
    if (guard >= pass_cap || (a.rmode != nullptr && guard >= PAR_RATE_PASSES && guard * n > pass_cap * f)) {
      bailed = true;  // uniform: guard and s_ctl[0] are
      break;
    }
    const uint32_t cn = min((uint32_t)PCH, n - f);

    // ====================== A: gather candidates (all waves, 4 chunk pods each)
    for (uint32_t i = tid; i < DH; i += PR_THREADS) {
      s_dh[i] = 0;
      s_do[i] = PNONE;
    }
    if (a.prof) {  // diagnostic: how long the prefetched windows are still in flight
      __builtin_amdgcn_s_waitcnt(0);
      clk.tick(12);
    }
    {
      // The wave's four pods side by side, so that their LDS round trips
      // overlap: scalar state in one batch, then the four first windows'
      // membership probes of M interleaved.
      uint32_t jt[PPW], nkt[PPW], bt[PPW], rept[PPW], dirt[PPW];
      uint64_t rkt[PPW], kt[PPW] = {kw0, kw1, kw2, kw3};
      bool on[PPW];
#pragma unroll
      for (int t = 0; t < PPW; ++t) {
        const uint32_t c = wid + PR_NW * t;
        on[t] = c < cn;
        jt[t] = f + (on[t] ? c : 0u);
        dirt[t] = s_dirty[jt[t]];
        rkt[t] = s_rk[jt[t]];
        nkt[t] = s_hdr[jt[t]].nkeys;
        bt[t] = s_lptr[jt[t]];
        rept[t] = s_rep[jt[t]];
      }
#pragma unroll
      for (int t = 0; t < PPW; ++t) {
        if (!on[t] || !dirt[t]) continue;
        // Rpre's node was re-taken: the max over every M node again
        const PQ q = s_q[jt[t]];
        uint64_t best = 0;
        const uint32_t mn = s_ctl[5];
        for (uint32_t m = lane; m < mn; m += WAVE) {
          const RNode &x = s_m[m];
          best = max64(best, pair_eval<EXT>(q, &s_px[EXT ? jt[t] : 0], a.clauses, x.row, &s_mx[EXT ? m : 0], x.slot,
                                            x.rc0, x.rm0, x.np0, a.w).key);
        }
        rkt[t] = wave_max_u64_dpp(best);
        if (lane == 0) {
          s_rk[jt[t]] = rkt[t];
          s_dirty[jt[t]] = 0;
          if (a.prof) atomicAdd((unsigned long long *)&s_clk[10], 1ull);
        }
      }
      // membership of the first windows' slots in M: four probe chains at once
      uint32_t ht[PPW], st[PPW];
      bool pend[PPW], inm[PPW];
#pragma unroll
      for (int t = 0; t < PPW; ++t) {
        st[t] = key_slot(kt[t]);
        pend[t] = on[t] && bt[t] + lane < nkt[t];
        inm[t] = false;
        ht[t] = rhash(st[t]);
      }
      while (__ballot(pend[0] || pend[1] || pend[2] || pend[3])) {
        uint32_t v[PPW];
#pragma unroll
        for (int t = 0; t < PPW; ++t) v[t] = pend[t] ? s_mh[ht[t]] : 0u;
#pragma unroll
        for (int t = 0; t < PPW; ++t) {
          if (!pend[t]) continue;
          if (v[t] == 0) {
            pend[t] = false;
          } else if (v[t] == st[t] + 1) {
            inm[t] = true;
            pend[t] = false;
          } else {
            ht[t] = (ht[t] + 1) & (PMH - 1);
          }
        }
      }
      clk.tick(13);  // wave 0: scalar state, dirty recomputes, M probes of the first windows
      static_for<PPW>([&](auto T) {
        constexpr int t = T;
        const uint32_t c = wid + PR_NW * t;
        if (c >= cn) return;
        const uint32_t j = jt[t], nk = nkt[t];
        const uint64_t rk = rkt[t];
        const uint64_t *keys = a.frec + (size_t)rept[t] * RW + REC_HDR_WORDS;
        uint32_t base = bt[t], cnt = 0, firstu = PNONE;
        bool more = false;
        uint64_t k = kt[t];
        bool in = inm[t];
        for (bool first_window = true; base < nk; first_window = false) {
          const uint32_t e = base + lane;
          const bool valid = e < nk;
          if (!first_window) in = valid && mh_find(key_slot(k)) != PNONE;  // later windows: one probe chain
          const bool unt = valid && !in;
          const uint64_t um = __ballot(unt);
          if (firstu == PNONE && um) firstu = base + (uint32_t)__builtin_ctzll(um);
          const bool take = unt && k > rk;
          const uint64_t tm = __ballot(take);
          const uint32_t r = cnt + (uint32_t)__popcll(tm & lt_mask);
          if (take && r < (uint32_t)NC) {
            s_ck[c][r] = k;
            s_ce[c][r] = (uint16_t)e;
          }
          cnt += (uint32_t)__popcll(tm);
          if (cnt >= (uint32_t)NC) {
            more = true;  // there may be more untaken entries above Rpre
            break;
          }
          if (__ballot(valid && k <= rk)) break;  // keys descend: the rest are below Rpre
          base += WAVE;
          k = base + lane < nk ? keys[base + lane] : 0ull;
          if (a.prof && lane == 0) atomicAdd((unsigned long long *)&s_clk[11], 1ull);
        }
        if (lane == 0) {
          s_cnc[c] = min(cnt, (uint32_t)NC);
          s_cmore[c] = more ? 1u : 0u;
          s_lptr[j] = firstu != PNONE ? firstu : min(base + WAVE, nk);
          const uint32_t feas = s_hdr[j].feasible - (uint32_t)s_dl[j];
          s_cpst[c] = feas == 0                                     ? PD_UNSCHED
                      : ((s_fl[j] & PF_PREF_ERR) && feas >= 2)     ? PD_ERROR
                      : norm_stop(j, EXT ? s_dn[EXT ? j : 0] : 0u) ? PD_STOP
                                                                   : PD_NODE;
        }
      });
      clk.tick(14);  // wave 0: the window scans
    }
    // the first NR candidates' rows of the wave's pods by LDS-DMA, lane r ->
    // row r, issued after every scan (the compiler waits for all outstanding
    // loads before a scan's key use); landed before the barrier.  (Issued with
    // the key windows a phase earlier instead, for the first NR list entries,
    // the gather kept its time and the Rpre phase grew by the issue: 55k ->
    // 76k cycles per round on the proxy.)
    static_for<PPW>([&](auto T) {
      const uint32_t c = wid + PR_NW * (uint32_t)T;
      if (c >= cn) return;
      if (lane < min(s_cnc[c], (uint32_t)NR)) {
        const size_t e = (size_t)s_rep[f + c] * a.K + s_ce[c][lane];
        const uint4 *src = (const uint4 *)(a.crow + e);
#pragma unroll
        for (int q = 0; q < ROW_PIECES; ++q)
          __builtin_amdgcn_global_load_lds((gvoid_t *)(src + q), (lvoid_t *)&s_crow[c][q][0], 16, 0, 0);
        if constexpr (EXT) {
          const uint4 *srx = (const uint4 *)(a.cext + e);
#pragma unroll
          for (int q = 0; q < EXT_PIECES; ++q)
            __builtin_amdgcn_global_load_lds((gvoid_t *)(srx + q), (lvoid_t *)&s_crowx[c][q][0], 16, 0, 0);
        }
      }
    });
    clk.tick(3);                    // wave 0: the row DMAs issued
    __builtin_amdgcn_s_waitcnt(0);  // this wave's row DMAs have landed
    clk.tick(5);                    // ... and its wait for them
    __syncthreads();
    clk.tick(1);

    // ================== B: proposals by deferred acceptance (wave 0, lane = pod)
    if (wid == 0) {
      const uint32_t c = lane, j = f + c;
      const bool in = c < cn;
      const uint32_t pst = in ? s_cpst[c] : PD_INCOMPLETE;
      const uint32_t nc = in ? s_cnc[c] : 0u;
      uint32_t ptr = 0, h = PNONE;
      bool active = in && pst == PD_NODE && nc > 0;
      // Pod c proposes its candidate ptr; every slot keeps the lowest pod that
      // ever proposed it (a holder only loses a slot to a lower pod, and a
      // slot once held stays held), so pods that see another owner move on.
      // The fixed point is the serial greedy: each pod takes its first
      // candidate no lower pod takes.
      for (uint32_t it = 0; it <= (uint32_t)(PCH * NC); ++it) {
        if (active && h == PNONE) h = dh_insert(key_slot(s_ck[c][ptr]));
        if (active) atomicMin(&s_do[h], c);
        const bool lost = active && s_do[h] != c;
        if (__ballot(lost) == 0) break;
        if (lost) {
          h = PNONE;
          if (++ptr >= nc) active = false;
        }
      }
      uint32_t code = pst, src = PNONE, ps = PNONE;
      uint64_t key = 0;
      if (in && pst == PD_NODE) {
        if (active) {
          key = s_ck[c][ptr];
          ps = key_slot(key);
          src = ptr;
        } else if (s_cmore[c]) {
          code = PD_INCOMPLETE;  // more candidates than gathered may be free
        } else {
          const uint64_t rk = s_rk[j];
          if (rk > s_hdr[j].bound) {
            key = rk;
            ps = key_slot(rk);
            src = PSRC_M | mh_find(ps);
          } else {
            code = PD_STOP;
          }
        }
      }
      // Rpre's node re-taken by a lower chunk pod: its state for this pod
      // changed, so Rpre is no longer known here
      const bool rp = in && code == PD_NODE && src >= PSRC_M;
      uint32_t hh = PNONE;
      if (rp) {
        hh = dh_insert(ps);
        atomicMin(&s_do[hh], c);
      }
      if (rp && s_do[hh] != c) {
        code = PD_INCOMPLETE;
        key = 0;
        ps = PNONE;
      }
      const uint64_t inc = __ballot(in && code == PD_INCOMPLETE), stp = __ballot(in && code == PD_STOP);
      uint32_t cut = cn;
      if (inc) cut = min(cut, (uint32_t)__builtin_ctzll(inc));
      if (stp) cut = min(cut, (uint32_t)__builtin_ctzll(stp) + 1u);
      const bool live = c < cut;
      if (!live) {
        key = 0;
        ps = PNONE;
      }
      // the proposed node's state at the chunk start
      if (live && code == PD_NODE) {
        if (src >= PSRC_M) {
          s_prow[c] = s_m[src & 0xFFFFu];
          if constexpr (EXT) s_prowx[c] = s_mx[src & 0xFFFFu];
        } else {
          prow_from_cand(c, c, j, src, ps);
        }
      }
      // lanes proposing the same slot: first of the group, next member
      s_gh[lane] = 0;
      s_gh[lane + WAVE] = 0;
      s_gm[lane] = 0;
      s_gm[lane + WAVE] = 0;
      const uint64_t g = group_of(ps, ps != PNONE);
      const uint64_t above = lane == 63 ? 0ull : g & ~((2ull << lane) - 1ull);
      s_pk[c] = key;
      s_ps[c] = ps;
      s_pfst[c] = (g & lt_mask) == 0 ? 1u : 0u;
      s_pnx[c] = above ? (uint32_t)__builtin_ctzll(above) : PNONE;
      s_ik[c] = 0;
      s_idl[c] = 0;
      if constexpr (EXT) s_idn[c] = 0;
      s_cpst[c] = code;  // proposal code from here on
      s_cdm[c] = src;    // proposal source (C reads it before reusing the slot)
      if (lane == 0) s_ctl[2] = cut;
    }
    __syncthreads();
    clk.tick(2);
    const uint32_t cut = s_ctl[2];

    // ============== chunk pairs: nodes taken earlier in the chunk, for every later pod
    {
      const uint32_t npairs = cut * (cut - 1) / 2;
      for (uint32_t t = tid; t < npairs; t += PR_THREADS) {
        // pair (jc, ic), ic < jc: t = jc (jc - 1) / 2 + ic
        uint32_t jc = (uint32_t)((1.0f + __builtin_sqrtf(1.0f + 8.0f * (float)t)) * 0.5f);
        while (jc * (jc - 1) / 2 > t) --jc;
        while ((jc + 1) * jc / 2 <= t) ++jc;
        const uint32_t ic = t - jc * (jc - 1) / 2;
        if (s_ps[ic] == PNONE || !s_pfst[ic]) continue;
        CandRow r = s_prow[ic].row;
        const double rc0 = r.rc, rm0 = r.rm;
        const int32_t np0 = r.np;
        for (uint32_t k = ic; k != PNONE && k < jc; k = s_pnx[k]) pq_add(r, s_q[f + k]);
        const PQ q = s_q[f + jc];
        const PairEval v = pair_eval<EXT>(q, &s_px[EXT ? f + jc : 0], a.clauses, r, &s_prowx[EXT ? ic : 0],
                                          s_prow[ic].slot, rc0, rm0, np0, a.w);
        if (v.key) atomicMax((unsigned long long *)&s_ik[jc], (unsigned long long)v.key);
        if (v.lost) atomicAdd(&s_idl[jc], v.lost);
        if (EXT && v.at_lost) atomicAdd(&s_idn[EXT ? jc : 0], (v.at_lost & 1u) | (v.at_lost >> 1) << 16);
      }
    }
    __syncthreads();
    clk.tick(4);

    // ===== C: exact decisions, the verified prefix committed (wave 0, lane = pod)
    if (wid == 0) {
      const uint32_t c = lane, j = f + c;
      const bool live = c < cut;
      const uint32_t pcode = live ? s_cpst[c] : PD_INCOMPLETE;
      const uint32_t psrc = live ? s_cdm[c] : PNONE;
      const uint64_t pkey = live ? s_pk[c] : 0ull;
      uint32_t code = PD_INCOMPLETE, feas = 0;
      uint64_t win = 0, ku = 0;
      uint32_t kidx = PNONE;
      if (live) {
        const ShardRecHdr &hd = s_hdr[j];
        feas = hd.feasible - (uint32_t)s_dl[j] - (uint32_t)s_idl[c];
        const uint64_t rk = s_rk[j], ik = s_ik[c];
        code = PD_NODE;
        if (feas == 0) {
          code = PD_UNSCHED;
        } else if ((s_fl[j] & PF_PREF_ERR) && feas >= 2) {
          code = PD_ERROR;
        } else if (norm_stop(j, EXT ? s_dn[EXT ? j : 0] + s_idn[EXT ? c : 0] : 0u)) {
          code = PD_STOP;
        } else {
          // the first candidate no lower pod took: the proposal's, unless the
          // pod had no proposal (its status changed with the chunk's commits)
          if (pcode == PD_NODE) {
            if (psrc < PSRC_M) {
              ku = pkey;
              kidx = psrc;
            }
          } else {
            const uint32_t nc = s_cnc[c];
            for (uint32_t l = 0; l < nc; ++l) {
              const uint32_t o = dh_owner(key_slot(s_ck[c][l]));
              if (o == PNONE || o >= c) {
                ku = s_ck[c][l];
                kidx = l;
                break;
              }
            }
          }
          // every gathered candidate scores above Rpre: with one free, Rpre's
          // node (re-taken or not) cannot win over it
          if (ku) {
            win = max64(ku, max64(rk, ik));
          } else {
            const uint32_t ro = rk ? dh_owner(key_slot(rk)) : PNONE;
            if (s_cmore[c] || (ro != PNONE && ro < c)) {
              code = PD_INCOMPLETE;
            } else {
              const uint64_t bm = max64(rk, ik);
              if (bm > hd.bound) win = bm;
              else code = PD_STOP;
            }
          }
        }
      }
      const bool mism = live && code != PD_INCOMPLETE && (code != pcode || (code == PD_NODE && win != pkey));
      const uint64_t mmask = __ballot(mism), imask = __ballot(live && code == PD_INCOMPLETE);
      const uint32_t mm = mmask ? (uint32_t)__builtin_ctzll(mmask) : PNONE;
      uint32_t ccut = cut;
      if (imask) ccut = min(ccut, (uint32_t)__builtin_ctzll(imask));
      // pods [0, nfix) get results; `stop`: the round ends at pod f + nfix.
      // ccut >= 1: the chunk's first pod is always decided (no lower pod
      // takes its candidates or Rpre's node)
      uint32_t nfix;
      bool stop;
      if (mm < ccut) {
        stop = __builtin_amdgcn_readlane(code, mm) == PD_STOP;
        nfix = stop ? mm : mm + 1;
      } else {
        stop = ccut > 0 && __builtin_amdgcn_readlane(code, ccut - 1) == PD_STOP;
        nfix = stop ? ccut - 1 : ccut;
      }
      if (c == mm && code == PD_NODE) {
        // the node the exact decision commits, at the chunk start
        const uint32_t ws = key_slot(win);
        if (win == ku) {
          prow_from_cand(c, c, j, kidx, ws);
        } else {
          uint32_t from = PNONE;
          for (uint32_t i = 0; i < c && from == PNONE; ++i)
            if (s_ps[i] == ws) from = i;
          if constexpr (EXT) {
            const uint32_t mi = from != PNONE ? PNONE : mh_find(ws);
            s_prow[c] = from != PNONE ? s_prow[from] : s_m[mi];
            s_prowx[c] = from != PNONE ? s_prowx[from] : s_mx[mi];
          } else {
            s_prow[c] = *(from != PNONE ? &s_prow[from] : &s_m[mh_find(ws)]);
          }
        }
      }
      const bool fx = c < nfix;
      if (!fx) win = 0;
      if (fx) {
        s_resc[j] = make_uint4((uint32_t)win, (uint32_t)(win >> 32), feas,
                               code == PD_UNSCHED ? 1u : code == PD_ERROR ? 2u : 0u);
        s_rdl[j] = s_dl[j] + s_idl[c];
      }
      // commit: the first fixed pod of each node adds every fixed pod's request on it
      const uint32_t ws = win ? key_slot(win) : PNONE;
      s_gh[lane] = 0;
      s_gh[lane + WAVE] = 0;
      s_gm[lane] = 0;
      s_gm[lane + WAVE] = 0;
      const uint64_t g = group_of(ws, ws != PNONE);
      const bool first = ws != PNONE && (g & lt_mask) == 0;
      const uint32_t mi0 = first ? mh_find(ws) : PNONE;
      const bool isnew = first && mi0 == PNONE;
      const uint64_t fm = __ballot(first), nm = __ballot(isnew);
      const uint32_t mn = s_ctl[5];
      if (first) {
        const uint32_t mi = isnew ? mn + (uint32_t)__popcll(nm & lt_mask) : mi0;
        // a new node enters M with its chunk-start row (piece by piece: a
        // struct copy through a selected pointer goes via scratch); then the
        // requests are summed in registers, in pod order, and stored back
        if (isnew) {
          const uint4 *sp = (const uint4 *)&s_prow[c];
          uint4 *dp = (uint4 *)&s_m[mi];
#pragma unroll
          for (int q = 0; q < (int)(sizeof(RNode) / 16); ++q) dp[q] = sp[q];
          if constexpr (EXT) {
            const uint4 *sx = (const uint4 *)&s_prowx[c];
            uint4 *dx = (uint4 *)&s_mx[mi];
#pragma unroll
            for (int q = 0; q < EXT_PIECES; ++q) dx[q] = sx[q];
          }
        }
        CandRow &xr = s_m[mi].row;
        double rc = xr.rc, rm = xr.rm, zc = xr.zc100, zm = xr.zm100;
        int32_t np = xr.np;
        const uint32_t d = (uint32_t)__popcll(fm & lt_mask);
        s_cdm[d] = mi;
        s_cdp[d][0] = rc;
        s_cdp[d][1] = rm;
        s_cdn[d] = np;
        s_cdr[d] = isnew ? 0u : 1u;
        for (uint64_t m = g; m; m &= m - 1) {  // pq_add
          const PQ &q = s_q[f + (uint32_t)__builtin_ctzll(m)];
          rc += q.rc;
          rm += q.rm;
          zc += q.zc;
          zm += q.zm;
          np += 1;
        }
        xr.rc = rc;
        xr.rm = rm;
        xr.zc100 = zc;
        xr.zm100 = zm;
        xr.np = np;
        if (isnew) {
          uint32_t h = rhash(ws);
          while (atomicCAS(&s_mh[h], 0u, ws + 1) != 0u) h = (h + 1) & (PMH - 1);
          s_mi[h] = mi;
        }
      }
      if (lane == 0) {
        s_ctl[4] = (uint32_t)__popcll(fm);
        s_ctl[5] = mn + (uint32_t)__popcll(nm);
        s_ctl[0] = f + nfix;
        s_ctl[1] = stop ? 1u : 0u;
        s_ctl[6] += 1;
      }
    }
    __syncthreads();
    clk.tick(6);

    // ===== Rpre / feasible-count updates of every later pod (pairs in parallel)
    {
      const uint32_t nf = s_ctl[0], nd = s_ctl[4];
      const uint32_t npend = n > nf ? n - nf : 0u;
      if (s_ctl[1] == 0 && npend > 0) {
        load_windows(nf, min((uint32_t)PCH, npend));  // the next chunk's first windows, in flight meanwhile
        const uint32_t total = nd * npend;
        for (uint32_t t = tid; t < total; t += PR_THREADS) {
          const uint32_t d = t / npend, jj = nf + t % npend;
          const RNode &x = s_m[s_cdm[d]];
          const PQ q = s_q[jj];
          const PairEval v = pair_eval<EXT>(q, &s_px[EXT ? jj : 0], a.clauses, x.row, &s_mx[EXT ? s_cdm[d] : 0],
                                            x.slot, s_cdp[d][0], s_cdp[d][1], s_cdn[d], a.w);
          const uint64_t key = v.key;
          if (v.lost) atomicAdd(&s_dl[jj], v.lost);
          if (EXT && v.at_lost) atomicAdd(&s_dn[EXT ? jj : 0], (v.at_lost & 1u) | (v.at_lost >> 1) << 16);
          if (s_cdr[d]) {
            // a re-taken node: its old key may be the one Rpre holds, which a
            // max cannot take back -- recompute Rpre when the pod is reached
            // (if another node's key is in Rpre already, the old one is not
            // the max and the max with the new one is exact)
            const uint64_t cur = s_rk[jj];
            if (cur != 0 && key_slot(cur) == x.slot) {
              s_dirty[jj] = 1;
              continue;
            }
          }
          if (key) atomicMax((unsigned long long *)&s_rk[jj], (unsigned long long)key);
        }
      }
    }
    __syncthreads();
    clk.tick(7);
  }

  if (bailed) {
    // Hand the whole round to the serial kernel launched behind this one
    // (RESOLVE_AUTO): nothing of it is written here, so the serial kernel
    // resolves it from its first pod, in full, and the next round's
    // speculative sweep stays valid.  It also takes the following b rounds,
    // b doubling per consecutive hand-over (rmode[2]) up to PAR_MAX_STRETCH
    // rounds (PAR_MAX_BACKOFF times serial_rounds when that is more).
    if (tid == 0) {
      const uint32_t b = max(a.rmode[2], a.serial_rounds);
      a.rmode[0] = b + 1;  // this round, then b more (resolve_kernel counts them down)
      a.rmode[2] = min(2 * b, max(PAR_MAX_STRETCH, PAR_MAX_BACKOFF * a.serial_rounds));
      a.counters[CTR_PAR_BAILS] += 1;
      a.counters[CTR_PAR_PASSES] += s_ctl[6];
    }
    clk.tick(8);
    clk.flush();
    return false;  // no completion signal: the serial commit gives it
  }

  // ---- results of the resolved pods, the modified nodes, the next round's start
  const uint32_t nres = s_ctl[0];
  {
    uint32_t *dst = (uint32_t *)((DevResult *)a.results + start);
    constexpr uint32_t RW32 = sizeof(DevResult) / 4;
    for (uint32_t i = tid; i < nres * RW32; i += PR_THREADS) {
      const uint32_t pr = i / RW32, w = i % RW32;
      const uint4 c = s_resc[pr];
      const uint64_t win = ((uint64_t)c.y << 32) | c.x;
      const int64_t total = win ? (int64_t)(win >> 32) - 1 : 0;
      uint32_t v;
      switch (w) {
        case 0: v = win ? key_slot(win) : 0xFFFFFFFFu; break;            // node_index (-1: none)
        case 1: v = c.w; break;                                           // status
        case 2: v = (uint32_t)total; break;                               // total_score
        case 3: v = (uint32_t)((uint64_t)total >> 32); break;
        case 4: v = c.z; break;                                           // feasible_nodes
        case 5: v = a.evaluated; break;                                   // evaluated_nodes
        case 6: case 7: case 8: case 9: v = s_hdr[pr].fails[w - 6]; break;  // fail_counts
        case 10: v = s_hdr[pr].fails[KS_PLUGIN_FIT_IDX] + (uint32_t)s_rdl[pr]; break;
        case 13: v = s_pfo[pr]; break;                                    // prefiltered
        case 14: v = (win && c.z == 1) ? 1u : 0u; break;                  // flags
        default: v = 0; break;                                            // spread_fail, ipa_fail, _pad
      }
      dst[i] = v;
    }
  }
  const uint32_t mn = s_ctl[5];
  for (uint32_t i = tid; i < mn; i += PR_THREADS) a.carry_out[i] = rnode_carry(s_m[i], s_mx[EXT ? i : 0], EXT);
  if (tid == 0) {
    *a.carry_out_n = mn;
    mark_pod(a.marks, start, MARK_ROUND_START);
    *a.act_next = start + nres;
    *a.d_start = start + nres;
    a.counters[0] += 1;     // rounds
    a.counters[1] += nres;  // pods resolved
    a.counters[CTR_PAR_PASSES] += s_ctl[6];
    a.counters[CTR_PAR_ROUNDS] += 1;
    if (fast) a.counters[CTR_PAR_ONESTEP] += 1;
    if (a.rmode != nullptr) {
      a.rmode[1] = a.seq;  // resolve_kernel, launched after this one, skips the round
      a.rmode[2] = 0;      // a round resolved here ends a run of hand-overs
    }
  }
  __syncthreads();
  clk.tick(8);
  clk.flush();
  if (tid == 0) signal_done(a.flag_res, a.seq, a.stall_us);
  return true;
#undef lt_mask
#undef s_q
#undef s_px
#undef s_dn
#undef s_fl
#undef s_hdr
#undef s_rep
#undef s_rk
#undef s_dl
#undef s_dirty
#undef s_lptr
#undef s_resc
#undef s_rdl
#undef s_pfo
#undef s_m
#undef s_mx
#undef s_mh
#undef s_mi
#undef s_ck
#undef s_ce
#undef s_crow
#undef s_crowx
#undef s_cnc
#undef s_cmore
#undef s_cpst
#undef s_dh
#undef s_do
#undef s_gh
#undef s_gm
#undef s_pk
#undef s_ps
#undef s_pnx
#undef s_pfst
#undef s_prow
#undef s_prowx
#undef s_ik
#undef s_idl
#undef s_idn
#undef s_cdm
#undef s_cdp
#undef s_cdn
#undef s_cdr
#undef s_ctl
#undef s_ek
#undef s_ex
#undef s_tx
#undef s_ic
#undef s_wt
#undef s_clk
}

// One launch per round on the resolve stream: the parallel commit, and the
// serial one in the same workgroup when the round is not the parallel
// commit's (RESOLVE_SERIAL, a serial stretch, a hand-over).  The two share
// one LDS allocation (a union: each is within the CU's 160 KB on its own);
// the serial commit reads nothing the parallel one wrote to LDS.
template <bool EXT, int LIST_SPAN>
__global__ __launch_bounds__(PR_THREADS) void resolve_kernel(RoundArgs a) {
  static_assert(PR_THREADS == RESOLVE_THREADS, "both commits run on one 1024-thread workgroup");
  if (resolve_parallel<EXT>(a)) return;
  __syncthreads();  // the parallel commit's last LDS reads, its hand-over writes (rmode)
  resolve_serial<EXT, LIST_SPAN>(a);
}

hipError_t launch_resolve(const RoundArgs &a, bool ext, hipStream_t st) {
  if (a.K <= (uint32_t)(RES_LIST_WAVES * LIST_SPAN_1)) {
    if (ext) resolve_kernel<true, LIST_SPAN_1><<<1, PR_THREADS, 0, st>>>(a);
    else resolve_kernel<false, LIST_SPAN_1><<<1, PR_THREADS, 0, st>>>(a);
  } else {
    if (ext) resolve_kernel<true, LIST_SPAN_2><<<1, PR_THREADS, 0, st>>>(a);
    else resolve_kernel<false, LIST_SPAN_2><<<1, PR_THREADS, 0, st>>>(a);
  }
  return hipGetLastError();
}

}  // namespace ks
