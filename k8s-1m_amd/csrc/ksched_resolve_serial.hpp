// ksched_resolve_serial.hpp — the serial in-order commit (one barrier per
// pod) of a round, as a device function over its own LDS struct: the resolve
// kernel (ksched_resolve.hip) runs it for rounds the parallel commit does not
// take (RESOLVE_SERIAL, AUTO hand-overs and serial stretches), in a union with
// the parallel commit's LDS.
#pragma once

#include <hip/hip_runtime.h>

#include <utility>

#include "ksched_dev.hpp"
#include "ksched_eval.hpp"
#include "ksched_instr.hpp"
#include "ksched_kernels.hpp"
#include "ksched_util.hpp"

namespace ks {

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


// The serial kernel's LDS, a member of the resolve kernel's LDS union
template <bool EXT, int LIST_SPAN>
struct SerialLds {
  PodDev s_pod[MAX_P];
  ShardRecHdr s_hdr[MAX_P];
  uint32_t s_rep[MAX_P];  // record of each pod (an identical pod's: RoundArgs::rep)
  uint32_t s_norm[MAX_P][2];
  uint32_t s_hkey[RHASH];  // slots modified this round (+1), linear probing
  CandExt s_modx[EXT ? MAX_P : 1];  // label / taint words of the modified nodes
  // owner waves' partials for pod i (written in iteration i-1), by parity of i
  RNode s_ocand[2][NCAND_OWN];   // best two nodes per wave
  CandExt s_ocandx[EXT ? 2 : 1][EXT ? NCAND_OWN : 1];
  uint64_t s_okey[2][NCAND_OWN];  // their keys for pod i, 0 = none
  uint32_t s_oidx[2][NCAND_OWN];  // their owner indices
  alignas(16) int32_t s_dsum[2][RES_OWN_WAVES][NFILT + 3];
  // list staging (LDS-DMA targets): listed keys by pod mod KSLOTS; the chosen
  // rows by pod mod RSLOTS as [list wave][16-byte piece][candidate]
  uint64_t s_keys[KSLOTS][MAX_K];
  uint4 s_lrowb[RSLOTS][RES_LIST_WAVES][ROW_PIECES + (EXT ? EXT_PIECES : 0)][LSEL];
  // list waves' candidates for pod i (chosen in iteration i - LAHEAD), by i mod RSLOTS
  uint64_t s_lkey[RSLOTS][NCAND_LIST];
  uint32_t s_lidx[RSLOTS][NCAND_LIST];  // list index, NONE32 = none
  // eval wave: each candidate of pod i committed, its key / status change for pod i+1 (by parity of i)
  RNode s_post[2][NCAND];
  CandExt s_postx[EXT ? 2 : 1][EXT ? NCAND : 1];
  uint64_t s_ekey[2][NCAND];
  alignas(16) int32_t s_edd[2][NCAND][NFILT + 3];
  // decider -> everyone: pod i's commit {valid, candidate lane, joins, owner index}
  alignas(16) uint32_t s_pend[2][4];
  // s_done[b]: set by the decider in an iteration of parity b, read by every
  // wave after that iteration's barrier.  Double-buffered: a single word let
  // the decider's next-iteration store (r == nround: immediately after the
  // barrier) overtake a slow wave's read of this iteration, which then left
  // the loop one barrier early
  uint32_t s_done[2], s_stop_at;
  // results of the round, written out after the loop (no global stores inside it)
  // per pod: {winning key lo, hi, feasible nodes, status} (one 16-B store by
  // the decider) and the failure counts (lanes of the decider); expanded into
  // DevResults after the loop
  uint4 s_resc[MAX_P];
  uint32_t s_rfail[MAX_P][NFILT];
};

// the serial commit's view of the resolve kernel's LDS buffer (ksched_resolve.hip)
template <bool EXT, int LIST_SPAN>
__device__ __forceinline__ SerialLds<EXT, LIST_SPAN> *ser_lds();

template <bool EXT, int LIST_SPAN>
__device__ __forceinline__ void resolve_serial(const RoundArgs &a) {
  constexpr bool TWO = LIST_SPAN == 2 * WAVE;
#define s_pod (ser_lds<EXT, LIST_SPAN>()->s_pod)
#define s_hdr (ser_lds<EXT, LIST_SPAN>()->s_hdr)
#define s_rep (ser_lds<EXT, LIST_SPAN>()->s_rep)
#define s_norm (ser_lds<EXT, LIST_SPAN>()->s_norm)
#define s_hkey (ser_lds<EXT, LIST_SPAN>()->s_hkey)
#define s_modx (ser_lds<EXT, LIST_SPAN>()->s_modx)
#define s_ocand (ser_lds<EXT, LIST_SPAN>()->s_ocand)
#define s_ocandx (ser_lds<EXT, LIST_SPAN>()->s_ocandx)
#define s_okey (ser_lds<EXT, LIST_SPAN>()->s_okey)
#define s_oidx (ser_lds<EXT, LIST_SPAN>()->s_oidx)
#define s_dsum (ser_lds<EXT, LIST_SPAN>()->s_dsum)
#define s_keys (ser_lds<EXT, LIST_SPAN>()->s_keys)
#define s_lrowb (ser_lds<EXT, LIST_SPAN>()->s_lrowb)
#define s_lkey (ser_lds<EXT, LIST_SPAN>()->s_lkey)
#define s_lidx (ser_lds<EXT, LIST_SPAN>()->s_lidx)
#define s_post (ser_lds<EXT, LIST_SPAN>()->s_post)
#define s_postx (ser_lds<EXT, LIST_SPAN>()->s_postx)
#define s_ekey (ser_lds<EXT, LIST_SPAN>()->s_ekey)
#define s_edd (ser_lds<EXT, LIST_SPAN>()->s_edd)
#define s_pend (ser_lds<EXT, LIST_SPAN>()->s_pend)
#define s_done (ser_lds<EXT, LIST_SPAN>()->s_done)
#define s_stop_at (ser_lds<EXT, LIST_SPAN>()->s_stop_at)
#define s_resc (ser_lds<EXT, LIST_SPAN>()->s_resc)
#define s_rfail (ser_lds<EXT, LIST_SPAN>()->s_rfail)

  // tid: hardware thread (staging loops); wid / rtid: the wave's role and the
  // thread's index in role order (list entry, owned node)
  const uint32_t tid = threadIdx.x, lane = tid % WAVE;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(res_role(tid / WAVE)), rtid = wid * WAVE + lane;
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
#undef s_pod
#undef s_hdr
#undef s_rep
#undef s_norm
#undef s_hkey
#undef s_modx
#undef s_ocand
#undef s_ocandx
#undef s_okey
#undef s_oidx
#undef s_dsum
#undef s_keys
#undef s_lrowb
#undef s_lkey
#undef s_lidx
#undef s_post
#undef s_postx
#undef s_ekey
#undef s_edd
#undef s_pend
#undef s_done
#undef s_stop_at
#undef s_resc
#undef s_rfail
}

}  // namespace ks
