// ksched_kernels.hpp — launch arguments and launchers of the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "ksched_dev.hpp"

namespace ks {

constexpr int MAX_PG = 64;    // pods per sweep block (LDS wave records)
constexpr int MAX_P = 256;    // pods per round (resolve stages the round in LDS)
constexpr int MAX_K = 512;    // candidates per pod record (two list entries per list-wave lane in the resolve)
constexpr uint32_t FIX_NONE = 0xFFFFFFFFu;  // fix_list tail
// device counters of the parallel commit (ksched_resolve.hip): chunk passes,
// rounds it resolved
constexpr int CTR_PAR_PASSES = 12, CTR_PAR_ROUNDS = 13, CTR_PAR_BAILS = 14, CTR_PAR_ONESTEP = 15;
// per-pod round marks (ks_batch_marks, include/ksched.h): where the round
// machinery changed course, for tests that place checks there
constexpr uint8_t MARK_FIX = 1;          // re-swept with measured normaliser maxima (FIX sweep)
constexpr uint8_t MARK_ROUND_START = 2;  // first pod of a resolved round
constexpr uint8_t MARK_AFTER_WASTE = 4;  // ... whose previous speculated round was wasted

struct RoundArgs {
  NodeTable t;
  const Shard *shards;        // geometry of every shard, device memory (global ids)
  uint32_t total_shards;      // S
  uint32_t shard0;            // first global shard handled by this launch (grid.z / grid.y)
  uint32_t npl;               // nodes per lane of the sweep kernel
  uint32_t sub;               // layout nodes-per-lane / kernel nodes-per-lane
  uint32_t P;                 // pods per round
  uint32_t pg;                // pods per sweep block
  uint32_t K;                 // candidates per pod record
  uint32_t npods;             // batch size
  uint32_t bstride;           // BlockRec stride between pods (max blocks per shard)
  uint32_t evaluated;         // present nodes (EvaluatedNodes with pct = 100)
  uint32_t lnpl;              // layout nodes per lane (positions of committed slots)
  const PodDev *pods;
  const uint64_t *clauses;
  uint32_t *d_start;          // next unresolved pod of the batch (latest, for the host)
  // Two-stage pipeline (sweep k+1 overlaps resolve k), slots indexed by round parity:
  uint32_t *sstart;           // this round's sweep start (speculative)
  const uint32_t *prev_sstart;  // previous round's sweep start
  uint32_t *act;              // this round's actual start (written by the previous resolve)
  uint32_t *act_next;         // next round's actual start (written by this resolve)
  const uint32_t *prev_act;   // previous round's actual start
  const CarryRec *carry_in;   // nodes the previous round's resolve modified (merged by the patch)
  const uint32_t *carry_in_n;
  CarryRec *carry_out;        // nodes this round's resolve modifies
  uint32_t *carry_out_n;
  uint32_t first;             // first round of a pipeline run (no previous round)
  uint32_t *norm_max;         // [P][2] max raw TaintToleration / NodeAffinity over feasible nodes (norm_check)
  double *norm_inv;           // [P][2] RN(1 / norm_max), 0 for 0 (norm_check; FIX-mode sweep)
  const double *guess_inv;    // [npods][2] RN(1 / tt_guess), RN(1 / na_guess) (host)
  PodStat *pstat;             // [P] measured maxima (merge, all shards); nullptr: no normalising pod
  uint32_t *fix_flag;         // [P] the pod's guessed maxima were wrong: re-swept in FIX mode
  uint32_t *fix_group;        // [P / MAX_PG] FIX-mode pod group g holds flagged pods (g * MAX_PG < count)
  uint32_t *fix_list;         // [P] flagged pods of the round in order, then FIX_NONE
  uint32_t fix;               // FIX-mode launch of sweep / merge
  uint32_t pstat_sweep;       // the sweep (not the merge) folds its maxima into pstat (one rank)
  uint32_t *flag_res;         // resolve: round number `seq` stored here when done (null: the host signals)
  uint32_t seq;
  uint32_t stall_us;          // ks_debug_stall: the resolve holds its signal back this long (0: never)
  // Which commit resolves a round (ksched_resolve.hip resolve_kernel runs the
  // parallel one, then the serial one in the same workgroup when needed),
  // RESOLVE_AUTO: rmode[0]: rounds left for the serial commit (the parallel
  // one steps aside while > 0); rmode[1]: seq of the last round the parallel
  // commit resolved; rmode[2]: the next serial stretch.  A round the parallel
  // commit bails on (more than par_max_passes passes, or too few pods per
  // pass) is handed whole to the serial commit, with the next rmode[2]
  // (>= serial_rounds, doubling per consecutive hand-over) rounds.
  // nullptr: RESOLVE_PARALLEL, or RESOLVE_SERIAL with serial_only set.
  uint32_t *rmode;
  uint32_t par_max_passes, serial_rounds;
  uint32_t serial_only;       // RESOLVE_SERIAL: the resolve kernel skips the parallel commit
  uint64_t *prof;             // ks_debug_set_profile: resolve_par_kernel phase cycle sums (null: off)
  uint8_t *marks;             // [npods] per-pod round marks of the batch (ks_batch_marks): KS_MARK_*
  // Identical pods (resource-only batches; null otherwise): pods of a round
  // with byte-identical descriptors have identical lists, so only the first
  // of each class in the round window is swept, merged, gathered and patched
  // and the others read its record.  cls[i]: the batch index of pod i's
  // first identical pod (host); per round (by parity), written by the
  // advance kernel: rep[r] (the window's first pod of r's class), ulist
  // (the representatives in window order) and nuniq (their count)
  const uint32_t *cls;
  uint32_t *rep, *ulist, *nuniq;
  BlockRec *brec;             // [local shards][P][bstride]
  uint64_t *srec;             // [S][P][rec_words(K)]
  uint64_t *frec;             // [P][rec_words(K)] (== srec when S == 1)
  void *results;              // DevResult[npods]
  CandRow *crow;              // [P][K] S0 rows of the final candidates
  CandExt *cext;              // [P][K] their label / taint columns (EXT batches)
  const uint32_t *slot_pos;   // slot -> position
  uint64_t *counters;         // [0] rounds, [1] pods resolved, [2] pods swept, [3] wasted rounds,
                              // [4] FIX re-swept pods, [7] identical pods not swept (their class's
                              // representative was; [2] counts representatives), [CTR_PAR_*]
  Weights w;
};

struct DumpArgs {
  NodeTable t;
  const uint32_t *slot_pos;   // position of each slot
  uint32_t nslots;
  const PodDev *pods;         // one pod
  const uint64_t *clauses;
  uint32_t *norm_max;         // [2], zeroed
  int32_t *out;               // [nslots][10]
  Weights w;
};

// PodTopologySpread path (ksched_spread.hip): one pod per launch chain.
constexpr uint32_t SLOT_NONE = 0xFFFFFFFFu;  // position holding no slot (shard padding)
// status, la, ba, tt raw/score, na raw/score, il, pts raw/score, total lo/hi, ipa raw/score
constexpr int SPREAD_DUMP_WORDS = 14;
// launch_spread_pod passes: prep (PodTopologySpread DoNotSchedule counts,
// InterPodAffinity domain counts), min (criticalPaths), score (ScheduleAnyway)
enum SpreadLaunch : uint32_t { SPL_PREP = 1u, SPL_MIN = 2u, SPL_SCORE = 4u, SPL_AFF = 8u /* InterPodAffinity records */ };
struct SpreadArgs {
  NodeTable t;
  const uint32_t *pos_slot;   // position -> slot (SLOT_NONE: padding)
  const uint32_t *slot_pos;   // slot -> position
  uint32_t npos;
  uint32_t pod;               // index of the pod in the batch
  const PodDev *pods;
  const uint64_t *clauses;    // label programs + SpreadDev records
  const uint64_t *cmask;      // [npods][CMASK_WORDS] selector classes each pod of the batch matches
  const uint32_t *dom;        // [MAX_TOPO_KEYS][npos] domain id per position (DOM_NONE: key absent)
  uint32_t *cnt;              // [MAX_CLASSES][npos] matching bound pods per position
  int64_t *xalloc, *xreq;     // [MAX_XRES][npos] extended resources: Allocatable, Requested
  uint32_t *dcnt;             // [MAX_SPREAD][dom_cap] per-constraint domain counts (zero between pods)
  uint32_t *dflag;            // [MAX_SPREAD][dom_cap] bit 0 Filter-eligible domain, bit 1 Score domain
  uint32_t *tcnt;             // [MAX_TERM_CLASSES][npos] bound pods carrying each term class
  uint32_t *adcnt;            // [MAX_AFF][dom_cap] InterPodAffinity domain counts per record (zero between pods)
  int64_t *ipa_raw;           // [npos] InterPodAffinity raw score (filter -> select)
  uint32_t dom_cap;
  uint32_t ndom[MAX_TOPO_KEYS];  // domain ids of every topology-key column (at launch)
  SpreadAcc *acc;
  int8_t *st;                 // [npos] status of every position for this pod
  int64_t *raw;               // [npos] PodTopologySpread raw score
  uint64_t *part;             // [npos] normalisation-free score parts of feasible nodes (filter -> select)
  DevResult *results;
  int32_t *dump;              // ks_plugin_scores: [slots][SPREAD_DUMP_WORDS] (null: schedule)
  uint32_t no_commit;         // dump / reset: no result, no AssumePod
  uint64_t *counters;
  Weights w;
  int32_t w_pts, w_ipa;
  uint32_t evaluated;         // present nodes
  // percentageOfNodesToScore < 100 (ksched_spread.hip spread_window_kernel):
  // win_mode 0 off, 1 the probe filter pass (writes win_st only), 2 the
  // filter pass over the window; win_st [nslots] bit 0 in the node list, bit 1
  // feasible; win [WIN_WORDS] 0 nextStartNodeIndex, 1 the window's first slot,
  // 2 its end slot (exclusive, round the list), 3 every node visited, then
  // [2 per 4096-slot chunk] the chunk's list / feasible counts
  uint32_t *win;
  uint8_t *win_st;
  uint32_t nslots;
  uint32_t win_mode;
  int32_t pct;
};
constexpr uint32_t WIN_WORDS = 4;

// Replica runs (ksched_spread.hip): consecutive identical pods
// whose constraints are ScheduleAnyway (at most one kubernetes.io/hostname and
// one other key; the other may be DoNotSchedule), scheduled by one workgroup
// after one filter pass.  Sort
// key of a feasible node, at its slot: group code (ignored << 19 | domain << 8
// | own hostname count) << s_bits | (2^s_bits - 1 - static score).
constexpr uint32_t RUN_GROUPS = 512;    // groups a run can hold (more: the run is refused)
constexpr uint32_t RUN_TOUCHED = 512;   // distinct nodes one run may take (then it ends)
constexpr uint32_t RUN_MIN_PODS = 4;    // shorter sequences take the per-pod chain
constexpr uint32_t RK_HK_NONE = 255;    // the node lacks the hostname key (counts 0..254)
constexpr uint32_t RK_DZ_NONE = 2047;   // the node lacks the other key (domain ids 0..2046)
constexpr uint32_t RK_IGN = 1u << 19;   // PreScore ignores the node (requireAllTopologies)
// The sort runs over 20 + s_bits bits and an infeasible node's key is ~0 there
// (code 0xFFFFF).  Every feasible code keeps bit 19 clear and the ignored code
// keeps bits 0..18 clear, so no feasible or ignored key equals it, whatever the
// static score (2^s_bits - 1 - S with S = 0 included).
static_assert((RK_DZ_NONE << 8 | RK_HK_NONE) < RK_IGN && (RK_IGN | 0x7FFFFu) == 0xFFFFFu &&
                  RK_IGN != 0xFFFFFu,
              "replica sort keys: feasible / ignored codes stay below the infeasible code");
enum RunStop : uint32_t { RUN_END = 0, RUN_FIT = 1, RUN_FULL = 2, RUN_REFUSED = 3 };
constexpr uint32_t RUN_CTL_WORDS = 8;
struct ReplicaArgs {
  uint64_t *keys, *sorted;  // [npos] sort keys, sorted
  uint64_t *val, *sval;     // [nslots] slot << 32 | position of each key, sorted with the keys
  uint32_t *gstart;         // [RUN_GROUPS] first sorted index of each group (unordered)
  uint32_t *ctl;            // [RUN_CTL_WORDS] 0 groups, 1 refuse (a hostname count beyond RK_HK_NONE - 1, an
                            // ignored candidate of a DoNotSchedule run), 2 next pod, 3 RunStop, 4 candidates
                            // only the skew check rejected (DoNotSchedule runs)
  uint32_t end;             // one past the run's last pod
  uint32_t nslots;          // keys sorted (one per slot)
  uint32_t s_bits;          // bits of the static score (2^s_bits > 100 x the static plugins' weights)
  uint64_t *prof;           // KS_RUN_PROFILE: [0..2] cycles of the pod loop's phases, [3] pods (null: off)
};

hipError_t launch_spread_pod(const SpreadArgs &a, uint32_t passes, hipStream_t st);
hipError_t launch_spread_reset(const SpreadArgs &a, hipStream_t st);
// [prep + min passes (passes: SPL_PREP / SPL_MIN, a DoNotSchedule
// constraint)], the filter pass for a.pod, keys, sort, groups, the run
// kernel; ctl zeroed first
hipError_t launch_replica_run(const SpreadArgs &a, const ReplicaArgs &r, void *sort_tmp, size_t sort_tmp_bytes,
                              uint32_t passes, hipStream_t st);
hipError_t launch_sort_pairs(const uint64_t *kin, uint64_t *kout, const uint64_t *vin, uint64_t *vout, uint32_t n,
                             uint32_t end_bit, void *tmp, size_t *tmp_bytes, hipStream_t st);
hipError_t launch_class_commit(const DevResult *res, const uint64_t *cmask, const uint32_t *slot_pos, uint32_t *cnt,
                               uint32_t npos, uint32_t lo, uint32_t hi, hipStream_t st);
hipError_t launch_scatter_u32(uint32_t *col, const uint64_t *idx, const uint32_t *val, uint32_t n, hipStream_t st);
hipError_t launch_add_u32(uint32_t *col, const uint64_t *idx, const int32_t *delta, uint32_t n, hipStream_t st);
hipError_t launch_umax_u32(uint32_t *dst, const uint32_t *src, uint32_t n, hipStream_t st);
hipError_t launch_scatter_i64(int64_t *col, const uint64_t *idx, const int64_t *val, uint32_t n, bool add,
                              hipStream_t st);

hipError_t launch_norm_check(const RoundArgs &a, hipStream_t st);
hipError_t launch_sweep(const RoundArgs &a, bool ext, uint32_t nblocks, uint32_t ngroups, uint32_t nshards,
                        hipStream_t st);
hipError_t launch_merge(const RoundArgs &a, uint32_t nshards, hipStream_t st);
hipError_t launch_merge_shards(const RoundArgs &a, hipStream_t st);
hipError_t launch_gather_cand(const RoundArgs &a, bool ext, hipStream_t st);
hipError_t launch_patch(const RoundArgs &a, bool ext, hipStream_t st);
hipError_t launch_resolve(const RoundArgs &a, bool ext, hipStream_t st);
hipError_t launch_advance(const RoundArgs &a, hipStream_t st);
hipError_t launch_advance_writeback(const RoundArgs &a, const CarryRec *carry, const uint32_t *n, hipStream_t st);
hipError_t launch_writeback(const NodeTable &t, const CarryRec *carry, const uint32_t *n, hipStream_t st);
hipError_t launch_scatter_rows(const NodeTable &t, const uint32_t *pos, const int64_t *core, const uint64_t *ext,
                               uint32_t n, uint32_t flags, hipStream_t st);
hipError_t launch_apply_deltas(const NodeTable &t, const uint32_t *pos, const int64_t *delta, uint32_t n,
                               hipStream_t st);
hipError_t launch_gather_rows(const NodeTable &t, const uint32_t *pos, int64_t *out, uint32_t n, hipStream_t st);
hipError_t launch_scatter_u64(uint64_t *col, const uint32_t *pos, const uint64_t *val, uint32_t n,
                              hipStream_t st);
hipError_t launch_dump(const DumpArgs &a, hipStream_t st);
// ks_debug_stall: one wave that waits `usec` microseconds of wall clock, then exits
hipError_t launch_stall(uint32_t usec, hipStream_t st);

}  // namespace ks
