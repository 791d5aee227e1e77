// ksched_dev.hpp — device-resident formats of the shard hot path (shared by
// the HIP kernels and the host encoder).  Layout rationale: DESIGN.md §3.
#pragma once

#include <stdint.h>

namespace ks {

// ------------------------------------------------------------------ limits
constexpr int LW = 4;           // label bitset words per node (256 dictionary bits)
constexpr int NNUM = 2;         // numeric label columns (Gt / Lt operands)
constexpr int NFILT = 5;        // filter plugins of the round kernels (KS_PLUGIN_* 0..4)
constexpr int PLUGIN_SPREAD = 5;  // KS_PLUGIN_POD_TOPOLOGY_SPREAD (one-pod path only)
constexpr int PLUGIN_IPA = 6;     // KS_PLUGIN_INTER_POD_AFFINITY (one-pod path only)
constexpr int WAVE = 64;
constexpr int SWEEP_THREADS = 256;
constexpr int BLOCK_KEYS = 4;   // candidates kept per sweep block and pod
constexpr int MAX_SHARDS = 16;
constexpr int MERGE_CAP = 4096; // candidates sorted per pod by the merge kernel
constexpr uint64_t UNSCHED_BIT = 1ull << 63;  // hard-taint word: spec.unschedulable pseudo-taint

// Filter status codes (first failing plugin); FEASIBLE = passed every filter.
constexpr int ST_FEASIBLE = -1;
constexpr int ST_EMPTY = -2;
// Outside NodeAffinity's PreFilterResult: no Filter plugin runs on the node
// and no plugin is blamed (ks_result.fail_counts[KS_FAIL_PREFILTER_RESULT]).
constexpr int ST_PREFILTERED = 7;

// ---------------------------------------------------------- node table (SoA)
// Columns are indexed by POSITION, not slot: a shard's slots are permuted so
// that (wave, lane, step) of the sweep read consecutive positions (coalesced)
// while consecutive slots land in different waves (long candidate prefixes).
struct NodeTable {
  int64_t *acpu, *amem;   // Allocatable
  int64_t *rcpu, *rmem;   // Requested
  int64_t *zcpu, *zmem;   // NonZeroRequested
  int32_t *apods;         // Allocatable pods; < 0 marks an empty slot
  int32_t *npods;         // len(NodeInfo.Pods)
  uint64_t *hard;         // untolerable-effect taint bits (+ UNSCHED_BIT)
  uint64_t *prefer;       // PreferNoSchedule taint bits
  uint64_t *lab;          // [LW][npos] label-pair / key-present / numeric-valid bits
  int64_t *num;           // [NNUM][npos] parsed numeric label values
  uint32_t npos;          // positions per column
  uint32_t lw;            // label words in use (0..LW)
};

// Shard geometry.  Local index l = slot - lo; wave w = l % W;
// lane t = (l / W) % 64; step j = l / (64 W); pos = base + w*64*npl + j*64 + t.
struct Shard {
  uint32_t lo, count;   // slot range [lo, lo + count)
  uint32_t waves;       // W (multiple of 4)
  uint32_t base;        // first position
};

__host__ __device__ inline uint32_t shard_pos(const Shard &s, uint32_t npl, uint32_t l) {
  const uint32_t w = l % s.waves;
  const uint32_t t = (l / s.waves) % WAVE;
  const uint32_t j = l / (s.waves * WAVE);
  return s.base + w * WAVE * npl + j * WAVE + t;
}

// ----------------------------------------------------------------- pods
enum PodFlags : uint32_t {
  PF_HAS_REQ = 1u,    // Fit checks cpu/memory (some request is non-zero)
  PF_EXT = 2u,        // needs taint / label / name columns
  PF_TT = 4u,         // TaintToleration raw score may be non-zero (normalisation active)
  PF_NA = 8u,         // NodeAffinity preferred terms parsed (normalisation active)
  PF_HAS_PREF = 16u,  // preferredDuringScheduling != nil (NodeAffinity not skipped)
  PF_PREF_ERR = 32u,  // preferred terms failed to parse: PreScore error with >= 2 feasible
  PF_AFF = 64u,       // required program present (nodeSelector and/or required terms)
  PF_PREFILTER = 128u,   // NodeAffinity PreFilterResult: only nodes passing the prefilter program are evaluated
  PF_NA_CONFLICT = 256u, // NodeAffinity PreFilter rejects (conflicting metadata.name terms): every node fails NodeAffinity
  PF_SOLO = 512u,        // scheduled one at a time by the spread path (ksched_spread.hip): topology
                         // spread constraints, extended resources or ImageLocality; SoloHdr at solo_off
  PF_SPREAD_ALLKEYS = 1024u,  // PreScore requireAllTopologies (the pod's own constraints, not system defaults)
};

struct alignas(16) PodDev {
  int64_t req_cpu, req_mem;  // PodRequests (Fit filter, BalancedAllocation)
  int64_t nz_cpu, nz_mem;    // PodRequests with non-missing defaults (LeastAllocated)
  double req_cpu_d, req_mem_d;  // the same, exact in binary64 (< 2^46)
  double nz100_cpu, nz100_mem;  // non-zero requests x 100, exact (< 2^53)
  uint64_t tol_hard;         // hard-taint bits tolerated (+ UNSCHED_BIT)
  uint64_t tol_prefer;       // prefer-taint bits tolerated by "" / PreferNoSchedule tolerations
  uint32_t flags;
  int32_t name_slot;         // spec.nodeName: -1 unset, -2 names no node, else slot
  uint32_t req_off, req_len; // required program: word offset in the label-program buffer, terms (OR)
  uint32_t pref_off, pref_len;  // preferred program: word offset, terms (weighted sum)
  uint32_t solo_off;         // PF_SOLO: word offset of the pod's SoloHdr in the label-program buffer
  // Normalising-plugin maxima the sweep scores with (PF_TT / PF_NA): the host's
  // guess of max raw over feasible nodes.  The merge measures the true maxima;
  // pods whose guess was wrong are re-swept with them (norm_check, fix sweep).
  uint32_t tt_guess, na_guess;
  // NodeAffinity PreFilterResult (PF_PREFILTER): pre_len slot words at
  // pre_off; prefilter_out = present nodes outside it (host count)
  uint32_t pre_off, pre_len;
  uint32_t prefilter_out;
};
static_assert(sizeof(PodDev) == 128, "PodDev layout");

// Label programs.  A pod's required node affinity is an OR of TERMS and its
// preferred affinity a weighted sum of TERMS; each term is compiled on the
// host from one NodeSelectorTerm (the pod's nodeSelector merged into every
// required term), as fixed-form masks over the node's label bitset:
//   w0         n_groups | n_num << 8 | n_name << 16 | (uint64)weight << 32
//   must[LW]   bits the node must carry (In with one value, Exists, the
//              nodeSelector's pairs, the numeric-valid bit of a Gt / Lt key)
//   mf[LW]     must | forbid (NotIn values, DoesNotExist keys): the node
//              passes the pair / key requirements iff (lab & mf) == must
//   groups     n_groups x LW words (In with several values): lab & g != 0
//   num        n_num x 2 words: col | op << 8 (TO_GT / TO_LT), int64 operand
//   name       n_name x 2 words: TO_NAME_IN / TO_NAME_NOT_IN, slot
//              (matchFields metadata.name; -1 = the name is no node's)
// The PreFilterResult program (PF_PREFILTER) is a plain list of slots.
constexpr int TERM_HDR_WORDS = 1 + 2 * LW;
enum TermOp : uint32_t { TO_GT = 0, TO_LT = 1, TO_NAME_IN = 0, TO_NAME_NOT_IN = 1 };
__host__ __device__ inline uint32_t term_words(uint64_t w0) {
  const uint32_t ng = (uint32_t)w0 & 0xFF, nn = ((uint32_t)w0 >> 8) & 0xFF, nm = ((uint32_t)w0 >> 16) & 0xFF;
  return TERM_HDR_WORDS + ng * LW + 2 * (nn + nm);
}

// PodTopologySpread (ksched_spread.hip).  A pod's constraints, compiled on the
// host: the topology key's domain-id column, the selector's class column
// (matching bound pods per node), and the constraint's parameters.
constexpr int MAX_SPREAD = 8;        // constraints per pod
constexpr int MAX_TOPO_KEYS = 16;    // topology-key domain columns
constexpr int MAX_CLASSES = 128;     // selector-class count columns
constexpr int CMASK_WORDS = MAX_CLASSES / 64;  // per-pod class bitmask words
constexpr uint32_t DOM_NONE = 0xFFFFFFFFu;  // node lacks the topology key
constexpr uint32_t CLS_NONE = 0xFFFFFFFFu;  // Empty() / Nothing() selector: counts are 0
enum SpreadFlags : uint32_t {
  SP_SCORE = 1u,   // ScheduleAnyway (Score); else DoNotSchedule (Filter)
  SP_AFF = 2u,     // nodeAffinityPolicy Honor
  SP_TAINT = 4u,   // nodeTaintsPolicy Honor
  SP_SELF = 8u,    // the selector matches the incoming pod's own labels
  SP_HOST = 16u,   // topologyKey == kubernetes.io/hostname (Score counts per node)
};
struct alignas(16) SpreadDev {
  uint32_t key;        // topology-key column
  uint32_t cls;        // selector-class column or CLS_NONE
  int32_t max_skew, min_domains;
  uint32_t flags;      // SP_*
  uint32_t _pad[3];
};
static_assert(sizeof(SpreadDev) == 32, "SpreadDev layout");
constexpr uint32_t SPREAD_WORDS = sizeof(SpreadDev) / 8;

// A one-pod-path program (16-byte aligned in the label-program buffer):
//   SoloHdr, n_spread SpreadDev, n_xres XResDev, n_img ImageDev, n_aff AffDev.
struct alignas(16) SoloHdr {
  uint32_t n_spread, n_xres, n_img;
  uint32_t n_containers;  // ImageLocality: len(initContainers) + len(containers)
  uint32_t n_aff;         // InterPodAffinity records
  uint32_t aff_flags;     // AFF_SELF
  uint32_t _pad[2];
};
// InterPodAffinity (interpodaffinity/filtering.go, scoring.go): one record per
// (term, count column) the pod's cycle reads.  Counts are summed per topology
// domain of the record's key over every node (PreFilter / PreScore maps keyed
// by topology pair); the count column is a selector-class column (the incoming
// pod's terms against bound pods) or a term-class column (bound pods' terms
// that match the incoming pod: per node, the carriers of a required term, the
// summed weights of the carriers of a preferred one).
constexpr int MAX_AFF = 64;             // records per pod
constexpr int MAX_TERM_CLASSES = 1024;  // term-class columns (allocated as they are needed)
enum AffKind : uint32_t {
  AF_REQ_AFF = 0,     // required affinity term; column: pods matching ALL such terms (affinityCounts)
  AF_REQ_ANTI = 1,    // required anti-affinity term (antiAffinityCounts)
  AF_EXIST_ANTI = 2,  // a bound pod's required anti-affinity term (existingAntiAffinityCounts)
  AF_SCORE = 3,       // topologyScore: weight x count
  AF_OWN = 4,         // a term class of the pod's own terms: +weight on commit
  AF_KIND = 15u,
  AF_TERM = 16u,      // the column is a term-class column
  AF_NODE = 32u,      // every domain of the key holds one node (hostnames): the domain sum is the
                      // node's own count, read in place (no prep pass, no scattered domain sums)
};
constexpr uint32_t AFF_SELF = 1u;  // the pod matches all its required affinity terms
struct alignas(16) AffDev {
  uint32_t key;    // topology-key column
  uint32_t col;    // class column
  uint32_t kind;   // AffKind | AF_TERM
  int32_t weight;  // AF_SCORE: multiplier of the domain sum; AF_OWN: the column unit
};
// NodeResourcesFit for an extended resource (ephemeral-storage or a scalar
// resource): the pod's request and the resource's column.
constexpr int MAX_XRES = 8;
struct alignas(16) XResDev {
  uint32_t col, _pad;
  int64_t req;
};
// ImageLocality: one container image present on some node: the label bit of
// the node-side "image present" key and scaledImageScore (size x NumNodes /
// totalNumNodes, host-computed).
struct alignas(16) ImageDev {
  uint32_t bit, _pad;
  int64_t scaled;
};
constexpr int MAX_IMG = 32;  // ImageDev records per pod (containers whose image some node reports)
static_assert(sizeof(SoloHdr) == 32 && sizeof(XResDev) == 16 && sizeof(ImageDev) == 16 && sizeof(AffDev) == 16,
              "solo program layout");

// Per-pod accumulators of the spread path (reset by its commit kernel).
// Blocks add into ACC_SHARDS copies (block b -> copy b % ACC_SHARDS) and
// readers combine the copies: hundreds of blocks' atomics on ONE address
// serialise in L2 (~20 ns each: 2048 blocks cost +30 us per pass).
constexpr int SPREAD_MAX_BLOCKS = 256;
constexpr int ACC_SHARDS = 16;
struct SpreadAccShard {
  uint32_t fail[NFILT + 2];            // first failures per plugin (+ PodTopologySpread, InterPodAffinity)
  uint32_t feasible, ignored;          // feasible nodes; feasible nodes PreScore ignores
  uint32_t tt_max, na_max;             // max raw TaintToleration / NodeAffinity over feasible nodes
  uint64_t pts_min, pts_max;           // raw PodTopologySpread min / max over non-ignored feasible nodes
  uint64_t ipa_min, ipa_max;           // raw InterPodAffinity min / max over feasible nodes (biased 2^63)
  uint64_t best;                       // packed key of the winner
};
struct SpreadAcc {
  uint32_t min_match[MAX_SPREAD];      // Filter: min matching pods over eligible domains
  uint32_t ndomains[MAX_SPREAD];       // Filter: eligible domains
  uint32_t topo_size[MAX_SPREAD];      // Score: domains of non-ignored feasible nodes
  uint32_t aff_any;                    // InterPodAffinity: affinityCounts non-empty
  uint32_t score_any;                  // InterPodAffinity: topologyScore non-empty (else PreScore Skip)
  uint32_t _pad[2];
  SpreadAccShard sh[ACC_SHARDS];
};

// ----------------------------------------------------------- round records
// Per (pod-in-round, sweep block): best keys of the block + bound + counts.
struct alignas(16) BlockRec {
  uint64_t keys[BLOCK_KEYS];  // descending; 0 = none
  uint64_t bound;             // every feasible node of the block not listed has key <= bound
  uint32_t feasible;
  uint32_t fails[NFILT];
  uint32_t tt_cnt, na_cnt;    // feasible nodes whose raw normalising score equals the max used
  uint32_t tt_max, na_max;    // max raw TaintToleration / NodeAffinity score over the feasible nodes
};
static_assert(sizeof(BlockRec) == 80, "BlockRec layout");

// Per pod of a round after the merge (max over blocks and shards, then RCCL
// all-reduce(max) across ranks): the measured normalising maxima and whether
// any node is feasible.  norm_check turns it into norm_max and the fix flags.
struct PodStat {
  uint32_t tt_max, na_max, any_feasible, _pad;
};
static_assert(sizeof(PodStat) == 16, "PodStat layout");

// Per (pod-in-round, shard): sorted candidate prefix.  Stored as a fixed
// header followed by K keys (stride rec_words(K) u64).
struct alignas(16) ShardRecHdr {
  uint64_t bound;
  uint32_t nkeys;
  uint32_t feasible;
  uint32_t fails[NFILT];
  uint32_t tt_cnt, na_cnt;
  uint32_t _pad;
};
static_assert(sizeof(ShardRecHdr) == 48, "ShardRecHdr layout");
constexpr uint32_t REC_HDR_WORDS = 6;
__host__ __device__ inline uint32_t rec_words(uint32_t k) { return REC_HDR_WORDS + k; }

// S0 row of a listed candidate, gathered next to its key after the merge, in
// the form the resolve computes in: every resource quantity is an integer
// below 2^53 held as an exact binary64, so commits are exact additions and no
// int64 -> binary64 conversion sits on the resolve's per-pod critical path.
struct alignas(16) CandRow {
  double acpu, amem;        // Allocatable (< 2^44)
  double inv_cpu, inv_mem;  // RN(1 / Allocatable), 0 for a zero allocatable
  double rc, rm;            // Requested
  double zc100, zm100;      // NonZeroRequested x 100 (< 2^51)
  int32_t apods, np;
  uint32_t pos, _pad;
};
static_assert(sizeof(CandRow) == 80, "CandRow layout");
struct alignas(16) CandExt {
  uint64_t w[2 + LW + NNUM];  // hard, prefer, lab[LW], num[NNUM]
};
static_assert(sizeof(CandExt) == 64, "CandExt layout");

// A node modified by round k's resolve, handed to round k+1's patch (its sweep
// ran concurrently with round k and saw the table before round k) and to the
// write-back that lands round k in the table before sweep k+2.
struct alignas(16) CarryRec {
  int64_t acpu, amem;
  int64_t rc0, rm0;          // Requested as sweep k+1 saw it (start of round k)
  int64_t rc, rm, zc, zm;    // live state after round k
  uint32_t slot, pos;
  int32_t apods, np0, np;
  uint32_t _pad;
  uint64_t ext[2 + LW + NNUM];  // hard, prefer, label words, numeric labels (EXT batches)
};
static_assert(sizeof(CarryRec) == 160, "CarryRec layout");

// Device copy of ks_result (identical layout).
struct DevResult {
  int32_t node_index;
  int32_t status;
  int64_t total_score;
  uint32_t feasible_nodes;
  uint32_t evaluated_nodes;
  uint32_t fail_counts[NFILT];
  uint32_t spread_fail;  // ks_result.fail_counts[KS_PLUGIN_POD_TOPOLOGY_SPREAD]
  uint32_t ipa_fail;     // ks_result.fail_counts[KS_PLUGIN_INTER_POD_AFFINITY]
  uint32_t prefiltered;  // ks_result.fail_counts[KS_FAIL_PREFILTER_RESULT]
  uint32_t flags;
  uint32_t _pad;
};
static_assert(sizeof(DevResult) == 64, "DevResult layout");

struct Weights {
  int32_t fit, ba, tt, na, il;
};

}  // namespace ks
