// ksched_host.cpp — libksched C ABI (include/ksched.h): node cache encoder,
// pod compiler, device-driven scheduling rounds, RCCL candidate gather.
//
// The encoder turns k8s-shaped nodes into the SoA node table of
// ksched_dev.hpp (labels / taints as dictionary bitsets), and k8s-shaped pods
// into PodDev descriptors + label-selector clauses.  Upstream semantics it
// restates (k8s.io/kubernetes v1.31.3 unless noted):
//   pkg/api/v1/resource/helpers.go#PodRequests           (pod requests, A2)
//   framework/types.go#calculateResource                  (AddPod / RemovePod)
//   k8s.io/api core/v1/toleration.go#ToleratesTaint       (taint masks, A8)
//   component-helpers nodeaffinity.go#newNodeSelectorTerm (clauses, A9/A15)
//   apimachinery labels.NewRequirement validation         (parse errors)
#include <atomic>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <thread>
#include <memory>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "ksched.h"
#include "ksched_dev.hpp"
#include "ksched_kernels.hpp"
#include "ksched_sync.hpp"

using namespace ks;

namespace {

constexpr int64_t kDefaultMilliCPURequest = 100;             // schedutil.DefaultMilliCPURequest
constexpr int64_t kDefaultMemoryRequest = 200ll * 1024 * 1024;  // schedutil.DefaultMemoryRequest
constexpr int64_t kMaxExact = 1ll << 46;  // pod request bound: exact binary64 sums
constexpr int64_t kMaxAlloc = 1ll << 44;  // node allocatable bound: exact truncated LeastAllocated

std::string str(const char *p) { return p ? std::string(p) : std::string(); }

// ------------------------------------------------- apimachinery validation
// Character classes of qualifiedNameFmt / labelValueFmt / DNS-1123 subdomain.
enum : uint8_t { C_ALNUM = 1, C_LOWER_ALNUM = 2, C_DASH = 4, C_UNDERSCORE_DOT = 8 };
struct CharTable {
  uint8_t c[256] = {};
  CharTable() {
    for (int i = 'a'; i <= 'z'; ++i) c[i] = C_ALNUM | C_LOWER_ALNUM;
    for (int i = 'A'; i <= 'Z'; ++i) c[i] = C_ALNUM;
    for (int i = '0'; i <= '9'; ++i) c[i] = C_ALNUM | C_LOWER_ALNUM;
    c[(int)'-'] = C_DASH;
    c[(int)'_'] = C_UNDERSCORE_DOT;
    c[(int)'.'] = C_UNDERSCORE_DOT;
  }
};
const CharTable kChars;
inline uint8_t cls(char ch) { return kChars.c[(uint8_t)ch]; }

// "([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]", non-empty
bool name_part_ok(const std::string &s) {
  if (s.empty() || !(cls(s.front()) & C_ALNUM) || !(cls(s.back()) & C_ALNUM)) return false;
  return std::all_of(s.begin(), s.end(), [](char ch) { return cls(ch) != 0; });
}

bool dns1123_subdomain_ok(const std::string &s) {
  if (s.empty() || s.size() > 253) return false;
  size_t b = 0;
  for (;;) {
    const size_t e = s.find('.', b);
    const size_t len = (e == std::string::npos ? s.size() : e) - b;
    if (len == 0) return false;
    if (!(cls(s[b]) & C_LOWER_ALNUM) || !(cls(s[b + len - 1]) & C_LOWER_ALNUM)) return false;
    for (size_t i = b; i < b + len; ++i)
      if (!(cls(s[i]) & (C_LOWER_ALNUM | C_DASH))) return false;
    if (e == std::string::npos) return true;
    b = e + 1;
  }
}

bool qualified_name_ok(const std::string &k) {  // validation.IsQualifiedName
  const size_t slash = k.find('/');
  if (slash == std::string::npos) return k.size() <= 63 && name_part_ok(k);
  if (k.find('/', slash + 1) != std::string::npos) return false;
  const std::string prefix = k.substr(0, slash), name = k.substr(slash + 1);
  return dns1123_subdomain_ok(prefix) && name.size() <= 63 && name_part_ok(name);
}

bool label_value_ok(const std::string &v) {  // validation.IsValidLabelValue
  return v.size() <= 63 && (v.empty() || name_part_ok(v));
}

bool parse_int64(const std::string &s, int64_t *out) {  // strconv.ParseInt(s, 10, 64)
  size_t i = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '+' || s[0] == '-')) { neg = s[0] == '-'; i = 1; }
  if (i == s.size()) return false;
  uint64_t v = 0;
  const uint64_t lim = neg ? (1ull << 63) : (uint64_t)INT64_MAX;
  for (; i < s.size(); ++i) {
    const unsigned d = (unsigned)(s[i] - '0');
    if (d > 9) return false;
    if (v > (lim - d) / 10) return false;
    v = v * 10 + d;
  }
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}

// imagelocality#normalizedImageName: a name without a tag gets ":latest".
std::string normalized_image(const char *p) {
  std::string n = str(p);
  const size_t colon = n.rfind(':'), slash = n.rfind('/');
  const long lc = colon == std::string::npos ? -1 : (long)colon, ls = slash == std::string::npos ? -1 : (long)slash;
  if (lc <= ls) n += ":latest";
  return n;
}

const char *unmodelled_name(uint32_t bits) {
  if (bits & KS_UNMODELLED_HOST_PORTS) return "host ports (NodePorts)";
  if (bits & KS_UNMODELLED_TOPOLOGY_SPREAD) return "topology spread constraints (PodTopologySpread)";
  if (bits & KS_UNMODELLED_POD_AFFINITY) return "pod (anti-)affinity (InterPodAffinity)";
  if (bits & KS_UNMODELLED_VOLUMES) return "volumes (VolumeBinding / VolumeRestrictions / VolumeZone / NodeVolumeLimits)";
  if (bits & KS_UNMODELLED_NOMINATED_NODE) return "a nominated node";
  if (bits & KS_UNMODELLED_RESOURCE_CLAIMS) return "resource claims (DynamicResources)";
  return "an unknown feature bit";
}

// ------------------------------------------------------------ host types

struct Tol {
  uint32_t key;  // string id; 0 = ""
  uint32_t value;
  int32_t op, effect;
};

struct HostNode {
  bool present = false;
  uint32_t name = 0;
  int64_t acpu = 0, amem = 0, apods = 0;
  bool unschedulable = false;
  std::vector<std::pair<uint32_t, uint32_t>> labels;  // (key id, value id)
  uint64_t hard = 0, prefer = 0;
  uint64_t lab[LW] = {};
  int64_t num[NNUM] = {};
  std::vector<std::pair<std::string, int64_t>> images;  // status.images names (as reported) and sizes
  // taints as interned ids (the taint dictionaries are rebuilt from these)
  std::vector<std::array<uint32_t, 3>> hard_taints;            // key, value, effect
  std::vector<std::pair<uint32_t, uint32_t>> prefer_taints;    // key, value
  // NodeInfo.Pods as interned (namespace, labels) sets, one entry per bound pod
  // (PodTopologySpread counts them through selector classes)
  std::vector<uint32_t> pod_sets;
};

// PodTopologySpread host state.  A bound pod's (namespace, labels) is interned
// as a label set; a spread constraint's (namespace, selector) is a selector
// CLASS with a device column of matching bound pods per node; a topology key
// has a device column of per-node domain ids (value -> id, "" = 0).
struct LabelSet {
  uint32_t ns;
  std::vector<std::pair<uint32_t, uint32_t>> labels;     // sorted (key id, value id)
  std::vector<std::pair<uint32_t, uint32_t>> ns_labels;  // the namespace's labels, sorted
  // InterPodAffinity term classes of the pod's own terms, with the unit the
  // pod adds to the class column (the weight of a preferred term, else 1)
  std::vector<std::pair<uint32_t, uint32_t>> terms;
  std::string key;              // set_of_key entry (sets with namespace labels or terms)
  bool ever_bound = false;      // some node's pod records held it (never cleared: class creation's shortcut)
};
struct SelReq {
  uint32_t key;
  int32_t op;                   // KS_OP_IN / NOT_IN / EXISTS / DOES_NOT_EXIST
  std::vector<uint32_t> vals;   // sorted value ids
};
// One conjunct of a pod matcher (framework.AffinityTerm.Matches): the pod's
// namespace listed or selected by the namespace selector, and its labels
// selected.  A spread constraint's selector is {own namespace, selector}.
struct Clause {
  std::vector<uint32_t> nss;    // sorted namespace ids
  bool ns_sel_set = false;      // namespaceSelector set (else Nothing())
  std::vector<SelReq> ns_sel;
  bool sel_nothing = false;     // labelSelector nil: matches no pod
  std::vector<SelReq> sel;
};
struct SpreadClass {
  bool live = false;
  std::vector<Clause> clauses;  // all must match
  std::string canon;
  uint32_t refs = 0;            // prepared batches using the class
  uint64_t last_use = 0;
  uint64_t born = 0;            // class_epoch at creation (batches whose cmask predates it: run_batch adds their pods)
  uint64_t held = 0;            // last run whose cmask holds the class (its commits count it): no reuse before it ends
};
// A pod (anti-)affinity term some bound pod carries (InterPodAffinity's
// existing-pod side): device column = bound pods carrying it, per node
// (MAX_TERM_CLASSES columns, ksched_dev.hpp).
struct TermClass {
  bool live = false;
  int32_t kind = 0;
  uint32_t key = 0;             // topology key id
  Clause clause;
  std::string canon;
  int64_t bound = 0;            // bound pods carrying the term (the column's sum)
  uint32_t refs = 0;            // prepared batches holding pods that carry it
  // pods matching the term take the one-pod path while some bound or
  // prepared pod carries it
  bool active() const { return live && (bound > 0 || refs > 0); }
};
struct TopoKey {
  uint32_t key = 0;
  std::unordered_map<uint32_t, uint32_t> dom;  // value id -> domain id ("" -> 0)
  uint32_t ndom = 1;
  // nodes per domain: while no domain holds two nodes (hostnames), a domain
  // sum is the node's own count (InterPodAffinity's per-node records, AF_NODE)
  std::vector<uint32_t> slot_dom;   // [cap] domain of each slot (DOM_NONE: absent / no key)
  std::vector<uint32_t> dom_nodes;  // [ndom]
  uint32_t shared = 0;              // domains holding two or more nodes
  void place(uint32_t slot, uint32_t d) {
    const uint32_t o = slot_dom[slot];
    if (o == d) return;
    if (o != DOM_NONE && --dom_nodes[o] == 1) --shared;
    if (d != DOM_NONE) {
      if (d >= dom_nodes.size()) dom_nodes.resize((size_t)d + 1, 0);
      if (++dom_nodes[d] == 2) ++shared;
    }
    slot_dom[slot] = d;
  }
};

struct TaintKey {
  uint32_t key, value;
  int32_t effect;
  bool operator<(const TaintKey &o) const {
    return std::tie(key, value, effect) < std::tie(o.key, o.value, o.effect);
  }
};

struct NumCol {
  uint32_t col;
  uint32_t valid_bit;
};

}  // namespace

// ================================================================= context

struct ks_batch {
  uint32_t n = 0;
  uint64_t cmask_epoch = 0;  // class_epoch when the run took the pods' class masks
  uint64_t run_seq = 0;
  uint32_t dict_version = 0;
  uint32_t names_version = 0;  // 0: no pod of the batch resolved a node name
  bool ext = false, norm = false;
  // pooled device buffers (capacities in pods / clause words) and the pinned
  // host copy of the results, filled at the end of the run
  uint32_t cap_pods = 0;
  size_t cap_words = 0;
  PodDev *d_pods = nullptr;
  double *d_pinv = nullptr;  // [n][2] reciprocals of the normalising guesses
  uint64_t *d_clauses = nullptr;
  DevResult *d_results = nullptr;
  DevResult *h_results = nullptr;
  // pinned host copies of the compiled batch: uploaded by ks_batch_prepare
  // when nothing is in flight, else by the run itself (uploaded = false)
  PodDev *h_pods = nullptr;
  double *h_pinv = nullptr;
  uint64_t *h_clauses = nullptr;
  size_t n_words = 0;
  bool uploaded = false;
  // PodTopologySpread: per-pod label-set ids (bound pods are recorded at the
  // end of the run), spread-path flags (1 spread pod, 2 DoNotSchedule
  // constraints, 4 ScheduleAnyway constraints), the selector classes the
  // batch references, and the pods' class masks (computed at run time)
  std::vector<uint32_t> set_ids;
  std::vector<uint8_t> spread;
  bool any_spread = false;
  // replica runs: 1 the run kernel models the pod's program,
  // 2 the pod is identical to the one before it (program, labels)
  std::vector<uint8_t> rep;
  std::vector<uint32_t> class_refs;
  std::vector<uint32_t> term_refs;  // term classes of the batch's pods' own terms (one per pod and term)
  uint64_t *d_cmask = nullptr, *h_cmask = nullptr;
  uint8_t *d_marks = nullptr;  // [cap_pods rounded to 4] round marks (ks_batch_marks)
  // identical pods (RoundArgs::cls): per pod the batch index of its first
  // byte-identical descriptor; dups = some pod repeats an earlier one
  uint32_t *d_cls = nullptr, *h_cls = nullptr;
  bool dups = false;
  // asynchronous run state (ks_batch_submit / ks_batch_wait)
  bool queued = false, done = false;
  ks_status run_status = KS_OK;
  std::string run_err;
};

// In-process communicator (ks_comm_init_local): the ranks are contexts of one
// process -- on one device or several -- each driven by its own host thread.
// A collective is a host rendezvous exchanging (event, device pointer) pairs,
// device-to-device copies ordered by stream waits on the peers' events, and a
// second rendezvous whose events hold every rank's stream until all peers have
// read its buffers: the ordering an RCCL collective gives, without RCCL (which
// refuses two ranks on one GPU).  Test plumbing for the multi-rank path.
struct LgPost {
  hipEvent_t ev = nullptr;
  const void *ptr = nullptr;
  std::vector<double> vals;
};
// (the rendezvous itself: ksched_sync.hpp, exercised under TSan / ASan by
// tools/sync_stress.cpp)
struct LocalGroup : Rendezvous<LgPost> {
  using Post = LgPost;
  explicit LocalGroup(uint32_t n) : Rendezvous<LgPost>(n) {}
};

struct ks_ctx {
  ks_config cfg{};
  std::string err;
  hipStream_t stream = nullptr;   // table updates, prescore / sweep / merge / gather, RCCL
  hipStream_t rstream = nullptr;  // resolve (overlaps the next round's sweep)
  hipStream_t sstream = nullptr;  // merge .. patch (overlap the next round's sweep)
  hipEvent_t ev_sw[2] = {nullptr, nullptr}, ev_res[2] = {nullptr, nullptr};  // by round parity
  hipEvent_t ev_swept[2] = {nullptr, nullptr}, ev_fixed[2] = {nullptr, nullptr};
  // cross-stream hand-offs as stream memory operations (write / wait-value on
  // monotone round numbers): [0] swept, [1] side done, [2] resolved, [3] fixed
  uint32_t *d_flags = nullptr;
  uint32_t round_seq = 0;         // rounds enqueued since open
  uint32_t seq_of[2] = {0, 0};    // round number by parity
  bool value_sync = true;
  // Device-stall guard (sync_bounded): every host wait on a stream is bounded;
  // a miss wedges the context.  flag_want[f]: the last round number enqueued
  // to be signalled on hand-off flag f (what a finished stream leaves there)
  uint32_t sync_timeout_ms = 60000;
  // set by the worker thread's drains (sync_bounded), read by API threads
  std::atomic<bool> wedged{false};
  // stall_report's read-back stream: created by the first report, not at
  // ks_open.  A fourth stream alive beside main / side / resolve cost the
  // round pipeline 37 % (C3, serial resolve: 640k -> 400k pods/s,
  // profiles/r4/bench_r4q_*.json; the streams then share hardware queues)
  hipStream_t diag_stream = nullptr;
  uint32_t flag_want[4] = {0, 0, 0, 0};
  uint32_t *h_diag = nullptr;  // pinned: flags read back by the stall report
  // ks_debug_stall: the next round holds back flag stall_flag's signal by stall_us
  int32_t stall_flag = -1;
  uint32_t stall_us = 0;
  // Execution options from ks_config (ks_open), per context, so one process
  // can open contexts with different settings (tests do).
  bool early_fix = true;
  // resolve kernel of resource-only rounds (ksched_resolve.hip): KS_RESOLVE_AUTO
  // launches the parallel commit with the serial kernel behind it as its
  // fallback (RoundArgs::rmode, the two words at d_flags + 4)
  uint32_t resolve_mode = KS_RESOLVE_AUTO;
  uint32_t par_max_passes = 32, serial_rounds = 4;
  bool res_profile = false;  // ks_debug_set_profile: phase clocks of the parallel commit
  bool dedup = true;        // dedup_identical_pods: sweep identical pods of a round once
  bool tuple_guess = true;  // normaliser guesses over node tuples (refine_guesses)
  uint32_t timing_every = 8, ext_npl = 2;
  // (block, pod group) pairs a sweep aims for: resource-only sweeps 4096
  // (bigger pod groups amortise each block's row loads: C3 sweep 0.365 ->
  // 0.356 ms, profiles/r3/sweep_blocks_ab/), label / taint sweeps 16384
  // (C4 sweep 1.117 -> 1.102 ms; 4096 measured 2 % slower than 8192, 32768
  // no better: profiles/r3/sweep_blocks_ab/c4_*): sweep_pairs / sweep_pairs_ext
  uint32_t sweep_blocks = 4096, sweep_blocks_ext = 16384;
  // KS_EVENT_PROFILE=1: per event kind, runs / events / seconds of ks_events_apply (stderr at ks_close)
  bool ev_profile = false;
  // KS_RUN_PROFILE=1: seconds per phase of the batch runs (stderr at ks_close):
  // [0] waiting for `mu` at run start, [1] enqueueing rounds, [2] drains, [3] runs,
  // [4] worker runs' wall time, [5] worker idle between submitted runs, [6] worker runs
  bool run_profile = false;
  double prof[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // [7..9] ks_batch_prepare: drain wait, compile, rest
  struct EvProf {
    uint64_t runs = 0, events = 0;
    double s = 0;
  } ev_prof[4];
  // geometry
  uint32_t cap = 0, S = 1, npl = 8, P = 256, K = 256;
  std::vector<Shard> shards;
  uint32_t npos = 0;
  std::vector<uint32_t> slot_pos;
  // device state
  NodeTable t{};
  NodeTable run_t{};  // t as the running batch's rounds see it (run_batch)
  Shard *d_shards = nullptr;
  uint32_t *d_slot_pos = nullptr;
  uint32_t *d_start = nullptr;
  uint32_t *h_start = nullptr;  // pinned
  uint32_t *d_norm = nullptr;     // [2][P][2] by round parity
  double *d_norm_inv = nullptr;   // [2][P][2] by round parity
  PodStat *d_pstat = nullptr;     // [P]
  uint32_t *d_fix = nullptr;      // [P] flags + [MAX_P / MAX_PG] group flags + [MAX_P] compacted list
  uint32_t *d_dedup = nullptr;    // by round parity: rep [MAX_P], ulist [MAX_P], nuniq (RoundArgs::cls)
  bool dedup_used[2] = {false, false};  // the last round of that parity read records through rep
  BlockRec *d_brec = nullptr;     // [2][...] by round parity (merge k reads while sweep k+1 writes)
  size_t brec_bytes = 0;          // per parity
  uint64_t *d_srec = nullptr, *d_frec = nullptr;
  uint64_t *d_counters = nullptr;
  CandRow *d_crow = nullptr;
  CandExt *d_cext = nullptr;
  // pipeline state: [0,1] sweep start, [2,3] actual start, [4,5] carry counts (by parity)
  uint32_t *d_pipe = nullptr;
  CarryRec *d_carry = nullptr;  // [2][MAX_P]
  // host mirror / dictionaries
  std::vector<HostNode> nodes;
  uint32_t n_present = 0;
  std::vector<uint8_t> present_map;  // HostNode::present by slot, compact (pod events check it per pod)
  // ks_snapshot_update: the last NodeInfo.Generation applied per slot, and the max
  std::vector<int64_t> slot_gen;
  int64_t snapshot_gen = 0;
  std::unordered_map<std::string, uint32_t> str_ids{{"", 0}};
  std::vector<std::string> strs{""};
  std::unordered_map<uint32_t, uint32_t> name_slot;  // name id -> slot
  std::map<TaintKey, uint32_t> hard_dict;             // NoSchedule / NoExecute taints
  std::vector<TaintKey> hard_list;
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> prefer_dict;
  std::vector<std::pair<uint32_t, uint32_t>> prefer_list;
  uint64_t hard_in_use = 0, prefer_in_use = 0;
  std::unordered_map<uint64_t, uint32_t> prefer_masks;  // prefer-taint word -> present nodes with it
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> pair_bit;
  std::unordered_map<uint32_t, uint32_t> key_bit;
  std::unordered_map<uint32_t, NumCol> num_col;
  uint32_t next_bit = 0, next_num = 0;
  uint64_t label_resets = 0, taint_rebuilds = 0;  // dictionary capacity reclaims (diagnostics)
  std::unordered_map<uint32_t, std::vector<uint32_t>> key_nodes;  // key id -> slots having it
  bool compile_used_names = false;  // set by compile_pod when a pod resolved a node name to a slot
  uint32_t dict_version = 1;   // taint dictionary / node image set (compiled masks and checks)
  // Normaliser guesses (PodDev::tt_guess / na_guess): the distinct (label
  // words, numeric labels, taint words) of the present nodes, rebuilt when a
  // node's words change (tuple_version), and per (required, preferred
  // program, tolerations) the max raw over the tuples a node could pass with
  struct NodeTuple {
    uint64_t w[LW + NNUM + 2];  // lab, num, hard, prefer
  };
  uint64_t tuple_version = 0, tuples_for = ~0ull;
  std::vector<NodeTuple> tuples;
  std::unordered_map<std::string, std::pair<uint32_t, uint32_t>> guess_memo;
  uint32_t names_version = 1;  // node name -> slot map (compiled NodeName / metadata.name slots)
  std::vector<uint32_t> dirty_ext;
  // ImageLocality: image name (as nodes report it) -> present nodes reporting
  // it and the size the first of them reported (upstream cache imageStates)
  struct ImageState {
    uint32_t nodes = 0;
    int64_t size = 0;
  };
  std::unordered_map<std::string, ImageState> images;
  // extended resources (ephemeral-storage, scalar resources): name id -> column
  std::unordered_map<uint32_t, uint32_t> xres_of;
  std::vector<uint32_t> xres_names;
  int64_t *d_xalloc = nullptr, *d_xreq = nullptr;  // [MAX_XRES][npos], one allocation
  // bound pods carrying pod (anti-)affinity terms (InterPodAffinity precondition)
  int64_t affinity_pods = 0;
  // PodTopologySpread (ksched_spread.hip; device columns allocated on first use)
  std::map<std::pair<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>>, uint32_t> set_ids;
  std::vector<LabelSet> label_sets;
  std::unordered_map<std::string, uint32_t> empty_set_of_ns;  // label-less pods: namespace -> set id
  std::unordered_map<std::string, uint32_t> set_of_key;       // pods with terms / namespace labels
  TermClass terms[MAX_TERM_CLASSES];
  uint32_t n_terms = 0;
  std::unordered_map<std::string, uint32_t> term_of;         // canonical term -> class
  uint32_t *d_tcnt = nullptr;                                // [tcnt_cap][npos]
  uint32_t tcnt_cap = 0;
  uint32_t *d_adcnt = nullptr;                               // [MAX_AFF][dom_cap] affinity domain counts
  int64_t *d_sraw2 = nullptr;                                // [npos] InterPodAffinity raw score
  // (slot, set) of pods the batches bound, appended at the end of each run and
  // applied to HostNode::pod_sets only when a reader needs them (flush_bound)
  // NodeInfo.Pods changes as a log of (slot, set, op): +1 bound, -1 removed,
  // 0 node deleted.  While no selector class is live and no pod carries an
  // affinity term nothing reads the per-node records, so pod events and node
  // deletions only append here (no random access into 1M HostNodes per
  // event); flush_bound replays the log in order when a reader needs them.
  struct PodRec {
    uint32_t slot, set;
    int32_t op;
  };
  std::vector<PodRec> pending_bound;
  SpreadClass classes[MAX_CLASSES];
  std::unordered_map<std::string, uint32_t> class_of;  // canonical selector -> class
  uint64_t class_seq = 0;
  uint64_t class_epoch = 0;     // selector classes created
  uint64_t runs_started = 0, runs_done = 0;  // batch runs (in order, on the worker)
  std::vector<TopoKey> topo;                            // topology-key columns
  std::unordered_map<uint32_t, uint32_t> topo_of;       // key id -> column
  uint32_t *d_dom = nullptr;       // [MAX_TOPO_KEYS][npos]
  uint32_t *d_cnt = nullptr;       // [MAX_CLASSES][npos]
  uint32_t *d_pos_slot = nullptr;  // [npos]
  uint32_t *d_dcnt = nullptr, *d_dflag = nullptr;  // [MAX_SPREAD][dom_cap]
  uint32_t dom_cap = 0;
  SpreadAcc *d_acc = nullptr;
  int8_t *d_sst = nullptr;
  // percentageOfNodesToScore < 100: every pod takes the one-pod
  // chain with a window pass; d_win [WIN_WORDS] (0: nextStartNodeIndex),
  // d_win_st [cap] list / feasible bytes of the probe pass
  int32_t pct = 100;
  uint32_t *d_win = nullptr;
  uint8_t *d_win_st = nullptr;
  int64_t *d_sraw = nullptr;
  uint64_t *d_spart = nullptr;
  // replica runs: sort keys and positions, group starts, control
  // words (ReplicaArgs::ctl; pinned copy), radix-sort scratch
  bool replica_runs = true;
  // ks_batch_prepare compiling while submitted batches may run: creating a
  // topology / selector-class / term / extended-resource column is refused
  // (KS_NEED_DRAIN), the caller drains and compiles again
  bool undrained = false;
  uint64_t *d_rk_keys = nullptr, *d_rk_sorted = nullptr;
  uint64_t *d_rk_val = nullptr, *d_rk_sval = nullptr;
  uint32_t *d_rk_gstart = nullptr, *d_rk_ctl = nullptr;
  uint8_t *d_rk_tmp = nullptr;
  size_t rk_tmp_bytes = 0;
  uint32_t *h_rk_ctl = nullptr;
  uint64_t *d_rk_prof = nullptr;  // KS_RUN_PROFILE: replica_run phase clocks (ReplicaArgs::prof)
  uint64_t rk_prof[4] = {0, 0, 0, 0};  // ... their totals after the last run
  uint32_t *h_seg = nullptr;       // pinned: start pod of a round-kernel segment
  // comm: RCCL, or an in-process group of contexts (tests of the multi-rank path on one GPU)
  ncclComm_t comm = nullptr;
  std::shared_ptr<LocalGroup> lgroup;
  hipEvent_t lg_ev[2] = {nullptr, nullptr};  // posted / finished
  uint32_t *d_lgstage = nullptr;             // all-reduce input as peers read it
  bool has_comm() const { return comm != nullptr || lgroup != nullptr; }
  // stats
  ks_stats stats{};
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_sweep, ev_resolve, ev_spread;
  struct RunEv {
    hipEvent_t e0, e1;
    uint32_t pods;  // pods the replica run scheduled
  };
  std::vector<RunEv> ev_runs;
  std::vector<hipEvent_t> ev_pool;
  uint64_t counters_base[4] = {0, 0, 0, 0};  // device counters at the last ks_reset_stats
  uint64_t sweeps_issued = 0;                // main sweep launches since then (timed or not)
  uint64_t spread_seq = 0;                   // spread-path pods issued (timing sample)
  // Host<->device transfers of one ABI call: a pinned host staging buffer and a
  // device scratch buffer, both bump-allocated and reset at xfer_sync (no
  // pageable hipMemcpyAsync anywhere), on `stream`.  No fourth stream: the
  // box gives a process 4 hardware queues (GPU_MAX_HW_QUEUES), and a stream
  // sharing the resolve's queue serialises resolve k behind sweep k+1.
  struct Xfer {
    hipStream_t st = nullptr;
    uint8_t *pin = nullptr, *dscr = nullptr;
    size_t pin_cap = 0, pin_used = 0, dscr_cap = 0, dscr_used = 0;
    struct Pending {
      void *dst;
      size_t off, bytes;
    };
    std::vector<Pending> d2h_pending;
  };
  Xfer xm;
  // device buffers replaced while work may be in flight: freed at ks_close
  // (hipFree synchronises the whole device)
  std::vector<void *> graveyard;
  std::vector<void *> pinned_graveyard;
  // batch pool (ks_batch_free returns batches here; buffers are reused)
  std::mutex pool_mu;
  std::vector<ks_batch *> pool;
  std::vector<ks_batch *> all_batches;
  // host dictionaries / node mirror: ks_batch_prepare vs the worker's reads of t.lw
  std::mutex mu;
  // the worker waits for `mu` (run start / end): a compile holding it yields
  // between pods (compile_yield), so a batch's run does not wait for the
  // whole compile of a later batch
  std::atomic<uint32_t> mu_wanted{0};
  std::mutex err_mu;
  // asynchronous runs (ks_batch_submit / ks_batch_wait): one worker thread
  // (ksched_sync.hpp), created at ks_open
  std::unique_ptr<RunQueue<ks_batch>> runq;

  uint32_t intern(const char *p) {
    std::string s = str(p);
    auto it = str_ids.find(s);
    if (it != str_ids.end()) return it->second;
    const uint32_t id = (uint32_t)strs.size();
    strs.push_back(s);
    str_ids.emplace(std::move(s), id);
    return id;
  }
  int32_t lookup(const char *p) const {
    auto it = str_ids.find(str(p));
    return it == str_ids.end() ? -1 : (int32_t)it->second;
  }
  ks_status fail(ks_status st, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    std::lock_guard<std::mutex> g(err_mu);
    err = buf;
    return st;
  }
};

// Internal (never returned through the ABI): a compile that must create a
// column while batches may be running; ks_batch_prepare drains and retries.
constexpr ks_status KS_NEED_DRAIN = (ks_status)0x7F;

#define HIPC(ctx, x)                                                                           \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess)                                                                      \
      return (ctx)->fail(KS_ERR_DEVICE, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, \
                         __LINE__);                                                            \
  } while (0)

#define NCCLC(ctx, x)                                                                                  \
  do {                                                                                                 \
    ncclResult_t r_ = (x);                                                                             \
    if (r_ != ncclSuccess) return (ctx)->fail(KS_ERR_COMM, "%s: %s", #x, ncclGetErrorString(r_)); \
  } while (0)

namespace {

// --------------------------------------------------------------- transfers

inline size_t xround(size_t b) { return (b + 255) & ~(size_t)255; }

using Xfer = ks_ctx::Xfer;

// ------------------------------------------------------------ stall guard

const char *const kFlagName[4] = {"0 (sweep done: main -> side stream)", "1 (side stream done: -> resolve)",
                                  "2 (round resolved: resolve kernel -> main / side)",
                                  "3 (FIX sweep done: side -> main)"};

// A stream missed the deadline: wedge the context and name what is stuck.
ks_status stall_report(ks_ctx *c, hipStream_t st, const char *what, double ms) {
  c->wedged = true;
  std::string busy;
  const std::pair<hipStream_t, const char *> ss[3] = {{c->stream, "main"}, {c->sstream, "side"}, {c->rstream, "resolve"}};
  for (auto &p : ss)
    if (p.first && hipStreamQuery(p.first) == hipErrorNotReady) busy += std::string(busy.empty() ? "" : ", ") + p.second;
  // the flags through a stream of their own (the context's streams are
  // stuck), created here on the first report (never at ks_open, see
  // diag_stream) and kept until ks_close, so a report destroys nothing; best
  // effort: on a hung device the copy may never finish, and the report then
  // says so rather than waiting for it
  std::string flags = "unreadable (the device did not answer the read-back within 2 s)";
  if (!c->diag_stream && hipStreamCreateWithFlags(&c->diag_stream, hipStreamNonBlocking) != hipSuccess)
    c->diag_stream = nullptr;
  hipStream_t d = c->diag_stream;
  if (c->d_flags && c->h_diag && d && hipStreamQuery(d) == hipSuccess) {
    if (hipMemcpyAsync(c->h_diag, c->d_flags, 16, hipMemcpyDeviceToHost, d) == hipSuccess) {
      const auto t0 = std::chrono::steady_clock::now();
      while (hipStreamQuery(d) == hipErrorNotReady &&
             std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2))
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      if (hipStreamQuery(d) == hipSuccess) {
        flags.clear();
        // the stuck hand-off: of the flags behind what was enqueued, the one
        // at the earliest round, ties in pipeline order (sweep, FIX, side,
        // resolve): the flags after it wait on it
        int stuck = -1;
        for (int f : {0, 3, 1, 2}) {
          char b[96];
          std::snprintf(b, sizeof b, "%sflag %d = %u (enqueued up to %u)", flags.empty() ? "" : "; ", f, c->h_diag[f],
                        c->flag_want[f]);
          flags += b;
          if (c->h_diag[f] < c->flag_want[f] && (stuck < 0 || c->h_diag[f] < c->h_diag[stuck])) stuck = f;
        }
        flags += stuck >= 0 ? std::string("; stuck: flag ") + kFlagName[stuck] : std::string("; every flag reached");
      }
    }
  }
  return c->fail(KS_ERR_DEVICE,
                 "device stall: %s stream work of %s not finished after %.0f ms (round %u); unfinished streams: %s; %s",
                 st == c->stream ? "main" : st == c->sstream ? "side" : st == c->rstream ? "resolve" : "a",
                 what, ms, c->round_seq, busy.empty() ? "none" : busy.c_str(), flags.c_str());
}

// hipStreamSynchronize with a deadline (sync_timeout_ms): polls, yielding for
// the first 20 ms (a drain normally ends within a few ms), then sleeping.
ks_status sync_bounded(ks_ctx *c, hipStream_t st, const char *what) {
  if (c->wedged) return c->fail(KS_ERR_DEVICE, "context wedged by an earlier device stall (%s)", what);
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(st);
    if (e == hipSuccess) return KS_OK;
    if (e != hipErrorNotReady)
      return c->fail(KS_ERR_DEVICE, "hipStreamQuery (%s): %s", what, hipGetErrorString(e));
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms > c->sync_timeout_ms) return stall_report(c, st, what, ms);
    if (ms < 20) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(ms < 1000 ? 50 : 1000));
  }
}

ks_status xfer_sync(ks_ctx *c, Xfer &x) {
  ks_status st0 = sync_bounded(c, x.st, "a host<->device transfer");
  if (st0) return st0;
  for (auto &p : x.d2h_pending) std::memcpy(p.dst, x.pin + p.off, p.bytes);
  x.d2h_pending.clear();
  x.pin_used = x.dscr_used = 0;
  return KS_OK;
}
ks_status xfer_sync(ks_ctx *c) { return xfer_sync(c, c->xm); }

// Start an ABI call's transfers: completes earlier work, then guarantees
// pin_bytes of staging and dev_bytes of device scratch (each segment is
// rounded to 256 B: callers include that slack).  Outgrown buffers are
// retired to the graveyard (freed at ks_close: hipFree would wait for the
// whole device, including batches running on the other streams).
ks_status xfer_begin(ks_ctx *c, Xfer &x, size_t pin_bytes, size_t dev_bytes) {
  ks_status st = xfer_sync(c, x);
  if (st) return st;
  if (pin_bytes > x.pin_cap) {
    if (x.pin) c->pinned_graveyard.push_back(x.pin);
    x.pin = nullptr;
    x.pin_cap = std::max<size_t>(pin_bytes, std::max<size_t>(2 * x.pin_cap, 1 << 20));
    HIPC(c, hipHostMalloc((void **)&x.pin, x.pin_cap, hipHostMallocDefault));
  }
  if (dev_bytes > x.dscr_cap) {
    if (x.dscr) c->graveyard.push_back(x.dscr);
    x.dscr = nullptr;
    x.dscr_cap = std::max<size_t>(dev_bytes, std::max<size_t>(2 * x.dscr_cap, 1 << 20));
    HIPC(c, hipMalloc((void **)&x.dscr, x.dscr_cap));
  }
  return KS_OK;
}
ks_status xfer_begin(ks_ctx *c, size_t pin_bytes, size_t dev_bytes) { return xfer_begin(c, c->xm, pin_bytes, dev_bytes); }

template <class T>
T *dscratch(Xfer &x, size_t count) {
  const size_t b = xround(std::max<size_t>(count, 1) * sizeof(T));
  if (x.dscr_used + b > x.dscr_cap) return nullptr;
  T *p = (T *)(x.dscr + x.dscr_used);
  x.dscr_used += b;
  return p;
}
template <class T>
T *dscratch(ks_ctx *c, size_t count) { return dscratch<T>(c->xm, count); }

ks_status h2d(ks_ctx *c, Xfer &x, void *dst, const void *src, size_t bytes) {
  if (!bytes) return KS_OK;
  const size_t b = xround(bytes);
  if (x.pin_used + b > x.pin_cap) return c->fail(KS_ERR_INVALID, "staging overflow (h2d %zu)", bytes);
  std::memcpy(x.pin + x.pin_used, src, bytes);
  HIPC(c, hipMemcpyAsync(dst, x.pin + x.pin_used, bytes, hipMemcpyHostToDevice, x.st));
  x.pin_used += b;
  return KS_OK;
}
ks_status h2d(ks_ctx *c, void *dst, const void *src, size_t bytes) { return h2d(c, c->xm, dst, src, bytes); }

// Completed (copied to dst) at the next xfer_sync.
ks_status d2h(ks_ctx *c, void *dst, const void *src, size_t bytes) {
  Xfer &x = c->xm;
  if (!bytes) return KS_OK;
  const size_t b = xround(bytes);
  if (x.pin_used + b > x.pin_cap) return c->fail(KS_ERR_INVALID, "staging overflow (d2h %zu)", bytes);
  HIPC(c, hipMemcpyAsync(x.pin + x.pin_used, src, bytes, hipMemcpyDeviceToHost, x.st));
  x.d2h_pending.push_back({dst, x.pin_used, bytes});
  x.pin_used += b;
  return KS_OK;
}

// --------------------------------------------------------- label encoding

void node_ext_bits(ks_ctx *c, HostNode &n) {
  uint64_t lab[LW] = {};
  int64_t num[NNUM] = {};
  for (auto &kv : n.labels) {
    auto pb = c->pair_bit.find(kv);
    if (pb != c->pair_bit.end()) lab[pb->second >> 6] |= 1ull << (pb->second & 63);
    auto kb = c->key_bit.find(kv.first);
    if (kb != c->key_bit.end()) lab[kb->second >> 6] |= 1ull << (kb->second & 63);
    auto nc = c->num_col.find(kv.first);
    if (nc != c->num_col.end()) {
      int64_t v;
      if (parse_int64(c->strs[kv.second], &v)) {
        lab[nc->second.valid_bit >> 6] |= 1ull << (nc->second.valid_bit & 63);
        num[nc->second.col] = v;
      }
    }
  }
  std::memcpy(n.lab, lab, sizeof lab);
  std::memcpy(n.num, num, sizeof num);
  c->tuple_version++;
}

ks_status alloc_bit(ks_ctx *c, uint32_t *bit) {
  if (c->next_bit >= (uint32_t)LW * 64) return c->fail(KS_ERR_CAPACITY, "label dictionary full (%d bits)", LW * 64);
  *bit = c->next_bit++;
  c->t.lw = std::max(c->t.lw, (*bit >> 6) + 1);
  return KS_OK;
}

// key_nodes lists are append-only (a slot is added for every label it is
// upserted with); entries are re-validated here and the list compacted.
void mark_key_nodes_dirty(ks_ctx *c, uint32_t key) {
  auto it = c->key_nodes.find(key);
  if (it == c->key_nodes.end()) return;
  std::vector<uint32_t> &v = it->second;
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  size_t keep = 0;
  for (uint32_t s : v) {
    const HostNode &h = c->nodes[s];
    if (!h.present) continue;
    bool has = false;
    for (auto &kv : h.labels) has |= kv.first == key;
    if (!has) continue;
    v[keep++] = s;
    node_ext_bits(c, c->nodes[s]);
    c->dirty_ext.push_back(s);
  }
  v.resize(keep);
}

ks_status get_pair_bit(ks_ctx *c, uint32_t key, uint32_t value, uint32_t *bit) {
  auto it = c->pair_bit.find({key, value});
  if (it != c->pair_bit.end()) { *bit = it->second; return KS_OK; }
  ks_status st = alloc_bit(c, bit);
  if (st) return st;
  c->pair_bit.emplace(std::make_pair(key, value), *bit);
  mark_key_nodes_dirty(c, key);
  return KS_OK;
}

ks_status get_key_bit(ks_ctx *c, uint32_t key, uint32_t *bit) {
  auto it = c->key_bit.find(key);
  if (it != c->key_bit.end()) { *bit = it->second; return KS_OK; }
  ks_status st = alloc_bit(c, bit);
  if (st) return st;
  c->key_bit.emplace(key, *bit);
  mark_key_nodes_dirty(c, key);
  return KS_OK;
}

ks_status get_num_col(ks_ctx *c, uint32_t key, NumCol *out) {
  auto it = c->num_col.find(key);
  if (it != c->num_col.end()) { *out = it->second; return KS_OK; }
  if (c->next_num >= (uint32_t)NNUM) return c->fail(KS_ERR_CAPACITY, "numeric label columns full (%d)", NNUM);
  NumCol nc;
  nc.col = c->next_num++;
  ks_status st = alloc_bit(c, &nc.valid_bit);
  if (st) return st;
  c->num_col.emplace(key, nc);
  mark_key_nodes_dirty(c, key);
  *out = nc;
  return KS_OK;
}

// Label dictionary reclaim.  Bits are pod-driven and only grow; when a batch
// cannot get the bits its label programs need, the dictionary restarts empty:
// every present node's label words are re-encoded (zero until the batch's
// own requirements allocate bits again, which re-encodes the nodes carrying
// those keys) and prepared batches turn stale (dict_version).  The caller
// has drained the submitted batches (their programs test the old bits).
void reset_label_dict(ks_ctx *c) {
  c->pair_bit.clear();
  c->key_bit.clear();
  c->num_col.clear();
  c->next_bit = c->next_num = 0;
  for (uint32_t s = 0; s < c->cap; ++s) {
    HostNode &h = c->nodes[s];
    if (!h.present) continue;
    bool any = false;
    for (int k = 0; k < LW; ++k) any |= h.lab[k] != 0;
    for (int k = 0; k < NNUM; ++k) any |= h.num[k] != 0;
    if (!any) continue;
    std::memset(h.lab, 0, sizeof h.lab);
    std::memset(h.num, 0, sizeof h.num);
    c->dirty_ext.push_back(s);
  }
  c->dict_version++;
  c->label_resets++;
  c->tuple_version++;
}

// ------------------------------------------------------------ pod compile

bool tolerates(const ks_ctx *c, const std::vector<Tol> &tols, uint32_t key, uint32_t value, int32_t effect) {
  for (auto &t : tols) {  // ToleratesTaint
    if (t.effect != KS_EFFECT_ALL && t.effect != effect) continue;
    if (t.key != 0 && t.key != key) continue;
    if (t.op == KS_TOL_EXISTS) return true;
    if (t.op == KS_TOL_EQUAL && t.value == value) return true;
  }
  return false;
}

// PodRequests (resourcehelper) for cpu / memory; non_missing applies the
// scheduler's non-zero defaults to containers that omit a request.
ks_status pod_requests(const ks_pod &p, bool non_missing, int64_t *cpu, int64_t *mem) {
  auto req = [&](const ks_container &k, int64_t *a, int64_t *b) -> bool {
    if (k.flags & KS_REQ_HAS_OTHER) return false;
    *a = (k.flags & KS_REQ_HAS_CPU) ? k.milli_cpu : (non_missing ? kDefaultMilliCPURequest : 0);
    *b = (k.flags & KS_REQ_HAS_MEMORY) ? k.memory : (non_missing ? kDefaultMemoryRequest : 0);
    return true;
  };
  int64_t sum_c = 0, sum_m = 0;
  for (uint32_t i = 0; i < p.n_containers; ++i) {
    int64_t a, b;
    if (!req(p.containers[i], &a, &b)) return KS_ERR_UNSUPPORTED;
    sum_c += a;
    sum_m += b;
  }
  // init containers: max over "sidecars so far + this init container"; sidecars also add to the sum
  int64_t side_c = 0, side_m = 0, init_c = 0, init_m = 0;
  for (uint32_t i = 0; i < p.n_init_containers; ++i) {
    int64_t a, b;
    if (!req(p.init_containers[i], &a, &b)) return KS_ERR_UNSUPPORTED;
    int64_t use_c, use_m;
    if (p.init_containers[i].restart_always) {
      sum_c += a;
      sum_m += b;
      side_c += a;
      side_m += b;
      use_c = side_c;
      use_m = side_m;
    } else {
      use_c = a + side_c;
      use_m = b + side_m;
    }
    init_c = std::max(init_c, use_c);
    init_m = std::max(init_m, use_m);
  }
  sum_c = std::max(sum_c, init_c);
  sum_m = std::max(sum_m, init_m);
  if (p.has_overhead) {
    sum_c += p.overhead_milli_cpu;
    sum_m += p.overhead_memory;
  }
  *cpu = sum_c;
  *mem = sum_m;
  return KS_OK;
}

// Label-program words of one batch (ksched_dev.hpp: terms, PreFilterResult slots).
struct ProgBuf {
  std::vector<uint64_t> w;
  uint32_t size() const { return (uint32_t)w.size(); }
  // Programs are content-addressed within a batch, so pods with identical
  // programs get identical offsets (and byte-identical descriptors: the
  // sweep's identical-pod classes, pod_classes).  intern(off): the words
  // [off, size) were just appended; returns the offset of their first copy
  // (dropping the new one), 0 for an empty program.
  std::unordered_map<std::string, uint32_t> progs;
  uint32_t intern(uint32_t off) {
    if (off == size()) return 0;
    std::string key((const char *)(w.data() + off), (size() - off) * 8);
    auto it = progs.find(key);
    if (it != progs.end()) {
      w.resize(off);
      return it->second;
    }
    progs.emplace(std::move(key), off);
    return off;
  }
};

inline void set_bit(uint64_t m[LW], uint32_t b) { m[b >> 6] |= 1ull << (b & 63); }

// One NodeSelectorTerm as fixed-form masks (ksched_dev.hpp).
struct TermBuild {
  uint64_t must[LW] = {}, forbid[LW] = {};
  std::vector<std::array<uint64_t, LW>> groups;
  std::vector<std::pair<uint64_t, uint64_t>> nums, names;
  // a pair / key both required and forbidden: the term matches no node
  bool contradictory() const {
    for (int k = 0; k < LW; ++k)
      if (must[k] & forbid[k]) return true;
    return false;
  }
  void emit(ProgBuf &out, int32_t weight) const {
    out.w.push_back((uint64_t)groups.size() | ((uint64_t)nums.size() << 8) | ((uint64_t)names.size() << 16) |
                    ((uint64_t)(uint32_t)weight << 32));
    for (int k = 0; k < LW; ++k) out.w.push_back(must[k]);
    for (int k = 0; k < LW; ++k) out.w.push_back(must[k] | forbid[k]);
    for (auto &g : groups) out.w.insert(out.w.end(), g.begin(), g.end());
    for (auto &x : nums) { out.w.push_back(x.first); out.w.push_back(x.second); }
    for (auto &x : names) { out.w.push_back(x.first); out.w.push_back(x.second); }
  }
};

// newNodeSelectorTerm -> TermBuild.  Returns false on a parse error (the term
// then matches nothing in a required selector; a preferred term's PreScore
// fails).  Capacity / unsupported errors propagate through *st.
bool compile_term(ks_ctx *c, const ks_term &t, TermBuild &tb, ks_status *st) {
  for (uint32_t i = 0; i < t.n_expressions; ++i) {
    const ks_requirement &e = t.match_expressions[i];
    const std::string key = str(e.key);
    std::vector<std::string> vals;
    for (uint32_t k = 0; k < e.n_values; ++k) vals.push_back(str(e.values[k]));
    // labels.NewRequirement validation
    bool ok;
    switch (e.op) {
      case KS_OP_IN:
      case KS_OP_NOT_IN: ok = !vals.empty(); break;
      case KS_OP_EXISTS:
      case KS_OP_DOES_NOT_EXIST: ok = vals.empty(); break;
      case KS_OP_GT:
      case KS_OP_LT: {
        int64_t x;
        ok = vals.size() == 1 && parse_int64(vals[0], &x);
        break;
      }
      default: ok = false;
    }
    for (auto &v : vals) ok = ok && label_value_ok(v);
    ok = ok && qualified_name_ok(key);
    if (!ok) return false;
    const uint32_t kid = c->intern(e.key);
    uint32_t bit;
    switch (e.op) {
      case KS_OP_IN: {  // one value: a required pair; several: any of the pairs
        std::array<uint64_t, LW> g{};
        for (auto &v : vals) {
          if ((*st = get_pair_bit(c, kid, c->intern(v.c_str()), &bit))) return false;
          set_bit(g.data(), bit);
        }
        int nb = 0;
        for (int k = 0; k < LW; ++k) nb += __builtin_popcountll(g[k]);
        if (nb == 1) {
          for (int k = 0; k < LW; ++k) tb.must[k] |= g[k];
        } else {
          tb.groups.push_back(g);
        }
        break;
      }
      case KS_OP_NOT_IN:  // no listed pair (true when the key is absent)
        for (auto &v : vals) {
          if ((*st = get_pair_bit(c, kid, c->intern(v.c_str()), &bit))) return false;
          set_bit(tb.forbid, bit);
        }
        break;
      case KS_OP_EXISTS:
      case KS_OP_DOES_NOT_EXIST:
        if ((*st = get_key_bit(c, kid, &bit))) return false;
        set_bit(e.op == KS_OP_EXISTS ? tb.must : tb.forbid, bit);
        break;
      default: {  // Gt / Lt: the label parses as an int64 (valid bit) and compares
        NumCol nc;
        if ((*st = get_num_col(c, kid, &nc))) return false;
        set_bit(tb.must, nc.valid_bit);
        int64_t x = 0;
        parse_int64(vals[0], &x);
        tb.nums.emplace_back((uint64_t)nc.col | ((uint64_t)(e.op == KS_OP_GT ? TO_GT : TO_LT) << 8), (uint64_t)x);
      }
    }
  }
  for (uint32_t i = 0; i < t.n_fields; ++i) {  // nodeSelectorRequirementsAsFieldSelector
    const ks_requirement &e = t.match_fields[i];
    if (str(e.key) != "metadata.name" || e.n_values != 1 || (e.op != KS_OP_IN && e.op != KS_OP_NOT_IN)) return false;
    const int32_t nid = c->lookup(e.values[0]);
    int64_t slot = -1;
    if (nid >= 0) {
      auto it = c->name_slot.find((uint32_t)nid);
      if (it != c->name_slot.end()) slot = it->second;
    }
    tb.names.emplace_back(e.op == KS_OP_IN ? TO_NAME_IN : TO_NAME_NOT_IN, (uint64_t)slot);
    c->compile_used_names = true;
  }
  return true;
}

// Reference count of the non-zero prefer-taint words of present nodes (the
// TaintToleration max guess of compile_pod).
void prefer_mask_ref(ks_ctx *c, uint64_t mask, int delta) {
  if (!mask) return;
  auto it = c->prefer_masks.find(mask);
  if (delta > 0) {
    if (it == c->prefer_masks.end()) c->prefer_masks.emplace(mask, 1u);
    else it->second++;
  } else if (it != c->prefer_masks.end() && --it->second == 0) {
    c->prefer_masks.erase(it);
  }
}

// NodeAffinity.PreFilter's PreFilterResult (upstream v1.31
// plugins/nodeaffinity/node_affinity.go#PreFilter), from the RAW required
// terms (parse errors and empty terms included, as upstream): when every term
// has matchFields metadata.name In requirements, the candidate nodes are the
// union over terms of the intersection of each term's name sets.  Returns
// false when some term names no node (all nodes eligible); *names = the union.
bool prefilter_names(const ks_pod &p, std::vector<std::string> *names) {
  if (!p.has_required || p.n_required_terms == 0) return false;
  std::vector<std::string> uni;
  for (uint32_t i = 0; i < p.n_required_terms; ++i) {
    const ks_term &t = p.required_terms[i];
    bool have = false;
    std::vector<std::string> inter;
    for (uint32_t k = 0; k < t.n_fields; ++k) {
      const ks_requirement &r = t.match_fields[k];
      if (str(r.key) != "metadata.name" || r.op != KS_OP_IN) continue;
      std::vector<std::string> vs;
      for (uint32_t v = 0; v < r.n_values; ++v) vs.push_back(str(r.values[v]));
      std::sort(vs.begin(), vs.end());
      vs.erase(std::unique(vs.begin(), vs.end()), vs.end());
      if (!have) {
        inter = vs;
        have = true;
      } else {
        std::vector<std::string> x;
        std::set_intersection(inter.begin(), inter.end(), vs.begin(), vs.end(), std::back_inserter(x));
        inter.swap(x);
      }
    }
    if (!have) return false;  // this term does not restrict node names
    uni.insert(uni.end(), inter.begin(), inter.end());
  }
  std::sort(uni.begin(), uni.end());
  uni.erase(std::unique(uni.begin(), uni.end()), uni.end());
  *names = std::move(uni);
  return true;
}

// Preconditions of the modelled plugin set: a pod the
// default profile would filter or score with a plugin ksched does not model is
// refused, never scheduled approximately.
ks_status check_modelled(ks_ctx *c, const ks_pod &p) {
  if (p.unmodelled)
    return c->fail(KS_ERR_UNSUPPORTED, "pod %s/%s carries %s", str(p.ns).c_str(), str(p.name).c_str(),
                   unmodelled_name(p.unmodelled));
  if (c->affinity_pods > 0)
    return c->fail(KS_ERR_UNSUPPORTED,
                   "%lld bound pod(s) carry pod (anti-)affinity terms: InterPodAffinity filters and scores every "
                   "incoming pod", (long long)c->affinity_pods);
  return KS_OK;
}

ks_status solo_compile(ks_ctx *c, const ks_pod &p, PodDev &d, ProgBuf &cl, bool create,
                       std::vector<uint32_t> *refs);
void refine_guesses(ks_ctx *c, PodDev &d, const ProgBuf &cl);

// A preferred term no node passing the pod's nodeSelector can match (a node
// holds one value per label key): In / NotIn / DoesNotExist on a key the
// nodeSelector pins to another value.  Its weight never counts toward the
// NodeAffinity max, so the normaliser guess leaves it out (a guess only has
// to be right often: a wrong one costs a FIX re-sweep, never a wrong result).
static bool pref_excluded_by_selector(const ks_pod &p, const ks_term &t) {
  for (uint32_t e = 0; e < t.n_expressions; ++e) {
    const ks_requirement &r = t.match_expressions[e];
    for (uint32_t s = 0; s < p.n_node_selector; ++s) {
      if (str(p.node_selector[s].key) != str(r.key)) continue;
      const std::string v = str(p.node_selector[s].value);
      bool in = false;
      for (uint32_t k = 0; k < r.n_values; ++k) in |= str(r.values[k]) == v;
      if ((r.op == KS_OP_IN && !in) || (r.op == KS_OP_NOT_IN && in) || r.op == KS_OP_DOES_NOT_EXIST) return true;
    }
  }
  return false;
}

ks_status compile_pod(ks_ctx *c, const ks_pod &p, PodDev &d, ProgBuf &cl, bool create_spread = false,
                      std::vector<uint32_t> *class_refs = nullptr) {
  std::memset(&d, 0, sizeof d);
  ks_status st;
  if ((st = check_modelled(c, p))) return st;
  if ((st = pod_requests(p, false, &d.req_cpu, &d.req_mem)) ||
      (st = pod_requests(p, true, &d.nz_cpu, &d.nz_mem)))
    return c->fail(st, "pod %s/%s requests a resource other than cpu/memory", str(p.ns).c_str(),
                   str(p.name).c_str());
  if (d.req_cpu < 0 || d.req_mem < 0 || d.req_cpu >= kMaxExact || d.req_mem >= kMaxExact)
    return c->fail(KS_ERR_RANGE, "pod %s requests outside [0, 2^46)", str(p.name).c_str());
  if (d.req_cpu != 0 || d.req_mem != 0) d.flags |= PF_HAS_REQ;
  if (d.nz_cpu >= kMaxExact || d.nz_mem >= kMaxExact)
    return c->fail(KS_ERR_RANGE, "pod %s requests outside [0, 2^46)", str(p.name).c_str());
  d.req_cpu_d = (double)d.req_cpu;
  d.req_mem_d = (double)d.req_mem;
  d.nz100_cpu = (double)d.nz_cpu * 100.0;
  d.nz100_mem = (double)d.nz_mem * 100.0;
  // tolerations -> dictionary masks
  std::vector<Tol> tols, tols_prefer;
  for (uint32_t i = 0; i < p.n_tolerations; ++i) {
    const ks_toleration &t = p.tolerations[i];
    Tol x{c->intern(t.key), c->intern(t.value), t.op, t.effect};  // "" interns to id 0
    tols.push_back(x);
    if (t.effect == KS_EFFECT_ALL || t.effect == KS_EFFECT_PREFER_NO_SCHEDULE) tols_prefer.push_back(x);
  }
  for (size_t b = 0; b < c->hard_list.size(); ++b)
    if (tolerates(c, tols, c->hard_list[b].key, c->hard_list[b].value, c->hard_list[b].effect))
      d.tol_hard |= 1ull << b;
  // NodeUnschedulable: Taint{Key: node.kubernetes.io/unschedulable, Effect: NoSchedule}
  if (tolerates(c, tols, c->intern("node.kubernetes.io/unschedulable"), 0, KS_EFFECT_NO_SCHEDULE))
    d.tol_hard |= UNSCHED_BIT;
  for (size_t b = 0; b < c->prefer_list.size(); ++b)
    if (tolerates(c, tols_prefer, c->prefer_list[b].first, c->prefer_list[b].second, KS_EFFECT_PREFER_NO_SCHEDULE))
      d.tol_prefer |= 1ull << b;
  if (c->prefer_in_use & ~d.tol_prefer) {
    d.flags |= PF_TT;
    // guess of max raw over feasible nodes: the max over the prefer-taint words
    // present in the cluster (exact unless no feasible node carries the worst one)
    uint32_t g = 0;
    if (c->prefer_masks.size() <= 256) {
      for (const auto &kv : c->prefer_masks) g = std::max<uint32_t>(g, (uint32_t)__builtin_popcountll(kv.first & ~d.tol_prefer));
    } else {
      g = (uint32_t)__builtin_popcountll(c->prefer_in_use & ~d.tol_prefer);
    }
    d.tt_guess = g;
  }
  // spec.nodeName
  d.name_slot = -1;
  if (p.node_name && p.node_name[0]) {
    d.name_slot = -2;
    const int32_t nid = c->lookup(p.node_name);
    if (nid >= 0) {
      auto it = c->name_slot.find((uint32_t)nid);
      if (it != c->name_slot.end()) d.name_slot = (int32_t)it->second;
    }
    c->compile_used_names = true;
  }
  // required: OR of the RequiredDuringScheduling terms, the nodeSelector's
  // pairs merged into each (RequiredNodeAffinity.Match: selector AND terms);
  // no usable term (all empty / parse errors / contradictory) matches nothing
  TermBuild sel;
  for (uint32_t i = 0; i < p.n_node_selector; ++i) {
    uint32_t bit;
    if ((st = get_pair_bit(c, c->intern(p.node_selector[i].key), c->intern(p.node_selector[i].value), &bit)))
      return st;
    set_bit(sel.must, bit);
  }
  d.req_off = cl.size();
  if (p.has_required) {
    for (uint32_t i = 0; i < p.n_required_terms; ++i) {
      const ks_term &t = p.required_terms[i];
      if (t.n_expressions == 0 && t.n_fields == 0) continue;  // empty term selects nothing: skipped
      TermBuild tb;
      st = KS_OK;
      if (!compile_term(c, t, tb, &st)) {
        if (st) return st;
        continue;  // parse error: the term never matches
      }
      for (int k = 0; k < LW; ++k) tb.must[k] |= sel.must[k];
      if (tb.contradictory()) continue;
      tb.emit(cl, 0);
      d.req_len++;
    }
  } else if (p.n_node_selector) {
    sel.emit(cl, 0);
    d.req_len = 1;
  }
  d.req_off = cl.intern(d.req_off);
  d.solo_off = 0;
  {
    std::vector<std::string> names;
    if (prefilter_names(p, &names)) {
      if (names.empty()) {
        d.flags |= PF_NA_CONFLICT;  // UnschedulableAndUnresolvable (errReasonConflict) at PreFilter
      } else {
        d.flags |= PF_PREFILTER;
        d.pre_off = cl.size();
        for (auto &nm : names) {
          auto id = c->str_ids.find(nm);
          if (id == c->str_ids.end()) continue;
          auto it = c->name_slot.find(id->second);
          if (it == c->name_slot.end()) continue;  // PreFilterResult names a node the snapshot lacks
          cl.w.push_back((uint64_t)it->second);
        }
        d.pre_len = cl.size() - d.pre_off;
        d.pre_off = cl.intern(d.pre_off);
        d.prefilter_out = c->n_present - d.pre_len;
      }
      c->compile_used_names = true;
    }
  }
  if (p.n_node_selector || p.has_required) d.flags |= PF_AFF;
  // preferred terms: Σ weight of the matching ones
  d.pref_off = cl.size();
  if (p.has_preferred) {
    d.flags |= PF_HAS_PREF;
    for (uint32_t i = 0; i < p.n_preferred; ++i) {
      const ks_preferred_term &t = p.preferred[i];
      if (t.weight == 0 || (t.preference.n_expressions == 0 && t.preference.n_fields == 0)) continue;
      if (t.weight < 0 || t.weight > 100)
        return c->fail(KS_ERR_UNSUPPORTED, "preferred term weight %d outside 1..100", t.weight);
      TermBuild tb;
      st = KS_OK;
      if (!compile_term(c, t.preference, tb, &st)) {
        if (st) return st;
        d.flags |= PF_PREF_ERR;
        continue;
      }
      if (tb.contradictory()) continue;  // matches no node: adds 0 everywhere
      tb.emit(cl, t.weight);
      d.pref_len++;
      // guess of max raw: every term matches some feasible node, except the
      // ones the pod's own nodeSelector rules out
      if (!pref_excluded_by_selector(p, t.preference)) d.na_guess += (uint32_t)t.weight;
    }
    if (d.pref_len) d.flags |= PF_NA;
  }
  d.pref_off = cl.intern(d.pref_off);
  if ((c->hard_in_use & ~d.tol_hard) || d.name_slot != -1 || (d.flags & (PF_AFF | PF_TT | PF_NA)))
    d.flags |= PF_EXT;
  refine_guesses(c, d, cl);
  return solo_compile(c, p, d, cl, create_spread, class_refs);
}

// One label-program term (ksched_dev.hpp) against a node tuple; false in
// *known for metadata.name entries (a per-node property).
bool tuple_term(const uint64_t *t, const ks_ctx::NodeTuple &x, bool *known) {
  const uint64_t w0 = t[0];
  const uint32_t ng = (uint32_t)w0 & 0xFF, nn = ((uint32_t)w0 >> 8) & 0xFF, nm = ((uint32_t)w0 >> 16) & 0xFF;
  if (nm) *known = false;
  bool ok = true;
  for (int k = 0; k < LW; ++k) ok &= ((x.w[k] & t[1 + LW + k]) ^ t[1 + k]) == 0;
  const uint64_t *g = t + TERM_HDR_WORDS;
  for (uint32_t i = 0; i < ng; ++i, g += LW) {
    uint64_t any = 0;
    for (int k = 0; k < LW; ++k) any |= x.w[k] & g[k];
    ok &= any != 0;
  }
  for (uint32_t i = 0; i < nn; ++i, g += 2) {
    const int64_t v = (int64_t)x.w[LW + ((g[0] & 0xFF) ? 1 : 0)];
    const int64_t o = (int64_t)g[1];
    ok &= ((g[0] >> 8) & 0xFF) == TO_GT ? v > o : v < o;
  }
  return ok;
}

// Normaliser guesses of a compiled pod: max raw TaintToleration / NodeAffinity
// over the node tuples that pass the pod's label and taint filters (every
// node of such a tuple fails only on resources, so with many nodes per tuple
// the guess is the measured max).  Memoised per program; name-based terms
// keep the caller's guesses.
void refine_guesses(ks_ctx *c, PodDev &d, const ProgBuf &cl) {
  if (!c->tuple_guess || !(d.flags & (PF_TT | PF_NA)) || (d.flags & (PF_PREFILTER | PF_NA_CONFLICT)) ||
      d.name_slot != -1)
    return;
  if (c->tuples_for != c->tuple_version) {
    struct H {
      size_t operator()(const ks_ctx::NodeTuple &x) const {
        uint64_t h = 1469598103934665603ull;
        for (uint64_t v : x.w) h = (h ^ v) * 1099511628211ull;
        return (size_t)h;
      }
    };
    struct E {
      bool operator()(const ks_ctx::NodeTuple &a, const ks_ctx::NodeTuple &b) const {
        return std::memcmp(a.w, b.w, sizeof a.w) == 0;
      }
    };
    std::unordered_set<ks_ctx::NodeTuple, H, E> seen;
    for (uint32_t sl = 0; sl < c->cap && seen.size() <= 4096; ++sl) {  // past 4096: simple guesses
      const HostNode &h = c->nodes[sl];
      if (!h.present) continue;
      ks_ctx::NodeTuple x;
      std::memcpy(x.w, h.lab, sizeof h.lab);
      std::memcpy(x.w + LW, h.num, sizeof h.num);
      x.w[LW + NNUM] = h.hard;
      x.w[LW + NNUM + 1] = h.prefer;
      seen.insert(x);
    }
    c->tuples.assign(seen.begin(), seen.end());
    c->guess_memo.clear();
    c->tuples_for = c->tuple_version;
  }
  if (c->tuples.size() > 4096) return;  // too many distinct tuples: keep the simple guesses
  const uint64_t *req = cl.w.data() + d.req_off, *pref = cl.w.data() + d.pref_off;
  size_t req_words = 0, pref_words = 0;
  for (uint32_t k = 0; k < d.req_len; ++k) req_words += term_words(req[req_words]);
  for (uint32_t k = 0; k < d.pref_len; ++k) pref_words += term_words(pref[pref_words]);
  std::string key((const char *)&d.tol_hard, 8);
  key.append((const char *)&d.tol_prefer, 8);
  const uint32_t f = d.flags & (PF_AFF | PF_TT | PF_NA);
  key.append((const char *)&f, 4);
  key.append((const char *)&d.req_len, 4);
  key.append((const char *)req, req_words * 8);
  key.append((const char *)pref, pref_words * 8);
  auto it = c->guess_memo.find(key);
  if (it == c->guess_memo.end()) {
    uint32_t tt = 0, na = 0;
    bool known = true, any = false;
    for (const ks_ctx::NodeTuple &x : c->tuples) {
      if (x.w[LW + NNUM] & ~d.tol_hard) continue;  // a hard taint (or unschedulable) the pod does not tolerate
      if (d.flags & PF_AFF) {
        bool m = false;
        const uint64_t *t = req;
        for (uint32_t k = 0; k < d.req_len; ++k, t += term_words(t[0])) m |= tuple_term(t, x, &known);
        if (!m) continue;
      }
      any = true;
      tt = std::max<uint32_t>(tt, (uint32_t)__builtin_popcountll(x.w[LW + NNUM + 1] & ~d.tol_prefer));
      uint32_t raw = 0;
      const uint64_t *t = pref;
      for (uint32_t k = 0; k < d.pref_len; ++k, t += term_words(t[0]))
        if (tuple_term(t, x, &known)) raw += (uint32_t)(t[0] >> 32);
      na = std::max(na, raw);
    }
    if (!known || !any) return;
    it = c->guess_memo.emplace(std::move(key), std::make_pair(tt, na)).first;
  }
  if (d.flags & PF_TT) d.tt_guess = it->second.first;
  if (d.flags & PF_NA) d.na_guess = it->second.second;
}

// Taint dictionaries (hard: NoSchedule / NoExecute, prefer: PreferNoSchedule)
// for one node from its stored taint ids.  Returns KS_ERR_CAPACITY when a new
// taint finds the dictionary full (63 hard taints + the unschedulable bit, 64
// prefer taints); *grew when a taint was new.
ks_status encode_taints(ks_ctx *c, HostNode &h, bool *grew) {
  c->tuple_version++;
  h.hard = h.unschedulable ? UNSCHED_BIT : 0;
  h.prefer = 0;
  for (auto &t : h.hard_taints) {
    TaintKey tk{t[0], t[1], (int32_t)t[2]};
    auto it = c->hard_dict.find(tk);
    uint32_t b;
    if (it == c->hard_dict.end()) {
      if (c->hard_list.size() >= 63) return KS_ERR_CAPACITY;
      b = (uint32_t)c->hard_list.size();
      c->hard_dict.emplace(tk, b);
      c->hard_list.push_back(tk);
      *grew = true;
    } else {
      b = it->second;
    }
    h.hard |= 1ull << b;
  }
  for (auto &pk : h.prefer_taints) {
    auto it = c->prefer_dict.find(pk);
    uint32_t b;
    if (it == c->prefer_dict.end()) {
      if (c->prefer_list.size() >= 64) return KS_ERR_CAPACITY;
      b = (uint32_t)c->prefer_list.size();
      c->prefer_dict.emplace(pk, b);
      c->prefer_list.push_back(pk);
      *grew = true;
    } else {
      b = it->second;
    }
    h.prefer |= 1ull << b;
  }
  return KS_OK;
}

// Taint dictionary reclaim: rebuilt from the taints present nodes carry now
// (deleted / updated nodes' taints drop out); every present node's taint
// words are re-encoded and prepared batches turn stale.  KS_ERR_CAPACITY when
// the present nodes alone carry more distinct taints than the words hold.
ks_status rebuild_taint_dicts(ks_ctx *c) {
  c->hard_dict.clear();
  c->hard_list.clear();
  c->prefer_dict.clear();
  c->prefer_list.clear();
  c->prefer_masks.clear();
  c->hard_in_use = c->prefer_in_use = 0;
  bool grew = false;
  ks_status st = KS_OK;
  for (uint32_t s = 0; s < c->cap; ++s) {
    HostNode &h = c->nodes[s];
    if (!h.present) continue;
    if (!st) st = encode_taints(c, h, &grew);
    if (st) h.hard = h.prefer = 0;  // keep the mirror consistent; the call fails
    c->hard_in_use |= h.hard;
    c->prefer_in_use |= h.prefer;
    prefer_mask_ref(c, h.prefer, +1);
    c->dirty_ext.push_back(s);
  }
  c->dict_version++;
  c->taint_rebuilds++;
  if (st) return c->fail(st, "present nodes carry more than 63 hard / 64 PreferNoSchedule distinct taints");
  return KS_OK;
}

// Node image set (ImageLocality precondition): reference counts of present
// nodes per normalised image name.  Returns true when a name is new.
bool node_images_ref(ks_ctx *c, HostNode &h, int delta) {
  bool grew = false;
  for (auto &im : h.images) {
    auto it = c->images.find(im.first);
    if (delta > 0) {
      if (it == c->images.end()) {  // addNodeImageStates: the first reporter's size
        c->images.emplace(im.first, ks_ctx::ImageState{1u, im.second});
        grew = true;
      } else {
        it->second.nodes++;
      }
    } else if (it != c->images.end() && --it->second.nodes == 0) {
      c->images.erase(it);  // removeNodeImageStates: the last node reporting it left
    }
  }
  return grew;
}

// Node-side "image present" key of ImageLocality (a label key no real label can have).
std::string image_key(const std::string &name) { return std::string("\x01image\x01") + name; }

// schedutil.IsScalarResourceName || ephemeral-storage (framework.Resource fields
// beyond cpu / memory / pods); other names are ignored upstream.
bool xres_name_ok(const std::string &n) {
  if (n == "ephemeral-storage") return true;
  if (n.rfind("hugepages-", 0) == 0 || n.rfind("attachable-volumes-", 0) == 0) return true;
  if (n.find("kubernetes.io/") != std::string::npos) return true;  // IsPrefixedNativeResource
  if (n.find('/') == std::string::npos) return false;               // IsNativeResource
  if (n.rfind("requests.", 0) == 0) return false;
  return qualified_name_ok("requests." + n);                        // IsExtendedResourceName
}

// Column of an extended resource (created on first sight, at most MAX_XRES).
ks_status xres_column(ks_ctx *c, uint32_t name, bool create, uint32_t *out) {
  auto it = c->xres_of.find(name);
  if (it != c->xres_of.end()) {
    *out = it->second;
    return KS_OK;
  }
  if (!create) {
    *out = UINT32_MAX;
    return KS_OK;
  }
  if (c->undrained) return KS_NEED_DRAIN;
  if (c->xres_names.size() >= (size_t)MAX_XRES)
    return c->fail(KS_ERR_UNSUPPORTED, "more than %d extended resource names (%s)", MAX_XRES, c->strs[name].c_str());
  if (!c->d_xalloc) {
    const size_t n = (size_t)MAX_XRES * c->npos;
    HIPC(c, hipMalloc((void **)&c->d_xalloc, 2 * n * 8));
    HIPC(c, hipMemsetAsync(c->d_xalloc, 0, 2 * n * 8, c->stream));
    c->d_xreq = c->d_xalloc + n;
  }
  *out = (uint32_t)c->xres_names.size();
  c->xres_of.emplace(name, *out);
  c->xres_names.push_back(name);
  return KS_OK;
}

// col[idx] = val (add: col[idx] += val) over the extended-resource columns
// (d_xalloc, then d_xreq at MAX_XRES * npos).
ks_status xres_scatter(ks_ctx *c, const std::vector<uint64_t> &idx, const std::vector<int64_t> &val, bool add) {
  if (idx.empty()) return KS_OK;
  const size_t bytes = idx.size() * 16 + 1024;
  ks_status st = xfer_begin(c, bytes, bytes);
  if (st) return st;
  uint64_t *d_idx = dscratch<uint64_t>(c, idx.size());
  int64_t *d_val = dscratch<int64_t>(c, val.size());
  if ((st = h2d(c, d_idx, idx.data(), idx.size() * 8)) || (st = h2d(c, d_val, val.data(), val.size() * 8))) return st;
  HIPC(c, launch_scatter_i64(c->d_xalloc, d_idx, d_val, (uint32_t)idx.size(), add, c->stream));
  return xfer_sync(c);
}

// PodRequests for the extended resources (resourcehelper.PodRequests: the
// containers' sum, init containers' max with sidecars) as (column, value) with
// value > 0.  KS_REQ_HAS_OTHER (a request the caller could not express) is
// refused; names framework.Resource ignores are skipped.
ks_status pod_xrequests(ks_ctx *c, const ks_pod &p, bool create, std::vector<std::pair<uint32_t, int64_t>> *out) {
  out->clear();
  bool any = false;
  auto scan = [&](const ks_container *cs, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) any |= cs[i].n_extended != 0;
  };
  scan(p.containers, p.n_containers);
  scan(p.init_containers, p.n_init_containers);
  if (!any) return KS_OK;
  std::map<uint32_t, int64_t> sum, side, init;  // by column
  auto each = [&](const ks_container &k, const std::function<ks_status(uint32_t, int64_t)> &f) -> ks_status {
    for (uint32_t j = 0; j < k.n_extended; ++j) {
      const std::string nm = str(k.extended[j].name);
      if (!xres_name_ok(nm)) continue;
      // extended columns are compared in exact int64 (no LeastAllocated
      // floor): any non-negative request, sums checked for overflow below
      if (k.extended[j].value < 0)
        return c->fail(KS_ERR_RANGE, "pod %s: negative %s request", str(p.name).c_str(), nm.c_str());
      uint32_t col;
      if (ks_status st = xres_column(c, c->intern(nm.c_str()), create, &col)) return st;
      if (col == UINT32_MAX) continue;  // ks_pods_check: no column yet (validation only)
      if (ks_status st = f(col, k.extended[j].value)) return st;
    }
    return KS_OK;
  };
  auto add = [&](int64_t &acc, int64_t v) -> ks_status {
    if (__builtin_add_overflow(acc, v, &acc))
      return c->fail(KS_ERR_RANGE, "pod %s: extended resource requests overflow int64", str(p.name).c_str());
    return KS_OK;
  };
  for (uint32_t i = 0; i < p.n_containers; ++i)
    if (ks_status st = each(p.containers[i], [&](uint32_t col, int64_t v) { return add(sum[col], v); }))
      return st;
  for (uint32_t i = 0; i < p.n_init_containers; ++i) {
    const ks_container &k = p.init_containers[i];
    std::map<uint32_t, int64_t> use;
    ks_status st;
    if (k.restart_always) {
      st = each(k, [&](uint32_t col, int64_t v) {
        ks_status e = add(sum[col], v);
        return e ? e : add(side[col], v);
      });
      use = side;
    } else {
      use = side;
      st = each(k, [&](uint32_t col, int64_t v) { return add(use[col], v); });
    }
    if (st) return st;
    for (auto &kv : use) init[kv.first] = std::max(init[kv.first], kv.second);
  }
  for (auto &kv : init) sum[kv.first] = std::max(sum[kv.first], kv.second);
  for (auto &kv : sum)
    if (kv.second > 0) out->emplace_back(kv.first, kv.second);
  return KS_OK;
}

// --------------------------------------------------------------- devices

ks_status upload_dirty_ext(ks_ctx *c, Xfer &x) {
  if (c->dirty_ext.empty()) return KS_OK;
  std::sort(c->dirty_ext.begin(), c->dirty_ext.end());
  c->dirty_ext.erase(std::unique(c->dirty_ext.begin(), c->dirty_ext.end()), c->dirty_ext.end());
  const uint32_t n = (uint32_t)c->dirty_ext.size();
  std::vector<uint32_t> pos(n);
  std::vector<uint64_t> ext((size_t)n * (2 + LW + NNUM));
  for (uint32_t i = 0; i < n; ++i) {
    const HostNode &h = c->nodes[c->dirty_ext[i]];
    pos[i] = c->slot_pos[c->dirty_ext[i]];
    uint64_t *e = &ext[(size_t)i * (2 + LW + NNUM)];
    e[0] = h.hard;
    e[1] = h.prefer;
    for (int k = 0; k < LW; ++k) e[2 + k] = h.lab[k];
    for (int k = 0; k < NNUM; ++k) e[2 + LW + k] = (uint64_t)h.num[k];
  }
  ks_status st = xfer_begin(c, x, n * 4 + ext.size() * 8 + 1024, n * 4 + ext.size() * 8 + 1024);
  if (st) return st;
  uint32_t *d_pos = dscratch<uint32_t>(x, n);
  uint64_t *d_ext = dscratch<uint64_t>(x, ext.size());
  if ((st = h2d(c, x, d_pos, pos.data(), n * 4)) || (st = h2d(c, x, d_ext, ext.data(), ext.size() * 8))) return st;
  HIPC(c, launch_scatter_rows(c->t, d_pos, nullptr, d_ext, n, 2u, x.st));
  if ((st = xfer_sync(c, x))) return st;
  c->dirty_ext.clear();
  return KS_OK;
}

template <class T>
ks_status dalloc(ks_ctx *c, T **p, size_t count) {
  HIPC(c, hipMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T)));
  HIPC(c, hipMemsetAsync(*p, 0, std::max<size_t>(count, 1) * sizeof(T), c->stream));
  return KS_OK;
}

uint32_t blocks_per_shard(const Shard &s, uint32_t sub) { return (s.waves * sub + 3) / 4; }

// Sweep / prescore kernel width: fewer nodes per lane when label/taint
// columns are held too (register budget).
uint32_t kernel_npl(const ks_ctx *c, bool ext) {
  return ext ? std::min<uint32_t>(c->npl, c->ext_npl) : c->npl;
}


// ====================================================== PodTopologySpread
// Host side of the spread path (ksched_spread.hip): label sets of bound pods,
// selector classes, topology-key domain columns, and the compilation of a
// pod's constraints (upstream podtopologyspread/common.go
// #filterTopologySpreadConstraints, LabelSelectorAsSelector,
// mergeLabelSetWithSelector).

ks_status term_get(ks_ctx *c, const ks_pod &p, const ks_pod_affinity_term &t, bool create, uint32_t *out);
bool term_valid(const ks_pod_affinity_term &t);

void term_activate(ks_ctx *c, uint32_t tc, int64_t bound_delta, int32_t refs_delta);

// Interned (namespace, labels, namespace labels, own affinity terms) of a
// pod; creates the term classes of its terms (invalid terms are dropped, as
// the oracle's cache does) and holds each (a reference in `hold`, released by
// the caller) so that no later term class creation reuses its slot.
ks_status intern_set(ks_ctx *c, const ks_pod &p, uint32_t *out, std::vector<uint32_t> *hold) {
  const bool plain = p.n_namespace_labels == 0 && p.n_affinity_terms == 0;
  if (plain && p.n_labels == 0) {  // the common case: one lookup by namespace
    auto it = c->empty_set_of_ns.find(str(p.ns));
    if (it != c->empty_set_of_ns.end()) {
      *out = it->second;
      return KS_OK;
    }
  }
  std::vector<std::pair<uint32_t, uint32_t>> l;
  l.reserve(p.n_labels);
  for (uint32_t k = 0; k < p.n_labels; ++k) l.emplace_back(c->intern(p.labels[k].key), c->intern(p.labels[k].value));
  std::sort(l.begin(), l.end());
  const uint32_t ns = c->intern(p.ns);
  if (plain) {
    auto key = std::make_pair(ns, std::move(l));
    auto it = c->set_ids.find(key);
    if (it != c->set_ids.end()) {
      *out = it->second;
      return KS_OK;
    }
    const uint32_t id = (uint32_t)c->label_sets.size();
    c->label_sets.push_back(LabelSet{key.first, key.second, {}, {}, {}});
    c->set_ids.emplace(std::move(key), id);
    if (p.n_labels == 0) c->empty_set_of_ns.emplace(str(p.ns), id);
    *out = id;
    return KS_OK;
  }
  std::vector<std::pair<uint32_t, uint32_t>> nl;
  for (uint32_t k = 0; k < p.n_namespace_labels; ++k)
    nl.emplace_back(c->intern(p.namespace_labels[k].key), c->intern(p.namespace_labels[k].value));
  std::sort(nl.begin(), nl.end());
  std::vector<std::pair<uint32_t, uint32_t>> terms;
  for (uint32_t k = 0; k < p.n_affinity_terms; ++k) {
    uint32_t t;
    if (!term_valid(p.affinity_terms[k])) continue;
    const ks_status st = term_get(c, p, p.affinity_terms[k], true, &t);
    if (st == KS_ERR_UNSUPPORTED) continue;  // selector parse error
    if (st) return st;
    term_activate(c, t, 0, +1);
    hold->push_back(t);
    terms.emplace_back(t, p.affinity_terms[k].kind >= KS_POD_AFFINITY_PREFERRED ? (uint32_t)p.affinity_terms[k].weight : 1u);
  }
  std::string key = std::to_string(ns);
  for (auto &kv : l) key += '|' + std::to_string(kv.first) + '=' + std::to_string(kv.second);
  key += "#";
  for (auto &kv : nl) key += '|' + std::to_string(kv.first) + '=' + std::to_string(kv.second);
  key += "#";
  for (auto &t : terms) key += ',' + std::to_string(t.first) + '*' + std::to_string(t.second);
  auto it = c->set_of_key.find(key);
  if (it != c->set_of_key.end()) {
    *out = it->second;
    return KS_OK;  // same term classes: held above
  }
  const uint32_t id = (uint32_t)c->label_sets.size();
  c->label_sets.push_back(LabelSet{ns, std::move(l), std::move(nl), std::move(terms), key});
  c->set_of_key.emplace(std::move(key), id);
  *out = id;
  return KS_OK;
}

// Apply the pending records of batch-bound pods to the nodes (before a
// reader: class creation, pod removal, node deletion).
void flush_bound(ks_ctx *c) {
  for (auto &b : c->pending_bound) {
    std::vector<uint32_t> &v = c->nodes[b.slot].pod_sets;
    if (b.op > 0) {
      v.push_back(b.set);
      c->label_sets[b.set].ever_bound = true;
    } else if (b.op < 0) {
      auto it = std::find(v.begin(), v.end(), b.set);
      if (it != v.end()) {  // never bound here: nothing to remove
        *it = v.back();     // a multiset: order is immaterial
        v.pop_back();
      }
    } else {
      v.clear();
    }
  }
  c->pending_bound.clear();
}

// Nothing reads the per-node pod records: no live selector class, no term class.
bool pod_records_unread(const ks_ctx *c) {
  if (c->n_terms) return false;
  for (int k = 0; k < MAX_CLASSES; ++k)
    if (c->classes[k].live) return false;
  return true;
}

// labels.Selector.Matches over sorted (key, value) ids.
bool reqs_match(const std::vector<SelReq> &reqs, const std::vector<std::pair<uint32_t, uint32_t>> &labels) {
  for (const SelReq &r : reqs) {
    auto it = std::lower_bound(labels.begin(), labels.end(), std::make_pair(r.key, 0u));
    const bool has = it != labels.end() && it->first == r.key;
    const bool in = has && std::binary_search(r.vals.begin(), r.vals.end(), it->second);
    switch (r.op) {
      case KS_OP_IN: if (!in) return false; break;
      case KS_OP_NOT_IN: if (in) return false; break;
      case KS_OP_EXISTS: if (!has) return false; break;
      default: if (has) return false; break;  // DoesNotExist
    }
  }
  return true;
}

// framework.AffinityTerm.Matches (namespace listed or selected, then the
// selector) of one clause.
bool clause_match(const Clause &k, uint32_t ns, const std::vector<std::pair<uint32_t, uint32_t>> &labels,
                  const std::vector<std::pair<uint32_t, uint32_t>> &ns_labels) {
  if (!std::binary_search(k.nss.begin(), k.nss.end(), ns) && !(k.ns_sel_set && reqs_match(k.ns_sel, ns_labels)))
    return false;
  return !k.sel_nothing && reqs_match(k.sel, labels);
}

void reqs_canon(std::string &s, const std::vector<SelReq> &reqs) {
  for (auto &r : reqs) {
    s += '|' + std::to_string(r.key) + ':' + std::to_string(r.op);
    for (uint32_t v : r.vals) s += ',' + std::to_string(v);
  }
}
std::string clause_canon(const Clause &k) {
  std::string s = "N";
  for (uint32_t n : k.nss) s += ',' + std::to_string(n);
  if (k.ns_sel_set) {
    s += "S";
    reqs_canon(s, k.ns_sel);
  }
  if (k.sel_nothing) s += "L-";
  else {
    s += "L";
    reqs_canon(s, k.sel);
  }
  return s;
}

bool class_matches(const ks_ctx *c, const SpreadClass &k, uint32_t set) {
  const LabelSet &ls = c->label_sets[set];
  for (const Clause &cl : k.clauses)
    if (!clause_match(cl, ls.ns, ls.labels, ls.ns_labels)) return false;
  return true;
}

ks_status spread_scratch(ks_ctx *c, uint32_t need) {
  if (need <= c->dom_cap) return KS_OK;
  // callers have drained every submitted batch (hipFree waits for the device)
  if (ks_status e_ = sync_bounded(c, c->stream, __func__)) return e_;
  if (c->d_dcnt) (void)hipFree(c->d_dcnt);
  if (c->d_dflag) (void)hipFree(c->d_dflag);
  if (c->d_adcnt) (void)hipFree(c->d_adcnt);
  c->d_dcnt = c->d_dflag = c->d_adcnt = nullptr;
  const uint32_t cap = std::max<uint32_t>({need, 2 * c->dom_cap, 1024});
  ks_status st;
  if ((st = dalloc(c, &c->d_dcnt, (size_t)MAX_SPREAD * cap)) || (st = dalloc(c, &c->d_dflag, (size_t)MAX_SPREAD * cap)) ||
      (st = dalloc(c, &c->d_adcnt, (size_t)MAX_AFF * cap)))
    return st;
  c->dom_cap = cap;
  return KS_OK;
}

// slots per list / feasible count of the window pass (ksched_spread.hip WIN_CHUNK)
constexpr size_t WIN_CHUNK_SLOTS = 1024;

ks_status spread_alloc(ks_ctx *c) {
  if (c->d_dom) return KS_OK;
  if (c->undrained) return KS_NEED_DRAIN;
  ks_status st;
  // domain columns then class columns, one allocation (one index space for scatters)
  if ((st = dalloc(c, &c->d_dom, (size_t)(MAX_TOPO_KEYS + MAX_CLASSES) * c->npos)) || (st = dalloc(c, &c->d_pos_slot, c->npos)) ||
      (st = dalloc(c, &c->d_acc, 1)) || (st = dalloc(c, &c->d_sst, c->npos)) || (st = dalloc(c, &c->d_sraw, c->npos)) ||
      (st = dalloc(c, &c->d_spart, c->npos)) || (st = dalloc(c, &c->d_sraw2, c->npos)))
    return st;
  if (c->pct != 100) {
    const size_t pieces = ((size_t)c->cap + WIN_CHUNK_SLOTS - 1) / WIN_CHUNK_SLOTS;
    if ((st = dalloc(c, &c->d_win, WIN_WORDS + 2 * pieces)) ||
        (st = dalloc(c, &c->d_win_st, ((size_t)c->cap + 15) & ~(size_t)15)))  // 16-byte loads
      return st;
  }
  c->d_cnt = c->d_dom + (size_t)MAX_TOPO_KEYS * c->npos;
  HIPC(c, hipMemsetAsync(c->d_dom, 0xFF, (size_t)MAX_TOPO_KEYS * c->npos * 4, c->stream));
  std::vector<uint32_t> ps(c->npos, SLOT_NONE);
  for (uint32_t sl = 0; sl < c->cap; ++sl) ps[c->slot_pos[sl]] = sl;
  SpreadAcc acc{};
  for (int k = 0; k < MAX_SPREAD; ++k) acc.min_match[k] = 0xFFFFFFFFu;
  for (int k = 0; k < ACC_SHARDS; ++k) acc.sh[k].pts_min = acc.sh[k].ipa_min = ~0ull;
  if ((st = xfer_begin(c, (size_t)c->npos * 4 + sizeof acc + 1024, 0)) ||
      (st = h2d(c, c->d_pos_slot, ps.data(), (size_t)c->npos * 4)) || (st = h2d(c, c->d_acc, &acc, sizeof acc)) ||
      (st = xfer_sync(c)))
    return st;
  return spread_scratch(c, 1024);
}

// Domain id of a node for one topology key (DOM_NONE: no such label; the value
// "" is domain 0); new values get the next id.
uint32_t node_domain(TopoKey &k, const HostNode &h) {
  for (auto &kv : h.labels) {
    if (kv.first != k.key) continue;
    if (kv.second == 0) return 0;
    auto it = k.dom.find(kv.second);
    if (it != k.dom.end()) return it->second;
    const uint32_t id = k.ndom++;
    k.dom.emplace(kv.second, id);
    return id;
  }
  return DOM_NONE;
}

// (Re)build topology-key column `ti` from the present nodes.
ks_status topo_build(ks_ctx *c, uint32_t ti) {
  TopoKey &k = c->topo[ti];
  k.dom.clear();
  k.ndom = 1;
  k.slot_dom.assign(c->cap, DOM_NONE);
  k.dom_nodes.clear();
  k.shared = 0;
  std::vector<uint32_t> col(c->npos, DOM_NONE);
  for (uint32_t sl = 0; sl < c->cap; ++sl)
    if (c->nodes[sl].present) {
      col[c->slot_pos[sl]] = node_domain(k, c->nodes[sl]);
      k.place(sl, col[c->slot_pos[sl]]);
    }
  ks_status st;
  if ((st = spread_scratch(c, k.ndom)) || (st = xfer_begin(c, (size_t)c->npos * 4 + 1024, 0)) ||
      (st = h2d(c, c->d_dom + (size_t)ti * c->npos, col.data(), (size_t)c->npos * 4)) || (st = xfer_sync(c)))
    return st;
  return KS_OK;
}

// Column of a topology key (created when `create`; the caller has drained).
ks_status topo_column(ks_ctx *c, uint32_t key, bool create, uint32_t *out) {
  auto it = c->topo_of.find(key);
  if (it != c->topo_of.end()) {
    *out = it->second;
    return KS_OK;
  }
  if (!create) {
    *out = 0;
    return KS_OK;
  }
  if (c->undrained) return KS_NEED_DRAIN;
  if (c->topo.size() >= (size_t)MAX_TOPO_KEYS)
    return c->fail(KS_ERR_CAPACITY, "more than %d topology keys in spread constraints", MAX_TOPO_KEYS);
  ks_status st;
  if ((st = spread_alloc(c))) return st;
  const uint32_t ti = (uint32_t)c->topo.size();
  c->topo.emplace_back();
  c->topo.back().key = key;
  c->topo_of.emplace(key, ti);
  if ((st = topo_build(c, ti))) return st;
  *out = ti;
  return KS_OK;
}

// Selector class of (namespace, requirements): its column counts the bound
// pods of every node that the selector matches (created when `create`, from
// the host's records of bound pods).
ks_status class_get(ks_ctx *c, std::vector<Clause> &&clauses, bool create, uint32_t *out) {
  std::string canon;
  for (const Clause &k : clauses) canon += clause_canon(k) + ';';
  auto it = c->class_of.find(canon);
  if (it != c->class_of.end()) {
    *out = it->second;
    c->classes[it->second].last_use = ++c->class_seq;
    return KS_OK;
  }
  if (!create) {
    *out = CLS_NONE;
    return KS_OK;
  }
  // With batches in flight (undrained), only a class no bound pod matches
  // so far (a new deployment's selector) is created: its column starts at
  // zero, and each batch whose class masks predate it adds the pods it bound
  // at the end of its run (run_batch); no running batch's commits may touch
  // the slot (a free one, or one whose last holder has ended).  Otherwise the
  // caller drains and compiles again.
  ks_status st;
  if ((st = spread_alloc(c))) return st;
  flush_bound(c);  // the column counts every bound pod
  SpreadClass nk;
  nk.live = true;
  nk.clauses = std::move(clauses);
  nk.canon = canon;
  // the label sets the selector matches; none that a bound pod ever carried
  // (a new deployment's selector): the column is zero, no walk over the nodes
  std::vector<int8_t> match(c->label_sets.size(), 0);
  bool any = false;
  for (uint32_t set = 0; set < match.size(); ++set) {
    match[set] = class_matches(c, nk, set) ? 1 : 0;
    any |= match[set] && c->label_sets[set].ever_bound;
  }
  if (c->undrained && any) return KS_NEED_DRAIN;
  int slot = -1;
  for (int k = 0; k < MAX_CLASSES && slot < 0; ++k)
    if (!c->classes[k].live) slot = k;
  if (slot < 0) {  // evict the least recently used class no prepared batch references
    uint64_t best = UINT64_MAX;
    for (int k = 0; k < MAX_CLASSES; ++k)
      if (c->classes[k].refs == 0 && c->classes[k].last_use < best &&
          (!c->undrained || c->classes[k].held <= c->runs_done)) {
        best = c->classes[k].last_use;
        slot = k;
      }
    if (slot < 0) {
      if (c->undrained) return KS_NEED_DRAIN;
      return c->fail(KS_ERR_CAPACITY, "%d spread selector classes referenced by prepared batches", MAX_CLASSES);
    }
    c->class_of.erase(c->classes[slot].canon);
  }
  SpreadClass &k = c->classes[slot];
  k = std::move(nk);
  k.last_use = ++c->class_seq;
  k.born = ++c->class_epoch;
  if (c->undrained) c->stats.classes_inflight++;
  c->class_of.emplace(canon, (uint32_t)slot);
  if (!any) {
    HIPC(c, hipMemsetAsync(c->d_cnt + (size_t)slot * c->npos, 0, (size_t)c->npos * 4, c->stream));
    *out = (uint32_t)slot;
    return KS_OK;
  }
  std::vector<uint32_t> col(c->npos, 0);
  for (uint32_t sl = 0; sl < c->cap; ++sl) {
    const HostNode &h = c->nodes[sl];
    if (!h.present) continue;
    uint32_t n = 0;
    for (uint32_t set : h.pod_sets) n += (uint32_t)match[set];
    col[c->slot_pos[sl]] = n;
  }
  if ((st = xfer_begin(c, (size_t)c->npos * 4 + 1024, 0)) ||
      (st = h2d(c, c->d_cnt + (size_t)slot * c->npos, col.data(), (size_t)c->npos * 4)) || (st = xfer_sync(c)))
    return st;
  *out = (uint32_t)slot;
  return KS_OK;
}

// A prepared batch's hold on a selector class (no eviction until ks_batch_free);
// taken as soon as the class is looked up, so that later pods of the same
// batch cannot evict it.
void class_hold(ks_ctx *c, std::vector<uint32_t> *refs, uint32_t k) {
  if (k == CLS_NONE) return;
  refs->push_back(k);
  c->classes[k].refs++;
}
void class_release(ks_ctx *c, std::vector<uint32_t> *refs) {
  for (uint32_t k : *refs)
    if (c->classes[k].refs) c->classes[k].refs--;
  refs->clear();
}

// metav1.LabelSelectorAsSelector: false on a parse error.
bool parse_label_selector(ks_ctx *c, const ks_label_selector &ls, std::vector<SelReq> *reqs) {
  auto add = [&](const char *key, int32_t op, const char *const *vals, uint32_t nv) {
    const std::string k = str(key);
    if (!qualified_name_ok(k)) return false;
    if ((op == KS_OP_IN || op == KS_OP_NOT_IN) && nv == 0) return false;
    if ((op == KS_OP_EXISTS || op == KS_OP_DOES_NOT_EXIST) && nv != 0) return false;
    SelReq r{c->intern(key), op, {}};
    for (uint32_t i = 0; i < nv; ++i) {
      if (!label_value_ok(str(vals[i]))) return false;
      r.vals.push_back(c->intern(vals[i]));
    }
    std::sort(r.vals.begin(), r.vals.end());
    r.vals.erase(std::unique(r.vals.begin(), r.vals.end()), r.vals.end());
    reqs->push_back(std::move(r));
    return true;
  };
  for (uint32_t i = 0; i < ls.n_match_labels; ++i) {
    const char *v = ls.match_labels[i].value;
    if (!add(ls.match_labels[i].key, KS_OP_IN, &v, 1)) return false;  // selection.Equals
  }
  for (uint32_t i = 0; i < ls.n_match_expressions; ++i) {
    const ks_requirement &e = ls.match_expressions[i];
    if (e.op != KS_OP_IN && e.op != KS_OP_NOT_IN && e.op != KS_OP_EXISTS && e.op != KS_OP_DOES_NOT_EXIST)
      return false;  // "is not a valid label selector operator"
    if (!add(e.key, e.op, e.values, e.n_values)) return false;
  }
  std::sort(reqs->begin(), reqs->end(), [](const SelReq &a, const SelReq &b) {
    return std::tie(a.key, a.op, a.vals) < std::tie(b.key, b.op, b.vals);
  });
  reqs->erase(std::unique(reqs->begin(), reqs->end(),
                          [](const SelReq &a, const SelReq &b) {
                            return a.key == b.key && a.op == b.op && a.vals == b.vals;
                          }),
              reqs->end());
  return true;
}

// framework/types.go#newAffinityTerm of one of pod p's terms: namespaces
// listed, else the pod's own when the namespace selector is nil; nil
// selectors are Nothing().  False on a parse error or an invalid term (the
// apiserver would reject it).
bool term_clause(ks_ctx *c, const ks_pod &p, const ks_pod_affinity_term &t, Clause *out) {
  Clause k;
  for (uint32_t i = 0; i < t.n_namespaces; ++i) k.nss.push_back(c->intern(t.namespaces[i]));
  if (k.nss.empty() && t.namespace_selector.is_nil) k.nss.push_back(c->intern(p.ns));
  std::sort(k.nss.begin(), k.nss.end());
  k.nss.erase(std::unique(k.nss.begin(), k.nss.end()), k.nss.end());
  k.ns_sel_set = !t.namespace_selector.is_nil;
  if (k.ns_sel_set && !parse_label_selector(c, t.namespace_selector, &k.ns_sel)) return false;
  k.sel_nothing = t.selector.is_nil != 0;
  if (!k.sel_nothing && !parse_label_selector(c, t.selector, &k.sel)) return false;
  *out = std::move(k);
  return true;
}

bool term_valid(const ks_pod_affinity_term &t) {
  if (!t.topology_key || !t.topology_key[0] || t.kind < KS_POD_AFFINITY_REQUIRED || t.kind > KS_POD_ANTI_AFFINITY_PREFERRED)
    return false;
  if (t.kind >= KS_POD_AFFINITY_PREFERRED && (t.weight < 1 || t.weight > 100)) return false;
  return true;
}

// Term class of one of a bound (or to-be-bound) pod's terms, created when
// `create` (its column starts at zero: no pod carrying it is bound yet).
// Classes no pod carries (bound or prepared) are reused when the table is full.
ks_status term_get(ks_ctx *c, const ks_pod &p, const ks_pod_affinity_term &t, bool create, uint32_t *out) {
  Clause k;
  if (!term_valid(t) || !term_clause(c, p, t, &k))
    return c->fail(KS_ERR_UNSUPPORTED, "pod %s/%s: invalid pod (anti-)affinity term", str(p.ns).c_str(),
                   str(p.name).c_str());
  const uint32_t key = c->intern(t.topology_key);
  // preferred terms of any weight share a class: its column sums the weights
  const std::string canon = std::to_string(t.kind) + '/' + std::to_string(key) + '/' + clause_canon(k);
  auto it = c->term_of.find(canon);
  if (it != c->term_of.end()) {
    *out = it->second;
    return KS_OK;
  }
  if (!create) {
    *out = UINT32_MAX;
    return KS_OK;
  }
  if (c->undrained) return KS_NEED_DRAIN;
  int slot = -1;
  for (int i = 0; i < MAX_TERM_CLASSES && slot < 0; ++i)
    if (!c->terms[i].live) slot = i;
  for (int i = 0; i < MAX_TERM_CLASSES && slot < 0; ++i)
    if (c->terms[i].bound == 0 && c->terms[i].refs == 0) {
      slot = i;
      c->term_of.erase(c->terms[i].canon);
      // label sets of pods carrying the old term (none bound or prepared) are
      // retired: a new such pod interns a fresh set
      for (LabelSet &ls : c->label_sets)
        if (std::any_of(ls.terms.begin(), ls.terms.end(), [&](const std::pair<uint32_t, uint32_t> &x) {
              return x.first == (uint32_t)i;
            })) {
          c->set_of_key.erase(ls.key);
          ls.terms.clear();
          ls.key.clear();
        }
    }
  if (slot < 0) return c->fail(KS_ERR_CAPACITY, "more than %d distinct pod (anti-)affinity terms", MAX_TERM_CLASSES);
  ks_status st;
  if ((st = spread_alloc(c))) return st;
  if ((uint32_t)slot >= c->tcnt_cap) {  // grow the columns (callers have drained)
    const uint32_t cap = std::min<uint32_t>(MAX_TERM_CLASSES, std::max<uint32_t>({16, 2 * c->tcnt_cap, (uint32_t)slot + 1}));
    uint32_t *nt = nullptr;
    if ((st = dalloc(c, &nt, (size_t)cap * c->npos))) return st;
    if (c->d_tcnt) {
      HIPC(c, hipMemcpyAsync(nt, c->d_tcnt, (size_t)c->tcnt_cap * c->npos * 4, hipMemcpyDeviceToDevice, c->stream));
      if (ks_status e_ = sync_bounded(c, c->stream, __func__)) return e_;
      (void)hipFree(c->d_tcnt);
    }
    c->d_tcnt = nt;
    c->tcnt_cap = cap;
  }
  uint32_t col;
  if ((st = topo_column(c, key, true, &col))) return st;
  TermClass &tc = c->terms[slot];
  tc = TermClass{};
  tc.live = true;
  tc.kind = t.kind;
  tc.key = key;
  tc.clause = std::move(k);
  tc.canon = canon;
  c->term_of.emplace(canon, (uint32_t)slot);
  c->n_terms = std::max<uint32_t>(c->n_terms, (uint32_t)slot + 1);
  *out = (uint32_t)slot;
  return KS_OK;
}

// A term class gains its first carrier: pods compiled before saw no such term
// (prepared batches go stale).
void term_activate(ks_ctx *c, uint32_t tc, int64_t bound_delta, int32_t refs_delta) {
  TermClass &t = c->terms[tc];
  const bool was = t.active();
  t.bound += bound_delta;
  t.refs += refs_delta;
  if (!was && t.active()) c->dict_version++;
}

// Interned, sorted labels and namespace labels of a pod.
void pod_label_ids(ks_ctx *c, const ks_pod &p, std::vector<std::pair<uint32_t, uint32_t>> *l,
                   std::vector<std::pair<uint32_t, uint32_t>> *nl) {
  for (uint32_t k = 0; k < p.n_labels; ++k) l->emplace_back(c->intern(p.labels[k].key), c->intern(p.labels[k].value));
  for (uint32_t k = 0; k < p.n_namespace_labels; ++k)
    nl->emplace_back(c->intern(p.namespace_labels[k].key), c->intern(p.namespace_labels[k].value));
  std::sort(l->begin(), l->end());
  std::sort(nl->begin(), nl->end());
}

// Whether some bound (or prepared) pod's term selects the pod: InterPodAffinity
// then filters (existing anti-affinity) or scores it.
bool matched_by_terms(ks_ctx *c, const ks_pod &p) {
  bool any = false;
  for (uint32_t t = 0; t < c->n_terms && !any; ++t) any = c->terms[t].active();
  if (!any) return false;
  std::vector<std::pair<uint32_t, uint32_t>> l, nl;
  pod_label_ids(c, p, &l, &nl);
  const uint32_t ns = c->intern(p.ns);
  for (uint32_t t = 0; t < c->n_terms; ++t)
    if (c->terms[t].active() && clause_match(c->terms[t].clause, ns, l, nl)) return true;
  return false;
}

// Whether compiling the pod may create one-pod-path state (columns, label
// bits, device buffers): ks_batch_prepare drains the submitted batches first.
bool may_need_solo(ks_ctx *c, const ks_pod &p) {
  if (p.n_spread || p.n_affinity_terms || c->pct != 100) return true;
  if (matched_by_terms(c, p)) return true;
  for (uint32_t i = 0; i < p.n_containers; ++i)
    if (p.containers[i].n_extended || (!c->images.empty() && p.containers[i].image && p.containers[i].image[0]))
      return true;
  for (uint32_t i = 0; i < p.n_init_containers; ++i)
    if (p.init_containers[i].n_extended ||
        (!c->images.empty() && p.init_containers[i].image && p.init_containers[i].image[0]))
      return true;
  return false;
}

// InterPodAffinity records of a pod (ksched_dev.hpp AffDev): its own required
// affinity terms (one selector class of all of them: affinityCounts counts
// pods matching every term), required anti-affinity and preferred terms (one
// class each), the bound pods' term classes that match it (existing
// anti-affinity; hardPodAffinityWeight x required and weighted preferred
// terms for the score), and its own term classes (counted on commit).
ks_status ipa_compile(ks_ctx *c, const ks_pod &p, bool create, std::vector<uint32_t> *refs, std::vector<AffDev> *out,
                      uint32_t *flags) {
  const std::string pn = str(p.ns) + "/" + str(p.name);
  ks_status st;
  std::vector<std::pair<uint32_t, uint32_t>> l, nl;
  pod_label_ids(c, p, &l, &nl);
  const uint32_t ns = c->intern(p.ns);
  std::vector<Clause> req_aff;
  std::vector<uint32_t> req_keys;
  for (uint32_t k = 0; k < p.n_affinity_terms; ++k) {
    const ks_pod_affinity_term &t = p.affinity_terms[k];
    Clause cl;
    if (!term_valid(t) || !term_clause(c, p, t, &cl))
      return c->fail(KS_ERR_UNSUPPORTED, "pod %s: pod (anti-)affinity term %u is invalid", pn.c_str(), k);
    uint32_t kc;
    if ((st = topo_column(c, c->intern(t.topology_key), create, &kc))) return st;
    if (t.kind == KS_POD_AFFINITY_REQUIRED) {
      req_aff.push_back(std::move(cl));
      req_keys.push_back(kc);
      continue;
    }
    std::vector<Clause> one(1, std::move(cl));
    uint32_t col;
    if ((st = class_get(c, std::move(one), create, &col))) return st;
    if (create && refs) class_hold(c, refs, col);
    const int32_t w = t.kind == KS_POD_AFFINITY_PREFERRED ? t.weight : -t.weight;
    out->push_back(AffDev{kc, col, t.kind == KS_POD_ANTI_AFFINITY_REQUIRED ? (uint32_t)AF_REQ_ANTI : (uint32_t)AF_SCORE,
                          t.kind == KS_POD_ANTI_AFFINITY_REQUIRED ? 0 : w});
  }
  if (!req_aff.empty()) {
    bool self = true;  // podMatchesAllAffinityTerms(terms, pod)
    for (const Clause &cl : req_aff) self = self && clause_match(cl, ns, l, nl);
    if (self) *flags |= AFF_SELF;
    uint32_t col;
    if ((st = class_get(c, std::move(req_aff), create, &col))) return st;
    if (create && refs) class_hold(c, refs, col);
    for (uint32_t kc : req_keys) out->push_back(AffDev{kc, col, AF_REQ_AFF, 0});
  }
  for (uint32_t t = 0; t < c->n_terms; ++t) {
    const TermClass &tc = c->terms[t];
    if (!tc.active() || !clause_match(tc.clause, ns, l, nl)) continue;
    uint32_t kc;
    if ((st = topo_column(c, tc.key, create, &kc))) return st;
    if (tc.kind == KS_POD_ANTI_AFFINITY_REQUIRED) out->push_back(AffDev{kc, t, AF_EXIST_ANTI | AF_TERM, 0});
    else if (tc.kind == KS_POD_AFFINITY_REQUIRED) {
      if (c->cfg.hard_pod_affinity_weight > 0)
        out->push_back(AffDev{kc, t, AF_SCORE | AF_TERM, c->cfg.hard_pod_affinity_weight});
    } else {
      out->push_back(AffDev{kc, t, AF_SCORE | AF_TERM, tc.kind == KS_POD_AFFINITY_PREFERRED ? 1 : -1});
    }
  }
  if (create)  // the pod's own term classes (ks_batch_prepare interned them)
    for (uint32_t k = 0; k < p.n_affinity_terms; ++k) {
      uint32_t t;
      if ((st = term_get(c, p, p.affinity_terms[k], false, &t))) return st;
      const ks_pod_affinity_term &tm = p.affinity_terms[k];
      if (t != UINT32_MAX)
        out->push_back(AffDev{0, t, AF_OWN | AF_TERM, tm.kind >= KS_POD_AFFINITY_PREFERRED ? tm.weight : 1});
    }
  if (out->size() > (size_t)MAX_AFF)
    return c->fail(KS_ERR_UNSUPPORTED, "pod %s: more than %d pod (anti-)affinity records (own and matching terms)",
                   pn.c_str(), MAX_AFF);
  if (create)  // keys whose every domain is one node (hostnames): per-node records
    for (AffDev &r : *out) {
      const uint32_t kind = r.kind & AF_KIND;
      if (kind != AF_REQ_AFF && kind != AF_OWN && r.key < c->topo.size() && c->topo[r.key].shared == 0)
        r.kind |= AF_NODE;
    }
  return KS_OK;
}

// Passes of the spread chain a one-pod program needs (SpreadLaunch).
uint32_t solo_passes(const SoloHdr *hd) {
  const SpreadDev *sd = reinterpret_cast<const SpreadDev *>(hd + 1);
  uint32_t f = 0;
  for (uint32_t k = 0; k < hd->n_spread; ++k) f |= (sd[k].flags & SP_SCORE) ? SPL_SCORE : (SPL_PREP | SPL_MIN);
  const AffDev *ad = reinterpret_cast<const AffDev *>(reinterpret_cast<const uint8_t *>(sd + hd->n_spread) +
                                                      hd->n_xres * sizeof(XResDev) + hd->n_img * sizeof(ImageDev));
  for (uint32_t k = 0; k < hd->n_aff; ++k)
    if ((ad[k].kind & AF_KIND) != AF_OWN && !(ad[k].kind & AF_NODE)) f |= SPL_PREP;
  if (hd->n_aff) f |= SPL_AFF;  // the filter variant that reads the records
  return f;
}

// Replica runs: the run kernel models a one-pod program with at
// most one kubernetes.io/hostname constraint (ScheduleAnyway) and one on
// another key, and no InterPodAffinity, extended-resource or image records.  The inclusion policies need no check: PreScore's per-node
// nodeAffinityPolicy / nodeTaintsPolicy tests pass on every node a pod can be
// committed to (a feasible node matches the pod's required affinity and
// tolerates its hard taints).
// Since round 6 the other key's constraint may be DoNotSchedule: the run
// then blocks and unblocks whole domains as their counts and the minimum
// move, for pods without a normalised TaintToleration / NodeAffinity score
// (those maxima range over the feasible nodes, which change in such a run).
bool replica_program(const PodDev &p, const SoloHdr *hd) {
  if (hd->n_spread == 0 || hd->n_aff || hd->n_xres || hd->n_img || (p.flags & PF_PREF_ERR)) return false;
  const SpreadDev *sd = reinterpret_cast<const SpreadDev *>(hd + 1);
  uint32_t host = 0, other = 0;
  bool dns = false;
  for (uint32_t k = 0; k < hd->n_spread; ++k) {
    const bool h = sd[k].flags & SP_HOST;
    if (!(sd[k].flags & SP_SCORE)) {
      if (h) return false;
      dns = true;
    }
    ++(h ? host : other);
  }
  if (dns && (p.flags & (PF_TT | PF_NA))) return false;
  return host <= 1 && other <= 1;
}

// Words of a label program of `terms` terms at `off` (ksched_dev.hpp layout).
size_t program_words(const uint64_t *w, uint32_t off, uint32_t terms) {
  size_t n = 0;
  for (uint32_t k = 0; k < terms; ++k) n += term_words(w[off + n]);
  return n;
}

// Two compiled pods the kernels cannot tell apart: equal descriptors up to
// the program offsets, equal programs (required / preferred / prefilter /
// one-pod records).  Their labels (class masks) are compared by the caller.
bool same_pod_program(const PodDev &a, const PodDev &b, const uint64_t *w) {
  PodDev x = a, y = b;
  x.req_off = y.req_off = x.pref_off = y.pref_off = x.solo_off = y.solo_off = x.pre_off = y.pre_off = 0;
  if (std::memcmp(&x, &y, sizeof x) != 0) return false;
  auto same = [&](uint32_t oa, uint32_t ob, size_t n) { return std::memcmp(w + oa, w + ob, n * 8) == 0; };
  if (!same(a.req_off, b.req_off, program_words(w, a.req_off, a.req_len))) return false;
  if (!same(a.pref_off, b.pref_off, program_words(w, a.pref_off, a.pref_len))) return false;
  if (!same(a.pre_off, b.pre_off, a.pre_len)) return false;
  if (a.flags & PF_SOLO) {
    const SoloHdr *h = reinterpret_cast<const SoloHdr *>(w + a.solo_off);
    const size_t bytes = sizeof(SoloHdr) + h->n_spread * sizeof(SpreadDev) + h->n_xres * sizeof(XResDev) +
                         h->n_img * sizeof(ImageDev) + h->n_aff * sizeof(AffDev);
    if (!same(a.solo_off, b.solo_off, bytes / 8)) return false;
  }
  return true;
}

// The one-pod-path program of a pod (ksched_dev.hpp SoloHdr): its spread
// constraints (SpreadDev), extended-resource requests (XResDev) and the
// ImageLocality terms of its images present on some node (ImageDev).  Pods
// with none of them stay on the round kernels.  Invalid constraints (the
// apiserver would reject them; upstream's PreFilter / PreScore would return
// an Error) are refused with KS_ERR_UNSUPPORTED, so the shim hands the pod to
// upstream.  Without `create` (ks_pods_check) only validates.
ks_status solo_compile(ks_ctx *c, const ks_pod &p, PodDev &d, ProgBuf &cl, bool create,
                       std::vector<uint32_t> *refs) {
  const std::string pn = str(p.ns) + "/" + str(p.name);
  ks_status st;
  std::vector<std::pair<uint32_t, int64_t>> xr;
  if ((st = pod_xrequests(c, p, create, &xr))) return st;
  // imagelocality#sumImageScores: every init and regular container whose
  // (normalised) image some node reports adds scaledImageScore
  std::vector<ImageDev> imgs;
  if (!c->images.empty()) {
    auto scan = [&](const ks_container *cs, uint32_t n) -> ks_status {
      for (uint32_t i = 0; i < n; ++i) {
        if (!cs[i].image || !cs[i].image[0]) continue;
        const std::string nm = normalized_image(cs[i].image);
        auto it = c->images.find(nm);
        if (it == c->images.end()) continue;
        ImageDev g{};
        if (create) {
          if (ks_status e = get_key_bit(c, c->intern(image_key(nm).c_str()), &g.bit)) return e;
        }
        // scaledImageScore: int64(float64(size) * (float64(numNodes) / float64(totalNumNodes)))
        g.scaled = (int64_t)((double)it->second.size * ((double)it->second.nodes / (double)c->n_present));
        imgs.push_back(g);
      }
      return KS_OK;
    };
    if ((st = scan(p.init_containers, p.n_init_containers)) || (st = scan(p.containers, p.n_containers))) return st;
    if (imgs.size() > (size_t)MAX_IMG)
      return c->fail(KS_ERR_UNSUPPORTED, "pod %s: more than %d containers with images present on nodes", pn.c_str(),
                     MAX_IMG);
    if (!imgs.empty()) c->compile_used_names = true;  // the node count enters the scores
  }
  std::vector<AffDev> aff;
  uint32_t aff_flags = 0;
  if (p.n_affinity_terms || c->n_terms) {
    if ((st = ipa_compile(c, p, create, refs, &aff, &aff_flags))) return st;
  }
  // (percentageOfNodesToScore < 100: every pod takes the chain, which holds the window pass)
  if (!p.n_spread && xr.empty() && imgs.empty() && aff.empty() && c->pct == 100) return KS_OK;
  // multi-rank contexts run the one-pod path replicated: every rank holds the
  // whole node table and every commit, so each rank's chain over
  // all positions gives the same result with no exchange
  if (create && (st = spread_alloc(c))) return st;
  if (p.n_spread > (uint32_t)MAX_SPREAD)
    return c->fail(KS_ERR_UNSUPPORTED, "pod %s: more than %d topology spread constraints", pn.c_str(), MAX_SPREAD);
  std::vector<std::pair<uint32_t, uint32_t>> own;  // the pod's labels (selfMatch)
  for (uint32_t k = 0; k < p.n_labels; ++k) own.emplace_back(c->intern(p.labels[k].key), c->intern(p.labels[k].value));
  std::sort(own.begin(), own.end());
  const uint32_t host_key = c->intern("kubernetes.io/hostname");
  std::vector<SpreadDev> recs;
  std::set<std::pair<uint32_t, int32_t>> seen;
  bool any_filter = false, any_score = false;
  for (uint32_t i = 0; i < p.n_spread; ++i) {
    const ks_spread_constraint &sc = p.spread[i];
    const uint32_t key = c->intern(sc.topology_key);
    if (!sc.topology_key || !sc.topology_key[0] || sc.max_skew < 1 ||
        (sc.when_unsatisfiable != KS_DO_NOT_SCHEDULE && sc.when_unsatisfiable != KS_SCHEDULE_ANYWAY) ||
        sc.min_domains < 0 || (sc.min_domains > 0 && sc.when_unsatisfiable != KS_DO_NOT_SCHEDULE) ||
        sc.node_affinity_policy < 0 || sc.node_affinity_policy > 2 || sc.node_taints_policy < 0 ||
        sc.node_taints_policy > 2 || !seen.emplace(key, sc.when_unsatisfiable).second)
      return c->fail(KS_ERR_UNSUPPORTED, "pod %s: topology spread constraint %u is invalid", pn.c_str(), i);
    SpreadDev r{};
    r.max_skew = sc.max_skew;
    r.min_domains = sc.min_domains ? sc.min_domains : 1;
    const bool score = sc.when_unsatisfiable == KS_SCHEDULE_ANYWAY;
    r.flags = (score ? SP_SCORE : 0u) | (key == host_key ? SP_HOST : 0u) |
              (sc.node_affinity_policy != KS_INCLUSION_IGNORE ? SP_AFF : 0u) |
              (sc.node_taints_policy == KS_INCLUSION_HONOR ? SP_TAINT : 0u);
    (score ? any_score : any_filter) = true;
    // selector (+ matchLabelKeys with the pod's own values; Nothing() stays Nothing())
    std::vector<SelReq> reqs;
    const bool nothing = sc.selector.is_nil != 0;
    if (!nothing && !parse_label_selector(c, sc.selector, &reqs))
      return c->fail(KS_ERR_UNSUPPORTED, "pod %s: topology spread constraint %u has an invalid label selector",
                     pn.c_str(), i);
    if (!nothing) {
      for (uint32_t k = 0; k < sc.n_match_label_keys; ++k) {
        const uint32_t mk = c->intern(sc.match_label_keys[k]);
        auto it = std::lower_bound(own.begin(), own.end(), std::make_pair(mk, 0u));
        if (it != own.end() && it->first == mk) reqs.push_back(SelReq{mk, KS_OP_IN, {it->second}});
      }
      std::sort(reqs.begin(), reqs.end(), [](const SelReq &a, const SelReq &b) {
        return std::tie(a.key, a.op, a.vals) < std::tie(b.key, b.op, b.vals);
      });
      reqs.erase(std::unique(reqs.begin(), reqs.end(),
                             [](const SelReq &a, const SelReq &b) {
                               return a.key == b.key && a.op == b.op && a.vals == b.vals;
                             }),
                 reqs.end());
    }
    if (!nothing && reqs_match(reqs, own)) r.flags |= SP_SELF;
    r.cls = CLS_NONE;  // Nothing() matches no pod; Empty() counts 0 (countPodsMatchSelector)
    if (!nothing && !reqs.empty()) {
      std::vector<Clause> cls(1);
      cls[0].nss = {c->intern(p.ns)};
      cls[0].sel = std::move(reqs);
      if ((st = class_get(c, std::move(cls), create, &r.cls))) return st;
      if (create && refs) class_hold(c, refs, r.cls);
    }
    if ((st = topo_column(c, key, create, &r.key))) return st;
    recs.push_back(r);
  }
  if (!create) return KS_OK;
  if (cl.w.size() & 1) cl.w.push_back(0);  // the records are 16-byte aligned
  d.solo_off = (uint32_t)cl.w.size();
  auto emit = [&](const void *rec, size_t bytes) {
    const size_t w0 = cl.w.size();
    cl.w.resize(w0 + bytes / 8);
    std::memcpy(cl.w.data() + w0, rec, bytes);
  };
  const SoloHdr hdr{(uint32_t)recs.size(), (uint32_t)xr.size(), (uint32_t)imgs.size(),
                    p.n_init_containers + p.n_containers, (uint32_t)aff.size(), aff_flags, {0, 0}};
  emit(&hdr, sizeof hdr);
  for (const SpreadDev &r : recs) emit(&r, sizeof r);
  for (auto &x : xr) {
    const XResDev r{x.first, 0, x.second};
    emit(&r, sizeof r);
  }
  for (const ImageDev &g : imgs) emit(&g, sizeof g);
  for (const AffDev &r : aff) emit(&r, sizeof r);
  d.flags |= PF_SOLO | (p.n_spread && !p.spread_defaulted ? PF_SPREAD_ALLKEYS : 0u);
  (void)any_filter;
  (void)any_score;
  return KS_OK;
}

// Device deltas of the selector-class and term-class columns for pods bound /
// removed on slots (sign +1 / -1), and the host records.
ks_status spread_pods_delta(ks_ctx *c, const uint32_t *sets, const uint32_t *slots, uint32_t n, int sign) {
  std::vector<uint64_t> idx, tidx;
  std::vector<int32_t> dv, tdv;
  if (pod_records_unread(c)) {  // log only (flush_bound replays it in order)
    for (uint32_t i = 0; i < n; ++i) c->pending_bound.push_back({slots[i], sets[i], sign});
    return KS_OK;
  }
  flush_bound(c);
  int live[MAX_CLASSES];  // live selector classes (the per-pod loop visits only these)
  int nlive = 0;
  for (int k = 0; k < MAX_CLASSES; ++k)
    if (c->classes[k].live) live[nlive++] = k;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t set = sets[i];
    HostNode &h = c->nodes[slots[i]];
    if (sign > 0) {
      h.pod_sets.push_back(set);
      c->label_sets[set].ever_bound = true;
    } else {
      auto it = std::find(h.pod_sets.begin(), h.pod_sets.end(), set);
      if (it == h.pod_sets.end()) continue;  // never bound here: no count to remove
      *it = h.pod_sets.back();  // a multiset: order is immaterial
      h.pod_sets.pop_back();
    }
    const uint32_t pos = c->slot_pos[slots[i]];
    for (int q = 0; q < nlive; ++q)
      if (const int k = live[q]; class_matches(c, c->classes[k], set)) {
        idx.push_back((uint64_t)k * c->npos + pos);
        dv.push_back(sign);
      }
    for (auto &t : c->label_sets[set].terms) {
      term_activate(c, t.first, sign, 0);
      tidx.push_back((uint64_t)t.first * c->npos + pos);
      tdv.push_back(sign * (int32_t)t.second);
    }
  }
  for (int pass = 0; pass < 2; ++pass) {
    auto &ix = pass ? tidx : idx;
    auto &dx = pass ? tdv : dv;
    if (ix.empty()) continue;
    const size_t bytes = ix.size() * 12 + 1024;
    ks_status st = xfer_begin(c, bytes, bytes);
    if (st) return st;
    uint64_t *d_idx = dscratch<uint64_t>(c, ix.size());
    int32_t *d_dv = dscratch<int32_t>(c, dx.size());
    if ((st = h2d(c, d_idx, ix.data(), ix.size() * 8)) || (st = h2d(c, d_dv, dx.data(), dx.size() * 4))) return st;
    HIPC(c, launch_add_u32(pass ? c->d_tcnt : c->d_cnt, d_idx, d_dv, (uint32_t)ix.size(), c->stream));
    if ((st = xfer_sync(c))) return st;
  }
  return KS_OK;
}

// Topology-key and class columns of nodes upserted (their labels may have
// changed; their bound pods stay) or deleted (pods leave with the node).
ks_status spread_nodes_changed(ks_ctx *c, const uint32_t *slots, uint32_t n, bool deleted) {
  if (!c->d_dom || !n) return KS_OK;
  std::vector<uint64_t> idx;
  std::vector<uint32_t> val;
  std::vector<uint32_t> rebuild;
  for (uint32_t ti = 0; ti < c->topo.size(); ++ti) {
    TopoKey &k = c->topo[ti];
    const bool unique = k.shared == 0;
    for (uint32_t i = 0; i < n; ++i) {
      idx.push_back((uint64_t)ti * c->npos + c->slot_pos[slots[i]]);
      val.push_back(deleted ? DOM_NONE : node_domain(k, c->nodes[slots[i]]));
      k.place(slots[i], val.back());
    }
    if (unique && k.shared) c->dict_version++;  // prepared per-node records no longer hold
    if (k.ndom > 2 * c->cap + 1024) rebuild.push_back(ti);  // churned values: renumber
  }
  if (deleted)
    for (int k = 0; k < MAX_CLASSES; ++k)
      if (c->classes[k].live)
        for (uint32_t i = 0; i < n; ++i) {
          idx.push_back((uint64_t)c->npos * MAX_TOPO_KEYS + (uint64_t)k * c->npos + c->slot_pos[slots[i]]);
          val.push_back(0);
        }
  ks_status st;
  uint32_t need = 0;
  for (auto &k : c->topo) need = std::max(need, k.ndom);
  if ((st = spread_scratch(c, need))) return st;
  if (!idx.empty()) {
    const size_t bytes = idx.size() * 12 + 1024;
    if ((st = xfer_begin(c, bytes, bytes))) return st;
    uint64_t *d_idx = dscratch<uint64_t>(c, idx.size());
    uint32_t *d_val = dscratch<uint32_t>(c, val.size());
    if ((st = h2d(c, d_idx, idx.data(), idx.size() * 8)) || (st = h2d(c, d_val, val.data(), val.size() * 4)))
      return st;
    // one index space: topology columns, then (offset by MAX_TOPO_KEYS columns) class columns
    HIPC(c, launch_scatter_u32(c->d_dom, d_idx, d_val, (uint32_t)idx.size(), c->stream));
    if ((st = xfer_sync(c))) return st;
  }
  if (deleted && c->d_tcnt && c->n_terms) {
    idx.clear();
    val.clear();
    for (uint32_t t = 0; t < c->n_terms; ++t)
      if (c->terms[t].live)
        for (uint32_t i = 0; i < n; ++i) {
          idx.push_back((uint64_t)t * c->npos + c->slot_pos[slots[i]]);
          val.push_back(0);
        }
    if (!idx.empty()) {
      const size_t bytes = idx.size() * 12 + 1024;
      if ((st = xfer_begin(c, bytes, bytes))) return st;
      uint64_t *d_idx = dscratch<uint64_t>(c, idx.size());
      uint32_t *d_val = dscratch<uint32_t>(c, val.size());
      if ((st = h2d(c, d_idx, idx.data(), idx.size() * 8)) || (st = h2d(c, d_val, val.data(), val.size() * 4)))
        return st;
      HIPC(c, launch_scatter_u32(c->d_tcnt, d_idx, d_val, (uint32_t)idx.size(), c->stream));
      if ((st = xfer_sync(c))) return st;
    }
  }
  for (uint32_t ti : rebuild)
    if ((st = topo_build(c, ti))) return st;
  return KS_OK;
}

hipEvent_t get_event(ks_ctx *c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

ks_status collect_timing(ks_ctx *c) {
  for (auto &pr : c->ev_sweep) {
    float ms = 0;
    HIPC(c, hipEventElapsedTime(&ms, pr.first, pr.second));
    c->stats.sweep_ms += ms;
    c->stats.sweep_launches++;
    c->ev_pool.push_back(pr.first);
    c->ev_pool.push_back(pr.second);
  }
  for (auto &pr : c->ev_resolve) {
    float ms = 0;
    HIPC(c, hipEventElapsedTime(&ms, pr.first, pr.second));
    c->stats.resolve_ms += ms;
    c->stats.resolve_launches++;
    c->ev_pool.push_back(pr.first);
    c->ev_pool.push_back(pr.second);
  }
  for (auto &pr : c->ev_spread) {
    float ms = 0;
    HIPC(c, hipEventElapsedTime(&ms, pr.first, pr.second));
    c->stats.spread_ms += ms;
    c->stats.spread_pods_timed++;
    c->ev_pool.push_back(pr.first);
    c->ev_pool.push_back(pr.second);
  }
  for (auto &r : c->ev_runs) {
    float ms = 0;
    HIPC(c, hipEventElapsedTime(&ms, r.e0, r.e1));
    c->stats.spread_ms += ms;
    c->stats.spread_pods_timed += r.pods;
    c->stats.replica_ms += ms;
    c->ev_pool.push_back(r.e0);
    c->ev_pool.push_back(r.e1);
  }
  c->ev_sweep.clear();
  c->ev_resolve.clear();
  c->ev_spread.clear();
  c->ev_runs.clear();
  return KS_OK;
}

// Cross-stream hand-off: `st` signals round number `seq` on flag f (or by the
// event, value_sync = 0); `wt` waits for it.
static ks_status hand_signal(ks_ctx *c, hipStream_t st, int f, hipEvent_t ev, uint32_t seq) {
  if (c->stall_flag == f) {  // ks_debug_stall
    HIPC(c, launch_stall(c->stall_us, st));
    c->stall_flag = -1;
  }
  c->flag_want[f] = seq;
  // with value hand-offs the event is not waited on (drain_rounds waits on
  // ev_res only): skip its marker packet
  if (c->value_sync) HIPC(c, hipStreamWriteValue32(st, c->d_flags + f, seq, 0));
  else HIPC(c, hipEventRecord(ev, st));
  return KS_OK;
}
static ks_status hand_wait(ks_ctx *c, hipStream_t wt, int f, hipEvent_t ev, uint32_t seq) {
  if (c->value_sync) HIPC(c, hipStreamWaitValue32(wt, c->d_flags + f, seq, hipStreamWaitValueGte, 0xFFFFFFFFu));
  else HIPC(c, hipStreamWaitEvent(wt, ev, 0));
  return KS_OK;
}

// ------------------------------------------------------------- collectives
// RCCL when ks_comm_init made a communicator, else the in-process group.

ks_status lg_exchange(ks_ctx *c, LocalGroup::Post p, std::vector<LocalGroup::Post> &out) {
  if (!c->lgroup->exchange(c->cfg.rank, std::move(p), out))
    return c->fail(KS_ERR_COMM, "in-process communicator failed: a peer rank did not arrive within 300 s");
  return KS_OK;
}

// Second rendezvous of a local collective: the stream continues only once
// every peer's copies out of this rank's buffers are done.
ks_status lg_finish(ks_ctx *c, hipStream_t st) {
  HIPC(c, hipEventRecord(c->lg_ev[1], st));
  std::vector<LocalGroup::Post> ps;
  ks_status e = lg_exchange(c, {c->lg_ev[1], nullptr, {}}, ps);
  if (e) return e;
  for (uint32_t j = 0; j < c->lgroup->world(); ++j)
    if (j != c->cfg.rank) HIPC(c, hipStreamWaitEvent(st, ps[j].ev, 0));
  return KS_OK;
}

// In place: rank r's slice [r * bytes, (r + 1) * bytes) of buf -> every rank's buf.
ks_status coll_allgather(ks_ctx *c, void *buf, size_t bytes, hipStream_t st) {
  const uint32_t r = c->cfg.rank;
  if (c->comm) {
    NCCLC(c, ncclAllGather((uint8_t *)buf + (size_t)r * bytes, buf, bytes, ncclUint8, c->comm, st));
    return KS_OK;
  }
  HIPC(c, hipEventRecord(c->lg_ev[0], st));
  std::vector<LocalGroup::Post> ps;
  ks_status e = lg_exchange(c, {c->lg_ev[0], buf, {}}, ps);
  if (e) return e;
  for (uint32_t j = 0; j < c->lgroup->world(); ++j) {
    if (j == r) continue;
    HIPC(c, hipStreamWaitEvent(st, ps[j].ev, 0));
    HIPC(c, hipMemcpyAsync((uint8_t *)buf + (size_t)j * bytes, (const uint8_t *)ps[j].ptr + (size_t)j * bytes, bytes,
                           hipMemcpyDeviceToDevice, st));
  }
  return lg_finish(c, st);
}

// In place: element-wise max of n uint32 over all ranks.
ks_status coll_allreduce_max_u32(ks_ctx *c, uint32_t *buf, size_t n, hipStream_t st) {
  if (c->comm) {
    NCCLC(c, ncclAllReduce(buf, buf, n, ncclUint32, ncclMax, c->comm, st));
    return KS_OK;
  }
  if (n > 4 * (size_t)MAX_P) return c->fail(KS_ERR_INVALID, "in-process all-reduce of %zu words", n);
  HIPC(c, hipMemcpyAsync(c->d_lgstage, buf, n * 4, hipMemcpyDeviceToDevice, st));
  HIPC(c, hipEventRecord(c->lg_ev[0], st));
  std::vector<LocalGroup::Post> ps;
  ks_status e = lg_exchange(c, {c->lg_ev[0], c->d_lgstage, {}}, ps);
  if (e) return e;
  for (uint32_t j = 0; j < c->lgroup->world(); ++j) {
    if (j == c->cfg.rank) continue;
    HIPC(c, hipStreamWaitEvent(st, ps[j].ev, 0));
    HIPC(c, launch_umax_u32(buf, (const uint32_t *)ps[j].ptr, (uint32_t)n, st));
  }
  return lg_finish(c, st);
}

// One device-driven round (all kernels read the queue head from d_start).
// Round k of a pipeline run (k = 0 starts it: the table holds every previous
// round).  Stream order, with sweep k+1 overlapping merge .. patch k and resolve k:
//   stream : [wait resolve k-2 (and FIX sweep k-1), write-back k-2] advance k,
//            sweep k, record ev_swept[k]
//   sstream: wait ev_swept[k], merge k, [norm_check, FIX sweep + merge k],
//            (RCCL), merge_shards k, gather k, [wait resolve k-1, patch k],
//            record ev_sw[k]
//   rstream: wait ev_sw[k], resolve k, record ev_res[k]
ks_status enqueue_round(ks_ctx *c, ks_batch *b, uint32_t k, uint32_t end) {
  // Timing events cost the main stream ~10 us of dispatch per sweep, so only
  // every KS_TIMING_EVERY-th round (default 8) is timed.
  const bool tm = c->timing && (c->round_seq + 1) % c->timing_every == 0;
  // multi-rank path whenever a communicator exists (also a 1-rank one: exercised by tests)
  const bool multi = c->has_comm();
  const uint32_t nloc = multi ? 1 : c->S;
  const uint32_t shard0 = multi ? c->cfg.rank : 0;
  const uint32_t knpl = kernel_npl(c, b->ext);
  ks_status st = KS_OK;
  const uint32_t sub = c->npl / knpl;
  uint32_t bmax = 0;
  for (uint32_t q = 0; q < nloc; ++q) bmax = std::max(bmax, blocks_per_shard(c->shards[shard0 + q], sub));
  // pods per block: enough (block, pod-group) pairs to fill 256 CUs x 8 waves
  const uint32_t want = b->ext ? c->sweep_blocks_ext : c->sweep_blocks;
  const uint32_t total_blocks = bmax * nloc;
  uint32_t groups = (want + total_blocks - 1) / total_blocks;
  groups = std::max<uint32_t>(1, std::min(groups, c->P));
  uint32_t pg = (c->P + groups - 1) / groups;
  pg = std::min<uint32_t>(std::max<uint32_t>(pg, 1), MAX_PG);
  groups = (c->P + pg - 1) / pg;

  RoundArgs a{};
  a.t = c->run_t;  // the table as this run sees it (run_batch), no lock per round
  a.shards = c->d_shards;
  a.total_shards = c->S;
  a.shard0 = shard0;
  a.npl = knpl;
  a.sub = sub;
  a.lnpl = c->npl;
  a.P = c->P;
  a.pg = pg;
  a.K = c->K;
  a.npods = end;  // the segment ends here (pods after it go to the spread path)
  a.bstride = bmax;
  a.evaluated = c->n_present;
  a.pods = b->d_pods;
  a.clauses = b->d_clauses;
  a.marks = b->d_marks;
  const uint32_t q = k & 1u, pq = q ^ 1u;
  c->dedup_used[q] = b->dups && c->dedup;
  if (c->dedup_used[q]) {
    uint32_t *dd = c->d_dedup + (size_t)q * (2 * MAX_P + 4);
    a.cls = b->d_cls;
    a.rep = dd;
    a.ulist = dd + MAX_P;
    a.nuniq = dd + 2 * MAX_P;
  }
  const size_t RW = rec_words(c->K);
  a.d_start = c->d_start;
  a.sstart = c->d_pipe + q;
  a.prev_sstart = c->d_pipe + pq;
  a.act = c->d_pipe + 2 + q;
  a.act_next = c->d_pipe + 2 + pq;
  a.prev_act = c->d_pipe + 2 + pq;
  a.carry_in = c->d_carry + (size_t)pq * MAX_P;
  a.carry_in_n = c->d_pipe + 4 + pq;
  a.carry_out = c->d_carry + (size_t)q * MAX_P;
  a.carry_out_n = c->d_pipe + 4 + q;
  a.first = k == 0;
  a.norm_max = c->d_norm + (size_t)q * 2 * c->P;
  a.norm_inv = c->d_norm_inv + (size_t)q * 2 * c->P;
  a.guess_inv = b->d_pinv;
  a.pstat = b->norm ? c->d_pstat : nullptr;
  a.fix_flag = c->d_fix;
  a.fix_group = c->d_fix + MAX_P;
  a.fix_list = c->d_fix + MAX_P + MAX_P / MAX_PG;
  a.fix = 0;
  a.brec = c->d_brec + (size_t)q * (c->brec_bytes / sizeof(BlockRec));
  a.srec = c->d_srec + (size_t)q * c->S * c->P * RW;
  a.frec = c->S == 1 ? a.srec : c->d_frec + (size_t)q * c->P * RW;
  a.results = b->d_results;
  a.counters = c->d_counters;
  a.crow = c->d_crow + (size_t)q * c->P * c->K;
  a.cext = c->d_cext + (size_t)q * c->P * c->K;
  a.slot_pos = c->d_slot_pos;
  a.w = Weights{c->cfg.weight_fit, c->cfg.weight_balanced, c->cfg.weight_taint, c->cfg.weight_affinity,
                c->cfg.weight_image};
  if ((size_t)nloc * c->P * bmax * sizeof(BlockRec) > c->brec_bytes)
    return c->fail(KS_ERR_INVALID, "block record buffer too small");

  // Sweep-kernel geometry is expressed with the kernel's own nodes-per-lane:
  // positions of layout wave w, steps [j0, j0 + knpl) are kernel wave w*sub + j0/knpl.
  // The kernels address positions as base + wave*64*knpl + j*64 + lane, which
  // equals the layout position when the layout's npl-step block of a wave is
  // split into `sub` consecutive kernel waves; slots follow from the layout.
  // early_fix (default 1, one rank): the sweep measures the normaliser
  // maxima itself and norm_check + the FIX sweep follow it on the main
  // stream, so sweep k+1 no longer waits for the side stream's merge k; the
  // merge then reads the FIX records of the flagged pods directly
  const bool early = b->norm && !multi && c->early_fix;
  a.pstat_sweep = early ? 1u : 0u;
  if (k >= 2) {  // round k-2 lands in the table before sweep k (sweep k-1 has finished reading it)
    if ((st = hand_wait(c, c->stream, 2, c->ev_res[q], c->seq_of[q]))) return st;
    if (b->norm && !early && (st = hand_wait(c, c->stream, 3, c->ev_fixed[pq], c->seq_of[pq]))) return st;  // ... and so has FIX sweep k-1
    HIPC(c, launch_advance_writeback(a, c->d_carry + (size_t)q * MAX_P, c->d_pipe + 4 + q, c->stream));
  } else {
    HIPC(c, launch_advance(a, c->stream));
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (tm) {
    e0 = get_event(c);
    e1 = get_event(c);
    HIPC(c, hipEventRecord(e0, c->stream));
  }
  if (early) HIPC(c, hipMemsetAsync(c->d_pstat, 0, (size_t)c->P * sizeof(PodStat), c->stream));
  HIPC(c, launch_sweep(a, b->ext, bmax, groups, nloc, c->stream));
  ++c->sweeps_issued;
  if (tm) {
    HIPC(c, hipEventRecord(e1, c->stream));
    c->ev_sweep.emplace_back(e0, e1);
  }
  // merge .. patch on the side stream, overlapping sweep k+1 (block records
  // by parity; gather k may read the table while the write-back of round k-1
  // lands: only rows of round k-1's nodes change, and patch k replaces those)
  const uint32_t seq = ++c->round_seq;
  c->seq_of[q] = seq;
  hipStream_t ss = c->sstream;
  if (early) {
    HIPC(c, launch_norm_check(a, c->stream));
    RoundArgs f = a;
    f.fix = 1;
    f.pg = MAX_PG;
    HIPC(c, launch_sweep(f, true, bmax, (c->P + MAX_PG - 1) / MAX_PG, nloc, c->stream));
  }
  if ((st = hand_signal(c, c->stream, 0, c->ev_swept[q], seq)) || (st = hand_wait(c, ss, 0, c->ev_swept[q], seq))) return st;
  if (b->norm && !early) HIPC(c, hipMemsetAsync(c->d_pstat, 0, (size_t)c->P * sizeof(PodStat), ss));
  HIPC(c, launch_merge(a, nloc, ss));
  if (b->norm && !early) {
    // the sweep scored normalising plugins with each pod's guessed maxima:
    // measure (all ranks), flag the wrong guesses, re-sweep + re-merge those pods
    if (multi && (st = coll_allreduce_max_u32(c, (uint32_t *)c->d_pstat, 4 * (size_t)c->P, ss))) return st;
    HIPC(c, launch_norm_check(a, ss));
    RoundArgs f = a;
    f.fix = 1;
    f.pg = MAX_PG;
    HIPC(c, launch_sweep(f, true, bmax, (c->P + MAX_PG - 1) / MAX_PG, nloc, ss));
    if ((st = hand_signal(c, ss, 3, c->ev_fixed[q], seq))) return st;  // the FIX sweep reads the table as sweep k did
    HIPC(c, launch_merge(f, nloc, ss));
  }
  if (multi) {
    const size_t words = (size_t)c->P * RW;
    if ((st = coll_allgather(c, a.srec, words * 8, ss))) return st;
  }
  if (c->S > 1) HIPC(c, launch_merge_shards(a, ss));
  HIPC(c, launch_gather_cand(a, b->ext, ss));
  if (k > 0) {
    // merge round k-1's commits into the lists once resolve k-1 is done
    if ((st = hand_wait(c, ss, 2, c->ev_res[pq], seq - 1))) return st;
    HIPC(c, launch_patch(a, b->ext, ss));
  }
  if ((st = hand_signal(c, ss, 1, c->ev_sw[q], seq)) || (st = hand_wait(c, c->rstream, 1, c->ev_sw[q], seq))) return st;
  if (tm) {
    e0 = get_event(c);
    e1 = get_event(c);
    HIPC(c, hipEventRecord(e0, c->rstream));
  }
  {
    RoundArgs ra = a;
    ra.flag_res = c->value_sync ? c->d_flags + 2 : nullptr;
    ra.seq = seq;
    ra.stall_us = 0;
    if (c->stall_flag == 2) {  // ks_debug_stall
      ra.stall_us = c->stall_us;
      c->stall_flag = -1;
    }
    c->flag_want[2] = seq;
    ra.par_max_passes = c->par_max_passes;
    ra.prof = c->res_profile ? c->d_counters + 16 : nullptr;
    ra.serial_rounds = c->serial_rounds;
    // one launch: the parallel commit, and the serial one in the same
    // workgroup for the rounds it does not take
    ra.rmode = c->resolve_mode == KS_RESOLVE_AUTO ? c->d_flags + 4 : nullptr;
    ra.serial_only = c->resolve_mode == KS_RESOLVE_SERIAL ? 1u : 0u;
    HIPC(c, launch_resolve(ra, b->ext, c->rstream));
  }
  if (tm) {
    HIPC(c, hipEventRecord(e1, c->rstream));
    c->ev_resolve.emplace_back(e0, e1);
  }
  // the resolve kernel stores `seq` in flag 2 itself (no stream write operation after it)
  HIPC(c, hipEventRecord(c->ev_res[q], c->rstream));
  return KS_OK;
}

// End of a pipeline run of `rounds` rounds: land the last two rounds in the
// table and wait for everything.
ks_status drain_rounds(ks_ctx *c, uint32_t rounds, void *h_res, const void *d_res, size_t res_bytes) {
  for (uint32_t k = rounds >= 2 ? rounds - 2 : 0; k < rounds; ++k) {
    const uint32_t q = k & 1u;
    HIPC(c, hipStreamWaitEvent(c->stream, c->ev_res[q], 0));
    HIPC(c, launch_writeback(c->t, c->d_carry + (size_t)q * MAX_P, c->d_pipe + 4 + q, c->stream));
  }
  if (res_bytes) HIPC(c, hipMemcpyAsync(h_res, d_res, res_bytes, hipMemcpyDeviceToHost, c->stream));
  HIPC(c, hipMemcpyAsync(c->h_start, c->d_start, 4, hipMemcpyDeviceToHost, c->stream));
  return sync_bounded(c, c->stream, "a pipeline run's drain");
}

// ------------------------------------------------------------- batches

// A pooled batch with room for n pods and `words` clause words: device
// buffers are allocated only when no pooled batch is large enough, and
// outgrown clause buffers are retired to the graveyard.
ks_status batch_acquire(ks_ctx *c, uint32_t n, size_t words, ks_batch **out) {
  const uint32_t need = std::max<uint32_t>(n, 1);
  ks_batch *b = nullptr;
  {
    std::lock_guard<std::mutex> g(c->pool_mu);
    size_t bi = SIZE_MAX;
    for (size_t i = 0; i < c->pool.size(); ++i)
      if (c->pool[i]->cap_pods >= need && (bi == SIZE_MAX || c->pool[i]->cap_pods < c->pool[bi]->cap_pods)) bi = i;
    if (bi != SIZE_MAX) {
      b = c->pool[bi];
      c->pool.erase(c->pool.begin() + (long)bi);
    }
  }
  if (!b) {
    b = new ks_batch();
    {
      std::lock_guard<std::mutex> g(c->pool_mu);
      c->all_batches.push_back(b);
    }
    HIPC(c, hipMalloc((void **)&b->d_pods, (size_t)need * sizeof(PodDev)));
    HIPC(c, hipMalloc((void **)&b->d_pinv, (size_t)need * 2 * sizeof(double)));
    HIPC(c, hipMalloc((void **)&b->d_results, (size_t)need * sizeof(DevResult)));
    HIPC(c, hipHostMalloc((void **)&b->h_results, (size_t)need * sizeof(DevResult), hipHostMallocDefault));
    HIPC(c, hipHostMalloc((void **)&b->h_pods, (size_t)need * sizeof(PodDev), hipHostMallocDefault));
    HIPC(c, hipHostMalloc((void **)&b->h_pinv, (size_t)need * 2 * sizeof(double), hipHostMallocDefault));
    HIPC(c, hipMalloc((void **)&b->d_cmask, (size_t)need * 8 * CMASK_WORDS));
    HIPC(c, hipHostMalloc((void **)&b->h_cmask, (size_t)need * 8 * CMASK_WORDS, hipHostMallocDefault));
    HIPC(c, hipMalloc((void **)&b->d_marks, ((size_t)need + 3) & ~(size_t)3));
    HIPC(c, hipMalloc((void **)&b->d_cls, (size_t)need * 4));
    HIPC(c, hipHostMalloc((void **)&b->h_cls, (size_t)need * 4, hipHostMallocDefault));
    b->cap_pods = need;
  }
  if (words > b->cap_words) {
    if (b->d_clauses) c->graveyard.push_back(b->d_clauses);
    if (b->h_clauses) c->pinned_graveyard.push_back(b->h_clauses);
    b->d_clauses = nullptr;
    b->h_clauses = nullptr;
    b->cap_words = std::max<size_t>(words, std::max<size_t>(2 * b->cap_words, 4096));
    HIPC(c, hipMalloc((void **)&b->d_clauses, b->cap_words * 8));
    HIPC(c, hipHostMalloc((void **)&b->h_clauses, b->cap_words * 8, hipHostMallocDefault));
  }
  b->n = 0;
  b->queued = b->done = false;
  b->run_status = KS_OK;
  b->run_err.clear();
  *out = b;
  return KS_OK;
}

void batch_release(ks_ctx *c, ks_batch *b) {
  std::lock_guard<std::mutex> g(c->pool_mu);
  b->queued = b->done = false;
  c->pool.push_back(b);
}

// Compiled batch (pinned host copies) -> device, on the scheduler stream.
// Identical pods of a resource-only batch (RoundArgs::cls): cls[i] = the index
// of the first pod whose compiled descriptor is byte-identical to pod i's
// (the sweep, Filter and Score read nothing else of a pod), i for pods of the
// one-pod path.  Returns whether some pod repeats an earlier one.
bool pod_classes(const PodDev *dev, uint32_t n, uint32_t *cls) {
  std::unordered_map<uint64_t, uint32_t> first;
  first.reserve(n);
  bool dups = false;
  for (uint32_t i = 0; i < n; ++i) {
    cls[i] = i;
    if (dev[i].flags & PF_SOLO) continue;
    uint64_t h = 1469598103934665603ull;  // FNV-1a over the descriptor's words
    const uint64_t *w = reinterpret_cast<const uint64_t *>(&dev[i]);
    for (size_t q = 0; q < sizeof(PodDev) / 8; ++q) h = (h ^ w[q]) * 1099511628211ull;
    for (;; ++h) {  // open addressing on the hash value itself (collisions probe h + 1)
      auto it = first.find(h);
      if (it == first.end()) {
        first.emplace(h, i);
        break;
      }
      if (std::memcmp(&dev[it->second], &dev[i], sizeof(PodDev)) == 0) {
        cls[i] = it->second;
        dups = true;
        break;
      }
    }
  }
  return dups;
}

ks_status upload_batch(ks_ctx *c, ks_batch *b) {
  const size_t np = std::max<uint32_t>(b->n, 1);
  HIPC(c, hipMemcpyAsync(b->d_pods, b->h_pods, np * sizeof(PodDev), hipMemcpyHostToDevice, c->stream));
  HIPC(c, hipMemcpyAsync(b->d_pinv, b->h_pinv, np * 2 * sizeof(double), hipMemcpyHostToDevice, c->stream));
  if (b->dups) HIPC(c, hipMemcpyAsync(b->d_cls, b->h_cls, np * 4, hipMemcpyHostToDevice, c->stream));
  HIPC(c, hipMemcpyAsync(b->d_clauses, b->h_clauses, b->n_words * 8, hipMemcpyHostToDevice, c->stream));
  HIPC(c, hipMemsetAsync(b->d_results, 0, np * sizeof(DevResult), c->stream));
  HIPC(c, hipMemsetAsync(b->d_marks, 0, (np + 3) & ~(size_t)3, c->stream));
  b->uploaded = true;
  return KS_OK;
}

// Replica runs: what the run kernel's key layout holds --
// domain ids of the other key below RK_DZ_NONE -- on a single-rank context
// (the one-pod path's condition).
bool replica_fits(const ks_ctx *c, const ks_batch *b, const SpreadArgs &sa, uint32_t i) {
  if (c->has_comm()) return false;
  const SoloHdr *hd = reinterpret_cast<const SoloHdr *>(b->h_clauses + b->h_pods[i].solo_off);
  const SpreadDev *sd = reinterpret_cast<const SpreadDev *>(hd + 1);
  for (uint32_t k = 0; k < hd->n_spread; ++k)
    if (!(sd[k].flags & SP_HOST) && sa.ndom[sd[k].key] > RK_DZ_NONE) return false;
  return true;
}

// One replica run over pods [lo, hi) of the batch: one filter pass, the sort,
// the run kernel; waits for it and returns the first pod it did not schedule
// (lo: refused) and why it stopped (RunStop).
ks_status replica_run(ks_ctx *c, ks_batch *b, SpreadArgs sa, uint32_t lo, uint32_t hi, uint32_t *next,
                      uint32_t *stop) {
  if (!c->d_rk_keys) {
    size_t bytes = 0;
    HIPC(c, launch_sort_pairs(nullptr, nullptr, nullptr, nullptr, c->cap, 64, nullptr, &bytes, c->stream));
    ks_status st;
    if ((st = dalloc(c, &c->d_rk_keys, c->npos)) || (st = dalloc(c, &c->d_rk_sorted, c->npos)) ||
        (st = dalloc(c, &c->d_rk_val, c->npos)) || (st = dalloc(c, &c->d_rk_sval, c->npos)) ||
        (st = dalloc(c, &c->d_rk_gstart, RUN_GROUPS)) || (st = dalloc(c, &c->d_rk_ctl, RUN_CTL_WORDS)) ||
        (st = dalloc(c, &c->d_rk_tmp, std::max<size_t>(bytes, 16))) ||
        (c->run_profile && (st = dalloc(c, &c->d_rk_prof, 4))))
      return st;
    c->rk_tmp_bytes = bytes;
    HIPC(c, hipHostMalloc((void **)&c->h_rk_ctl, 16, hipHostMallocDefault));
  }
  // static score < 100 x (the weights of LeastAllocated, BalancedAllocation,
  // TaintToleration, NodeAffinity) + 1; ImageLocality adds 0 (no image records)
  const uint32_t s_max = 100u * (uint32_t)(c->cfg.weight_fit + c->cfg.weight_balanced + c->cfg.weight_taint +
                                           c->cfg.weight_affinity);
  uint32_t s_bits = 1;
  while (s_bits < 32 && (s_max >> s_bits) != 0) ++s_bits;
  ReplicaArgs r{c->d_rk_keys, c->d_rk_sorted, c->d_rk_val, c->d_rk_sval, c->d_rk_gstart, c->d_rk_ctl, hi, c->cap,
                s_bits, c->d_rk_prof};
  sa.pod = lo;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->timing) {
    e0 = get_event(c);
    e1 = get_event(c);
    HIPC(c, hipEventRecord(e0, c->stream));
  }
  HIPC(c, launch_replica_run(sa, r, c->d_rk_tmp, c->rk_tmp_bytes, b->spread[lo] & 0x7Fu, c->stream));
  if (c->timing) HIPC(c, hipEventRecord(e1, c->stream));
  HIPC(c, hipMemcpyAsync(c->h_rk_ctl, c->d_rk_ctl, 16, hipMemcpyDeviceToHost, c->stream));
  if (ks_status st = sync_bounded(c, c->stream, "a replica run")) return st;
  *next = c->h_rk_ctl[2];
  *stop = c->h_rk_ctl[3];
  if (c->d_rk_prof) HIPC(c, hipMemcpy(c->rk_prof, c->d_rk_prof, sizeof c->rk_prof, hipMemcpyDeviceToHost));
  if (*next < lo || *next > hi || (*next == lo) != (*stop == RUN_REFUSED))
    return c->fail(KS_ERR_DEVICE, "replica run over pods [%u, %u) ended at %u (stop %u)", lo, hi, *next, *stop);
  const uint32_t done = *next - lo;
  c->stats.spread_pods += done;
  c->stats.replica_pods += done;
  c->stats.replica_runs += done ? 1 : 0;
  if (c->timing) {
    if (done) {
      c->ev_runs.push_back({e0, e1, done});
    } else {
      c->ev_pool.push_back(e0);
      c->ev_pool.push_back(e1);
    }
  }
  return KS_OK;
}

// Selector classes created while batch b was in flight (class_get,
// undrained): +1 in their columns for every pod b bound that they select.
// Called under mu at the end of b's run.
ks_status late_class_counts(ks_ctx *c, const ks_batch *b) {
  std::vector<uint64_t> idx;
  std::vector<int32_t> dv;
  for (int k = 0; k < MAX_CLASSES; ++k) {
    const SpreadClass &q = c->classes[k];
    if (!q.live || q.born <= b->cmask_epoch) continue;
    std::vector<int8_t> memo(c->label_sets.size(), -1);
    for (uint32_t i = 0; i < b->n; ++i) {
      if (b->h_results[i].status != KS_POD_SCHEDULED) continue;
      const uint32_t set = b->set_ids[i];
      if (memo[set] < 0) memo[set] = class_matches(c, q, set) ? 1 : 0;
      if (!memo[set]) continue;
      idx.push_back((uint64_t)k * c->npos + c->slot_pos[b->h_results[i].node_index]);
      dv.push_back(1);
    }
  }
  if (idx.empty()) return KS_OK;
  c->stats.late_class_pods += idx.size();
  const size_t bytes = idx.size() * 12 + 1024;
  ks_status st = xfer_begin(c, bytes, bytes);
  if (st) return st;
  uint64_t *d_idx = dscratch<uint64_t>(c, idx.size());
  int32_t *d_dv = dscratch<int32_t>(c, dv.size());
  if ((st = h2d(c, d_idx, idx.data(), idx.size() * 8)) || (st = h2d(c, d_dv, dv.data(), dv.size() * 4))) return st;
  HIPC(c, launch_add_u32(c->d_cnt, d_idx, d_dv, (uint32_t)idx.size(), c->stream));
  return xfer_sync(c);
}

// Run a prepared batch to completion on the scheduler streams; the results
// land in the batch's pinned host buffer.
ks_status run_batch(ks_ctx *c, ks_batch *b) {
  if (b->dict_version != c->dict_version)
    return c->fail(KS_ERR_STALE, "batch compiled against taint dictionary / node image set v%u, cache is at v%u",
                   b->dict_version, c->dict_version);
  if (b->names_version && b->names_version != c->names_version)
    return c->fail(KS_ERR_STALE, "batch resolved node names before the node set changed");
  if (c->cfg.world_size > 1 && !c->has_comm()) return c->fail(KS_ERR_COMM, "world_size > 1 but ks_comm_init not called");
  if (c->has_comm() && c->S != c->cfg.world_size)
    return c->fail(KS_ERR_INVALID, "RCCL sharding needs one shard per rank (virtual_shards must be 1)");
  HIPC(c, hipSetDevice(c->cfg.device));
  ks_status st0;
  // One critical section (a second one let the next batch's compile, which
  // holds `mu` for milliseconds, stall this run between the two):
  //  * label words of nodes that gained dictionary bits since the last upload
  //    (bits of this batch or a later-prepared one: a superset is harmless);
  //  * the table as the rounds read it (ks_batch_prepare of the next batch may
  //    widen t.lw meanwhile: its label words are uploaded by its own run);
  //  * the selector classes each pod matches, against the classes live now:
  //    the spread path's commits and the round kernels' (class_commit) count them.
  bool classes = false;
  {
    const auto tw = std::chrono::steady_clock::now();
    c->mu_wanted.fetch_add(1);
    std::lock_guard<std::mutex> g(c->mu);
    c->mu_wanted.fetch_sub(1);
    if (c->run_profile) c->prof[0] += std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count();
    if ((st0 = upload_dirty_ext(c, c->xm))) return st0;
    c->run_t = c->t;
    b->run_seq = ++c->runs_started;
    b->cmask_epoch = c->class_epoch;
    for (int k = 0; k < MAX_CLASSES; ++k) {
      classes |= c->classes[k].live;
      if (c->classes[k].live) c->classes[k].held = b->run_seq;
    }
    if (classes || b->any_spread) {
      std::vector<int32_t> memo(c->label_sets.size(), -1);  // set -> first pod index with it
      for (uint32_t i = 0; i < b->n; ++i) {
        const uint32_t set = b->set_ids[i];
        uint64_t *m = b->h_cmask + (size_t)i * CMASK_WORDS;
        if (memo[set] >= 0) {
          std::memcpy(m, b->h_cmask + (size_t)memo[set] * CMASK_WORDS, 8 * CMASK_WORDS);
          continue;
        }
        for (int w = 0; w < CMASK_WORDS; ++w) m[w] = 0;
        for (int k = 0; k < MAX_CLASSES; ++k)
          if (c->classes[k].live && class_matches(c, c->classes[k], set)) m[k / 64] |= 1ull << (k % 64);
        memo[set] = (int32_t)i;
      }
    }
  }
  const auto tu = std::chrono::steady_clock::now();
  if (!b->uploaded && (st0 = upload_batch(c, b))) return st0;
  if (c->run_profile) c->prof[5] += std::chrono::duration<double>(std::chrono::steady_clock::now() - tu).count();
  if (classes || b->any_spread)
    HIPC(c, hipMemcpyAsync(b->d_cmask, b->h_cmask, (size_t)std::max<uint32_t>(b->n, 1) * 8 * CMASK_WORDS, hipMemcpyHostToDevice,
                           c->stream));
  // Segments in queue order: runs of pods without spread constraints through
  // the pipelined rounds, spread pods one at a time through ksched_spread.hip.
  for (uint32_t lo = 0; lo < b->n;) {
    uint32_t hi = lo;
    if (b->any_spread && b->spread[lo]) {
      SpreadArgs sa{};
      {
        std::lock_guard<std::mutex> g(c->mu);
        sa.t = c->t;
        for (uint32_t k = 0; k < c->topo.size(); ++k) sa.ndom[k] = c->topo[k].ndom;
      }
      sa.pos_slot = c->d_pos_slot;
      sa.slot_pos = c->d_slot_pos;
      sa.npos = c->npos;
      sa.pods = b->d_pods;
      sa.clauses = b->d_clauses;
      sa.cmask = b->d_cmask;
      sa.dom = c->d_dom;
      sa.cnt = c->d_cnt;
      sa.xalloc = c->d_xalloc;
      sa.xreq = c->d_xreq;
      sa.dcnt = c->d_dcnt;
      sa.dflag = c->d_dflag;
      sa.tcnt = c->d_tcnt;
      sa.adcnt = c->d_adcnt;
      sa.ipa_raw = c->d_sraw2;
      sa.dom_cap = c->dom_cap;
      sa.acc = c->d_acc;
      sa.st = c->d_sst;
      sa.raw = c->d_sraw;
      sa.part = c->d_spart;
      sa.results = b->d_results;
      sa.counters = c->d_counters;
      sa.w = Weights{c->cfg.weight_fit, c->cfg.weight_balanced, c->cfg.weight_taint, c->cfg.weight_affinity,
                     c->cfg.weight_image};
      sa.w_pts = c->cfg.weight_topology_spread;
      sa.w_ipa = c->cfg.weight_inter_pod_affinity;
      sa.evaluated = c->n_present;
      if (c->pct != 100) {
        sa.win = c->d_win;
        sa.win_st = c->d_win_st;
        sa.nslots = c->cap;
        sa.win_mode = 2;
        sa.pct = c->pct;
      }
      // one pod through the per-pod chain
      auto chain = [&](uint32_t i) -> ks_status {
        sa.pod = i;
        // timing events on every KS_TIMING_EVERY-th spread pod
        const bool tm = c->timing && ++c->spread_seq % c->timing_every == 0;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (tm) {
          e0 = get_event(c);
          e1 = get_event(c);
          HIPC(c, hipEventRecord(e0, c->stream));
        }
        HIPC(c, launch_spread_pod(sa, b->spread[i] & 0x7Fu, c->stream));
        if (tm) {
          HIPC(c, hipEventRecord(e1, c->stream));
          c->ev_spread.emplace_back(e0, e1);
        }
        c->stats.spread_pods++;
        return KS_OK;
      };
      uint32_t chain_until = lo;  // pods before it take the chain (runs there stopped short)
      while (hi < b->n && b->spread[hi]) {
        // replica run: pod hi and the identical pods after it
        uint32_t e = hi + 1;
        if (c->replica_runs && c->pct == 100 && b->rep[hi] && hi >= chain_until)
          while (e < b->n && (b->rep[e] & 2)) ++e;
        if (e - hi >= RUN_MIN_PODS && replica_fits(c, b, sa, hi)) {
          uint32_t next = hi, stop = RUN_END;
          if (ks_status st = replica_run(c, b, sa, hi, e, &next, &stop)) return st;
          // refused (more groups than a run holds), or stopped short by a Fit
          // loss: the rest of these identical pods take the chain
          if (next == hi || (stop == RUN_FIT && next - hi < RUN_MIN_PODS)) chain_until = e;
          hi = next;
          continue;
        }
        if (ks_status st = chain(hi)) return st;
        ++hi;
      }
      HIPC(c, hipMemcpyAsync(b->h_results + lo, b->d_results + lo, (size_t)(hi - lo) * sizeof(DevResult),
                             hipMemcpyDeviceToHost, c->stream));
    } else {
      while (hi < b->n && !(b->any_spread && b->spread[hi])) ++hi;
      *c->h_seg = lo;
      HIPC(c, hipMemcpyAsync(c->d_start, c->h_seg, 4, hipMemcpyHostToDevice, c->stream));
      uint32_t host_start = lo;
      while (host_start < hi) {
        // Assume full rounds (an early stop costs the speculated round after it)
        // and check; each pipeline run resolves at least one pod.
        // Up to 256 rounds per run (a 50,000-pod batch): every run ends in a
        // drain, ~0.19 ms of idle GPU (C2 trace, profiles/r4/); 64 cost C2 two
        // extra drains per 20,000-pod batch.
        uint32_t rounds = (hi - host_start + c->P - 1) / c->P;
        rounds = std::min<uint32_t>(rounds, 256);
        const auto te = std::chrono::steady_clock::now();
        for (uint32_t r = 0; r < rounds; ++r) {
          ks_status st = enqueue_round(c, b, r, hi);
          if (st) return st;
        }
        const auto td = std::chrono::steady_clock::now();
        // results of every pod this pipeline run can resolve, behind its last round
        const uint32_t top = std::min<uint32_t>(hi, host_start + rounds * c->P);
        ks_status st = drain_rounds(c, rounds, b->h_results + host_start, b->d_results + host_start,
                                    (size_t)(top - host_start) * sizeof(DevResult));
        if (st) return st;
        if (c->run_profile) {
          c->prof[1] += std::chrono::duration<double>(td - te).count();
          c->prof[2] += std::chrono::duration<double>(std::chrono::steady_clock::now() - td).count();
        }
        if (*c->h_start <= host_start) return c->fail(KS_ERR_DEVICE, "no progress in scheduling rounds");
        host_start = *c->h_start;
      }
      if (classes)
        HIPC(c, launch_class_commit(b->d_results, b->d_cmask, c->d_slot_pos, c->d_cnt, c->npos, lo, hi, c->stream));
    }
    lo = hi;
  }
  {
    ks_status st1 = sync_bounded(c, c->stream, "a batch run");
    if (st1) return st1;
  }
  {
    // NodeInfo.Pods of the nodes this batch bound pods to (later selector
    // classes count them): appended to a log, applied when read
    const auto tw = std::chrono::steady_clock::now();
    c->mu_wanted.fetch_add(1);
    std::lock_guard<std::mutex> g(c->mu);
    c->mu_wanted.fetch_sub(1);
    if (c->run_profile) c->prof[4] += std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count();
    if (c->pending_bound.size() > (1u << 24)) flush_bound(c);
    for (uint32_t i = 0; i < b->n; ++i)
      if (b->h_results[i].status == KS_POD_SCHEDULED) {
        c->pending_bound.push_back({(uint32_t)b->h_results[i].node_index, b->set_ids[i], +1});
        for (auto &t : c->label_sets[b->set_ids[i]].terms) c->terms[t.first].bound++;  // the commit counted it
      }
    // classes created while this batch ran (after its class masks): its
    // commits did not count them, so its bound pods are added here, before
    // any later batch runs on the stream
    if (ks_status st = late_class_counts(c, b)) return st;
    c->runs_done = b->run_seq;
  }
  if (c->timing) {
    const auto tt = std::chrono::steady_clock::now();
    ks_status st = collect_timing(c);
    if (c->run_profile) c->prof[6] += std::chrono::duration<double>(std::chrono::steady_clock::now() - tt).count();
    if (st) return st;
  }
  c->prof[3] += 1;
  return KS_OK;
}

// RunQueue callbacks (ks_batch_submit's worker thread)
void worker_init(void *ctx) { (void)hipSetDevice(static_cast<ks_ctx *>(ctx)->cfg.device); }
int32_t worker_run(void *ctx, ks_batch *b, std::string *err) {
  ks_ctx *c = static_cast<ks_ctx *>(ctx);
  const ks_status st = run_batch(c, b);
  if (st) {
    std::lock_guard<std::mutex> g(c->err_mu);
    *err = c->err;
  }
  return st;
}

// Every ABI call except prepare / submit / wait / results / free first lets
// the submitted batches finish (they own the scheduler streams and the table).
ks_status drain_async(ks_ctx *c) {
  c->runq->drain();
  return KS_OK;
}

}  // namespace

// ================================================================== C ABI

extern "C" {

void ks_config_default(ks_config *cfg) {
  std::memset(cfg, 0, sizeof *cfg);
  cfg->device = 0;
  cfg->node_capacity = 1024;
  cfg->pods_per_round = 256;
  cfg->topk = 0;
  cfg->nodes_per_lane = 4;
  cfg->world_size = 1;
  cfg->rank = 0;
  cfg->virtual_shards = 1;
  cfg->weight_fit = 1;
  cfg->weight_balanced = 1;
  cfg->weight_taint = 3;
  cfg->weight_affinity = 2;
  cfg->weight_image = 1;
  cfg->weight_topology_spread = 2;
  cfg->weight_inter_pod_affinity = 2;
  cfg->hard_pod_affinity_weight = 1;
  cfg->percentage_of_nodes_to_score = 100;
  cfg->resolve_mode = KS_RESOLVE_AUTO;
  cfg->resolve_par_max_passes = 32;
  cfg->resolve_serial_rounds = 4;
  cfg->dedup_identical_pods = 1;
  cfg->early_fix = 1;
  cfg->tuple_guess = 1;
  cfg->ext_nodes_per_lane = 2;
  cfg->sweep_pairs = 4096;
  cfg->sweep_pairs_ext = 16384;
  cfg->resolve_cus = 1;
  cfg->side_cus = 0;
  cfg->value_sync = 1;
  cfg->sync_timeout_ms = 60000;
  cfg->spread_replica_runs = 1;
}

int32_t ks_abi_version(void) { return KSCHED_ABI_VERSION; }

const char *ks_last_error(const ks_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

ks_status ks_open(const ks_config *cfg, ks_ctx **out) {
  if (!cfg || !out) return KS_ERR_INVALID;
  *out = nullptr;
  auto c = std::make_unique<ks_ctx>();
  c->cfg = *cfg;
  c->runq = std::make_unique<RunQueue<ks_batch>>(c.get(), &worker_run, &worker_init);
  if (cfg->node_capacity == 0) return KS_ERR_INVALID;
  c->cap = cfg->node_capacity;
  c->npl = cfg->nodes_per_lane ? cfg->nodes_per_lane : 4;
  if (c->npl != 2 && c->npl != 4 && c->npl != 8) return KS_ERR_INVALID;
  c->P = cfg->pods_per_round ? cfg->pods_per_round : 256;
  if (c->P > (uint32_t)MAX_P) return KS_ERR_INVALID;
  c->K = cfg->topk ? cfg->topk : c->P;
  if (c->K > (uint32_t)MAX_K) return KS_ERR_INVALID;  // resolve: two listed candidates per list-wave lane
  const uint32_t world = cfg->world_size ? cfg->world_size : 1;
  c->cfg.world_size = world;
  if (cfg->rank >= world) return KS_ERR_INVALID;
  c->S = world > 1 ? world : std::max<uint32_t>(1, cfg->virtual_shards);
  if (c->S > (uint32_t)MAX_SHARDS) return KS_ERR_INVALID;
  // weights are small non-negative integers (the kernels add them in 32 bits)
  for (int32_t w : {cfg->weight_fit, cfg->weight_balanced, cfg->weight_taint, cfg->weight_affinity, cfg->weight_image,
                    cfg->weight_topology_spread, cfg->weight_inter_pod_affinity, cfg->hard_pod_affinity_weight})
    if (w < 0 || w > 10000) return KS_ERR_INVALID;
  // percentageOfNodesToScore (ksched.h): below 100 on one GPU shard only
  if (cfg->percentage_of_nodes_to_score < 0 || cfg->percentage_of_nodes_to_score > 100) return KS_ERR_INVALID;
  if (cfg->percentage_of_nodes_to_score != 100 && c->S > 1) return KS_ERR_UNSUPPORTED;
  c->pct = cfg->percentage_of_nodes_to_score;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return KS_ERR_DEVICE;
  if (cfg->device < 0 || cfg->device >= ndev) return KS_ERR_DEVICE;
  if (hipSetDevice(cfg->device) != hipSuccess) return KS_ERR_DEVICE;
  ks_ctx *x = c.get();
  {
    // execution options (ks_config; none changes a result)
    // (pass and round caps bounded so the resolve's uint32 products
    // pass_cap * n and backoff * serial_rounds cannot wrap)
    if (cfg->resolve_mode > KS_RESOLVE_PARALLEL || cfg->resolve_par_max_passes == 0 ||
        cfg->resolve_par_max_passes > (uint32_t)MAX_P + 1 || cfg->resolve_serial_rounds > (1u << 20) ||
        (cfg->ext_nodes_per_lane != 2 && cfg->ext_nodes_per_lane != 4 && cfg->ext_nodes_per_lane != 8) ||
        cfg->sweep_pairs == 0 || cfg->sweep_pairs_ext == 0 || cfg->sync_timeout_ms == 0 || cfg->resolve_cus > 64 ||
        cfg->side_cus > 64)
      return KS_ERR_INVALID;
    x->resolve_mode = cfg->resolve_mode;
    x->par_max_passes = cfg->resolve_par_max_passes;
    x->serial_rounds = cfg->resolve_serial_rounds;
    x->dedup = cfg->dedup_identical_pods != 0;
    x->early_fix = cfg->early_fix != 0;
    x->tuple_guess = cfg->tuple_guess != 0;
    x->ext_npl = cfg->ext_nodes_per_lane;
    x->sweep_blocks = cfg->sweep_pairs;
    x->sweep_blocks_ext = cfg->sweep_pairs_ext;
    x->sync_timeout_ms = cfg->sync_timeout_ms;
    x->replica_runs = cfg->spread_replica_runs != 0;
    // diagnostics only (stderr reports, timing sample rate): they change no
    // scheduling decision
    auto env_u = [](const char *name, int dflt) {
      const char *e = std::getenv(name);
      return e ? std::atoi(e) : dflt;
    };
    x->ev_profile = env_u("KS_EVENT_PROFILE", 0) != 0;
    x->run_profile = env_u("KS_RUN_PROFILE", 0) != 0;
    x->timing_every = (uint32_t)std::max(1, env_u("KS_TIMING_EVERY", 8));
  }
  {
    // Resolve runs on a high-priority stream on resolve_cus (default 1) CUs
    // of its own: the main and side streams are masked off them, so a resolve
    // launch never waits for a CU to drain the next round's sweep blocks (the
    // sweep loses 1/256 of the chip, measured ~4 % slower).  0: no mask.
    const int nres = (int)cfg->resolve_cus;
    hipDeviceProp_t prop{};
    HIPC(x, hipGetDeviceProperties(&prop, cfg->device));
    const int ncu = prop.multiProcessorCount;
    // side_cus (default 0): CUs the main stream (sweeps) leaves to the side
    // stream, so merge / gather / patch blocks start without waiting for sweep
    // blocks to drain
    const int nside = (int)cfg->side_cus;
    if (nres > 0 && nres + nside < ncu) {
      std::vector<uint32_t> main_mask((ncu + 31) / 32, 0u), side_mask((ncu + 31) / 32, 0u),
          res_mask((ncu + 31) / 32, 0u);
      for (int i = 0; i < ncu; ++i) {
        if (i >= ncu - nres) res_mask[i / 32] |= 1u << (i % 32);
        else side_mask[i / 32] |= 1u << (i % 32);
        if (i < ncu - nres - nside) main_mask[i / 32] |= 1u << (i % 32);
      }
      HIPC(x, hipExtStreamCreateWithCUMask(&x->stream, (uint32_t)main_mask.size(), main_mask.data()));
      HIPC(x, hipExtStreamCreateWithCUMask(&x->rstream, (uint32_t)res_mask.size(), res_mask.data()));
      HIPC(x, hipExtStreamCreateWithCUMask(&x->sstream, (uint32_t)side_mask.size(), side_mask.data()));
    } else {
      int lo = 0, hi = 0;
      HIPC(x, hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking));
      HIPC(x, hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIPC(x, hipStreamCreateWithPriority(&x->rstream, hipStreamNonBlocking, hi));
      HIPC(x, hipStreamCreateWithPriority(&x->sstream, hipStreamNonBlocking, hi));
    }
    x->xm.st = x->stream;
    {  // value_sync = 0: cross-stream hand-offs by event waits instead
      int can = 0;
      (void)hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, cfg->device);
      x->value_sync = can != 0 && cfg->value_sync != 0;
    }
    for (int q = 0; q < 2; ++q) {
      HIPC(x, hipEventCreateWithFlags(&x->ev_sw[q], hipEventDisableTiming));
      HIPC(x, hipEventCreateWithFlags(&x->ev_res[q], hipEventDisableTiming));
      HIPC(x, hipEventCreateWithFlags(&x->ev_swept[q], hipEventDisableTiming));
      HIPC(x, hipEventCreateWithFlags(&x->ev_fixed[q], hipEventDisableTiming));
    }
  }
  // shard geometry: contiguous slot ranges; waves rounded to a multiple of 4
  uint32_t base = 0;
  for (uint32_t s = 0; s < x->S; ++s) {
    Shard sh;
    sh.lo = (uint32_t)((uint64_t)x->cap * s / x->S);
    const uint32_t hi = (uint32_t)((uint64_t)x->cap * (s + 1) / x->S);
    sh.count = hi - sh.lo;
    uint32_t lanes = (sh.count + x->npl - 1) / x->npl;
    uint32_t waves = (lanes + WAVE - 1) / WAVE;
    waves = std::max<uint32_t>(4, (waves + 3) & ~3u);
    sh.waves = waves;
    sh.base = base;
    base += waves * WAVE * x->npl;
    x->shards.push_back(sh);
  }
  x->npos = base;
  x->slot_pos.resize(x->cap);
  for (auto &sh : x->shards)
    for (uint32_t l = 0; l < sh.count; ++l) x->slot_pos[sh.lo + l] = shard_pos(sh, x->npl, l);
  x->nodes.resize(x->cap);
  x->present_map.assign(x->cap, 0);
  // device table
  ks_status st;
  NodeTable &t = x->t;
  t.npos = x->npos;
  t.lw = 0;
  if ((st = dalloc(x, &t.acpu, x->npos)) || (st = dalloc(x, &t.amem, x->npos)) ||
      (st = dalloc(x, &t.rcpu, x->npos)) || (st = dalloc(x, &t.rmem, x->npos)) ||
      (st = dalloc(x, &t.zcpu, x->npos)) || (st = dalloc(x, &t.zmem, x->npos)) ||
      (st = dalloc(x, &t.apods, x->npos)) || (st = dalloc(x, &t.npods, x->npos)) ||
      (st = dalloc(x, &t.hard, x->npos)) || (st = dalloc(x, &t.prefer, x->npos)) ||
      (st = dalloc(x, &t.lab, (size_t)LW * x->npos)) || (st = dalloc(x, &t.num, (size_t)NNUM * x->npos)))
    return st;
  HIPC(x, hipMemsetAsync(t.apods, 0xFF, (size_t)x->npos * 4, x->stream));  // every position empty
  if ((st = dalloc(x, &x->d_shards, x->S)) || (st = dalloc(x, &x->d_slot_pos, x->cap)) ||
      (st = dalloc(x, &x->d_start, 1)) || (st = dalloc(x, &x->d_norm, 2 * 2 * (size_t)x->P)) ||
      (st = dalloc(x, &x->d_norm_inv, 2 * 2 * (size_t)x->P)) ||
      (st = dalloc(x, &x->d_pstat, (size_t)x->P)) || (st = dalloc(x, &x->d_fix, 2 * MAX_P + MAX_P / MAX_PG)) ||
      (st = dalloc(x, &x->d_dedup, 2 * (2 * (size_t)MAX_P + 4))) ||
      (st = dalloc(x, &x->d_pipe, 8)) || (st = dalloc(x, &x->d_flags, 8)) || (st = dalloc(x, &x->d_carry, 2 * (size_t)MAX_P)) ||
      (st = dalloc(x, &x->d_counters, 32)))
    return st;
  if ((st = xfer_begin(x, x->S * sizeof(Shard) + (size_t)x->cap * 4 + 1024, 0)) ||
      (st = h2d(x, x->d_shards, x->shards.data(), x->S * sizeof(Shard))) ||
      (st = h2d(x, x->d_slot_pos, x->slot_pos.data(), (size_t)x->cap * 4)))
    return st;
  HIPC(x, hipHostMalloc((void **)&x->h_start, 4, hipHostMallocDefault));
  HIPC(x, hipHostMalloc((void **)&x->h_seg, 4, hipHostMallocDefault));
  HIPC(x, hipHostMalloc((void **)&x->h_diag, 64, hipHostMallocDefault));
  // round records: blocks of the widest kernel (npl 2 -> sub = npl / 2)
  uint32_t bmax = 0;
  for (auto &sh : x->shards) bmax = std::max(bmax, blocks_per_shard(sh, x->npl / std::min<uint32_t>(x->npl, 2)));
  const uint32_t nloc = world > 1 ? 1 : x->S;
  x->brec_bytes = (size_t)nloc * x->P * bmax * sizeof(BlockRec);
  if ((st = dalloc(x, (uint8_t **)&x->d_brec, 2 * x->brec_bytes))) return st;
  const size_t recs = (size_t)x->S * x->P * rec_words(x->K);  // per round parity
  // +2 words: the resolve's 16-byte key DMA may read 8 bytes past the last record
  if ((st = dalloc(x, &x->d_srec, 2 * recs + 2)) ||
      (st = dalloc(x, &x->d_frec, 2 * (size_t)x->P * rec_words(x->K) + 2)) ||
      (st = dalloc(x, &x->d_crow, 2 * (size_t)x->P * x->K)) || (st = dalloc(x, &x->d_cext, 2 * (size_t)x->P * x->K)))
    return st;
  if ((st = xfer_sync(x))) return st;  // all initialisation is stream-ordered
  *out = c.release();
  return KS_OK;
}

void ks_close(ks_ctx *c) {
  if (!c) return;
  drain_async(c);  // batches still queued or running count in the profile below
  double wp[3];
  c->runq->profile(wp);
  if (c->run_profile)
    std::fprintf(stderr,
                 "ksched runs: %.0f runs: lock wait %.3f s (at the end %.3f s), enqueue %.3f s, drains %.3f s; "
                 "worker: %.0f runs %.3f s, idle between runs %.3f s; prepare: drain wait %.3f s, compile %.3f s, "
                 "acquire / copy / upload %.3f s; in runs: upload %.3f s, timing read-back %.3f s\n",
                 c->prof[3], c->prof[0], c->prof[4], c->prof[1], c->prof[2], wp[2], wp[0], wp[1], c->prof[7],
                 c->prof[8], c->prof[9], c->prof[5], c->prof[6]);
  if (c->run_profile && c->rk_prof[3]) {
    const uint64_t *h = c->rk_prof;
    const double n = (double)h[3];
    std::fprintf(stderr, "ksched replica runs: %llu pods; cycles per pod: min/max raw %.0f, argmax %.0f, commit %.0f\n",
                 (unsigned long long)h[3], h[0] / n, h[1] / n, h[2] / n);
  }
  if (c->ev_profile)
    for (int k = 0; k < 4; ++k)
      std::fprintf(stderr, "ksched events kind %d: %llu runs, %llu events, %.3f s\n", k,
                   (unsigned long long)c->ev_prof[k].runs, (unsigned long long)c->ev_prof[k].events, c->ev_prof[k].s);
  c->runq->stop();
  (void)hipSetDevice(c->cfg.device);
  // bounded (a wedged context gets one more full timeout to finish)
  const bool was_wedged = c->wedged.load();
  c->wedged = false;
  for (hipStream_t st : {c->stream, c->rstream, c->sstream})
    if (st && !c->wedged) (void)sync_bounded(c, st, "ks_close");
  if (was_wedged && !c->wedged)
    std::fprintf(stderr, "ksched: the stalled device work of a wedged context finished before ks_close\n");
  if (c->wedged) {
    // device work of this context may never finish: free nothing it may use
    std::fprintf(stderr, "ksched: closing a wedged context; its device memory and streams are left allocated\n");
    delete c;
    return;
  }
  if (c->comm) ncclCommDestroy(c->comm);
  for (auto &e : c->lg_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->d_lgstage) (void)hipFree(c->d_lgstage);
  void *bufs[] = {c->t.acpu, c->t.amem, c->t.rcpu, c->t.rmem, c->t.zcpu, c->t.zmem, c->t.apods,
                  c->t.npods, c->t.hard, c->t.prefer, c->t.lab, c->t.num, c->d_shards, c->d_slot_pos,
                  c->d_start, c->d_norm, c->d_norm_inv, c->d_pstat, c->d_fix, c->d_brec, c->d_srec, c->d_frec,
                  c->d_counters, c->d_crow, c->d_cext, c->d_pipe, c->d_carry, c->d_flags, c->d_dom, c->d_dedup,
                  c->d_pos_slot, c->d_dcnt, c->d_dflag, c->d_acc, c->d_sst, c->d_sraw, c->d_spart,
                  c->d_xalloc, c->d_tcnt, c->d_adcnt, c->d_sraw2, c->d_rk_keys, c->d_rk_sorted, c->d_rk_val,
                  c->d_rk_sval, c->d_rk_gstart, c->d_rk_ctl, c->d_rk_tmp, c->d_rk_prof, c->d_win, c->d_win_st};
  for (void *b : bufs)
    if (b) (void)hipFree(b);
  if (c->h_start) (void)hipHostFree(c->h_start);
  if (c->h_seg) (void)hipHostFree(c->h_seg);
  if (c->h_rk_ctl) (void)hipHostFree(c->h_rk_ctl);
  if (c->h_diag) (void)hipHostFree(c->h_diag);
  if (c->xm.pin) (void)hipHostFree(c->xm.pin);
  if (c->xm.dscr) (void)hipFree(c->xm.dscr);
  for (void *g : c->graveyard) (void)hipFree(g);
  for (void *g : c->pinned_graveyard) (void)hipHostFree(g);
  for (ks_batch *b : c->all_batches) {
    for (void *p : {(void *)b->d_pods, (void *)b->d_pinv, (void *)b->d_clauses, (void *)b->d_results,
                    (void *)b->d_cmask, (void *)b->d_marks, (void *)b->d_cls})
      if (p) (void)hipFree(p);
    for (void *p : {(void *)b->h_results, (void *)b->h_pods, (void *)b->h_pinv, (void *)b->h_clauses,
                    (void *)b->h_cmask, (void *)b->h_cls})
      if (p) (void)hipHostFree(p);
    delete b;
  }
  for (auto &pr : c->ev_sweep) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
  for (auto &pr : c->ev_resolve) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
  for (auto &pr : c->ev_spread) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
  for (auto &r : c->ev_runs) { (void)hipEventDestroy(r.e0); (void)hipEventDestroy(r.e1); }
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  for (int q = 0; q < 2; ++q) {
    if (c->ev_sw[q]) (void)hipEventDestroy(c->ev_sw[q]);
    if (c->ev_res[q]) (void)hipEventDestroy(c->ev_res[q]);
    if (c->ev_swept[q]) (void)hipEventDestroy(c->ev_swept[q]);
    if (c->ev_fixed[q]) (void)hipEventDestroy(c->ev_fixed[q]);
  }
  if (c->diag_stream && hipStreamQuery(c->diag_stream) == hipSuccess) (void)hipStreamDestroy(c->diag_stream);
  if (c->rstream) (void)hipStreamDestroy(c->rstream);
  if (c->sstream) (void)hipStreamDestroy(c->sstream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

ks_status ks_nodes_upsert(ks_ctx *c, const ks_node *nodes, const uint32_t *slots, uint32_t n) {
  const uint32_t nodes_n = n;
  if (!c || (n && (!nodes || !slots))) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  c->tuple_version++;
  HIPC(c, hipSetDevice(c->cfg.device));
  // Events are applied in order; a slot named twice in one call ends in its
  // last state (one device row per distinct slot, so the scatter is race-free).
  std::vector<uint32_t> pos;
  std::vector<int64_t> core;
  std::vector<uint64_t> ext;
  std::unordered_map<uint32_t, uint32_t> row_of;  // slot -> row in the upload
  bool grew = false;
  // Validate the whole call first so that a rejected call changes nothing.
  {
    std::unordered_set<uint32_t> in_call(slots, slots + n);
    std::unordered_map<std::string, uint32_t> call_names;
    for (uint32_t i = 0; i < n; ++i) {
      const ks_node &s = nodes[i];
      const uint32_t slot = slots[i];
      if (slot >= c->cap) return c->fail(KS_ERR_NOT_FOUND, "slot %u >= capacity %u", slot, c->cap);
      if (s.alloc_milli_cpu < 0 || s.alloc_milli_cpu >= kMaxAlloc || s.alloc_memory < 0 ||
          s.alloc_memory >= kMaxAlloc || s.alloc_pods < 0 || s.alloc_pods > INT32_MAX - 1)
        return c->fail(KS_ERR_RANGE, "node %s allocatable outside the exact range", str(s.name).c_str());
      // extended / ephemeral columns are only compared (Fit: request >
      // Allocatable - Requested, exact int64), so any non-negative int64 is
      // exact; the 2^44 bound is LeastAllocated's (cpu and memory only)
      for (uint32_t k = 0; k < s.n_extended; ++k)
        if (s.extended && s.extended[k].value < 0)
          return c->fail(KS_ERR_RANGE, "node %s extended allocatable negative", str(s.name).c_str());
      // node names are unique (metadata.name matchFields resolve a name to one slot)
      const std::string nm = str(s.name);
      auto ci = call_names.emplace(nm, slot);
      if (!ci.second && ci.first->second != slot)
        return c->fail(KS_ERR_INVALID, "node name %s given to slots %u and %u", nm.c_str(), ci.first->second, slot);
      const int64_t nid = c->lookup(s.name);
      if (nid >= 0) {
        auto it = c->name_slot.find((uint32_t)nid);
        if (it != c->name_slot.end() && it->second != slot && c->nodes[it->second].present &&
            !in_call.count(it->second))
          return c->fail(KS_ERR_INVALID, "node name %s already names slot %u", nm.c_str(), it->second);
      }
    }
  }
  for (uint32_t i = 0; i < n; ++i) {
    const ks_node &s = nodes[i];
    const uint32_t slot = slots[i];
    HostNode &h = c->nodes[slot];
    const bool is_new = !h.present;
    const uint32_t nid = c->intern(s.name);
    if (is_new || h.name != nid) c->names_version++;
    if (!is_new) {
      c->name_slot.erase(h.name);  // key_nodes entries are re-validated lazily
      node_images_ref(c, h, -1);
    } else {
      c->n_present++;
    }
    h.present = true;
    c->present_map[slot] = 1;
    h.name = nid;
    c->name_slot[h.name] = slot;
    std::vector<std::pair<std::string, int64_t>> old_images;
    old_images.swap(h.images);
    {
      // one entry per name, the first occurrence's size (addNodeImageStates)
      std::unordered_set<std::string> seen;
      for (uint32_t k = 0; k < s.n_images; ++k)
        if (s.images && s.images[k].name && s.images[k].name[0] && seen.insert(str(s.images[k].name)).second)
          h.images.emplace_back(str(s.images[k].name), s.images[k].size_bytes);
      std::sort(h.images.begin(), h.images.end());
    }
    node_images_ref(c, h, +1);
    // prepared pods' ImageLocality terms (sizes, node counts) may have changed
    if (h.images != old_images || (is_new && !h.images.empty())) grew = true;
    h.acpu = s.alloc_milli_cpu;
    h.amem = s.alloc_memory;
    h.apods = s.alloc_pods;
    h.unschedulable = s.unschedulable != 0;
    h.labels.clear();
    for (uint32_t k = 0; k < s.n_labels; ++k) {
      const uint32_t key = c->intern(s.labels[k].key);
      h.labels.emplace_back(key, c->intern(s.labels[k].value));
      c->key_nodes[key].push_back(slot);
    }
    for (auto &im : h.images) {  // ImageLocality: "image present" keys in the label bitset
      const uint32_t key = c->intern(image_key(im.first).c_str());
      h.labels.emplace_back(key, 0u);
      c->key_nodes[key].push_back(slot);
    }
    if (!is_new) prefer_mask_ref(c, h.prefer, -1);
    h.hard_taints.clear();
    h.prefer_taints.clear();
    for (uint32_t k = 0; k < s.n_taints; ++k) {
      const ks_taint &tt = s.taints[k];
      const uint32_t key = c->intern(tt.key), val = c->intern(tt.value);
      if (tt.effect == KS_EFFECT_NO_SCHEDULE || tt.effect == KS_EFFECT_NO_EXECUTE)
        h.hard_taints.push_back({key, val, (uint32_t)tt.effect});
      else if (tt.effect == KS_EFFECT_PREFER_NO_SCHEDULE)
        h.prefer_taints.emplace_back(key, val);
      // other effects are ignored by both TaintToleration filters and scores
    }
    bool rebuilt = false;
    if (encode_taints(c, h, &grew) == KS_ERR_CAPACITY) {
      // dictionary full of taints no present node may carry any more: rebuild
      // it from the present nodes (this one included) and re-encode them all
      if (ks_status st = rebuild_taint_dicts(c)) return st;
      grew = rebuilt = true;
    }
    if ((h.hard & ~c->hard_in_use) || (h.prefer & ~c->prefer_in_use)) grew = true;
    c->hard_in_use |= h.hard;
    c->prefer_in_use |= h.prefer;
    if (!rebuilt) prefer_mask_ref(c, h.prefer, +1);  // (the rebuild counted it)
    node_ext_bits(c, h);
    auto ins = row_of.emplace(slot, (uint32_t)pos.size());
    const uint32_t row = ins.first->second;
    if (ins.second) {
      pos.push_back(c->slot_pos[slot]);
      core.resize(core.size() + 8);
      ext.resize(ext.size() + 2 + LW + NNUM);
      core[(size_t)row * 8 + 3] = is_new ? 1 : 0;  // reset Requested iff absent before this call
    }
    int64_t *cr = &core[(size_t)row * 8];
    cr[0] = h.acpu;
    cr[1] = h.amem;
    cr[2] = h.apods;
    uint64_t *e = &ext[(size_t)row * (2 + LW + NNUM)];
    e[0] = h.hard;
    e[1] = h.prefer;
    for (int k = 0; k < LW; ++k) e[2 + k] = h.lab[k];
    for (int k = 0; k < NNUM; ++k) e[2 + LW + k] = (uint64_t)h.num[k];
  }
  if (grew) c->dict_version++;
  n = (uint32_t)pos.size();
  if (!n) return KS_OK;
  const size_t bytes = (size_t)n * 4 + core.size() * 8 + ext.size() * 8 + 1024;
  ks_status st = xfer_begin(c, bytes, bytes);
  if (st) return st;
  uint32_t *d_pos = dscratch<uint32_t>(c, n);
  int64_t *d_core = dscratch<int64_t>(c, core.size());
  uint64_t *d_ext = dscratch<uint64_t>(c, ext.size());
  if ((st = h2d(c, d_pos, pos.data(), (size_t)n * 4)) || (st = h2d(c, d_core, core.data(), core.size() * 8)) ||
      (st = h2d(c, d_ext, ext.data(), ext.size() * 8)))
    return st;
  HIPC(c, launch_scatter_rows(c->t, d_pos, d_core, d_ext, n, 1u, c->stream));
  if ((st = xfer_sync(c))) return st;
  std::vector<uint32_t> changed;
  changed.reserve(row_of.size());
  for (auto &kv : row_of) changed.push_back(kv.first);
  // extended allocatable (ephemeral-storage, scalar resources): columns for
  // every name first, then every column's value of every upserted node; a new
  // node's Requested starts at 0
  std::unordered_map<uint32_t, uint32_t> last;  // slot -> index of its last state in the call
  for (uint32_t i = 0; i < nodes_n; ++i) last[slots[i]] = i;
  for (uint32_t i = 0; i < nodes_n; ++i)
    for (uint32_t k = 0; k < nodes[i].n_extended; ++k) {
      const std::string nm = str(nodes[i].extended[k].name);
      if (!xres_name_ok(nm)) continue;
      uint32_t col;
      if ((st = xres_column(c, c->intern(nm.c_str()), true, &col)) == KS_ERR_UNSUPPORTED) continue;  // ignored
      if (st) return st;
    }
  if (!c->xres_names.empty()) {
    std::vector<uint64_t> idx;
    std::vector<int64_t> val;
    const uint64_t nx = (uint64_t)MAX_XRES * c->npos;
    for (auto &kv : last) {
      const ks_node &nd = nodes[kv.second];
      const uint64_t pos = c->slot_pos[kv.first];
      std::vector<int64_t> a(c->xres_names.size(), 0);
      for (uint32_t k = 0; k < nd.n_extended; ++k) {
        auto it = c->xres_of.find((uint32_t)c->lookup(nd.extended[k].name));
        if (nd.extended[k].name && it != c->xres_of.end() && xres_name_ok(str(nd.extended[k].name)))
          a[it->second] = nd.extended[k].value;
      }
      for (uint32_t col = 0; col < a.size(); ++col) {  // (values validated above: >= 0)
        idx.push_back(col * (uint64_t)c->npos + pos);
        val.push_back(a[col]);
        if (core[(size_t)row_of[kv.first] * 8 + 3]) {  // new node: Requested = 0
          idx.push_back(nx + col * (uint64_t)c->npos + pos);
          val.push_back(0);
        }
      }
    }
    if ((st = xres_scatter(c, idx, val, false))) return st;
  }
  return spread_nodes_changed(c, changed.data(), (uint32_t)changed.size(), false);
}

// Per-item form (include/ksched.h): every item is validated on its own and
// only the valid ones are applied, as one ks_nodes_upsert call.
ks_status ks_nodes_upsert_each(ks_ctx *c, const ks_node *nodes, const uint32_t *slots, uint32_t n, ks_status *status) {
  if (!c || !status || (n && (!nodes || !slots))) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  std::vector<ks_node> ok_nodes;
  std::vector<uint32_t> ok_slots, ok_idx;
  ks_status first = KS_OK;
  std::string first_err;
  std::vector<std::string> why(n);
  // Pass 1: what each item decides alone (slot, ranges).
  for (uint32_t i = 0; i < n; ++i) {
    const ks_node &s = nodes[i];
    const uint32_t slot = slots[i];
    ks_status st = KS_OK;
    const std::string nm = str(s.name);
    if (slot >= c->cap) {
      st = KS_ERR_NOT_FOUND;
      why[i] = "slot " + std::to_string(slot) + " >= capacity";
    } else if (s.alloc_milli_cpu < 0 || s.alloc_milli_cpu >= kMaxAlloc || s.alloc_memory < 0 ||
               s.alloc_memory >= kMaxAlloc || s.alloc_pods < 0 || s.alloc_pods > INT32_MAX - 1) {
      st = KS_ERR_RANGE;
      why[i] = "node " + nm + " allocatable outside the exact range";
    } else {
      for (uint32_t k = 0; k < s.n_extended && !st; ++k)
        if (s.extended && s.extended[k].value < 0) {
          st = KS_ERR_RANGE;
          why[i] = "node " + nm + " extended allocatable negative";
        }
    }
    status[i] = st;
  }
  // Pass 2: node-name uniqueness, judged against the items still accepted.
  // A name may move off a slot only if that slot's own item is applied too,
  // so a rejection can reject another item: repeat until nothing changes
  // (rejections only shrink the accepted set, so this ends).
  for (bool changed = true; changed;) {
    changed = false;
    std::unordered_set<uint32_t> in_call;
    for (uint32_t i = 0; i < n; ++i)
      if (!status[i]) in_call.insert(slots[i]);
    std::unordered_map<std::string, uint32_t> call_names;  // accepted items' names -> slot
    for (uint32_t i = 0; i < n; ++i) {
      if (status[i]) continue;
      const ks_node &s = nodes[i];
      const uint32_t slot = slots[i];
      const std::string nm = str(s.name);
      auto ci = call_names.emplace(nm, slot);
      if (!ci.second && ci.first->second != slot) {
        status[i] = KS_ERR_INVALID;
        why[i] = "node name " + nm + " given to two slots";
        changed = true;
        continue;
      }
      const int64_t nid = c->lookup(s.name);
      if (nid >= 0) {
        auto it = c->name_slot.find((uint32_t)nid);
        if (it != c->name_slot.end() && it->second != slot && c->nodes[it->second].present &&
            !in_call.count(it->second)) {
          status[i] = KS_ERR_INVALID;
          why[i] = "node name " + nm + " already names another slot";
          changed = true;
        }
      }
    }
  }
  for (uint32_t i = 0; i < n; ++i) {
    if (status[i]) {
      if (!first) {
        first = status[i];
        first_err = why[i];
      }
      continue;
    }
    ok_nodes.push_back(nodes[i]);
    ok_slots.push_back(slots[i]);
    ok_idx.push_back(i);
  }
  if (!ok_nodes.empty()) {
    if (ks_status st = ks_nodes_upsert(c, ok_nodes.data(), ok_slots.data(), (uint32_t)ok_nodes.size())) {
      for (uint32_t i : ok_idx) status[i] = st;  // a call-level failure (capacity, device): nothing applied
      return st;
    }
  }
  if (first) return c->fail(first, "%s (the other items were applied)", first_err.c_str());
  return KS_OK;
}

ks_status ks_nodes_delete(ks_ctx *c, const uint32_t *slots, uint32_t n) {
  if (!c || (n && !slots)) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  c->tuple_version++;
  HIPC(c, hipSetDevice(c->cfg.device));
  // every slot is checked before anything changes: a missing or repeated
  // slot fails the call with the host mirror and the device table untouched
  {
    std::unordered_set<uint32_t> seen;
    for (uint32_t i = 0; i < n; ++i) {
      if (slots[i] >= c->cap || !c->nodes[slots[i]].present)
        return c->fail(KS_ERR_NOT_FOUND, "slot %u not present", slots[i]);
      if (!seen.insert(slots[i]).second) return c->fail(KS_ERR_INVALID, "slot %u deleted twice in one call", slots[i]);
    }
  }
  // the deleted nodes' records go with them: replayed now when term counts
  // need them, else a clear entry in the log
  const bool unread = pod_records_unread(c);
  if (!unread) flush_bound(c);
  std::vector<uint32_t> pos(n);
  std::vector<int64_t> core((size_t)n * 8, 0);
  for (uint32_t i = 0; i < n; ++i) {
    HostNode &h = c->nodes[slots[i]];
    if (unread) c->pending_bound.push_back({slots[i], 0u, 0});
    for (uint32_t set : h.pod_sets)
      for (auto &t : c->label_sets[set].terms) c->terms[t.first].bound--;
    c->name_slot.erase(h.name);
    c->names_version++;
    prefer_mask_ref(c, h.prefer, -1);
    node_images_ref(c, h, -1);
    h = HostNode();
    c->present_map[slots[i]] = 0;
    c->n_present--;
    pos[i] = c->slot_pos[slots[i]];
    core[(size_t)i * 8 + 2] = -1;  // apods < 0: empty slot
    core[(size_t)i * 8 + 3] = 1;   // reset requested state
  }
  if (!n) return KS_OK;
  const size_t bytes = (size_t)n * 4 + core.size() * 8 + 1024;
  ks_status st = xfer_begin(c, bytes, bytes);
  if (st) return st;
  uint32_t *d_pos = dscratch<uint32_t>(c, n);
  int64_t *d_core = dscratch<int64_t>(c, core.size());
  if ((st = h2d(c, d_pos, pos.data(), (size_t)n * 4)) || (st = h2d(c, d_core, core.data(), core.size() * 8)))
    return st;
  HIPC(c, launch_scatter_rows(c->t, d_pos, d_core, nullptr, n, 0u, c->stream));
  if ((st = xfer_sync(c))) return st;
  if (!c->xres_names.empty()) {  // extended Allocatable / Requested leave with the node
    std::vector<uint64_t> idx;
    std::vector<int64_t> val;
    const uint64_t nx = (uint64_t)MAX_XRES * c->npos;
    for (uint32_t i = 0; i < n; ++i)
      for (uint32_t col = 0; col < c->xres_names.size(); ++col) {
        idx.push_back(col * (uint64_t)c->npos + pos[i]);
        idx.push_back(nx + col * (uint64_t)c->npos + pos[i]);
        val.push_back(0);
        val.push_back(0);
      }
    if ((st = xres_scatter(c, idx, val, false))) return st;
  }
  return spread_nodes_changed(c, slots, n, true);
}

// pods[i] points at pod i (ks_events_apply passes its events' pointers: no
// copy of the ks_pod structs)
static ks_status pods_delta(ks_ctx *c, const ks_pod *const *pods, const uint32_t *slots, uint32_t n, int sign) {
  if (!c || (n && (!pods || !slots))) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  if (!n) return KS_OK;
  HIPC(c, hipSetDevice(c->cfg.device));
  std::vector<uint32_t> pos(n);
  std::vector<int64_t> d((size_t)n * 5);
  int64_t aff = 0;
  // NodeInfo.Requested of the extended resources (validated before any device work)
  std::vector<uint64_t> xidx;
  std::vector<int64_t> xval;
  std::vector<std::pair<uint32_t, int64_t>> xr;
  std::vector<uint32_t> sets(n);
  // term classes held until the bound counts are applied (released on every return)
  struct Hold {
    ks_ctx *c;
    std::vector<uint32_t> v;
    ~Hold() {
      for (uint32_t t : v) term_activate(c, t, 0, -1);
    }
  } hold{c, {}};
  // Large logs (a burst's bound-pod deletions: ~150k pods): the per-pod work
  // that reads only the pod and the slot maps runs on a few threads (it is
  // memory-latency bound: scattered pod structs and slot entries).  Pods
  // that need more (an interned label set other than a namespace's empty
  // one, extended resources) and every error take the serial loop below,
  // which then reproduces the first failure exactly.
  std::vector<uint8_t> done(n, 0);
  if (n >= 8192) {
    const uint32_t T = std::min<uint32_t>(8, std::max(1u, std::thread::hardware_concurrency()));
    std::vector<int64_t> affs(T, 0);
    parallel_chunks(n, T, [&](uint32_t t, uint32_t lo, uint32_t hi) {
      for (uint32_t i = lo; i < hi; ++i) {
        if (slots[i] >= c->cap || !c->present_map[slots[i]]) continue;
        const ks_pod &pd = *pods[i];
        if (pd.n_namespace_labels || pd.n_affinity_terms || pd.n_labels) continue;
        bool ext = false;
        for (uint32_t k = 0; k < pd.n_containers; ++k) ext |= pd.containers[k].n_extended != 0;
        for (uint32_t k = 0; k < pd.n_init_containers; ++k) ext |= pd.init_containers[k].n_extended != 0;
        if (ext) continue;
        auto it = c->empty_set_of_ns.find(str(pd.ns));  // read-only here: no thread interns
        if (it == c->empty_set_of_ns.end()) continue;
        int64_t rc, rm, zc, zm;
        if (pod_requests(pd, false, &rc, &rm) || pod_requests(pd, true, &zc, &zm)) continue;
        sets[i] = it->second;
        if (pd.unmodelled & KS_UNMODELLED_POD_AFFINITY) affs[t] += sign;
        pos[i] = c->slot_pos[slots[i]];
        int64_t *x = &d[(size_t)i * 5];
        x[0] = sign * rc;
        x[1] = sign * rm;
        x[2] = sign * zc;
        x[3] = sign * zm;
        x[4] = sign;
        done[i] = 1;
      }
    });
    for (int64_t v : affs) aff += v;
  }
  for (uint32_t i = 0; i < n; ++i) {
    if (done[i]) continue;
    if (slots[i] >= c->cap || !c->present_map[slots[i]])
      return c->fail(KS_ERR_NOT_FOUND, "slot %u not present", slots[i]);
    int64_t rc, rm, zc, zm;
    ks_status st;
    const ks_pod &pd = *pods[i];
    if ((st = intern_set(c, pd, &sets[i], &hold.v))) return st;
    if ((st = pod_requests(pd, false, &rc, &rm)) || (st = pod_requests(pd, true, &zc, &zm)))
      return c->fail(st, "pod requests a resource it cannot express (KS_REQ_HAS_OTHER)");
    if ((st = pod_xrequests(c, pd, true, &xr))) return st;
    for (auto &x : xr) {
      xidx.push_back((uint64_t)MAX_XRES * c->npos + x.first * (uint64_t)c->npos + c->slot_pos[slots[i]]);
      xval.push_back(sign * x.second);
    }
    if (pd.unmodelled & KS_UNMODELLED_POD_AFFINITY) aff += sign;
    pos[i] = c->slot_pos[slots[i]];
    int64_t *x = &d[(size_t)i * 5];
    x[0] = sign * rc;
    x[1] = sign * rm;
    x[2] = sign * zc;
    x[3] = sign * zm;
    x[4] = sign;
  }
  const size_t bytes = (size_t)n * 4 + d.size() * 8 + 1024;
  ks_status st = xfer_begin(c, bytes, bytes);
  if (st) return st;
  uint32_t *d_pos = dscratch<uint32_t>(c, n);
  int64_t *d_d = dscratch<int64_t>(c, d.size());
  if ((st = h2d(c, d_pos, pos.data(), (size_t)n * 4)) || (st = h2d(c, d_d, d.data(), d.size() * 8))) return st;
  HIPC(c, launch_apply_deltas(c->t, d_pos, d_d, n, c->stream));
  c->affinity_pods += aff;
  if ((st = xfer_sync(c))) return st;
  if ((st = xres_scatter(c, xidx, xval, true))) return st;
  return spread_pods_delta(c, sets.data(), slots, n, sign);
}

static std::vector<const ks_pod *> pod_ptrs(const ks_pod *pods, uint32_t n) {
  std::vector<const ks_pod *> v(n);
  for (uint32_t i = 0; i < n; ++i) v[i] = pods + i;
  return v;
}

ks_status ks_pods_add(ks_ctx *c, const ks_pod *pods, const uint32_t *slots, uint32_t n) {
  if (n && !pods) return KS_ERR_INVALID;
  return pods_delta(c, pod_ptrs(pods, n).data(), slots, n, +1);
}
ks_status ks_pods_remove(ks_ctx *c, const ks_pod *pods, const uint32_t *slots, uint32_t n) {
  if (n && !pods) return KS_ERR_INVALID;
  return pods_delta(c, pod_ptrs(pods, n).data(), slots, n, -1);
}

ks_status ks_snapshot_update(ks_ctx *c, const ks_node_info *items, uint32_t n, int64_t *generation,
                             uint32_t *applied) {
  if (!c || (n && !items)) return KS_ERR_INVALID;
  if (c->slot_gen.size() != c->cap) c->slot_gen.assign(c->cap, INT64_MIN);
  // newest item per slot (validated before anything changes)
  std::unordered_map<uint32_t, uint32_t> best;
  for (uint32_t i = 0; i < n; ++i) {
    const ks_node_info &it = items[i];
    if (it.slot >= c->cap) return c->fail(KS_ERR_NOT_FOUND, "item %u: slot %u >= capacity %u", i, it.slot, c->cap);
    if (!it.deleted && !it.node) return c->fail(KS_ERR_INVALID, "item %u: no node", i);
    if (it.generation <= c->slot_gen[it.slot]) continue;  // already in the snapshot
    auto r = best.emplace(it.slot, i);
    if (!r.second && items[r.first->second].generation < it.generation) r.first->second = i;
  }
  std::vector<uint32_t> order;
  order.reserve(best.size());
  for (auto &kv : best) order.push_back(kv.second);
  std::sort(order.begin(), order.end());  // call order (deterministic)
  std::vector<uint32_t> del;
  std::vector<uint32_t> up_slots;
  std::vector<ks_node> up;
  for (uint32_t i : order) {
    const ks_node_info &it = items[i];
    if (it.deleted) {
      if (c->nodes[it.slot].present) del.push_back(it.slot);
    } else {
      up_slots.push_back(it.slot);
      up.push_back(*it.node);
    }
  }
  ks_status st;
  auto record = [&](bool deleted) {
    for (uint32_t i : order)
      if ((items[i].deleted != 0) == deleted) {
        c->slot_gen[items[i].slot] = items[i].generation;
        c->snapshot_gen = std::max(c->snapshot_gen, items[i].generation);
      }
  };
  if (!del.empty() && (st = ks_nodes_delete(c, del.data(), (uint32_t)del.size()))) return st;  // nothing changed
  record(true);  // the deletions are in: a failing upsert below leaves them recorded (a retry skips them)
  if (!up.empty() && (st = ks_nodes_upsert(c, up.data(), up_slots.data(), (uint32_t)up.size()))) {
    std::string e = ks_last_error(c);
    return c->fail(st, "%s (the call's %zu deletions were applied)", e.c_str(), del.size());
  }
  record(false);
  if (generation) *generation = c->snapshot_gen;
  if (applied) *applied = (uint32_t)order.size();
  return KS_OK;
}

ks_status ks_events_apply(ks_ctx *c, const ks_event *ev, uint32_t n) {
  if (!c || (n && !ev)) return KS_ERR_INVALID;
  std::vector<const ks_pod *> pods;
  std::vector<ks_node> nodes;
  std::vector<uint32_t> slots;
  for (uint32_t i = 0; i < n;) {
    const int32_t kind = ev[i].kind;
    if (kind < KS_EV_POD_ADD || kind > KS_EV_NODE_DELETE)
      return c->fail(KS_ERR_INVALID, "event %u: unknown kind %d", i, kind);
    uint32_t j = i;
    pods.clear();
    nodes.clear();
    slots.clear();
    for (; j < n && ev[j].kind == kind; ++j) {
      slots.push_back(ev[j].slot);
      if (kind == KS_EV_POD_ADD || kind == KS_EV_POD_REMOVE) {
        if (!ev[j].pod) return c->fail(KS_ERR_INVALID, "event %u: no pod", j);
        pods.push_back(ev[j].pod);
      } else if (kind == KS_EV_NODE_UPSERT) {
        if (!ev[j].node) return c->fail(KS_ERR_INVALID, "event %u: no node", j);
        nodes.push_back(*ev[j].node);
      }
    }
    const uint32_t m = j - i;
    ks_status st = KS_OK;
    const auto t0 = std::chrono::steady_clock::now();
    switch (kind) {
      case KS_EV_POD_ADD: st = pods_delta(c, pods.data(), slots.data(), m, +1); break;
      case KS_EV_POD_REMOVE: st = pods_delta(c, pods.data(), slots.data(), m, -1); break;
      case KS_EV_NODE_UPSERT: st = ks_nodes_upsert(c, nodes.data(), slots.data(), m); break;
      default: st = ks_nodes_delete(c, slots.data(), m); break;
    }
    if (c->ev_profile) {
      c->ev_prof[kind].runs++;
      c->ev_prof[kind].events += m;
      c->ev_prof[kind].s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    if (st) return st;
    i = j;
  }
  return KS_OK;
}

// Compile a batch's pods into dev / cl under c->mu.  When the label
// dictionary runs out of bits, reclaim it once (reset_label_dict, after the
// submitted batches drained) and compile the batch again from its first pod.
// Between two pods of a compile under `mu`: when the batch worker waits for
// `mu` (the start or end of a run), let it in.  Every pod's compile leaves the
// dictionaries, label sets and classes consistent, and what the worker does
// there reads them or uploads label rows (a superset of what the running
// batch needs is harmless), so a compile may be interleaved with it.
static void compile_yield(ks_ctx *c, std::unique_lock<std::mutex> &lk, uint32_t i) {
  if ((i & 255u) != 255u || c->mu_wanted.load(std::memory_order_relaxed) == 0) return;
  lk.unlock();
  const auto t0 = std::chrono::steady_clock::now();
  while (c->mu_wanted.load() != 0 && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(20))
    std::this_thread::yield();
  lk.lock();
}

static ks_status compile_batch(ks_ctx *c, const ks_pod *pods, uint32_t n, PodDev *dev, ProgBuf &cl,
                               std::unique_lock<std::mutex> &lk, bool create_spread = false,
                               std::vector<uint32_t> *class_refs = nullptr) {
  for (int attempt = 0;; ++attempt) {
    cl.w.clear();
    c->compile_used_names = false;
    if (class_refs) class_release(c, class_refs);
    ks_status st = KS_OK;
    for (uint32_t i = 0; i < n && !st; ++i) {
      st = compile_pod(c, pods[i], dev[i], cl, create_spread, class_refs);
      compile_yield(c, lk, i);
    }
    if (st && class_refs) class_release(c, class_refs);
    if (st != KS_ERR_CAPACITY || attempt > 0 || c->next_bit == 0) return st;
    lk.unlock();
    drain_async(c);
    lk.lock();
    c->undrained = false;  // drained: the retry may create columns
    reset_label_dict(c);
  }
}

ks_status ks_pods_check(ks_ctx *c, const ks_pod *pods, uint32_t n, ks_status *status) {
  if (!c || (n && (!pods || !status))) return KS_ERR_INVALID;
  std::unique_lock<std::mutex> g(c->mu);
  ks_status first = KS_OK;
  std::string first_err;
  for (uint32_t i = 0; i < n; ++i) {
    PodDev d;
    ProgBuf cl;
    status[i] = compile_batch(c, &pods[i], 1, &d, cl, g);
    if (status[i] && !first) {
      first = status[i];
      std::lock_guard<std::mutex> ge(c->err_mu);
      first_err = "pod " + std::to_string(i) + ": " + c->err;
    }
  }
  if (first) c->fail(first, "%s", first_err.c_str());
  return first;
}

ks_status ks_batch_prepare(ks_ctx *c, const ks_pod *pods, uint32_t n, ks_batch **out) {
  if (!c || !out || (n && !pods)) return KS_ERR_INVALID;
  *out = nullptr;
  HIPC(c, hipSetDevice(c->cfg.device));
  std::vector<PodDev> dev(std::max<uint32_t>(n, 1));
  ProgBuf cl;
  bool ext = false, norm = false;
  uint32_t dict_v, names_v;
  ks_status st;
  // Spread pods may create topology / selector-class / term columns, computed
  // from the host's records of bound pods, which needs every submitted batch
  // finished.  The compile first runs without waiting and refuses to create
  // any (KS_NEED_DRAIN): a running deployment's batches reference columns
  // that exist, and their compile overlaps the batch in flight.  Otherwise it
  // drains and compiles again.
  bool any_solo = false;
  {
    std::lock_guard<std::mutex> g(c->mu);
    for (uint32_t i = 0; i < n && !any_solo; ++i) any_solo = may_need_solo(c, pods[i]);
  }
  bool drained = !any_solo;
  if (!drained) drained = c->runq->idle();
  const auto tp0 = std::chrono::steady_clock::now();
  auto tp1 = tp0;
  std::vector<uint32_t> set_ids(n), refs, term_refs;
  for (;;) {
    {
      // compile against the host dictionaries (the worker reads t.lw and the
      // dirty label rows under mu)
      std::unique_lock<std::mutex> g(c->mu);
      c->undrained = !drained;
      // label sets first: they create the term classes of the pods' own terms,
      // which every later pod of the batch that they select must see
      st = KS_OK;
      for (uint32_t i = 0; i < n && !st; ++i) {
        st = intern_set(c, pods[i], &set_ids[i], &term_refs);
        compile_yield(c, g, i);
      }
      if (!st) st = compile_batch(c, pods, n, dev.data(), cl, g, true, &refs);
      c->undrained = false;
      if (st) {
        for (uint32_t t : term_refs) term_activate(c, t, 0, -1);
        class_release(c, &refs);
        if (st != KS_NEED_DRAIN) return st;
        term_refs.clear();
        set_ids.assign(n, 0);
        dev.assign(std::max<uint32_t>(n, 1), PodDev{});
        cl = ProgBuf();
      } else {
        for (uint32_t i = 0; i < n; ++i) {
          if (dev[i].flags & PF_SOLO) continue;  // the one-pod path evaluates it
          if (dev[i].flags & PF_EXT) ext = true;
          if (dev[i].flags & (PF_TT | PF_NA)) norm = true;
        }
        dict_v = c->dict_version;
        names_v = c->compile_used_names ? c->names_version : 0;
      }
    }
    if (st != KS_NEED_DRAIN) break;
    drain_async(c);
    drained = true;
    tp1 = std::chrono::steady_clock::now();
  }
  const auto tp2 = std::chrono::steady_clock::now();
  if (norm) ext = true;
  if (cl.w.empty()) cl.w.push_back(0);
  ks_batch *b = nullptr;
  if ((st = batch_acquire(c, n, cl.w.size(), &b))) {
    std::lock_guard<std::mutex> g(c->mu);
    class_release(c, &refs);
    for (uint32_t t : term_refs) term_activate(c, t, 0, -1);
    return st;
  }
  b->n = n;
  b->ext = ext;
  b->norm = norm;
  b->dict_version = dict_v;
  b->names_version = names_v;
  b->n_words = cl.w.size();
  b->set_ids = std::move(set_ids);
  b->class_refs = std::move(refs);
  b->term_refs = std::move(term_refs);
  b->spread.assign(n, 0);
  b->any_spread = false;
  b->rep.assign(n, 0);
  for (uint32_t i = 0; i < n; ++i) {
    if (!(dev[i].flags & PF_SOLO)) continue;
    const SoloHdr *hd = reinterpret_cast<const SoloHdr *>(cl.w.data() + dev[i].solo_off);
    b->spread[i] = (uint8_t)(0x80u | solo_passes(hd));
    b->any_spread = true;
    if (!replica_program(dev[i], hd)) continue;
    b->rep[i] = 1;
    if (i > 0 && b->rep[i - 1] && b->set_ids[i] == b->set_ids[i - 1] &&
        same_pod_program(dev[i - 1], dev[i], cl.w.data()))
      b->rep[i] |= 2;
  }
  std::memcpy(b->h_pods, dev.data(), dev.size() * sizeof(PodDev));
  b->dups = pod_classes(dev.data(), n, b->h_cls);
  for (size_t i = 0; i < dev.size(); ++i) {
    b->h_pinv[2 * i] = dev[i].tt_guess ? 1.0 / (double)dev[i].tt_guess : 0.0;
    b->h_pinv[2 * i + 1] = dev[i].na_guess ? 1.0 / (double)dev[i].na_guess : 0.0;
  }
  std::memcpy(b->h_clauses, cl.w.data(), cl.w.size() * 8);
  b->uploaded = false;
  if (c->runq->idle()) {
    // nothing in flight: upload now, so the run starts with every input
    // resident in HBM (the scheduler stream is ours until ks_batch_submit)
    {
      std::lock_guard<std::mutex> g(c->mu);
      if ((st = upload_dirty_ext(c, c->xm))) {
        batch_release(c, b);
        return st;
      }
    }
    if ((st = upload_batch(c, b)) || (st = xfer_sync(c))) {
      batch_release(c, b);
      return st;
    }
  }
  if (c->run_profile) {
    c->prof[7] += std::chrono::duration<double>(tp1 - tp0).count();
    c->prof[8] += std::chrono::duration<double>(tp2 - tp1).count();
    c->prof[9] += std::chrono::duration<double>(std::chrono::steady_clock::now() - tp2).count();
  }
  *out = b;
  return KS_OK;
}

ks_status ks_batch_run(ks_ctx *c, ks_batch *b) {
  if (!c || !b) return KS_ERR_INVALID;
  ks_status st = drain_async(c);
  if (st) return st;
  return run_batch(c, b);
}

ks_status ks_batch_submit(ks_ctx *c, ks_batch *b) {
  if (!c || !b) return KS_ERR_INVALID;
  if (!c->runq->submit(b)) return c->fail(KS_ERR_INVALID, "batch already submitted");
  return KS_OK;
}

ks_status ks_batch_wait(ks_ctx *c, ks_batch *b) {
  if (!c || !b) return KS_ERR_INVALID;
  if (!c->runq->wait(b)) return c->fail(KS_ERR_INVALID, "batch was not submitted");
  if (b->run_status) c->fail(b->run_status, "%s", b->run_err.c_str());
  return b->run_status;
}

ks_status ks_batch_results(ks_ctx *c, const ks_batch *b, ks_result *out) {
  if (!c || !b || (b->n && !out)) return KS_ERR_INVALID;
  static_assert(sizeof(ks_result) == sizeof(DevResult), "result layout");
  if (c->runq->running(b)) return c->fail(KS_ERR_INVALID, "batch still running (ks_batch_wait first)");
  // the run copied the results into the batch's pinned buffer
  std::memcpy(out, b->h_results, (size_t)b->n * sizeof(DevResult));
  uint64_t sched = 0;
  for (uint32_t i = 0; i < b->n; ++i) sched += out[i].status == KS_POD_SCHEDULED;
  c->stats.pods_scheduled += sched;
  return KS_OK;
}

ks_status ks_batch_marks(ks_ctx *c, const ks_batch *b, uint8_t *out) {
  if (!c || !b || (b->n && !out)) return KS_ERR_INVALID;
  if (c->runq->running(b)) return c->fail(KS_ERR_INVALID, "batch still running (ks_batch_wait first)");
  if (!b->n) return KS_OK;
  ks_status st;
  if ((st = xfer_begin(c, xround(b->n), 0))) return st;
  if ((st = d2h(c, out, b->d_marks, b->n))) return st;
  return xfer_sync(c);
}

void ks_batch_free(ks_ctx *c, ks_batch *b) {
  if (!b) return;
  if (!c) return;  // pooled buffers belong to the context (ks_close frees them)
  c->runq->settle(b);
  {
    std::lock_guard<std::mutex> g(c->mu);
    class_release(c, &b->class_refs);
    for (uint32_t t : b->term_refs) term_activate(c, t, 0, -1);
    b->term_refs.clear();
  }
  batch_release(c, b);
}

ks_status ks_schedule(ks_ctx *c, const ks_pod *pods, uint32_t n, ks_result *out) {
  ks_batch *b = nullptr;
  ks_status st = ks_batch_prepare(c, pods, n, &b);
  if (st) return st;
  st = ks_batch_run(c, b);
  if (!st) st = ks_batch_results(c, b, out);
  ks_batch_free(c, b);
  return st;
}

}  // extern "C"

namespace {

// SpreadArgs of the context's columns and scratch (the batch fields are the caller's).
SpreadArgs spread_args(ks_ctx *c) {
  SpreadArgs sa{};
  {
    std::lock_guard<std::mutex> g(c->mu);
    sa.t = c->t;
    for (uint32_t k = 0; k < c->topo.size(); ++k) sa.ndom[k] = c->topo[k].ndom;
  }
  sa.pos_slot = c->d_pos_slot;
  sa.slot_pos = c->d_slot_pos;
  sa.npos = c->npos;
  sa.dom = c->d_dom;
  sa.cnt = c->d_cnt;
  sa.xalloc = c->d_xalloc;
  sa.xreq = c->d_xreq;
  sa.dcnt = c->d_dcnt;
  sa.dflag = c->d_dflag;
  sa.tcnt = c->d_tcnt;
  sa.adcnt = c->d_adcnt;
  sa.ipa_raw = c->d_sraw2;
  sa.dom_cap = c->dom_cap;
  sa.acc = c->d_acc;
  sa.st = c->d_sst;
  sa.raw = c->d_sraw;
  sa.part = c->d_spart;
  sa.counters = c->d_counters;
  sa.w = Weights{c->cfg.weight_fit, c->cfg.weight_balanced, c->cfg.weight_taint, c->cfg.weight_affinity,
                 c->cfg.weight_image};
  sa.w_pts = c->cfg.weight_topology_spread;
  sa.w_ipa = c->cfg.weight_inter_pod_affinity;
  sa.evaluated = c->n_present;
  return sa;
}

// ks_plugin_scores of a pod with spread constraints: the spread chain in dump mode.
ks_status spread_plugin_scores(ks_ctx *c, const PodDev &d, const ProgBuf &cl, ks_node_score *out) {
  std::vector<int32_t> raw((size_t)c->cap * SPREAD_DUMP_WORDS);
  const size_t bytes = sizeof(PodDev) + cl.w.size() * 8 + raw.size() * 4 + 2048;
  ks_status st;
  if ((st = xfer_begin(c, bytes, bytes))) return st;
  PodDev *d_pod = dscratch<PodDev>(c, 1);
  uint64_t *d_cl = dscratch<uint64_t>(c, cl.w.size());
  int32_t *d_out = dscratch<int32_t>(c, raw.size());
  if ((st = h2d(c, d_pod, &d, sizeof d)) || (st = h2d(c, d_cl, cl.w.data(), cl.w.size() * 8))) return st;
  SpreadArgs sa = spread_args(c);
  sa.pods = d_pod;
  sa.clauses = d_cl;
  sa.pod = 0;
  sa.dump = d_out;
  sa.no_commit = 1;
  const SoloHdr *hd = reinterpret_cast<const SoloHdr *>(cl.w.data() + d.solo_off);
  HIPC(c, launch_spread_pod(sa, solo_passes(hd), c->stream));
  if ((st = d2h(c, raw.data(), d_out, raw.size() * 4)) || (st = xfer_sync(c))) return st;
  for (uint32_t i = 0; i < c->cap; ++i) {
    const int32_t *o = &raw[(size_t)i * SPREAD_DUMP_WORDS];
    ks_node_score s{};
    s.status = o[0];
    s.least_allocated = o[1];
    s.balanced_allocation = o[2];
    s.taint_raw = o[3];
    s.taint_score = o[4];
    s.affinity_raw = o[5];
    s.affinity_score = o[6];
    s.image_locality = o[7];
    s.spread_raw = o[8];
    s.spread_score = o[9];
    s.total_score = (int64_t)(((uint64_t)(uint32_t)o[11] << 32) | (uint32_t)o[10]);
    s.affinity_pod_raw = o[12];
    s.affinity_pod_score = o[13];
    out[i] = s;
  }
  return KS_OK;
}

}  // namespace

extern "C" {

ks_status ks_plugin_scores(ks_ctx *c, const ks_pod *pod, ks_node_score *out) {
  if (!c || !pod || !out) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  HIPC(c, hipSetDevice(c->cfg.device));
  PodDev d;
  ProgBuf cl;
  ks_status st;
  {
    std::unique_lock<std::mutex> g(c->mu);
    if ((st = compile_batch(c, pod, 1, &d, cl, g, true))) return st;
    if ((st = upload_dirty_ext(c, c->xm))) return st;
  }
  if (cl.w.empty()) cl.w.push_back(0);
  if (d.flags & PF_SOLO) return spread_plugin_scores(c, d, cl, out);
  DumpArgs a{};
  a.t = c->t;
  a.nslots = c->cap;
  a.w = Weights{c->cfg.weight_fit, c->cfg.weight_balanced, c->cfg.weight_taint, c->cfg.weight_affinity,
                c->cfg.weight_image};
  a.slot_pos = c->d_slot_pos;
  std::vector<int32_t> raw((size_t)c->cap * 10);
  const size_t bytes = sizeof(PodDev) + cl.w.size() * 8 + 8 + raw.size() * 4 + 2048;
  if ((st = xfer_begin(c, bytes, bytes))) return st;
  PodDev *d_pod = dscratch<PodDev>(c, 1);
  uint64_t *d_cl = dscratch<uint64_t>(c, cl.w.size());
  uint32_t *d_norm = dscratch<uint32_t>(c, 2);
  int32_t *d_out = dscratch<int32_t>(c, raw.size());
  if ((st = h2d(c, d_pod, &d, sizeof d)) || (st = h2d(c, d_cl, cl.w.data(), cl.w.size() * 8))) return st;
  HIPC(c, hipMemsetAsync(d_norm, 0, 8, c->stream));
  a.pods = d_pod;
  a.clauses = d_cl;
  a.norm_max = d_norm;
  a.out = d_out;
  HIPC(c, launch_dump(a, c->stream));
  if ((st = d2h(c, raw.data(), d_out, raw.size() * 4)) || (st = xfer_sync(c))) return st;
  for (uint32_t i = 0; i < c->cap; ++i) {
    const int32_t *o = &raw[(size_t)i * 10];
    ks_node_score s{};
    s.status = o[0];
    s.least_allocated = o[1];
    s.balanced_allocation = o[2];
    s.taint_raw = o[3];
    s.taint_score = o[4];
    s.affinity_raw = o[5];
    s.affinity_score = o[6];
    s.image_locality = o[7];
    s.spread_raw = 0;
    s.spread_score = 0;
    s.affinity_pod_raw = 0;
    s.affinity_pod_score = 0;
    s.total_score = (int64_t)(((uint64_t)(uint32_t)o[9] << 32) | (uint32_t)o[8]);
    out[i] = s;
  }
  return KS_OK;
}

ks_status ks_node_states(ks_ctx *c, const uint32_t *slots, uint32_t n, ks_node_state *out) {
  if (!c || (n && (!slots || !out))) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  if (!n) return KS_OK;
  HIPC(c, hipSetDevice(c->cfg.device));
  std::vector<uint32_t> pos(n);
  for (uint32_t i = 0; i < n; ++i) {
    if (slots[i] >= c->cap) return c->fail(KS_ERR_NOT_FOUND, "slot %u >= capacity", slots[i]);
    pos[i] = c->slot_pos[slots[i]];
  }
  std::vector<int64_t> raw((size_t)n * 8);
  const size_t bytes = (size_t)n * 4 + raw.size() * 8 + 1024;
  ks_status st = xfer_begin(c, bytes, bytes);
  if (st) return st;
  uint32_t *d_pos = dscratch<uint32_t>(c, n);
  int64_t *d_out = dscratch<int64_t>(c, raw.size());
  if ((st = h2d(c, d_pos, pos.data(), (size_t)n * 4))) return st;
  HIPC(c, launch_gather_rows(c->t, d_pos, d_out, n, c->stream));
  if ((st = d2h(c, raw.data(), d_out, raw.size() * 8)) || (st = xfer_sync(c))) return st;
  for (uint32_t i = 0; i < n; ++i) {
    const int64_t *r = &raw[(size_t)i * 8];
    ks_node_state s{};
    s.alloc_milli_cpu = r[0];
    s.alloc_memory = r[1];
    s.req_milli_cpu = r[2];
    s.req_memory = r[3];
    s.nonzero_milli_cpu = r[4];
    s.nonzero_memory = r[5];
    s.alloc_pods = (int32_t)r[6];
    s.pod_count = s.alloc_pods < 0 ? -1 : (int32_t)r[7];
    if (s.alloc_pods < 0) s = ks_node_state{0, 0, 0, 0, 0, 0, 0, -1};
    out[i] = s;
  }
  return KS_OK;
}

ks_status ks_comm_unique_id(uint8_t out[KS_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == KS_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return KS_ERR_COMM;
  std::memcpy(out, &id, sizeof id);
  return KS_OK;
}

ks_status ks_comm_init(ks_ctx *c, const uint8_t id[KS_COMM_ID_BYTES]) {
  if (!c || !id) return KS_ERR_INVALID;
  if (c->has_comm()) return c->fail(KS_ERR_INVALID, "the context already has a communicator");
  if (ks_status dst_ = drain_async(c)) return dst_;
  HIPC(c, hipSetDevice(c->cfg.device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  NCCLC(c, ncclCommInitRank(&c->comm, (int)c->cfg.world_size, uid, (int)c->cfg.rank));
  return KS_OK;
}

ks_status ks_comm_init_local(ks_ctx *const *ctxs, uint32_t n) {
  if (!ctxs || n == 0 || n > (uint32_t)MAX_SHARDS) return KS_ERR_INVALID;
  for (uint32_t r = 0; r < n; ++r) {
    ks_ctx *c = ctxs[r];
    if (!c) return KS_ERR_INVALID;
    if (c->cfg.world_size != n || c->cfg.rank != r)
      return c->fail(KS_ERR_INVALID, "context %u: world_size %u rank %u, expected %u / %u", r, c->cfg.world_size,
                     c->cfg.rank, n, r);
    if (c->has_comm()) return c->fail(KS_ERR_INVALID, "context %u already has a communicator", r);
  }
  auto g = std::make_shared<LocalGroup>(n);
  for (uint32_t r = 0; r < n; ++r) {
    ks_ctx *c = ctxs[r];
    if (ks_status dst_ = drain_async(c)) return dst_;
    HIPC(c, hipSetDevice(c->cfg.device));
    for (auto &e : c->lg_ev) HIPC(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPC(c, hipMalloc((void **)&c->d_lgstage, 4 * (size_t)MAX_P * sizeof(uint32_t)));
    c->lgroup = g;
  }
  return KS_OK;
}

ks_status ks_comm_allreduce_max(ks_ctx *c, double *values, uint32_t n) {
  if (!c || (n && !values)) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  if (!c->has_comm()) return c->fail(KS_ERR_COMM, "ks_comm_init not called");
  HIPC(c, hipSetDevice(c->cfg.device));
  if (c->lgroup) {  // host values: a rendezvous after this rank's queued work has finished
    if (ks_status e_ = sync_bounded(c, c->stream, __func__)) return e_;
    std::vector<LocalGroup::Post> ps;
    ks_status e = lg_exchange(c, {nullptr, nullptr, std::vector<double>(values, values + n)}, ps);
    if (e) return e;
    for (const auto &p : ps)
      for (uint32_t i = 0; i < n && i < p.vals.size(); ++i) values[i] = std::max(values[i], p.vals[i]);
    return KS_OK;
  }
  ks_status st = xfer_begin(c, 2 * (size_t)n * 8 + 1024, (size_t)n * 8 + 1024);
  if (st) return st;
  double *d = dscratch<double>(c, n);
  if ((st = h2d(c, d, values, (size_t)n * 8))) return st;
  NCCLC(c, ncclAllReduce(d, d, n, ncclFloat64, ncclMax, c->comm, c->stream));
  if ((st = d2h(c, values, d, (size_t)n * 8))) return st;
  return xfer_sync(c);
}

static ks_status read_counters(ks_ctx *c, uint64_t out[4]) {
  HIPC(c, hipSetDevice(c->cfg.device));
  ks_status st;
  if ((st = xfer_begin(c, 1024, 0)) || (st = d2h(c, out, c->d_counters, 4 * sizeof(uint64_t)))) return st;
  return xfer_sync(c);
}

ks_status ks_get_stats(ks_ctx *c, ks_stats *out) {
  if (!c || !out) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  uint64_t k[4];
  ks_status st = read_counters(c, k);
  if (st) return st;
  *out = c->stats;
  // (pod, node) evaluations of this rank's sweeps: pods swept x present local nodes
  const bool multi = c->has_comm();
  uint64_t local = 0;
  for (uint32_t q = 0; q < c->S; ++q) {
    if (multi && q != c->cfg.rank) continue;
    const Shard &sh = c->shards[q];
    for (uint32_t l = 0; l < sh.count; ++l) local += c->nodes[sh.lo + l].present;
  }
  // evaluations by the timed launches: all evaluations apportioned by launch
  // count (every launch but a batch's last sweeps P pods)
  const uint64_t all_evals = (k[2] - c->counters_base[2]) * local;
  out->sweep_evals = c->sweeps_issued ? (uint64_t)((double)all_evals * (double)c->stats.sweep_launches /
                                                   (double)c->sweeps_issued)
                                      : 0;
  out->rounds = k[0] - c->counters_base[0];
  out->pods_resolved = k[1] - c->counters_base[1];
  return KS_OK;
}

ks_status ks_reset_stats(ks_ctx *c) {
  if (!c) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  c->stats = ks_stats{};
  c->sweeps_issued = 0;
  return read_counters(c, c->counters_base);
}

ks_status ks_debug_round_record(ks_ctx *c, uint32_t r, uint64_t *out) {
  if (!c || !out) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  if (r >= c->P) return c->fail(KS_ERR_INVALID, "pod %u of a %u-pod round", r, c->P);
  HIPC(c, hipSetDevice(c->cfg.device));
  const size_t RW = rec_words(c->K);
  // round 0 = parity 0; with several shards the merged record (merge_shards)
  ks_status st;
  if (c->dedup_used[0]) {  // an identical pod's record serves pod r
    uint32_t rr = r;
    if ((st = xfer_begin(c, 1024, 0)) || (st = d2h(c, &rr, c->d_dedup + r, 4)) || (st = xfer_sync(c))) return st;
    r = rr;
  }
  const uint64_t *rec = (c->S == 1 ? c->d_srec : c->d_frec) + (size_t)r * RW;
  std::vector<uint64_t> w(RW);
  if ((st = xfer_begin(c, RW * 8 + 1024, 0)) || (st = d2h(c, w.data(), rec, RW * 8)) || (st = xfer_sync(c)))
    return st;
  const ShardRecHdr *h = (const ShardRecHdr *)w.data();
  out[0] = h->bound;
  out[1] = h->nkeys;
  for (uint32_t i = 0; i < c->K; ++i) out[2 + i] = i < h->nkeys ? w[REC_HDR_WORDS + i] : 0ull;
  return KS_OK;
}

ks_status ks_debug_set_profile(ks_ctx *c, int32_t on) {
  if (!c) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  c->res_profile = on != 0;
  return KS_OK;
}

ks_status ks_debug_resolve_profile(ks_ctx *c, uint64_t out[16]) {
  if (!c || !out) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  HIPC(c, hipSetDevice(c->cfg.device));
  ks_status st;
  if ((st = xfer_begin(c, 1024, 0)) || (st = d2h(c, out, c->d_counters + 16, 16 * sizeof(uint64_t))) ||
      (st = xfer_sync(c)))
    return st;
  return KS_OK;
}

ks_status ks_debug_counters(ks_ctx *c, uint64_t out[16]) {
  if (!c || !out) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  HIPC(c, hipSetDevice(c->cfg.device));
  ks_status st;
  if ((st = xfer_begin(c, 1024, 0)) || (st = d2h(c, out, c->d_counters, 16 * sizeof(uint64_t))) ||
      (st = xfer_sync(c)))
    return st;
  out[5] = c->label_resets;
  out[6] = c->taint_rebuilds;
  return KS_OK;
}

ks_status ks_set_timing(ks_ctx *c, int32_t enabled) {
  if (!c) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  c->timing = enabled != 0;
  return KS_OK;
}

ks_status ks_set_sync_timeout(ks_ctx *c, uint32_t ms) {
  if (!c || ms == 0) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  c->sync_timeout_ms = ms;
  return KS_OK;
}

ks_status ks_next_start_index(ks_ctx *c, uint64_t *out) {
  if (!c || !out) return KS_ERR_INVALID;
  *out = 0;
  if (c->pct == 100 || !c->d_win) return KS_OK;
  if (ks_status dst_ = drain_async(c)) return dst_;
  uint32_t v = 0;
  ks_status st;
  if ((st = xfer_begin(c, 64, 0)) || (st = d2h(c, &v, c->d_win, sizeof v)) || (st = xfer_sync(c))) return st;
  *out = v;
  return KS_OK;
}

ks_status ks_debug_runs_started(ks_ctx *c, uint64_t *out) {
  if (!c || !out) return KS_ERR_INVALID;
  std::lock_guard<std::mutex> g(c->mu);  // run_batch counts under mu; no drain here
  *out = c->runs_started;
  return KS_OK;
}

ks_status ks_debug_stall(ks_ctx *c, uint32_t flag, uint32_t usec) {
  if (!c || flag > 3 || usec > 600u * 1000u * 1000u) return KS_ERR_INVALID;
  if (ks_status dst_ = drain_async(c)) return dst_;
  c->stall_flag = (int32_t)flag;
  c->stall_us = usec;
  return KS_OK;
}

}  // extern "C"
