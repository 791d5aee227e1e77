// oracle.cpp — CPU restatement of upstream kube-scheduler v1.31.3 for the
// dist-scheduler shard path.  TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// PARITY UNPINNED (oracle.h): the forked scheduler the reference compiles
// (dist-scheduler/go.mod:133,138) is absent; this file restates the public
// upstream v1.31.3 sources, cited as upstream:<file>#<func>.  It deliberately
// works on the k8s-shaped objects (string maps, taint/toleration lists) with no
// dictionary or bitset encoding, so that it also checks the product's encoder.
//
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off).  Floating point follows
// Go on amd64 (GOAMD64=v1: no FMA fusion), i.e. IEEE binary64 with one
// rounding per operation.
#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int64_t kMaxNodeScore = 100;                      // framework.MaxNodeScore
constexpr int64_t kDefaultMilliCPURequest = 100;            // upstream:pkg/scheduler/util#DefaultMilliCPURequest
constexpr int64_t kDefaultMemoryRequest = 200 * 1024 * 1024; // upstream:pkg/scheduler/util#DefaultMemoryRequest

std::string S(const char *p) { return p ? std::string(p) : std::string(); }

// ------------------------------------------------------------------ objects

struct Taint {
  std::string key, value;
  int32_t effect;
};
struct Toleration {
  std::string key, value;
  int32_t op, effect;
};

struct AffTerm;  // interpodaffinity term of a bound pod (defined below)

struct Node {
  bool present = false;
  std::string name;
  int64_t alloc_cpu = 0, alloc_mem = 0, alloc_pods = 0;
  std::map<std::string, std::string> labels;
  std::vector<Taint> taints;
  bool unschedulable = false;
  // NodeInfo.Requested / NonZeroRequested / len(Pods)
  int64_t req_cpu = 0, req_mem = 0, nz_cpu = 0, nz_mem = 0;
  int64_t pods = 0;
  // framework.Resource beyond cpu / memory / pods: ephemeral-storage and scalar
  // resources (Allocatable, Requested)
  std::map<std::string, int64_t> xalloc, xreq;
  // status.images names (as reported) -> the entry's size (first occurrence)
  std::vector<std::pair<std::string, int64_t>> images;
  // NodeInfo.Pods' namespace and labels (PodTopologySpread counts them)
  struct PodRec {
    std::string ns;
    std::map<std::string, std::string> labels, ns_labels;
    std::vector<AffTerm> terms;  // the pod's pod (anti-)affinity terms
    std::string key;             // identity for RemovePod
    bool operator==(const PodRec &o) const { return key == o.key; }
  };
  std::vector<PodRec> pod_recs;
  // NodeInfo.PodsWithAffinity / PodsWithRequiredAntiAffinity sizes: upstream's
  // HavePodsWithAffinityList / HavePodsWithRequiredAntiAffinityList restrict
  // InterPodAffinity's scans to these nodes (same results, upstream's cost)
  int64_t pods_with_affinity = 0, pods_with_req_anti = 0;
};

// k8s.io/api/core/v1/toleration.go#ToleratesTaint
bool ToleratesTaint(const Toleration &t, const Taint &taint) {
  if (t.effect != KS_EFFECT_ALL && t.effect != taint.effect) return false;
  if (!t.key.empty() && t.key != taint.key) return false;
  switch (t.op) {
    case KS_TOL_EQUAL: return t.value == taint.value;
    case KS_TOL_EXISTS: return true;
    default: return false;
  }
}

// component-helpers/scheduling/corev1#TolerationsTolerateTaint
bool TolerationsTolerateTaint(const std::vector<Toleration> &tols, const Taint &taint) {
  for (auto &t : tols)
    if (ToleratesTaint(t, taint)) return true;
  return false;
}

// ---------------------------------------------- apimachinery validation

bool alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }

// qualifiedNameFmt "([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]"; labelValueFmt adds "empty ok".
bool matches_qualified_name_part(const std::string &s) {
  if (s.empty()) return false;
  if (!alnum(s.front()) || !alnum(s.back())) return false;
  for (char c : s)
    if (!(alnum(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}

// validation.IsDNS1123Subdomain
bool is_dns1123_subdomain(const std::string &s) {
  if (s.empty() || s.size() > 253) return false;
  size_t start = 0;
  while (true) {
    size_t dot = s.find('.', start);
    std::string lab = s.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
    if (lab.empty()) return false;
    auto lower_alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!lower_alnum(lab.front()) || !lower_alnum(lab.back())) return false;
    for (char c : lab)
      if (!(lower_alnum(c) || c == '-')) return false;
    if (dot == std::string::npos) break;
    start = dot + 1;
  }
  return true;
}

// apimachinery/pkg/util/validation#IsQualifiedName
bool IsQualifiedName(const std::string &v) {
  std::string name;
  size_t slash = v.find('/');
  if (slash == std::string::npos) {
    name = v;
  } else {
    if (v.find('/', slash + 1) != std::string::npos) return false;
    std::string prefix = v.substr(0, slash);
    name = v.substr(slash + 1);
    if (prefix.empty() || !is_dns1123_subdomain(prefix)) return false;
  }
  if (name.empty() || name.size() > 63) return false;
  return matches_qualified_name_part(name);
}

// apimachinery/pkg/util/validation#IsValidLabelValue
bool IsValidLabelValue(const std::string &v) {
  if (v.size() > 63) return false;
  return v.empty() || matches_qualified_name_part(v);
}

// strconv.ParseInt(s, 10, 64)
bool ParseInt64(const std::string &s, int64_t *out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  unsigned __int128 acc = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    acc = acc * 10 + (unsigned)(s[i] - '0');
    if (acc > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && acc > (unsigned __int128)INT64_MAX) return false;
  *out = neg ? (int64_t)(-(__int128)acc) : (int64_t)acc;
  return true;
}

// ------------------------------------------------- label selector requirement

enum SelOp { SEL_IN, SEL_NOT_IN, SEL_EXISTS, SEL_DOES_NOT_EXIST, SEL_GT, SEL_LT, SEL_EQUALS };

struct Requirement {  // apimachinery/pkg/labels#Requirement
  std::string key;
  SelOp op;
  std::vector<std::string> values;
};

// labels.NewRequirement validation; returns false on any error.
bool NewRequirement(const std::string &key, SelOp op, const std::vector<std::string> &vals,
                    Requirement *out) {
  bool ok = true;
  switch (op) {
    case SEL_IN:
    case SEL_NOT_IN:
      if (vals.empty()) ok = false;
      break;
    case SEL_EXISTS:
    case SEL_DOES_NOT_EXIST:
      if (!vals.empty()) ok = false;
      break;
    case SEL_EQUALS:
      if (vals.size() != 1) ok = false;
      break;
    case SEL_GT:
    case SEL_LT:
      if (vals.size() != 1) ok = false;
      for (auto &v : vals) {
        int64_t x;
        if (!ParseInt64(v, &x)) ok = false;
      }
      break;
    default: ok = false;
  }
  for (auto &v : vals)
    if (!IsValidLabelValue(v)) ok = false;
  if (!IsQualifiedName(key)) ok = false;
  if (ok) *out = Requirement{key, op, vals};
  return ok;
}

// labels.Requirement.Matches
bool Matches(const Requirement &r, const std::map<std::string, std::string> &ls) {
  auto it = ls.find(r.key);
  bool has = it != ls.end();
  auto hasValue = [&](const std::string &v) {
    return std::find(r.values.begin(), r.values.end(), v) != r.values.end();
  };
  switch (r.op) {
    case SEL_IN:
    case SEL_EQUALS:
      if (!has) return false;
      return hasValue(it->second);
    case SEL_NOT_IN:
      if (!has) return true;
      return !hasValue(it->second);
    case SEL_EXISTS: return has;
    case SEL_DOES_NOT_EXIST: return !has;
    case SEL_GT:
    case SEL_LT: {
      if (!has) return false;
      int64_t lv, rv;
      if (!ParseInt64(it->second, &lv)) return false;
      if (r.values.size() != 1) return false;
      if (!ParseInt64(r.values[0], &rv)) return false;
      return (r.op == SEL_GT && lv > rv) || (r.op == SEL_LT && lv < rv);
    }
  }
  return false;
}

// ------------------------------------------------------ node selector terms

struct FieldReq {
  std::string value;
  bool equal;  // In -> name == value, NotIn -> name != value
};

// component-helpers/scheduling/corev1/nodeaffinity#nodeSelectorTerm
struct NodeSelectorTerm {
  bool has_labels = false;
  std::vector<Requirement> labels;
  bool has_fields = false;
  std::vector<FieldReq> fields;
  bool parse_error = false;

  bool match(const Node &n) const {
    if (parse_error) return false;
    if (has_labels) {
      for (auto &r : labels)
        if (!Matches(r, n.labels)) return false;
    }
    if (has_fields && !n.name.empty()) {  // len(nodeFields) > 0
      for (auto &f : fields)
        if ((n.name == f.value) != f.equal) return false;
    }
    return true;
  }
};

bool is_empty_term(const ks_term &t) { return t.n_expressions == 0 && t.n_fields == 0; }

// nodeaffinity#newNodeSelectorTerm
NodeSelectorTerm newNodeSelectorTerm(const ks_term &t) {
  NodeSelectorTerm out;
  if (t.n_expressions != 0) {
    // nodeSelectorRequirementsAsSelector
    out.has_labels = true;
    for (uint32_t i = 0; i < t.n_expressions; ++i) {
      const ks_requirement &e = t.match_expressions[i];
      SelOp op;
      switch (e.op) {
        case KS_OP_IN: op = SEL_IN; break;
        case KS_OP_NOT_IN: op = SEL_NOT_IN; break;
        case KS_OP_EXISTS: op = SEL_EXISTS; break;
        case KS_OP_DOES_NOT_EXIST: op = SEL_DOES_NOT_EXIST; break;
        case KS_OP_GT: op = SEL_GT; break;
        case KS_OP_LT: op = SEL_LT; break;
        default: out.parse_error = true; continue;
      }
      std::vector<std::string> vals;
      for (uint32_t k = 0; k < e.n_values; ++k) vals.push_back(S(e.values[k]));
      Requirement r;
      if (!NewRequirement(S(e.key), op, vals, &r)) out.parse_error = true;
      else out.labels.push_back(r);
    }
  }
  if (t.n_fields != 0) {
    // nodeSelectorRequirementsAsFieldSelector
    out.has_fields = true;
    for (uint32_t i = 0; i < t.n_fields; ++i) {
      const ks_requirement &e = t.match_fields[i];
      if (S(e.key) != "metadata.name") { out.parse_error = true; continue; }
      if (e.n_values != 1) { out.parse_error = true; continue; }
      if (e.op == KS_OP_IN) out.fields.push_back({S(e.values[0]), true});
      else if (e.op == KS_OP_NOT_IN) out.fields.push_back({S(e.values[0]), false});
      else out.parse_error = true;
    }
  }
  return out;
}

// ------------------------------------------------------ labels.Selector

// apimachinery/pkg/labels: the internalSelector of LabelSelectorAsSelector
// (Everything() = no requirement, Nothing() = nil LabelSelector).
struct Selector {
  bool nothing = false;
  std::vector<Requirement> reqs;
  bool Empty() const { return !nothing && reqs.empty(); }
  bool Match(const std::map<std::string, std::string> &ls) const {
    if (nothing) return false;
    for (auto &r : reqs)
      if (!Matches(r, ls)) return false;
    return true;
  }
};

// metav1.LabelSelectorAsSelector; false on a parse error.
bool LabelSelectorAsSelector(const ks_label_selector &ls, Selector *out) {
  *out = Selector{};
  if (ls.is_nil) {
    out->nothing = true;
    return true;
  }
  for (uint32_t i = 0; i < ls.n_match_labels; ++i) {
    Requirement r;
    if (!NewRequirement(S(ls.match_labels[i].key), SEL_EQUALS, {S(ls.match_labels[i].value)}, &r)) return false;
    out->reqs.push_back(r);
  }
  for (uint32_t i = 0; i < ls.n_match_expressions; ++i) {
    const ks_requirement &e = ls.match_expressions[i];
    SelOp op;
    switch (e.op) {
      case KS_OP_IN: op = SEL_IN; break;
      case KS_OP_NOT_IN: op = SEL_NOT_IN; break;
      case KS_OP_EXISTS: op = SEL_EXISTS; break;
      case KS_OP_DOES_NOT_EXIST: op = SEL_DOES_NOT_EXIST; break;
      default: return false;  // "is not a valid label selector operator"
    }
    std::vector<std::string> vals;
    for (uint32_t k = 0; k < e.n_values; ++k) vals.push_back(S(e.values[k]));
    Requirement r;
    if (!NewRequirement(S(e.key), op, vals, &r)) return false;
    out->reqs.push_back(r);
  }
  return true;
}

// podtopologyspread/common.go: one constraint after filterTopologySpreadConstraints.
struct SpreadConstraint {
  int32_t max_skew = 1;
  std::string key;
  Selector sel;
  int32_t min_domains = 1;
  bool aff_honor = true, taint_honor = false;
  bool hostname = false;  // topologyKey == v1.LabelHostname (scoring counts per node)
};

// interpodaffinity: framework.AffinityTerm (framework/types.go#newAffinityTerm)
struct AffTerm {
  int32_t kind = 0;    // KS_POD_*AFFINITY_*
  int64_t weight = 0;  // preferred terms
  std::set<std::string> namespaces;
  Selector ns_sel;     // NamespaceSelector (nil -> Nothing())
  Selector sel;
  std::string key;
  // AffinityTerm.Matches(pod, nsLabels): namespace listed or selected, then the selector
  bool Matches(const std::string &ns, const std::map<std::string, std::string> &labels,
               const std::map<std::string, std::string> &ns_labels) const {
    if (!namespaces.count(ns) && !ns_sel.Match(ns_labels)) return false;
    return sel.Match(labels);
  }
};

// newAffinityTerm for one of pod p's terms; false on a selector parse error.
bool NewAffinityTerm(const ks_pod &p, const ks_pod_affinity_term &t, AffTerm *out) {
  AffTerm a;
  a.kind = t.kind;
  a.weight = t.weight;
  a.key = S(t.topology_key);
  for (uint32_t i = 0; i < t.n_namespaces; ++i) a.namespaces.insert(S(t.namespaces[i]));
  if (a.namespaces.empty() && t.namespace_selector.is_nil) a.namespaces.insert(S(p.ns));
  if (!LabelSelectorAsSelector(t.selector, &a.sel) || !LabelSelectorAsSelector(t.namespace_selector, &a.ns_sel))
    return false;
  *out = a;
  return true;
}

// ------------------------------------------------------------ pod state

struct PodState {
  // NodeResourcesFit PreFilter: computePodResourceRequest (actual requests)
  int64_t req_cpu = 0, req_mem = 0;
  bool req_other = false;
  // resourceAllocationScorer: non-zero (LeastAllocated) and actual (BalancedAllocation)
  int64_t nz_cpu = 0, nz_mem = 0;
  std::vector<Toleration> tolerations;
  std::vector<Toleration> tolerations_prefer;  // getAllTolerationPreferNoSchedule
  std::string node_name;
  // NodeAffinity PreFilter: GetRequiredNodeAffinity
  bool affinity_skip = true;
  std::vector<Requirement> node_selector;
  bool has_required = false;
  std::vector<NodeSelectorTerm> required;  // non-empty terms only
  // NodeAffinity PreFilter: PreFilterResult.NodeNames (prefilter) or a
  // conflicting name set (conflict: UnschedulableAndUnresolvable)
  bool prefilter = false, conflict = false;
  std::vector<std::string> prefilter_names;  // sorted
  // NodeAffinity PreScore: PreferredSchedulingTerms
  bool has_preferred = false;
  bool preferred_error = false;
  std::vector<std::pair<int64_t, NodeSelectorTerm>> preferred;
  // PodTopologySpread: DoNotSchedule (Filter) and ScheduleAnyway (Score)
  // constraints; requireAllTopologies = !spread_defaulted
  std::string ns;
  std::map<std::string, std::string> labels;
  std::vector<SpreadConstraint> spread_filter, spread_score;
  bool spread_defaulted = false;
  bool spread_error = false;  // a selector failed to parse (the product refuses the pod)
  // NodeResourcesFit beyond cpu / memory; ImageLocality inputs
  std::map<std::string, int64_t> xreq;
  std::vector<std::string> images;  // normalised, init containers then containers ("" = none)
  int64_t n_containers = 0;
  // InterPodAffinity: the pod's terms by kind, its namespace's labels
  std::vector<AffTerm> ipa[4];
  std::map<std::string, std::string> ns_labels;
  bool ipa_error = false;  // a term's selector failed to parse (the product refuses the pod)
};

// v1helper.IsScalarResourceName (extended, hugepages-, attachable-volumes-,
// kubernetes.io/-prefixed native) or ephemeral-storage: the resources
// framework.Resource keeps beyond cpu / memory / pods.
bool ExtendedResourceName(const std::string &n) {
  if (n == "ephemeral-storage") return true;
  if (n.rfind("hugepages-", 0) == 0 || n.rfind("attachable-volumes-", 0) == 0) return true;
  const bool prefixed_native = n.find("kubernetes.io/") != std::string::npos;
  if (prefixed_native) return true;
  if (n.find('/') == std::string::npos) return false;  // native, not scalar
  if (n.rfind("requests.", 0) == 0) return false;
  return IsQualifiedName("requests." + n);  // IsExtendedResourceName
}

// PodRequests for the extended resources: containers' sum, init containers'
// max with sidecars (the same rules as cpu / memory).
std::map<std::string, int64_t> PodXRequests(const ks_pod &p) {
  auto get = [](const ks_container &c) {
    std::map<std::string, int64_t> r;
    for (uint32_t k = 0; k < c.n_extended; ++k) {
      const std::string nm = S(c.extended[k].name);
      if (ExtendedResourceName(nm)) r[nm] += c.extended[k].value;
    }
    return r;
  };
  std::map<std::string, int64_t> sum, side, init;
  for (uint32_t i = 0; i < p.n_containers; ++i)
    for (auto &kv : get(p.containers[i])) sum[kv.first] += kv.second;
  for (uint32_t i = 0; i < p.n_init_containers; ++i) {
    auto r = get(p.init_containers[i]);
    std::map<std::string, int64_t> use;
    if (p.init_containers[i].restart_always) {
      for (auto &kv : r) {
        sum[kv.first] += kv.second;
        side[kv.first] += kv.second;
      }
      use = side;
    } else {
      use = side;
      for (auto &kv : r) use[kv.first] += kv.second;
    }
    for (auto &kv : use) init[kv.first] = std::max(init[kv.first], kv.second);
  }
  for (auto &kv : init) sum[kv.first] = std::max(sum[kv.first], kv.second);
  return sum;
}

// imagelocality#normalizedImageName
std::string NormalizedImageName(const std::string &name) {
  const size_t c = name.rfind(':'), sl = name.rfind('/');
  const long lc = c == std::string::npos ? -1 : (long)c, ls = sl == std::string::npos ? -1 : (long)sl;
  return lc <= ls ? name + ":latest" : name;
}

// upstream:pkg/api/v1/resource/helpers.go#PodRequests for cpu/memory.
void PodRequests(const ks_pod &p, bool non_missing, int64_t *cpu, int64_t *mem, bool *other) {
  auto get = [&](const ks_container &c, int64_t *ccpu, int64_t *cmem) {
    *ccpu = (c.flags & KS_REQ_HAS_CPU) ? c.milli_cpu : (non_missing ? kDefaultMilliCPURequest : 0);
    *cmem = (c.flags & KS_REQ_HAS_MEMORY) ? c.memory : (non_missing ? kDefaultMemoryRequest : 0);
    if (c.flags & KS_REQ_HAS_OTHER) *other = true;
  };
  int64_t rc = 0, rm = 0;
  for (uint32_t i = 0; i < p.n_containers; ++i) {
    int64_t a, b;
    get(p.containers[i], &a, &b);
    rc += a;
    rm += b;
  }
  int64_t sidecar_c = 0, sidecar_m = 0, init_c = 0, init_m = 0;
  for (uint32_t i = 0; i < p.n_init_containers; ++i) {
    int64_t a, b;
    get(p.init_containers[i], &a, &b);
    if (p.init_containers[i].restart_always) {
      rc += a;
      rm += b;
      sidecar_c += a;
      sidecar_m += b;
      a = sidecar_c;
      b = sidecar_m;
    } else {
      a += sidecar_c;
      b += sidecar_m;
    }
    init_c = std::max(init_c, a);
    init_m = std::max(init_m, b);
  }
  rc = std::max(rc, init_c);
  rm = std::max(rm, init_m);
  if (p.has_overhead) {
    rc += p.overhead_milli_cpu;
    rm += p.overhead_memory;
  }
  *cpu = rc;
  *mem = rm;
}

PodState compile_pod(const ks_pod &p) {
  PodState st;
  bool other = false;
  PodRequests(p, false, &st.req_cpu, &st.req_mem, &other);
  PodRequests(p, true, &st.nz_cpu, &st.nz_mem, &other);
  st.req_other = other;
  for (uint32_t i = 0; i < p.n_tolerations; ++i) {
    const ks_toleration &t = p.tolerations[i];
    Toleration tt{S(t.key), S(t.value), t.op, t.effect};
    st.tolerations.push_back(tt);
    if (t.effect == KS_EFFECT_ALL || t.effect == KS_EFFECT_PREFER_NO_SCHEDULE)
      st.tolerations_prefer.push_back(tt);
  }
  st.node_name = S(p.node_name);
  // NodeAffinity.PreFilter: Skip when no required affinity and no nodeSelector.
  st.has_required = p.has_required != 0;
  st.affinity_skip = !st.has_required && p.n_node_selector == 0;
  for (uint32_t i = 0; i < p.n_node_selector; ++i)
    st.node_selector.push_back(
        Requirement{S(p.node_selector[i].key), SEL_EQUALS, {S(p.node_selector[i].value)}});
  for (uint32_t i = 0; i < p.n_required_terms; ++i) {
    if (is_empty_term(p.required_terms[i])) continue;  // NewLazyErrorNodeSelector
    st.required.push_back(newNodeSelectorTerm(p.required_terms[i]));
  }
  // nodeaffinity#PreFilter: when every required term carries matchFields
  // metadata.name In requirements, PreFilterResult.NodeNames = the union over
  // terms of the intersection of each term's value sets (raw values, before
  // any parsing); an empty union rejects the pod (errReasonConflict).
  if (st.has_required && p.n_required_terms > 0) {
    bool all = true;
    std::vector<std::string> uni;
    for (uint32_t i = 0; i < p.n_required_terms && all; ++i) {
      const ks_term &t = p.required_terms[i];
      bool have = false;
      std::vector<std::string> term_names;
      for (uint32_t k = 0; k < t.n_fields; ++k) {
        const ks_requirement &r = t.match_fields[k];
        if (S(r.key) != "metadata.name" || r.op != KS_OP_IN) continue;
        std::vector<std::string> vs;
        for (uint32_t v = 0; v < r.n_values; ++v) vs.push_back(S(r.values[v]));
        if (!have) {
          term_names = vs;
          have = true;
        } else {  // sets.Intersection
          std::vector<std::string> keep;
          for (auto &x : term_names)
            if (std::find(vs.begin(), vs.end(), x) != vs.end()) keep.push_back(x);
          term_names = keep;
        }
      }
      if (!have) all = false;  // "all nodes are eligible because the terms are ORed"
      else uni.insert(uni.end(), term_names.begin(), term_names.end());
    }
    if (all) {
      std::sort(uni.begin(), uni.end());
      uni.erase(std::unique(uni.begin(), uni.end()), uni.end());
      if (uni.empty()) st.conflict = true;
      else {
        st.prefilter = true;
        st.prefilter_names = uni;
      }
    }
  }
  st.xreq = PodXRequests(p);
  for (uint32_t i = 0; i < p.n_init_containers; ++i)
    st.images.push_back(p.init_containers[i].image && p.init_containers[i].image[0]
                            ? NormalizedImageName(S(p.init_containers[i].image)) : std::string());
  for (uint32_t i = 0; i < p.n_containers; ++i)
    st.images.push_back(p.containers[i].image && p.containers[i].image[0]
                            ? NormalizedImageName(S(p.containers[i].image)) : std::string());
  st.n_containers = (int64_t)p.n_init_containers + p.n_containers;
  for (uint32_t i = 0; i < p.n_namespace_labels; ++i)
    st.ns_labels[S(p.namespace_labels[i].key)] = S(p.namespace_labels[i].value);
  for (uint32_t i = 0; i < p.n_affinity_terms; ++i) {
    AffTerm a;
    if (!NewAffinityTerm(p, p.affinity_terms[i], &a) || a.kind < 0 || a.kind > 3) st.ipa_error = true;
    else st.ipa[a.kind].push_back(a);
  }
  st.ns = S(p.ns);
  for (uint32_t i = 0; i < p.n_labels; ++i) st.labels[S(p.labels[i].key)] = S(p.labels[i].value);
  // podtopologyspread/common.go#filterTopologySpreadConstraints, per action
  st.spread_defaulted = p.spread_defaulted != 0;
  for (uint32_t i = 0; i < p.n_spread; ++i) {
    const ks_spread_constraint &c = p.spread[i];
    SpreadConstraint sc;
    sc.max_skew = c.max_skew;
    sc.key = S(c.topology_key);
    sc.hostname = sc.key == "kubernetes.io/hostname";
    if (!LabelSelectorAsSelector(c.selector, &sc.sel)) st.spread_error = true;
    // MatchLabelKeys: the incoming pod's values merged into the selector
    // (mergeLabelSetWithSelector: a Nothing() selector stays Nothing())
    std::vector<Requirement> extra;
    for (uint32_t k = 0; k < c.n_match_label_keys; ++k) {
      auto it = st.labels.find(S(c.match_label_keys[k]));
      if (it != st.labels.end()) extra.push_back(Requirement{it->first, SEL_EQUALS, {it->second}});
    }
    if (!extra.empty() && !sc.sel.nothing) sc.sel.reqs.insert(sc.sel.reqs.begin(), extra.begin(), extra.end());
    if (c.min_domains != 0) sc.min_domains = c.min_domains;
    if (c.node_affinity_policy != KS_INCLUSION_DEFAULT) sc.aff_honor = c.node_affinity_policy == KS_INCLUSION_HONOR;
    if (c.node_taints_policy != KS_INCLUSION_DEFAULT) sc.taint_honor = c.node_taints_policy == KS_INCLUSION_HONOR;
    (c.when_unsatisfiable == KS_DO_NOT_SCHEDULE ? st.spread_filter : st.spread_score).push_back(sc);
  }
  st.has_preferred = p.has_preferred != 0;
  for (uint32_t i = 0; i < p.n_preferred; ++i) {
    const ks_preferred_term &t = p.preferred[i];
    if (t.weight == 0 || is_empty_term(t.preference)) continue;  // NewPreferredSchedulingTerms
    NodeSelectorTerm term = newNodeSelectorTerm(t.preference);
    if (term.parse_error) st.preferred_error = true;
    else st.preferred.emplace_back((int64_t)t.weight, term);
  }
  return st;
}

// nodeaffinity.GetRequiredNodeAffinity(pod).Match(node), parse errors ignored
bool RequiredMatch(const PodState &st, const Node &n) {
  if (st.affinity_skip) return true;
  for (auto &r : st.node_selector)
    if (!Matches(r, n.labels)) return false;
  if (st.has_required) {
    for (auto &t : st.required)
      if (t.match(n)) return true;
    return false;
  }
  return true;
}

// v1helper.FindMatchingUntoleratedTaint(taints, tolerations, DoNotScheduleTaintsFilterFunc)
bool HasUntoleratedDoNotSchedule(const PodState &st, const Node &n) {
  for (auto &t : n.taints) {
    if (t.effect != KS_EFFECT_NO_SCHEDULE && t.effect != KS_EFFECT_NO_EXECUTE) continue;
    if (!TolerationsTolerateTaint(st.tolerations, t)) return true;
  }
  return false;
}

// -------------------------------------------------------------- filters
// Returns -1 (Success) or the KS_PLUGIN_* index of the first failing filter,
// in default-profile order (frameworkImpl.RunFilterPlugins stops at the first
// non-success status).

int Filter(const PodState &st, const Node &n) {
  // PreFilter outcome (schedule_one.go#findNodesThatFitPod): a rejecting
  // NodeAffinity PreFilter gives every node its status; nodes outside the
  // PreFilterResult get UnschedulableAndUnresolvable with no plugin and no
  // Filter runs on them (KS_FAIL_PREFILTER_RESULT)
  if (st.conflict) return KS_PLUGIN_NODE_AFFINITY;
  if (st.prefilter && !std::binary_search(st.prefilter_names.begin(), st.prefilter_names.end(), n.name))
    return KS_FAIL_PREFILTER_RESULT;
  // nodeunschedulable#Filter
  if (n.unschedulable &&
      !TolerationsTolerateTaint(st.tolerations,
                                Taint{"node.kubernetes.io/unschedulable", "", KS_EFFECT_NO_SCHEDULE}))
    return KS_PLUGIN_NODE_UNSCHEDULABLE;
  // nodename#Filter
  if (!st.node_name.empty() && st.node_name != n.name) return KS_PLUGIN_NODE_NAME;
  // tainttoleration#Filter: FindMatchingUntoleratedTaint(DoNotScheduleTaintsFilterFunc)
  for (auto &t : n.taints) {
    if (t.effect != KS_EFFECT_NO_SCHEDULE && t.effect != KS_EFFECT_NO_EXECUTE) continue;
    if (!TolerationsTolerateTaint(st.tolerations, t)) return KS_PLUGIN_TAINT_TOLERATION;
  }
  // nodeaffinity#Filter: RequiredNodeAffinity.Match (parse errors ignored)
  if (!RequiredMatch(st, n)) return KS_PLUGIN_NODE_AFFINITY;
  // noderesources/fit.go#fitsRequest
  bool fail = false;
  if (n.pods + 1 > n.alloc_pods) fail = true;
  if (!(st.req_cpu == 0 && st.req_mem == 0 && !st.req_other && st.xreq.empty())) {
    if (st.req_cpu > 0 && st.req_cpu > n.alloc_cpu - n.req_cpu) fail = true;
    if (st.req_mem > 0 && st.req_mem > n.alloc_mem - n.req_mem) fail = true;
    // ephemeral-storage (> 0) and every scalar resource (rQuant == 0 skipped)
    for (auto &kv : st.xreq) {
      if (kv.second == 0) continue;
      auto a = n.xalloc.find(kv.first);
      auto r = n.xreq.find(kv.first);
      const int64_t alloc = a == n.xalloc.end() ? 0 : a->second, req = r == n.xreq.end() ? 0 : r->second;
      if (kv.second > alloc - req) fail = true;
    }
  }
  if (fail) return KS_PLUGIN_NODE_RESOURCES_FIT;
  return -1;
}

// -------------------------------------------------------------- scores

// noderesources/least_allocated.go#leastRequestedScore
int64_t leastRequestedScore(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  return ((capacity - requested) * kMaxNodeScore) / capacity;
}

// resource_allocation.go#score + least_allocated.go#leastResourceScorer (cpu:1, memory:1),
// useRequested=false: node NonZeroRequested + pod non-zero request.
int64_t LeastAllocated(int64_t acpu, int64_t amem, int64_t ncpu, int64_t nmem, int64_t pcpu, int64_t pmem) {
  const int64_t alloc[2] = {acpu, amem};
  const int64_t req[2] = {ncpu + pcpu, nmem + pmem};
  int64_t nodeScore = 0, weightSum = 0;
  for (int i = 0; i < 2; ++i) {
    if (alloc[i] == 0) continue;
    nodeScore += leastRequestedScore(req[i], alloc[i]) * 1;
    weightSum += 1;
  }
  if (weightSum == 0) return 0;
  return nodeScore / weightSum;
}

// balanced_allocation.go#balancedResourceScorer, useRequested=true.
int64_t BalancedAllocation(int64_t acpu, int64_t amem, int64_t ncpu, int64_t nmem, int64_t pcpu, int64_t pmem) {
  const int64_t alloc[2] = {acpu, amem};
  const int64_t req[2] = {ncpu + pcpu, nmem + pmem};
  double fractions[2];
  int nf = 0;
  double totalFraction = 0;
  for (int i = 0; i < 2; ++i) {
    if (alloc[i] == 0) continue;
    double fraction = (double)req[i] / (double)alloc[i];
    if (fraction > 1) fraction = 1;
    totalFraction += fraction;
    fractions[nf++] = fraction;
  }
  (void)totalFraction;
  double std = 0.0;
  if (nf == 2) std = std::fabs((fractions[0] - fractions[1]) / 2);
  return (int64_t)((1 - std) * (double)kMaxNodeScore);
}

// tainttoleration#countIntolerableTaintsPreferNoSchedule
int64_t TaintRaw(const PodState &st, const Node &n) {
  int64_t c = 0;
  for (auto &t : n.taints) {
    if (t.effect != KS_EFFECT_PREFER_NO_SCHEDULE) continue;
    if (!TolerationsTolerateTaint(st.tolerations_prefer, t)) ++c;
  }
  return c;
}

// nodeaffinity#PreferredSchedulingTerms.Score
int64_t AffinityRaw(const PodState &st, const Node &n) {
  int64_t s = 0;
  for (auto &wt : st.preferred)
    if (wt.second.match(n)) s += wt.first;
  return s;
}

// plugins/helper/normalize_score.go#DefaultNormalizeScore for one element.
int64_t Normalize(int64_t score, int64_t maxCount, bool reverse) {
  if (maxCount == 0) return reverse ? kMaxNodeScore : 0;
  int64_t s = kMaxNodeScore * score / maxCount;
  return reverse ? kMaxNodeScore - s : s;
}

// Go math.Log (pure-Go log.go, the fdlibm e_log.c algorithm; the amd64
// assembly version performs the same operations), no FMA contraction.
double GoLog(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (std::isnan(x) || std::isinf(x)) return x;
  if (x < 0) return std::nan("");
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = std::frexp(x, &ki);
  if (f1 < 0.70710678118654752440 /* Sqrt2/2 */) {
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

// podtopologyspread/common.go#countPodsMatchSelector
int64_t CountPodsMatchSelector(const Node &n, const Selector &sel, const std::string &ns) {
  if (sel.Empty()) return 0;
  int64_t c = 0;
  for (auto &r : n.pod_recs)
    if (r.ns == ns && sel.Match(r.labels)) ++c;
  return c;
}

// common.go#nodeLabelsMatchSpreadConstraints
bool HasAllKeys(const Node &n, const std::vector<SpreadConstraint> &cs) {
  for (auto &c : cs)
    if (!n.labels.count(c.key)) return false;
  return true;
}

// topologySpreadConstraint.matchNodeInclusionPolicies
bool MatchInclusion(const SpreadConstraint &c, const PodState &st, const Node &n) {
  if (c.aff_honor && !RequiredMatch(st, n)) return false;
  if (c.taint_honor && HasUntoleratedDoNotSchedule(st, n)) return false;
  return true;
}

// Parallel node loop: parallelize.Until chunking, chunk = min(sqrt(N), N/threads + 1).
// fn(lo, hi, thread) over [lo, hi); the reductions built on it are
// order-independent (sums, min / max, set unions).
void ParallelNodes(int threads, uint32_t lo, uint32_t hi, const std::function<void(uint32_t, uint32_t, int)> &fn) {
  const uint32_t N = hi - lo;
  if (threads <= 1 || N < 1024) {
    fn(lo, hi, 0);
    return;
  }
  uint32_t chunk = std::min<uint32_t>((uint32_t)std::sqrt((double)N), N / threads + 1);
  if (chunk == 0) chunk = 1;
  std::atomic<uint32_t> next{lo};
  std::vector<std::thread> ws;
  for (int t = 0; t < threads; ++t) {
    ws.emplace_back([&, t] {
      while (true) {
        uint32_t s = next.fetch_add(chunk);
        if (s >= hi) break;
        fn(s, std::min(hi, s + chunk), t);
      }
    });
  }
  for (auto &w : ws) w.join();
}

template <class K>
void MergeCounts(std::map<K, int64_t> &into, const std::map<K, int64_t> &from) {
  for (auto &kv : from) into[kv.first] += kv.second;
}

// filtering.go#calPreFilterState: matching pods per topology value of every
// DoNotSchedule constraint over all nodes, and the global minimum
// (criticalPaths[0], 0 when fewer domains than minDomains).
struct SpreadFilterState {
  std::vector<std::map<std::string, int64_t>> counts;
  std::vector<int64_t> min_match;
};

SpreadFilterState SpreadPreFilter(const PodState &st, const std::vector<Node> &nodes, int threads) {
  SpreadFilterState s;
  const size_t nc = st.spread_filter.size();
  s.counts.resize(nc);
  s.min_match.assign(nc, 0);
  std::vector<std::vector<std::map<std::string, int64_t>>> part(threads < 1 ? 1 : threads,
                                                                std::vector<std::map<std::string, int64_t>>(nc));
  ParallelNodes(threads, 0, (uint32_t)nodes.size(), [&](uint32_t a, uint32_t b, int t) {
    for (uint32_t j = a; j < b; ++j) {
      const Node &n = nodes[j];
      if (!n.present || !HasAllKeys(n, st.spread_filter)) continue;
      for (size_t i = 0; i < nc; ++i) {
        const SpreadConstraint &c = st.spread_filter[i];
        if (!MatchInclusion(c, st, n)) continue;
        part[t][i][n.labels.at(c.key)] += CountPodsMatchSelector(n, c.sel, st.ns);
      }
    }
  });
  for (auto &q : part)
    for (size_t i = 0; i < nc; ++i) MergeCounts(s.counts[i], q[i]);
  for (size_t i = 0; i < nc; ++i) {
    int64_t m = INT32_MAX;  // newCriticalPaths: MatchNum = math.MaxInt32
    for (auto &kv : s.counts[i]) m = std::min(m, kv.second);
    if ((int64_t)s.counts[i].size() < st.spread_filter[i].min_domains) m = 0;  // minMatchNum
    s.min_match[i] = m;
  }
  return s;
}

// filtering.go#Filter: 'existing matching num' + 'self-match' - 'global min' <= maxSkew
bool SpreadFilter(const PodState &st, const SpreadFilterState &s, const Node &n) {
  for (size_t i = 0; i < st.spread_filter.size(); ++i) {
    const SpreadConstraint &c = st.spread_filter[i];
    auto it = n.labels.find(c.key);
    if (it == n.labels.end()) return false;  // ErrReasonNodeLabelNotMatch
    const int64_t self = c.sel.Match(st.labels) ? 1 : 0;
    auto m = s.counts[i].find(it->second);
    const int64_t match = m == s.counts[i].end() ? 0 : m->second;
    if (match + self - s.min_match[i] > (int64_t)c.max_skew) return false;  // ErrReasonConstraintsNotMatch
  }
  return true;
}

// interpodaffinity/filtering.go#PreFilter: existingAntiAffinityCounts (the
// existing pods' required anti-affinity terms the incoming pod matches),
// affinityCounts (existing pods matching ALL the incoming pod's required
// affinity terms, per term's topology pair) and antiAffinityCounts.
using TopoPair = std::pair<std::string, std::string>;
struct IpaFilterState {
  bool active = false;
  std::map<TopoPair, int64_t> existing_anti, aff, anti;
};

IpaFilterState IpaPreFilter(const PodState &st, const std::vector<Node> &nodes, int threads) {
  IpaFilterState s;
  const auto &req_aff = st.ipa[KS_POD_AFFINITY_REQUIRED], &req_anti = st.ipa[KS_POD_ANTI_AFFINITY_REQUIRED];
  // getIncomingAffinityAntiAffinityCounts visits every node only for a pod
  // with required terms; getExistingAntiAffinityCounts only the nodes with
  // pods carrying required anti-affinity
  const bool incoming = !req_aff.empty() || !req_anti.empty();
  std::vector<IpaFilterState> part(threads < 1 ? 1 : threads);
  ParallelNodes(threads, 0, (uint32_t)nodes.size(), [&](uint32_t a, uint32_t b, int th) {
  IpaFilterState &s = part[th];
  for (uint32_t j = a; j < b; ++j) {
    const Node &n = nodes[j];
    if (!n.present || (!incoming && n.pods_with_req_anti == 0)) continue;
    for (auto &e : n.pod_recs) {
      if (!incoming && e.terms.empty()) continue;
      for (auto &t : e.terms) {  // updateWithAntiAffinityTerms(existing terms, incoming pod)
        if (t.kind != KS_POD_ANTI_AFFINITY_REQUIRED || !t.Matches(st.ns, st.labels, st.ns_labels)) continue;
        auto it = n.labels.find(t.key);
        if (it != n.labels.end()) s.existing_anti[{t.key, it->second}] += 1;
      }
      bool all = !req_aff.empty();  // podMatchesAllAffinityTerms (merged namespaces)
      for (auto &t : req_aff) all = all && t.Matches(e.ns, e.labels, e.ns_labels);
      if (all)
        for (auto &t : req_aff) {
          auto it = n.labels.find(t.key);
          if (it != n.labels.end()) s.aff[{t.key, it->second}] += 1;
        }
      for (auto &t : req_anti) {
        if (!t.Matches(e.ns, e.labels, e.ns_labels)) continue;
        auto it = n.labels.find(t.key);
        if (it != n.labels.end()) s.anti[{t.key, it->second}] += 1;
      }
    }
  }
  });
  for (auto &q : part) {
    MergeCounts(s.existing_anti, q.existing_anti);
    MergeCounts(s.aff, q.aff);
    MergeCounts(s.anti, q.anti);
  }
  s.active = !(s.existing_anti.empty() && req_aff.empty() && req_anti.empty());  // else PreFilter Skip
  return s;
}

// filtering.go#Filter: satisfyPodAffinity, satisfyPodAntiAffinity, satisfyExistingPodsAntiAffinity
bool IpaFilter(const PodState &st, const IpaFilterState &s, const Node &n) {
  const auto &req_aff = st.ipa[KS_POD_AFFINITY_REQUIRED];
  bool exist = true;
  for (auto &t : req_aff) {
    auto it = n.labels.find(t.key);
    if (it == n.labels.end()) return false;  // all topology labels must exist on the node
    auto c = s.aff.find({t.key, it->second});
    if (c == s.aff.end() || c->second <= 0) exist = false;
  }
  if (!exist) {
    // the first pod of a series with affinity to itself
    bool self = !req_aff.empty();
    for (auto &t : req_aff) self = self && t.Matches(st.ns, st.labels, st.ns_labels);
    if (!(s.aff.empty() && self)) return false;
  }
  if (!s.anti.empty())
    for (auto &t : st.ipa[KS_POD_ANTI_AFFINITY_REQUIRED]) {
      auto it = n.labels.find(t.key);
      if (it == n.labels.end()) continue;
      auto c = s.anti.find({t.key, it->second});
      if (c != s.anti.end() && c->second > 0) return false;
    }
  if (!s.existing_anti.empty())
    for (auto &kv : n.labels) {
      auto c = s.existing_anti.find({kv.first, kv.second});
      if (c != s.existing_anti.end() && c->second > 0) return false;
    }
  return true;
}

// schedule_one.go#numFeasibleNodesToFind (minFeasibleNodesToFind 100,
// minFeasibleNodesPercentageToFind 5; int32 arithmetic, exact for any
// node count below 2^31 / 100)
int64_t NumFeasibleNodesToFind(int32_t pct, int64_t n) {
  if (n < 100) return n;
  int64_t p = pct;
  if (p == 0) {
    p = 50 - n / 125;
    if (p < 5) p = 5;
  }
  const int64_t k = n * p / 100;
  return k < 100 ? 100 : k;
}

inline uint64_t PackKey(int64_t total, uint32_t slot) {
  return ((uint64_t)(total + 1) << 32) | (uint64_t)(0xFFFFFFFFu - slot);
}

}  // namespace

// ================================================================ oracle

struct oracle {
  std::vector<Node> nodes;
  // cache imageStates: name -> (size of the first reporter, nodes reporting it)
  struct ImageState {
    int64_t size = 0;
    int64_t nodes = 0;
  };
  std::map<std::string, ImageState> image_states;
  int64_t n_present = 0;

  void images_ref(const Node &n, int sign) {
    for (auto &im : n.images) {
      auto it = image_states.find(im.first);
      if (sign > 0) {
        if (it == image_states.end()) image_states.emplace(im.first, ImageState{im.second, 1});
        else it->second.nodes++;
      } else if (it != image_states.end() && --it->second.nodes == 0) {
        image_states.erase(it);
      }
    }
  }

  // imagelocality Score: calculatePriority(sumImageScores, #containers)
  int64_t ImageLocality(const PodState &st, const Node &n) const {
    int64_t sum = 0;
    for (auto &nm : st.images) {
      if (nm.empty()) continue;
      bool on = false;
      for (auto &im : n.images) on |= im.first == nm;
      if (!on) continue;
      const ImageState &s = image_states.at(nm);
      sum += (int64_t)((double)s.size * ((double)s.nodes / (double)n_present));  // scaledImageScore
    }
    const int64_t mb = 1024 * 1024, minT = 23 * mb, maxT = 1000 * mb * st.n_containers;
    if (sum < minT) sum = minT;
    else if (sum > maxT) sum = maxT;
    return kMaxNodeScore * (sum - minT) / (maxT - minT);
  }
  int64_t w_fit, w_ba, w_tt, w_na, w_il, w_pts = 2, w_ipa = 2, hard_weight = 1;
  int threads = 1;
  int32_t pct = 100;        // percentageOfNodesToScore
  uint64_t next_start = 0;  // Scheduler.nextStartNodeIndex
  static constexpr int kNotVisited = 1000;  // ev[i].status of a node the window skipped

  struct Eval {
    int status;
    int64_t la, ba, tt_raw, na_raw;
    int64_t pts_raw, pts;  // PodTopologySpread raw / normalized (ScheduleAnyway constraints)
    int64_t il;            // ImageLocality
    int64_t ipa_raw, ipa;  // InterPodAffinity raw / normalized
  };
  std::vector<Eval> ev;  // per-node scratch, reused across pods

  Eval eval(const PodState &st, const Node &n, const SpreadFilterState *sf = nullptr,
            const IpaFilterState *af = nullptr) const {
    Eval e{};
    e.status = Filter(st, n);
    // PodTopologySpread.Filter follows NodeResourcesFit in the default profile
    if (e.status < 0 && sf && !st.spread_filter.empty() && !SpreadFilter(st, *sf, n))
      e.status = KS_PLUGIN_POD_TOPOLOGY_SPREAD;
    if (e.status < 0 && af && af->active && !IpaFilter(st, *af, n)) e.status = KS_PLUGIN_INTER_POD_AFFINITY;
    if (e.status >= 0) return e;
    e.la = LeastAllocated(n.alloc_cpu, n.alloc_mem, n.nz_cpu, n.nz_mem, st.nz_cpu, st.nz_mem);
    e.ba = BalancedAllocation(n.alloc_cpu, n.alloc_mem, n.req_cpu, n.req_mem, st.req_cpu, st.req_mem);
    e.tt_raw = TaintRaw(st, n);
    e.na_raw = st.has_preferred ? AffinityRaw(st, n) : 0;
    e.il = ImageLocality(st, n);
    return e;
  }

  int64_t total(const PodState &st, const Eval &e, int64_t tt_max, int64_t na_max) const {
    // frameworkImpl.RunScorePlugins: Σ weight × normalized score.  ImageLocality
    // scores 0 (nodes report no images); NodeAffinity is skipped without
    // preferred terms (PreScore Skip) and contributes nothing either way.
    int64_t t = w_fit * e.la + w_ba * e.ba + w_tt * Normalize(e.tt_raw, tt_max, true) + w_il * e.il;
    if (st.has_preferred) t += w_na * Normalize(e.na_raw, na_max, false);
    if (!st.spread_score.empty()) t += w_pts * e.pts;  // PreScore Skip without ScheduleAnyway constraints
    t += w_ipa * e.ipa;  // 0 when its PreScore skips (no topology score at all)
    return t;
  }

  void add_pod(Node &n, const ks_pod &p, int sign) {
    Node::PodRec rec;
    rec.ns = S(p.ns);
    for (uint32_t k = 0; k < p.n_labels; ++k) rec.labels[S(p.labels[k].key)] = S(p.labels[k].value);
    for (uint32_t k = 0; k < p.n_namespace_labels; ++k)
      rec.ns_labels[S(p.namespace_labels[k].key)] = S(p.namespace_labels[k].value);
    rec.key = rec.ns + "\x01" + S(p.name);
    for (auto &kv : rec.labels) rec.key += "\x01" + kv.first + "=" + kv.second;
    for (uint32_t k = 0; k < p.n_affinity_terms; ++k) {
      AffTerm a;
      if (NewAffinityTerm(p, p.affinity_terms[k], &a)) rec.terms.push_back(a);
    }
    auto counts = [&n](const Node::PodRec &r, int64_t d) {
      bool anti = false;
      for (auto &t : r.terms) anti |= t.kind == KS_POD_ANTI_AFFINITY_REQUIRED;
      n.pods_with_affinity += r.terms.empty() ? 0 : d;
      n.pods_with_req_anti += anti ? d : 0;
    };
    if (sign > 0) {
      counts(rec, +1);
      n.pod_recs.push_back(std::move(rec));
    } else {
      auto it = std::find(n.pod_recs.begin(), n.pod_recs.end(), rec);
      if (it != n.pod_recs.end()) {
        counts(*it, -1);
        n.pod_recs.erase(it);
      }
    }
    // framework/types.go#NodeInfo.update via calculateResource
    int64_t rc, rm, zc, zm;
    bool other = false;
    PodRequests(p, false, &rc, &rm, &other);
    PodRequests(p, true, &zc, &zm, &other);
    n.req_cpu += sign * rc;
    n.req_mem += sign * rm;
    for (auto &kv : PodXRequests(p)) n.xreq[kv.first] += sign * kv.second;
    n.nz_cpu += sign * zc;
    n.nz_mem += sign * zm;
    n.pods += sign;
  }

  void for_nodes(uint32_t lo, uint32_t hi, const std::function<void(uint32_t, uint32_t, int)> &fn) const {
    ParallelNodes(threads, lo, hi, fn);
  }

  // PodTopologySpread PreScore / Score / NormalizeScore (scoring.go) over the
  // feasible nodes (ev[i].status < 0): fills ev[i].pts_raw / ev[i].pts.
  void spread_score(const PodState &st, std::vector<Eval> &ev) const {
    const auto &cs = st.spread_score;
    if (cs.empty()) return;
    const bool requireAll = !st.spread_defaulted;
    const uint32_t N = (uint32_t)nodes.size();
    const size_t nc = cs.size();
    std::vector<char> ignored(N, 0);
    int64_t n_filtered = 0, n_ignored = 0;
    // initPreScoreState: topology values of the filtered (feasible) nodes
    struct Part {
      int64_t filtered = 0, ignored = 0, mn = INT64_MAX, mx = 0;
      std::vector<std::map<std::string, int64_t>> counts;
    };
    std::vector<Part> part(threads < 1 ? 1 : threads);
    for (auto &q : part) q.counts.resize(nc);
    for_nodes(0, N, [&](uint32_t a, uint32_t b, int t) {
      Part &q = part[t];
      for (uint32_t i = a; i < b; ++i) {
        if (!nodes[i].present || ev[i].status >= 0) continue;
        ++q.filtered;
        if (requireAll && !HasAllKeys(nodes[i], cs)) {
          ignored[i] = 1;
          ++q.ignored;
          continue;
        }
        for (size_t c = 0; c < nc; ++c) {
          if (cs[c].hostname) continue;
          auto it = nodes[i].labels.find(cs[c].key);
          q.counts[c].emplace(it == nodes[i].labels.end() ? std::string() : it->second, 0);
        }
      }
    });
    std::vector<std::map<std::string, int64_t>> counts(nc);
    for (auto &q : part) {
      n_filtered += q.filtered;
      n_ignored += q.ignored;
      for (size_t c = 0; c < nc; ++c) MergeCounts(counts[c], q.counts[c]);
      for (auto &m : q.counts) m.clear();
    }
    std::vector<double> weight(nc);
    for (size_t c = 0; c < nc; ++c) {
      const int64_t sz = cs[c].hostname ? n_filtered - n_ignored : (int64_t)counts[c].size();
      weight[c] = GoLog((double)(sz + 2));  // topologyNormalizingWeight
    }
    // PreScore processAllNode: matching pods of every node in a filtered domain
    for_nodes(0, N, [&](uint32_t a, uint32_t b, int t) {
      Part &q = part[t];
      for (uint32_t i = a; i < b; ++i) {
        const Node &n = nodes[i];
        if (!n.present) continue;
        if (requireAll && !HasAllKeys(n, cs)) continue;
        for (size_t c = 0; c < nc; ++c) {
          if (cs[c].hostname || !MatchInclusion(cs[c], st, n)) continue;
          auto it = n.labels.find(cs[c].key);
          const std::string &v = it == n.labels.end() ? std::string() : it->second;
          if (!counts[c].count(v)) continue;
          q.counts[c][v] += CountPodsMatchSelector(n, cs[c].sel, st.ns);
        }
      }
    });
    for (auto &q : part)
      for (size_t c = 0; c < nc; ++c) MergeCounts(counts[c], q.counts[c]);
    // Score: Σ cnt * weight + (maxSkew - 1), math.Round; NormalizeScore: min / max
    for_nodes(0, N, [&](uint32_t a, uint32_t b, int t) {
      Part &q = part[t];
      for (uint32_t i = a; i < b; ++i) {
        if (!nodes[i].present || ev[i].status >= 0 || ignored[i]) continue;
        const Node &n = nodes[i];
        double score = 0;
        for (size_t c = 0; c < nc; ++c) {
          auto it = n.labels.find(cs[c].key);
          if (it == n.labels.end()) continue;
          const int64_t cnt = cs[c].hostname ? CountPodsMatchSelector(n, cs[c].sel, st.ns) : counts[c].at(it->second);
          score += (double)cnt * weight[c] + (double)(cs[c].max_skew - 1);  // scoreForCount
        }
        ev[i].pts_raw = (int64_t)std::round(score);
        q.mn = std::min(q.mn, ev[i].pts_raw);
        q.mx = std::max(q.mx, ev[i].pts_raw);
      }
    });
    int64_t mn = INT64_MAX, mx = 0;
    for (auto &q : part) {
      mn = std::min(mn, q.mn);
      mx = std::max(mx, q.mx);
    }
    for (uint32_t i = 0; i < N; ++i) {
      if (!nodes[i].present || ev[i].status >= 0) continue;
      if (ignored[i]) ev[i].pts = 0;
      else if (mx == 0) ev[i].pts = kMaxNodeScore;
      else ev[i].pts = kMaxNodeScore * (mx + mn - ev[i].pts_raw) / mx;
    }
  }

  // InterPodAffinity PreScore / Score / NormalizeScore (scoring.go) over the
  // feasible nodes: topologyScore[key][value] from the incoming pod's
  // preferred terms against existing pods and the existing pods' required
  // (hardPodAffinityWeight) and preferred terms against the incoming pod;
  // min-max normalised in float64.  Fills ev[i].ipa_raw / ev[i].ipa.
  void ipa_score(const PodState &st, std::vector<Eval> &ev) const {
    std::map<std::string, std::map<std::string, int64_t>> ts;
    const uint32_t N = (uint32_t)nodes.size();
    // scoring.go#PreScore: without preferred terms of its own only the pods
    // with affinity (HavePodsWithAffinityList, NodeInfo.PodsWithAffinity) count
    const bool own = !st.ipa[KS_POD_AFFINITY_PREFERRED].empty() || !st.ipa[KS_POD_ANTI_AFFINITY_PREFERRED].empty();
    std::vector<std::map<std::string, std::map<std::string, int64_t>>> part(threads < 1 ? 1 : threads);
    for_nodes(0, N, [&](uint32_t a, uint32_t b, int th) {
    auto &ts = part[th];
    for (uint32_t i = a; i < b; ++i) {
      const Node &n = nodes[i];
      if (!n.present || n.labels.empty() || (!own && n.pods_with_affinity == 0)) continue;
      auto add = [&](const AffTerm &t, int64_t w) {
        auto it = n.labels.find(t.key);
        if (it != n.labels.end()) ts[t.key][it->second] += w;
      };
      for (auto &e : n.pod_recs) {
        if (!own && e.terms.empty()) continue;
        for (auto &t : st.ipa[KS_POD_AFFINITY_PREFERRED])
          if (t.Matches(e.ns, e.labels, e.ns_labels)) add(t, t.weight);
        for (auto &t : st.ipa[KS_POD_ANTI_AFFINITY_PREFERRED])
          if (t.Matches(e.ns, e.labels, e.ns_labels)) add(t, -t.weight);
        for (auto &t : e.terms) {
          if (!t.Matches(st.ns, st.labels, st.ns_labels)) continue;
          if (t.kind == KS_POD_AFFINITY_REQUIRED && hard_weight > 0) add(t, hard_weight);
          else if (t.kind == KS_POD_AFFINITY_PREFERRED) add(t, t.weight);
          else if (t.kind == KS_POD_ANTI_AFFINITY_PREFERRED) add(t, -t.weight);
        }
      }
    }
    });
    for (auto &q : part)
      for (auto &kv : q) MergeCounts(ts[kv.first], kv.second);
    if (ts.empty()) return;  // PreScore Skip: every score stays 0
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    for (uint32_t i = 0; i < N; ++i) {
      if (!nodes[i].present || ev[i].status >= 0) continue;
      int64_t sc = 0;
      for (auto &kv : ts) {
        auto it = nodes[i].labels.find(kv.first);
        if (it == nodes[i].labels.end()) continue;
        auto v = kv.second.find(it->second);
        if (v != kv.second.end()) sc += v->second;
      }
      ev[i].ipa_raw = sc;
      mn = std::min(mn, sc);
      mx = std::max(mx, sc);
    }
    const int64_t diff = mx - mn;
    for (uint32_t i = 0; i < N; ++i) {
      if (!nodes[i].present || ev[i].status >= 0) continue;
      double f = 0;
      if (diff > 0) f = (double)kMaxNodeScore * ((double)(ev[i].ipa_raw - mn) / (double)diff);
      ev[i].ipa = (int64_t)f;
    }
  }

  // findNodesThatPassFilters with percentageOfNodesToScore < 100
  // (schedule_one.go:findNodesThatFitPod / findNodesThatPassFilters /
  // numFeasibleNodesToFind), restated sequentially: upstream checks nodes with
  // parallelize.Until and keeps the first numNodesToFind that report feasible,
  // which with parallelism > 1 depends on goroutine timing; with one worker
  // it is this loop.  The node list is the present nodes in slot order
  // (upstream: the snapshot's list order), without the nodes a NodeAffinity
  // PreFilterResult excludes (upstream visits only the PreFilterResult's
  // nodes; they keep their KS_FAIL_PREFILTER_RESULT status here, never
  // visited).  Visiting starts at nextStartNodeIndex % len(list) and goes
  // round the list; the worker cancels at the (k+1)-th feasible node, so the
  // processed nodes (len(feasibleNodes) + len(NodeToStatus)) are the nodes
  // before it: k feasible and the infeasible ones between them.  Fewer than
  // k+1 feasible: every node is processed.  nextStartNodeIndex = (it +
  // processed) % len(allNodes).  Nodes after the window get kNotVisited.
  void window() {
    const uint32_t N = (uint32_t)nodes.size();
    std::vector<uint32_t> list;
    for (uint32_t i = 0; i < N; ++i)
      if (nodes[i].present && ev[i].status != KS_FAIL_PREFILTER_RESULT) list.push_back(i);
    const uint64_t nl = list.size();
    const int64_t k = NumFeasibleNodesToFind(pct, (int64_t)nl);
    uint64_t processed = nl;
    if (nl) {
      const uint64_t s = next_start % nl;
      int64_t found = 0;
      for (uint64_t j = 0; j < nl; ++j)
        if (ev[list[(s + j) % nl]].status < 0 && ++found == k + 1) {
          processed = j;
          break;
        }
      for (uint64_t j = processed; j < nl; ++j) ev[list[(s + j) % nl]].status = kNotVisited;
    }
    if (n_present) next_start = (next_start + processed) % (uint64_t)n_present;
  }

  // schedulePod (schedule_one.go): findNodesThatFitPod -> prioritizeNodes -> selectHost.
  ks_result schedule_one(const ks_pod &p) {
    ks_result r{};
    r.node_index = -1;
    PodState st = compile_pod(p);
    const uint32_t N = (uint32_t)nodes.size();
    ev.resize(N);
    SpreadFilterState sf;
    if (!st.spread_filter.empty()) sf = SpreadPreFilter(st, nodes, threads);
    const IpaFilterState af = IpaPreFilter(st, nodes, threads);
    // Filter + raw scores in parallel (findNodesThatPassFilters / RunScorePlugins
    // both fan out with parallelize.Until); counts and normaliser maxima are
    // order-independent reductions, combined from per-thread partials.
    struct Part {
      uint32_t evaluated = 0, feasible = 0, only = 0;
      uint32_t fail[KS_NUM_FAIL_COUNTS] = {};
      int64_t tt_max = 0, na_max = 0;
      uint64_t best = 0;
    };
    std::vector<Part> part(threads < 1 ? 1 : threads);
    for_nodes(0, N, [&](uint32_t a, uint32_t b, int) {
      for (uint32_t i = a; i < b; ++i)
        if (nodes[i].present) ev[i] = eval(st, nodes[i], &sf, &af);
    });
    if (pct != 100) window();
    for_nodes(0, N, [&](uint32_t a, uint32_t b, int t) {
      Part &q = part[t];
      for (uint32_t i = a; i < b; ++i) {
        if (!nodes[i].present || ev[i].status == kNotVisited) continue;
        ++q.evaluated;
        if (ev[i].status >= 0) {
          q.fail[ev[i].status]++;
          continue;
        }
        ++q.feasible;
        q.only = i;
        q.tt_max = std::max(q.tt_max, ev[i].tt_raw);
        q.na_max = std::max(q.na_max, ev[i].na_raw);
      }
    });
    uint32_t evaluated = 0, feasible = 0;
    int64_t tt_max = 0, na_max = 0;
    uint32_t only = 0;
    for (const Part &q : part) {
      evaluated += q.evaluated;
      feasible += q.feasible;
      if (q.feasible) only = q.only;
      for (int k = 0; k < KS_NUM_FAIL_COUNTS; ++k) r.fail_counts[k] += q.fail[k];
      tt_max = std::max(tt_max, q.tt_max);
      na_max = std::max(na_max, q.na_max);
    }
    r.evaluated_nodes = evaluated;
    r.feasible_nodes = feasible;
    if (feasible == 0) {
      r.status = KS_POD_UNSCHEDULABLE;  // FitError{NumAllNodes, Diagnosis}
      return r;
    }
    if (feasible == 1) {
      // "When only one node after predicate, just use it." No scoring upstream;
      // the build still reports that node's TotalScore.
      spread_score(st, ev);
      ipa_score(st, ev);
      r.flags |= KS_RESULT_SINGLE_FEASIBLE;
      r.node_index = (int32_t)only;
      r.total_score = total(st, ev[only], tt_max, na_max);
      r.status = KS_POD_SCHEDULED;
      return r;
    }
    if (st.has_preferred && st.preferred_error) {  // NodeAffinity.PreScore error
      r.status = KS_POD_ERROR;
      return r;
    }
    spread_score(st, ev);
    ipa_score(st, ev);
    for_nodes(0, N, [&](uint32_t a, uint32_t b, int t) {
      uint64_t &best = part[t].best;
      for (uint32_t i = a; i < b; ++i) {
        if (!nodes[i].present || ev[i].status >= 0) continue;
        uint64_t k = PackKey(total(st, ev[i], tt_max, na_max), i);
        if (k > best) best = k;  // max TotalScore, tie -> lowest slot
      }
    });
    uint64_t best = 0;
    for (const Part &q : part) best = std::max(best, q.best);
    r.node_index = (int32_t)(0xFFFFFFFFu - (uint32_t)best);
    r.total_score = (int64_t)(best >> 32) - 1;
    r.status = KS_POD_SCHEDULED;
    return r;
  }
};

extern "C" {

oracle *oracle_new(uint32_t cap, int32_t w_fit, int32_t w_ba, int32_t w_tt, int32_t w_na, int32_t w_il) {
  auto *o = new oracle();
  o->nodes.resize(cap);
  o->w_fit = w_fit;
  o->w_ba = w_ba;
  o->w_tt = w_tt;
  o->w_na = w_na;
  o->w_il = w_il;
  return o;
}
void oracle_free(oracle *o) { delete o; }
void oracle_set_threads(oracle *o, int32_t t) { o->threads = t < 1 ? 1 : t; }
void oracle_set_weight_spread(oracle *o, int32_t w) { o->w_pts = w; }
void oracle_set_weight_inter_pod_affinity(oracle *o, int32_t w, int32_t hard) {
  o->w_ipa = w;
  o->hard_weight = hard;
}
void oracle_set_percentage(oracle *o, int32_t pct) {
  o->pct = pct;
  o->next_start = 0;
}
uint64_t oracle_next_start(const oracle *o) { return o->next_start; }
int64_t oracle_num_feasible_nodes_to_find(int32_t pct, int64_t n) { return NumFeasibleNodesToFind(pct, n); }
double oracle_go_log(double x) { return GoLog(x); }

int32_t oracle_nodes_upsert(oracle *o, const ks_node *nodes, const uint32_t *slots, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    if (slots[i] >= o->nodes.size()) return KS_ERR_NOT_FOUND;
    Node &d = o->nodes[slots[i]];
    const ks_node &s = nodes[i];
    if (!d.present) {
      d = Node();
      o->n_present++;
    } else {
      o->images_ref(d, -1);  // UpdateNode: removeNodeImageStates, then add
    }
    d.present = true;
    d.images.clear();
    {
      std::set<std::string> seen;
      for (uint32_t k = 0; k < s.n_images; ++k)
        if (s.images[k].name && s.images[k].name[0] && seen.insert(S(s.images[k].name)).second)
          d.images.emplace_back(S(s.images[k].name), s.images[k].size_bytes);
    }
    o->images_ref(d, +1);
    d.xalloc.clear();
    for (uint32_t k = 0; k < s.n_extended; ++k)
      if (ExtendedResourceName(S(s.extended[k].name))) d.xalloc[S(s.extended[k].name)] = s.extended[k].value;
    d.name = S(s.name);
    d.alloc_cpu = s.alloc_milli_cpu;
    d.alloc_mem = s.alloc_memory;
    d.alloc_pods = s.alloc_pods;
    d.unschedulable = s.unschedulable != 0;
    d.labels.clear();
    for (uint32_t k = 0; k < s.n_labels; ++k) d.labels[S(s.labels[k].key)] = S(s.labels[k].value);
    d.taints.clear();
    for (uint32_t k = 0; k < s.n_taints; ++k)
      d.taints.push_back({S(s.taints[k].key), S(s.taints[k].value), s.taints[k].effect});
  }
  return KS_OK;
}

int32_t oracle_nodes_delete(oracle *o, const uint32_t *slots, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    if (slots[i] >= o->nodes.size()) return KS_ERR_NOT_FOUND;
    if (o->nodes[slots[i]].present) {
      o->images_ref(o->nodes[slots[i]], -1);
      o->n_present--;
    }
    o->nodes[slots[i]] = Node();
  }
  return KS_OK;
}

int32_t oracle_pods_add(oracle *o, const ks_pod *pods, const uint32_t *slots, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    if (slots[i] >= o->nodes.size() || !o->nodes[slots[i]].present) return KS_ERR_NOT_FOUND;
    o->add_pod(o->nodes[slots[i]], pods[i], +1);
  }
  return KS_OK;
}

int32_t oracle_pods_remove(oracle *o, const ks_pod *pods, const uint32_t *slots, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    if (slots[i] >= o->nodes.size() || !o->nodes[slots[i]].present) return KS_ERR_NOT_FOUND;
    o->add_pod(o->nodes[slots[i]], pods[i], -1);
  }
  return KS_OK;
}

int32_t oracle_schedule(oracle *o, const ks_pod *pods, uint32_t n, ks_result *out) {
  for (uint32_t i = 0; i < n; ++i) {
    out[i] = o->schedule_one(pods[i]);
    if (out[i].status == KS_POD_SCHEDULED)
      o->add_pod(o->nodes[out[i].node_index], pods[i], +1);  // assume -> NodeInfo.AddPod
  }
  return KS_OK;
}

int32_t oracle_plugin_scores(oracle *o, const ks_pod *pod, ks_node_score *out) {
  PodState st = compile_pod(*pod);
  const uint32_t N = (uint32_t)o->nodes.size();
  std::vector<oracle::Eval> ev(N);
  int64_t tt_max = 0, na_max = 0;
  SpreadFilterState sf;
  if (!st.spread_filter.empty()) sf = SpreadPreFilter(st, o->nodes, o->threads);
  const IpaFilterState af = IpaPreFilter(st, o->nodes, o->threads);
  for (uint32_t i = 0; i < N; ++i) {
    if (!o->nodes[i].present) {
      ev[i].status = -2;
      continue;
    }
    ev[i] = o->eval(st, o->nodes[i], &sf, &af);
    if (ev[i].status < 0) {
      tt_max = std::max(tt_max, ev[i].tt_raw);
      na_max = std::max(na_max, ev[i].na_raw);
    }
  }
  for (uint32_t i = 0; i < N; ++i) {
    ks_node_score s{};
    if (i == 0) {  // PodTopologySpread and InterPodAffinity over the feasible set
      o->spread_score(st, ev);
      o->ipa_score(st, ev);
    }
    if (!o->nodes[i].present) {
      s.status = -2;
    } else if (ev[i].status >= 0) {
      s.status = ev[i].status;
    } else {
      s.status = -1;
      s.least_allocated = (int32_t)ev[i].la;
      s.balanced_allocation = (int32_t)ev[i].ba;
      s.taint_raw = (int32_t)ev[i].tt_raw;
      s.taint_score = (int32_t)Normalize(ev[i].tt_raw, tt_max, true);
      s.affinity_raw = (int32_t)ev[i].na_raw;
      s.affinity_score = st.has_preferred ? (int32_t)Normalize(ev[i].na_raw, na_max, false) : 0;
      s.image_locality = (int32_t)ev[i].il;
      s.spread_raw = (int32_t)ev[i].pts_raw;
      s.spread_score = st.spread_score.empty() ? 0 : (int32_t)ev[i].pts;
      s.affinity_pod_raw = (int32_t)ev[i].ipa_raw;
      s.affinity_pod_score = (int32_t)ev[i].ipa;
      s.total_score = o->total(st, ev[i], tt_max, na_max);
    }
    out[i] = s;
  }
  return KS_OK;
}

int32_t oracle_node_states(oracle *o, const uint32_t *slots, uint32_t n, ks_node_state *out) {
  for (uint32_t i = 0; i < n; ++i) {
    if (slots[i] >= o->nodes.size()) return KS_ERR_NOT_FOUND;
    const Node &d = o->nodes[slots[i]];
    ks_node_state s{};
    if (d.present) {
      s.alloc_milli_cpu = d.alloc_cpu;
      s.alloc_memory = d.alloc_mem;
      s.req_milli_cpu = d.req_cpu;
      s.req_memory = d.req_mem;
      s.nonzero_milli_cpu = d.nz_cpu;
      s.nonzero_memory = d.nz_mem;
      s.alloc_pods = (int32_t)d.alloc_pods;
      s.pod_count = (int32_t)d.pods;
    } else {
      s.pod_count = -1;
    }
    out[i] = s;
  }
  return KS_OK;
}

int32_t oracle_shard_prescore_run(oracle *o, const ks_pod *pod, uint32_t lo, uint32_t hi,
                                  oracle_shard_prescore *out) {
  PodState st = compile_pod(*pod);
  oracle_shard_prescore r{};
  hi = std::min<uint32_t>(hi, (uint32_t)o->nodes.size());
  for (uint32_t i = lo; i < hi; ++i) {
    if (!o->nodes[i].present) continue;
    oracle::Eval e = o->eval(st, o->nodes[i]);
    if (e.status >= 0) {
      r.fail_counts[e.status]++;
      continue;
    }
    r.feasible++;
    if (e.tt_raw > r.taint_max) { r.taint_max = e.tt_raw; r.taint_count = 0; }
    if (e.tt_raw == r.taint_max) r.taint_count++;
    if (e.na_raw > r.affinity_max) { r.affinity_max = e.na_raw; r.affinity_count = 0; }
    if (e.na_raw == r.affinity_max) r.affinity_count++;
  }
  r.error = (st.has_preferred && st.preferred_error) ? 1 : 0;
  *out = r;
  return KS_OK;
}

uint64_t oracle_shard_best(oracle *o, const ks_pod *pod, uint32_t lo, uint32_t hi, int64_t tt_max,
                           int64_t na_max) {
  PodState st = compile_pod(*pod);
  uint64_t best = 0;
  hi = std::min<uint32_t>(hi, (uint32_t)o->nodes.size());
  for (uint32_t i = lo; i < hi; ++i) {
    if (!o->nodes[i].present) continue;
    oracle::Eval e = o->eval(st, o->nodes[i]);
    if (e.status >= 0) continue;
    best = std::max(best, PackKey(o->total(st, e, tt_max, na_max), i));
  }
  return best;
}

int32_t oracle_commit(oracle *o, const ks_pod *pod, uint32_t slot) {
  if (slot >= o->nodes.size() || !o->nodes[slot].present) return KS_ERR_NOT_FOUND;
  o->add_pod(o->nodes[slot], *pod, +1);
  return KS_OK;
}

int64_t oracle_least_allocated(int64_t acpu, int64_t amem, int64_t ncpu, int64_t nmem, int64_t pcpu,
                               int64_t pmem) {
  return LeastAllocated(acpu, amem, ncpu, nmem, pcpu, pmem);
}

int64_t oracle_balanced_allocation(int64_t acpu, int64_t amem, int64_t ncpu, int64_t nmem,
                                   int64_t pcpu, int64_t pmem) {
  return BalancedAllocation(acpu, amem, ncpu, nmem, pcpu, pmem);
}

int32_t oracle_pod_requests(const ks_pod *pod, int64_t out[4]) {
  bool other = false;
  PodRequests(*pod, false, &out[0], &out[1], &other);
  PodRequests(*pod, true, &out[2], &out[3], &other);
  return other ? KS_ERR_UNSUPPORTED : KS_OK;
}

}  // extern "C"
