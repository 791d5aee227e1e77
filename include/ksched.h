/*
 * ksched.h — C ABI of the MI355X-native dist-scheduler shard core (libksched.so).
 *
 * This is the drop-in boundary for ONE path of bchess/k8s-1m: the dist-scheduler
 * shard's Filter -> Score -> NormalizeScore -> select -> commit loop.  In the
 * reference that loop is the forked kube-scheduler's `schedulePod` (upstream
 * k8s.io/kubernetes v1.31.3 pkg/scheduler/schedule_one.go), reached from
 *   dist-scheduler/cmd/dist-scheduler/scheduler.go:543   (ScheduleOne goroutine)
 * and its result is consumed by
 *   dist-scheduler/pkg/distpermit/distpermit.go:51-72    (NodePluginScoresState -> TotalScore)
 *   dist-scheduler/pkg/distpermit/distpermit.go:81-121   (SendScore, int32 score, 0 = no candidate)
 *   dist-scheduler/cmd/dist-scheduler/scheduler.go:372-401 (podScheduleFailure: FitError path)
 * A Go shim overrides the upstream `Scheduler.SchedulePod` function field next to
 * the `NextPod` / `FailureHandler` overrides the reference already installs
 * (scheduler.go:307-321) and calls these entry points through cgo; see
 * INTEGRATION.md for the binding.
 *
 * Conventions
 *  - Every entry point returns ks_status (0 = KS_OK).  No C++ exception crosses
 *    the ABI; the last error text of a context is available via ks_last_error().
 *  - All buffers are caller-owned.  Pointers passed in are only read during the
 *    call; nothing is retained.  No callbacks.
 *  - One ks_ctx per GPU.  Calls on one context must be externally serialised.
 *  - Resource quantities are integers in canonical units: CPU in millicores
 *    (Quantity.MilliValue()), memory in bytes (Quantity.Value()).
 *  - Node identity is a caller-chosen slot index in [0, node_capacity); the
 *    node index is also the deterministic tie-break key (lowest index wins).
 */
#ifndef KSCHED_H
#define KSCHED_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KSCHED_ABI_VERSION 6

/* ---------------------------------------------------------------- status */
typedef int32_t ks_status;
enum {
  KS_OK = 0,
  KS_ERR_INVALID = 1,     /* bad argument / malformed object                 */
  KS_ERR_DEVICE = 2,      /* HIP runtime error (no device, launch failure)   */
  KS_ERR_CAPACITY = 3,    /* dictionary / slot capacity exhausted            */
  KS_ERR_UNSUPPORTED = 4, /* feature outside the implemented plugin subset   */
  KS_ERR_RANGE = 5,       /* value outside the exact-arithmetic range        */
  KS_ERR_NOT_FOUND = 6,   /* unknown node slot                               */
  KS_ERR_COMM = 7,        /* RCCL error                                      */
  KS_ERR_STALE = 8        /* batch compiled against an older node dictionary */
};

/* ------------------------------------------------------- k8s-shaped input */
/* Mirrors k8s.io/api/core/v1 types restricted to the fields the path reads. */

typedef struct {
  const char *key;
  const char *value;
} ks_label;

/* v1.TaintEffect */
enum {
  KS_EFFECT_ALL = 0, /* "" (only meaningful on a toleration: matches every effect) */
  KS_EFFECT_NO_SCHEDULE = 1,
  KS_EFFECT_PREFER_NO_SCHEDULE = 2,
  KS_EFFECT_NO_EXECUTE = 3
};

typedef struct {
  const char *key;
  const char *value;
  int32_t effect; /* KS_EFFECT_* (never KS_EFFECT_ALL on a taint) */
  int32_t _pad;
} ks_taint;

/* v1.TolerationOperator */
enum { KS_TOL_EQUAL = 0 /* "" or "Equal" */, KS_TOL_EXISTS = 1, KS_TOL_INVALID = 2 };

typedef struct {
  const char *key;   /* "" / NULL = any key (only valid with Exists)  */
  const char *value; /* NULL treated as ""                             */
  int32_t op;        /* KS_TOL_*                                       */
  int32_t effect;    /* KS_EFFECT_* ; KS_EFFECT_ALL = "" (all effects) */
} ks_toleration;

/* A resource quantity other than cpu / memory / pods: ephemeral-storage
 * (bytes) or a scalar resource (extended "vendor.example/x", hugepages-*,
 * attachable-volumes-*, kubernetes.io/-prefixed), as Quantity.Value().  Other
 * names are ignored, as upstream's framework.Resource ignores them. */
typedef struct {
  const char *name;
  int64_t value;
} ks_resource;

/* One name of a status.images entry with the entry's sizeBytes (an entry with
 * several names appears once per name). */
typedef struct {
  const char *name;
  int64_t size_bytes;
} ks_image;

/* v1.Node (name, labels, spec.taints, spec.unschedulable, status.allocatable,
 * status.images).  images: every name of every status.images entry; upstream's
 * cache keys ImageStates by those names (internal/cache/cache.go
 * #addNodeImageStates: the size is the first reporting node's, the node count
 * the number of nodes reporting the name). */
typedef struct {
  const char *name;
  int64_t alloc_milli_cpu;
  int64_t alloc_memory;
  int64_t alloc_pods;
  const ks_label *labels;
  const ks_taint *taints;
  uint32_t n_labels;
  uint32_t n_taints;
  uint32_t unschedulable;
  uint32_t n_images;
  const ks_image *images;
  const ks_resource *extended;  /* status.allocatable beyond cpu / memory / pods */
  uint32_t n_extended;
  uint32_t _pad;
} ks_node;

/* One container's resources.requests.  A resource that is ABSENT from the
 * requests map is distinguished from an explicit 0 (upstream
 * resourcehelper.PodRequests NonMissingContainerRequests semantics). */
enum { KS_REQ_HAS_CPU = 1u, KS_REQ_HAS_MEMORY = 2u, KS_REQ_HAS_OTHER = 4u };
typedef struct {
  int64_t milli_cpu;
  int64_t memory;
  uint32_t flags;          /* KS_REQ_* presence bits; HAS_OTHER = a request the caller cannot
                              express in `extended` (refused) */
  uint32_t restart_always; /* init containers only: restartPolicy: Always (sidecar) */
  const char *image;       /* container image (NULL / "" = none): ImageLocality */
  const ks_resource *extended;  /* requests beyond cpu / memory (ephemeral-storage, scalar) */
  uint32_t n_extended;
  uint32_t _pad;
} ks_container;

/* v1.NodeSelectorOperator */
enum {
  KS_OP_IN = 0,
  KS_OP_NOT_IN = 1,
  KS_OP_EXISTS = 2,
  KS_OP_DOES_NOT_EXIST = 3,
  KS_OP_GT = 4,
  KS_OP_LT = 5,
  KS_OP_INVALID = 6
};

typedef struct {
  const char *key;
  const char *const *values;
  uint32_t n_values;
  int32_t op; /* KS_OP_* */
} ks_requirement;

typedef struct {
  const ks_requirement *match_expressions;
  const ks_requirement *match_fields;
  uint32_t n_expressions;
  uint32_t n_fields;
} ks_term;

typedef struct {
  ks_term preference;
  int32_t weight;
  int32_t _pad;
} ks_preferred_term;

/* metav1.LabelSelector (labels.Selector after LabelSelectorAsSelector): every
 * match_labels pair and every expression (KS_OP_IN / NOT_IN / EXISTS /
 * DOES_NOT_EXIST) must hold.  is_nil = 1: the selector field is nil, which
 * selects no pod. */
typedef struct {
  const ks_label *match_labels;
  const ks_requirement *match_expressions;
  uint32_t n_match_labels;
  uint32_t n_match_expressions;
  uint32_t is_nil;
  uint32_t _pad;
} ks_label_selector;

/* v1.UnsatisfiableConstraintAction and v1.NodeInclusionPolicy */
enum { KS_DO_NOT_SCHEDULE = 0, KS_SCHEDULE_ANYWAY = 1 };
enum { KS_INCLUSION_DEFAULT = 0 /* field nil */, KS_INCLUSION_HONOR = 1, KS_INCLUSION_IGNORE = 2 };

/* v1.TopologySpreadConstraint (PodTopologySpread plugin, upstream
 * pkg/scheduler/framework/plugins/podtopologyspread).  Defaults of nil
 * fields as upstream's filterTopologySpreadConstraints: min_domains 0 = 1,
 * node_affinity_policy Honor, node_taints_policy Ignore.  match_label_keys
 * are merged into the selector with the incoming pod's values
 * (MatchLabelKeysInPodTopologySpread, on by default in v1.31). */
typedef struct {
  const char *topology_key;
  ks_label_selector selector;
  const char *const *match_label_keys;
  uint32_t n_match_label_keys;
  int32_t max_skew;
  int32_t when_unsatisfiable;   /* KS_DO_NOT_SCHEDULE / KS_SCHEDULE_ANYWAY   */
  int32_t min_domains;          /* 0 = nil                                   */
  int32_t node_affinity_policy; /* KS_INCLUSION_*                            */
  int32_t node_taints_policy;   /* KS_INCLUSION_*                            */
} ks_spread_constraint;

/* v1.PodAffinityTerm / WeightedPodAffinityTerm (InterPodAffinity plugin,
 * upstream pkg/scheduler/framework/plugins/interpodaffinity).  namespaces
 * empty and namespace_selector nil = the pod's own namespace.  A
 * namespace_selector is matched against the labels of a pod's namespace,
 * which every ks_pod carries (namespace_labels).  matchLabelKeys /
 * mismatchLabelKeys are merged into labelSelector by the apiserver (v1.31). */
enum {
  KS_POD_AFFINITY_REQUIRED = 0,       /* podAffinity.requiredDuringScheduling...      */
  KS_POD_ANTI_AFFINITY_REQUIRED = 1,  /* podAntiAffinity.requiredDuringScheduling...  */
  KS_POD_AFFINITY_PREFERRED = 2,      /* podAffinity.preferredDuringScheduling...     */
  KS_POD_ANTI_AFFINITY_PREFERRED = 3  /* podAntiAffinity.preferredDuringScheduling... */
};
typedef struct {
  ks_label_selector selector;            /* labelSelector (is_nil: matches no pod)  */
  ks_label_selector namespace_selector;  /* is_nil: the field is not set            */
  const char *const *namespaces;
  const char *topology_key;
  uint32_t n_namespaces;
  int32_t kind;                          /* KS_POD_*AFFINITY_*                      */
  int32_t weight;                        /* preferred terms: 1..100                 */
  int32_t _pad;
} ks_pod_affinity_term;

/* Pod features whose plugins ksched does not model.
 * The caller sets the bit when the pod carries the feature; a pod with any
 * bit set is refused with KS_ERR_UNSUPPORTED (ks_pods_check names it) and
 * the shim falls back to upstream schedulePod for it.  The
 * default profile's plugins that read them: */
enum {
  KS_UNMODELLED_HOST_PORTS = 1u,       /* NodePorts: a container port with hostPort != 0             */
  KS_UNMODELLED_TOPOLOGY_SPREAD = 2u,  /* PodTopologySpread constraints the caller could not express
                                          as ks_pod.spread (ksched models the plugin itself: pass the
                                          pod's constraints, or its system-default ones, there)      */
  KS_UNMODELLED_POD_AFFINITY = 4u,     /* InterPodAffinity terms the caller could not express as
                                          ks_pod.affinity_terms.  On a pod bound through ks_pods_add /
                                          KS_EV_POD_ADD it makes every later batch refuse until that
                                          pod is removed (existing pods' terms filter and score the
                                          incoming pod)                                             */
  KS_UNMODELLED_VOLUMES = 8u,          /* VolumeBinding / VolumeRestrictions / VolumeZone /
                                          NodeVolumeLimits: PVC, ephemeral or CSI volumes           */
  KS_UNMODELLED_NOMINATED_NODE = 16u,  /* status.nominatedNodeName (evaluateNominatedNode)          */
  KS_UNMODELLED_RESOURCE_CLAIMS = 32u, /* DynamicResources: spec.resourceClaims                     */
  KS_UNMODELLED_ALL = 63u
};

/* v1.Pod restricted to scheduling-relevant fields. */
typedef struct {
  const char *ns;
  const char *name;
  const ks_container *containers;
  const ks_container *init_containers;
  const ks_toleration *tolerations;
  const ks_label *node_selector;          /* spec.nodeSelector                     */
  const ks_term *required_terms;          /* requiredDuringScheduling...NodeSelectorTerms */
  const ks_preferred_term *preferred;     /* preferredDuringScheduling...          */
  const char *node_name;                  /* spec.nodeName (NULL/"" = unset)       */
  int64_t overhead_milli_cpu;             /* spec.overhead (if has_overhead)       */
  int64_t overhead_memory;
  uint32_t n_containers;
  uint32_t n_init_containers;
  uint32_t n_tolerations;
  uint32_t n_node_selector;
  uint32_t n_required_terms;
  uint32_t has_required;  /* RequiredDuringSchedulingIgnoredDuringExecution != nil */
  uint32_t n_preferred;
  uint32_t has_preferred; /* PreferredDuringSchedulingIgnoredDuringExecution != nil */
  uint32_t has_overhead;
  uint32_t unmodelled;    /* KS_UNMODELLED_* bits */
  /* PodTopologySpread inputs.  labels / ns of a pod bound through ks_pods_add,
   * KS_EV_POD_ADD or a batch are what later pods' spread selectors count
   * (countPodsMatchSelector: same namespace, selector match).  spread holds
   * the pod's topologySpreadConstraints; when it has none and upstream's
   * system defaulting applies (the pod is selected by a Service or owned by a
   * ReplicaSet / StatefulSet / ReplicationController: helper.DefaultSelector
   * is non-empty), the caller passes the two system-default constraints
   * (kubernetes.io/hostname maxSkew 3, topology.kubernetes.io/zone maxSkew 5,
   * ScheduleAnyway, selector = DefaultSelector) and sets spread_defaulted = 1,
   * which makes PreScore keep nodes lacking a topology key
   * (requireAllTopologies = false). */
  const ks_label *labels;              /* metadata.labels */
  const ks_spread_constraint *spread;
  uint32_t n_labels;
  uint32_t n_spread;
  uint32_t spread_defaulted;
  uint32_t _pad2;
  /* InterPodAffinity: the pod's pod (anti-)affinity terms, and the labels of
   * its namespace (namespace selectors of other pods' terms match them). */
  const ks_pod_affinity_term *affinity_terms;
  const ks_label *namespace_labels;
  uint32_t n_affinity_terms;
  uint32_t n_namespace_labels;
} ks_pod;

/* ------------------------------------------------------------- outputs */
/* Filter plugins in default-profile order (v1.31 apis/config/v1 default plugins). */
enum {
  KS_PLUGIN_NODE_UNSCHEDULABLE = 0,
  KS_PLUGIN_NODE_NAME = 1,
  KS_PLUGIN_TAINT_TOLERATION = 2,
  KS_PLUGIN_NODE_AFFINITY = 3,
  KS_PLUGIN_NODE_RESOURCES_FIT = 4,
  KS_PLUGIN_POD_TOPOLOGY_SPREAD = 5,
  KS_PLUGIN_INTER_POD_AFFINITY = 6,
  KS_NUM_FILTER_PLUGINS = 7
};

enum {
  KS_POD_SCHEDULED = 0,     /* node_index valid                                  */
  KS_POD_UNSCHEDULABLE = 1, /* FitError: no feasible node; fail_counts = Diagnosis */
  KS_POD_ERROR = 2          /* framework Error status (e.g. preferred-term parse error) */
};

enum { KS_RESULT_SINGLE_FEASIBLE = 1u /* upstream returns without scoring */ };

/* fail_counts[KS_FAIL_PREFILTER_RESULT]: nodes outside NodeAffinity's
 * PreFilterResult (required terms that all name nodes by matchFields
 * metadata.name In), which upstream v1.31 records as
 * UnschedulableAndUnresolvable "node is filtered out by the prefilter result"
 * without running any Filter plugin on them (schedule_one.go#findNodesThatFitPod). */
enum { KS_FAIL_PREFILTER_RESULT = KS_NUM_FILTER_PLUGINS, KS_NUM_FAIL_COUNTS = KS_NUM_FILTER_PLUGINS + 1 };

/* ScheduleResult{SuggestedHost, EvaluatedNodes, FeasibleNodes} or FitError. */
typedef struct {
  int32_t node_index;     /* chosen node slot, -1 if none                        */
  int32_t status;         /* KS_POD_*                                            */
  int64_t total_score;    /* TotalScore of the chosen node (NodePluginScores)    */
  uint32_t feasible_nodes;
  uint32_t evaluated_nodes;
  uint32_t fail_counts[KS_NUM_FAIL_COUNTS]; /* nodes rejected first by each filter plugin, then
                                               nodes excluded by the PreFilterResult */
  uint32_t flags;         /* KS_RESULT_*                                         */
  uint32_t _pad;
} ks_result;

/* Per-node plugin scores of one pod (parity dump; NodePluginScores analogue). */
typedef struct {
  int32_t status;        /* -1 feasible, else KS_PLUGIN_* of the first failing filter, -2 empty slot */
  int32_t least_allocated;      /* NodeResourcesFit (LeastAllocated)     */
  int32_t balanced_allocation;  /* NodeResourcesBalancedAllocation       */
  int32_t taint_raw;            /* TaintToleration raw (before normalize) */
  int32_t taint_score;          /* TaintToleration normalized            */
  int32_t affinity_raw;         /* NodeAffinity raw                      */
  int32_t affinity_score;       /* NodeAffinity normalized               */
  int32_t image_locality;       /* ImageLocality (0: nodes report no images) */
  int32_t spread_raw;           /* PodTopologySpread raw (0 when its PreScore skips) */
  int32_t spread_score;         /* PodTopologySpread normalized          */
  int32_t affinity_pod_raw;     /* InterPodAffinity raw (0 when its PreScore skips) */
  int32_t affinity_pod_score;   /* InterPodAffinity normalized           */
  int64_t total_score;          /* Σ weight × score over non-skipped plugins */
} ks_node_score;

/* Node resource state (NodeInfo.Requested / NonZeroRequested / len(Pods)). */
typedef struct {
  int64_t alloc_milli_cpu, alloc_memory;
  int64_t req_milli_cpu, req_memory;
  int64_t nonzero_milli_cpu, nonzero_memory;
  int32_t alloc_pods;
  int32_t pod_count; /* -1 for an empty slot */
} ks_node_state;

/* ------------------------------------------------------------- context */
typedef struct {
  int32_t device;            /* HIP device ordinal                               */
  uint32_t node_capacity;    /* node slots (index space)                         */
  uint32_t pods_per_round;   /* P: pods evaluated per sweep (0 = default 256)    */
  uint32_t topk;             /* K: candidates kept per pod (0 = P)               */
  uint32_t nodes_per_lane;   /* nodes held per GPU lane in the sweep (0 = 4)     */
  uint32_t world_size;       /* GPUs sharding the node index space (1 = no RCCL) */
  uint32_t rank;             /* this GPU's shard                                 */
  uint32_t virtual_shards;   /* >1: emulate that many shards on this one device  */
  /* Score plugin weights (default profile: 1, 1, 3, 2, 1). */
  int32_t weight_fit;        /* NodeResourcesFit                                */
  int32_t weight_balanced;   /* NodeResourcesBalancedAllocation                 */
  int32_t weight_taint;      /* TaintToleration                                 */
  int32_t weight_affinity;   /* NodeAffinity                                    */
  int32_t weight_image;      /* ImageLocality                                   */
  /* (weight_topology_spread: after percentage_of_nodes_to_score) */
  /* KubeSchedulerProfile.percentageOfNodesToScore, 0..100.  100 (the default
   * here and the reference's dist-scheduler/deployment.yaml:95) scores every
   * node.  Below 100 (0 = upstream's adaptive 50 - N/125; the published run's
   * 5 at terraform/kubernetes/dist-scheduler.tf:562) each pod visits the node
   * list (present nodes in slot order) from nextStartNodeIndex and stops at
   * numFeasibleNodesToFind feasible nodes, as upstream's findNodesThatPassFilters
   * does with one worker (schedule_one.go; with more workers upstream's set
   * depends on goroutine timing); nextStartNodeIndex advances by the nodes
   * processed (ks_next_start_index).  Every pod then takes the one-pod chain.
   * Below 100 with world_size > 1 or virtual_shards > 1: KS_ERR_UNSUPPORTED. */
  int32_t percentage_of_nodes_to_score;
  int32_t weight_topology_spread; /* PodTopologySpread (default profile: 2)     */
  int32_t weight_inter_pod_affinity; /* InterPodAffinity (default profile: 2)    */
  int32_t hard_pod_affinity_weight;  /* InterPodAffinityArgs.hardPodAffinityWeight (1) */
  /* Execution options (ks_config_default sets each default).  None of them
   * changes a result -- every combination schedules exactly as upstream's
   * sequential loop does (the tests pin each one); they choose how the device
   * gets there.  ks_open reads no environment variable that selects any of
   * this. */
  uint32_t resolve_mode;          /* in-order commit of every round (resource-only and label / taint):
                                     KS_RESOLVE_AUTO (default: the parallel proposal / verify commit,
                                     handing rounds where pods pile onto the same nodes to the serial
                                     commit in the same launch), KS_RESOLVE_SERIAL, KS_RESOLVE_PARALLEL
                                      */
  uint32_t resolve_par_max_passes;  /* AUTO: a round needing more chunk passes than this (32, 1..257),
                                       or on pace (after 4) to need more, goes whole to the serial
                                       commit, with ...                                                */
  uint32_t resolve_serial_rounds;   /* ... this many following rounds (4, <= 2^20; doubled per
                                       consecutive hand-over, up to 256 rounds or 16x)                 */
  uint32_t dedup_identical_pods;  /* 1 (default): a round's byte-identical pods are swept once (§5.5) */
  uint32_t early_fix;             /* 1 (default): on one rank the normaliser FIX re-sweep follows the
                                     sweep on its stream (§5.2); 0: behind the merge (multi-rank order) */
  uint32_t tuple_guess;           /* 1 (default): normaliser maxima guessed from node label / taint
                                     tuples; 0: from the pod alone (more FIX re-sweeps)               */
  uint32_t ext_nodes_per_lane;    /* nodes per lane of the label / taint sweep: 2 (default), 4 or 8  */
  uint32_t sweep_pairs;           /* (block, pod group) pairs of a resource-only sweep (4096)        */
  uint32_t sweep_pairs_ext;       /* ... of a label / taint sweep (16384)                            */
  uint32_t resolve_cus;           /* CUs reserved for the resolve stream (1; 0: no CU masks)         */
  uint32_t side_cus;              /* CUs the sweep stream leaves to the side stream (0)              */
  uint32_t value_sync;            /* 1 (default): cross-stream hand-offs by stream wait-value packets;
                                     0: by events (profilers that serialise dispatches)              */
  uint32_t sync_timeout_ms;       /* bound on every host wait for device work (60000), see
                                     ks_set_sync_timeout                                            */
  uint32_t spread_replica_runs;   /* 1 (default): runs of >= 4 identical one-pod-path pods with at
                                     most a kubernetes.io/hostname ScheduleAnyway constraint and one on
                                     another key (ScheduleAnyway, or since round 6 DoNotSchedule) --
                                     deployment replicas under the system defaults or their own
                                     zone constraints -- are scheduled by one filter pass and one
                                     workgroup per run; 0: the per-pod chain.
                                     Off when percentage_of_nodes_to_score < 100            */
} ks_config;

enum { KS_RESOLVE_AUTO = 0, KS_RESOLVE_SERIAL = 1, KS_RESOLVE_PARALLEL = 2 };

typedef struct ks_ctx ks_ctx;
typedef struct ks_batch ks_batch;

/* Fill *cfg with the default-profile configuration. */
void ks_config_default(ks_config *cfg);

/* Scheduler construction (replaces scheduler.NewN's per-shard NodeInfo cache,
 * dist-scheduler/cmd/dist-scheduler/scheduler.go:281-300). */
ks_status ks_open(const ks_config *cfg, ks_ctx **out);
void ks_close(ks_ctx *ctx);
const char *ks_last_error(const ks_ctx *ctx);
int32_t ks_abi_version(void);

/* Node cache events (filtered node informer, scheduler.go:200-219 ->
 * upstream internal/cache AddNode/UpdateNode/RemoveNode).  Upsert of an
 * existing slot keeps its Requested/NonZeroRequested/pod count. */
ks_status ks_nodes_upsert(ks_ctx *ctx, const ks_node *nodes, const uint32_t *slots, uint32_t n);
/* Per-item form: each item is validated on its own (slot, name, cpu / memory
 * allocatable below 2^44 -- LeastAllocated's exact-floor bound, DESIGN.md §4 --
 * non-negative extended / ephemeral-storage allocatable, any int64 size) and
 * status[i] = KS_OK or that item's error; the valid items are applied as one
 * ks_nodes_upsert.  Returns KS_OK when every item was applied, else the first
 * failing item's status (ks_last_error names it).  ks_nodes_upsert itself
 * applies nothing when any item is invalid. */
ks_status ks_nodes_upsert_each(ks_ctx *ctx, const ks_node *nodes, const uint32_t *slots, uint32_t n,
                               ks_status *status);
ks_status ks_nodes_delete(ks_ctx *ctx, const uint32_t *slots, uint32_t n);

/* Generation-based snapshot update (upstream Cache.UpdateSnapshot,
 * pkg/scheduler/internal/cache/cache.go; the reference's shards call it once
 * per ScheduleOne through the fork, scheduler.go:543): the cache's NodeInfos
 * -- all of them, or any superset of those changed since the last call --
 * each with its NodeInfo.Generation.  An item whose generation is not above
 * the last one applied to its slot is already in the snapshot and skipped
 * (replayed or reordered deliveries are harmless); of several items for one
 * slot in a call the highest generation wins.  deleted = 1 is RemoveNode
 * (the node leaves with its pods; skipped if the slot is empty), otherwise
 * AddNode / UpdateNode of `node` (the slot's pods stay: pods arrive through
 * ks_pods_add / ks_pods_remove / ks_events_apply).  Deletions are applied
 * before upserts, so a name may move to another slot within one call.
 * *generation receives the highest generation applied so far (the snapshot's
 * generation), *applied the number of items applied (either may be null). */
typedef struct {
  uint32_t slot;
  uint32_t deleted;
  int64_t generation;
  const ks_node *node; /* deleted = 0 */
} ks_node_info;
ks_status ks_snapshot_update(ks_ctx *ctx, const ks_node_info *items, uint32_t n, int64_t *generation,
                             uint32_t *applied);

/* Pod cache events: NodeInfo.AddPod (bind / assume) and RemovePod (delete). */
ks_status ks_pods_add(ks_ctx *ctx, const ks_pod *pods, const uint32_t *slots, uint32_t n);
ks_status ks_pods_remove(ks_ctx *ctx, const ks_pod *pods, const uint32_t *slots, uint32_t n);

/* One informer event of an ordered log (the delta feed of SURVEY §8(f) F2:
 * upstream internal/cache AddPod / RemovePod / AddNode / UpdateNode /
 * RemoveNode as the reference's informers deliver them, scheduler.go:200-228).
 * kind selects the payload: pod (KS_EV_POD_*) or node (KS_EV_NODE_UPSERT);
 * slot is the node slot the event applies to. */
enum {
  KS_EV_POD_ADD = 0,     /* NodeInfo.AddPod: a pod bound (or assumed) on slot */
  KS_EV_POD_REMOVE = 1,  /* NodeInfo.RemovePod: a pod deleted from slot */
  KS_EV_NODE_UPSERT = 2, /* AddNode / UpdateNode (keeps the slot's pods) */
  KS_EV_NODE_DELETE = 3, /* RemoveNode (its pods leave with it) */
};
typedef struct {
  int32_t kind;
  uint32_t slot;
  const ks_pod *pod;   /* KS_EV_POD_ADD / KS_EV_POD_REMOVE */
  const ks_node *node; /* KS_EV_NODE_UPSERT */
} ks_event;

/* Apply an event log in order: the state afterwards equals applying each
 * event alone, one after the other.  Consecutive events of one kind go to the
 * device as one batch (pod deltas commute; upserts of one slot keep the last
 * state).  On error the events before the failing run are applied. */
ks_status ks_events_apply(ks_ctx *ctx, const ks_event *events, uint32_t n);

/* schedulePod for a stream of pods, in order: each pod is scheduled against
 * the cache as left by the previous one (AssumePod commit), exactly as
 * sequential ScheduleOne calls.  out[i] receives pod i's result. */
ks_status ks_schedule(ks_ctx *ctx, const ks_pod *pods, uint32_t n, ks_result *out);

/* Per-pod admission check without scheduling: status[i] = KS_OK, or the
 * ks_status ks_batch_prepare would fail pod i with (KS_ERR_UNSUPPORTED for a
 * KS_UNMODELLED_* feature, an unsupported resource or a container image some
 * node reports; KS_ERR_RANGE; KS_ERR_CAPACITY).  Returns KS_OK when every pod
 * passes, else the first failing pod's status (ks_last_error names it).  The
 * shim splits a batch at refused pods and hands those to upstream schedulePod. */
ks_status ks_pods_check(ks_ctx *ctx, const ks_pod *pods, uint32_t n, ks_status *status);

/* Split form of ks_schedule: compile + upload once (prepare), then run with
 * all inputs resident in HBM (the timed hot path), then fetch results.
 * Batch buffers come from a per-context pool (no device allocation per batch
 * once the pool holds a batch of that size; ks_batch_free returns them). */
ks_status ks_batch_prepare(ks_ctx *ctx, const ks_pod *pods, uint32_t n, ks_batch **out);
ks_status ks_batch_run(ks_ctx *ctx, ks_batch *batch);
ks_status ks_batch_results(ks_ctx *ctx, const ks_batch *batch, ks_result *out);
void ks_batch_free(ks_ctx *ctx, ks_batch *batch);

/* Asynchronous run: ks_batch_submit queues a prepared batch on the context's
 * worker thread (batches run in submission order, each against the cache the
 * previous one left) and returns at once; ks_batch_wait blocks until that
 * batch has run and returns its run status.  While batches are in flight the
 * caller may ks_batch_prepare (compile + upload on a stream of its own, so
 * compiling batch k+1 overlaps running batch k), ks_batch_results of a waited
 * batch, and ks_batch_free; every other call on the context first waits for
 * all submitted batches. */
ks_status ks_batch_submit(ks_ctx *ctx, ks_batch *batch);
ks_status ks_batch_wait(ks_ctx *ctx, ks_batch *batch);

/* Per-plugin scores of `pod` on every node slot against the current cache
 * (out has node_capacity entries).  Parity dump of NodePluginScores. */
ks_status ks_plugin_scores(ks_ctx *ctx, const ks_pod *pod, ks_node_score *out);

/* Read back node resource state. */
ks_status ks_node_states(ks_ctx *ctx, const uint32_t *slots, uint32_t n, ks_node_state *out);

/* Cross-GPU candidate gather over RCCL (replaces CollectScore fan-in,
 * dist-scheduler/cmd/dist-scheduler/grpc_server.go:116-127 and
 * pkg/scoreevaluator/scoreevaluator.go:45-126, for co-located shards). */
#define KS_COMM_ID_BYTES 128
ks_status ks_comm_unique_id(uint8_t out[KS_COMM_ID_BYTES]);
ks_status ks_comm_init(ks_ctx *ctx, const uint8_t id[KS_COMM_ID_BYTES]);
/* In-process communicator: ctxs[r] (world_size n, rank r) are contexts of
 * this process -- one device or several -- each then driven by its own host
 * thread; the collectives above run as device copies ordered by stream events
 * instead of RCCL (which refuses two ranks on one GPU).  It exists so the
 * multi-rank path can be tested on one GPU; a deployment uses ks_comm_init. */
ks_status ks_comm_init_local(ks_ctx *const *ctxs, uint32_t n);
/* Element-wise max of n doubles over all ranks (in place); also a barrier. */
ks_status ks_comm_allreduce_max(ks_ctx *ctx, double *values, uint32_t n);

/* Parity dump of the round kernels' own output: the merged candidate record
 * of pod `pod_in_round` of the LAST batch's first round (read after
 * ks_schedule / ks_batch_run returns; valid while that round resolved every
 * pod it swept, i.e. for batches of at most pods_per_round pods): out[0] the
 * bound (>= every unlisted feasible packed key), out[1] the key count, then
 * the packed keys ((TotalScore + 1) << 32 | ~slot, descending) as the sweep
 * computed them against the round-start state; out has room for 2 + topk
 * words.  Lets tests compare the fused sweep's per-node scores with the
 * oracle for every listed node, not only the chosen one. */
ks_status ks_debug_round_record(ks_ctx *ctx, uint32_t pod_in_round, uint64_t *out);

/* Counters for measurement. */
typedef struct {
  uint64_t rounds;          /* sweep rounds issued                         */
  uint64_t pods_resolved;
  uint64_t pods_scheduled;
  uint64_t sweep_launches;  /* launches of the sweep kernel (timed)        */
  double sweep_ms;          /* Σ device time of sweep launches (HIP events) */
  uint64_t sweep_evals;     /* Σ (pod, node) evaluations by timed sweeps   */
  double resolve_ms;        /* Σ device time of resolve launches           */
  uint64_t resolve_launches;
  double spread_ms;         /* Σ device time of timed spread-path pods (whole kernel chain) */
  uint64_t spread_pods_timed;
  uint64_t spread_pods;     /* pods scheduled by the spread path           */
  uint64_t replica_runs;    /* replica runs of the spread path (spread_replica_runs) */
  uint64_t replica_pods;    /* pods they scheduled (counted in spread_pods too)      */
  double replica_ms;        /* Σ device time of timed replica runs (in spread_ms too) */
  uint64_t classes_inflight; /* selector classes ks_batch_prepare created while batches ran (no drain) */
  uint64_t late_class_pods;  /* pods those batches bound that a new class selects, counted at their end */
} ks_stats;
ks_status ks_get_stats(ks_ctx *ctx, ks_stats *out);
ks_status ks_reset_stats(ks_ctx *ctx);
/* Raw counters: [0] rounds [1] pods resolved [2] pods swept
 * [3] speculated rounds wasted [4] pods re-swept because their guessed
 * normalising maxima were wrong, [5] label-dictionary reclaims, [6] taint
 * dictionary rebuilds, [7] identical pods not swept, [12] passes of the
 * parallel commit, [13] rounds it resolved, [14] of those it cut short and
 * handed over to the serial kernel (AUTO), [15] of those resolved in one step
 * (one class of identical request-less pods).  (The instrumented stamps builds,
 * k8s-1m_amd/csrc/ksched_instr.hpp, put phase cycle sums in [8..15].) */
ks_status ks_debug_counters(ks_ctx *ctx, uint64_t out[16]);
/* Diagnostics of the parallel commit: with the profile
 * on, every round accumulates s_memtime cycles per phase: out[0] stage,
 * [1] gather barrier, [2] proposals, [3] wave 0's row DMA issue, [4] chunk
 * pairs, [5] its DMA wait, [6] decide + commit, [7] Rpre updates, [8]
 * epilogue, [12] wave 0's wait for its prefetched windows, [13] its scalar
 * state and M probes, [14] its window scans; out[9] counts the rounds
 * profiled, [10] dirty Rpre recomputes, [11] extra list windows. */
ks_status ks_debug_set_profile(ks_ctx *ctx, int32_t on);
ks_status ks_debug_resolve_profile(ks_ctx *ctx, uint64_t out[16]);
/* Round marks of a finished batch (diagnostics for tests that place parity
 * checks where the round machinery changed course): out[i] for pod i of the
 * batch, bits KS_MARK_*.  Valid after ks_batch_run / ks_batch_wait. */
#define KS_MARK_FIX 1u          /* re-swept with the measured normaliser maxima  */
#define KS_MARK_ROUND_START 2u  /* first pod of a resolved round                 */
#define KS_MARK_AFTER_WASTE 4u  /* ... whose previous speculated round was wasted */
ks_status ks_batch_marks(ks_ctx *ctx, const ks_batch *batch, uint8_t *out);
/* Device-stall guard.  Every wait of the library on the device is bounded
 * (ks_config.sync_timeout_ms at ks_open, default 60000, or this call).  A stream
 * that has not finished in time makes the call return KS_ERR_DEVICE with
 * ks_last_error naming the unfinished streams, the hand-off flags' device
 * values and the round numbers they were expected to reach; the context is
 * then wedged: every later call that waits on the device fails at once, and
 * ks_close frees nothing the device may still use. */
ks_status ks_set_sync_timeout(ks_ctx *ctx, uint32_t ms);
/* Fault injection for that guard (tests): the next scheduling round holds
 * back the signal of cross-stream hand-off flag `flag` (0 sweep done, 1 side
 * stream done, 2 round resolved, 3 FIX sweep done) by `usec` microseconds of
 * bounded device-side waiting, then signals as usual. */
ks_status ks_debug_stall(ks_ctx *ctx, uint32_t flag, uint32_t usec);
/* Scheduler.nextStartNodeIndex (percentageOfNodesToScore < 100; 0 otherwise),
 * after the submitted batches. */
ks_status ks_next_start_index(ks_ctx *ctx, uint64_t *out);
/* Batch runs the context has started (the worker took their selector-class
 * masks and table view); returns at once, without waiting for submitted
 * batches -- tests order a ks_batch_prepare after a submitted run's start. */
ks_status ks_debug_runs_started(ks_ctx *ctx, uint64_t *out);
/* 1 = time sweep / resolve launches with HIP events (every KS_TIMING_EVERY-th
 * round, default 8; sweep_evals counts the timed launches' share), 0 = off. */
ks_status ks_set_timing(ks_ctx *ctx, int32_t enabled);

#ifdef __cplusplus
}
#endif

#endif /* KSCHED_H */
