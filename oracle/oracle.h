/*
 * oracle.h — CPU restatement of the dist-scheduler shard hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so, and only as the checker
 * (or as the timed CPU baseline).  The product path (libksched.so) never
 * links, loads or calls it.
 *
 * PARITY UNPINNED: the reference's implementation of this path lives in the
 * forked kube-scheduler submodule (dist-scheduler/.gitmodules:1-3,
 * dist-scheduler/go.mod:133,138), which is empty in /root/reference, and no Go
 * toolchain exists here; the reference holds no test or fixture for this path
 * (SURVEY.md §8(c)).  The oracle restates upstream k8s.io/kubernetes v1.31.3
 * and k8s.io/component-helpers v0.31.3 / k8s.io/api v0.31.3 semantics
 * (SURVEY.md Appendix A); its arithmetic is pinned only by the hand-derived
 * known-answer tests of SURVEY.md Appendix B (tests/test_oracle_kat.py).
 */
#ifndef KSCHED_ORACLE_H
#define KSCHED_ORACLE_H

#include <stdint.h>
#include "ksched.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle oracle;

oracle *oracle_new(uint32_t node_capacity, int32_t w_fit, int32_t w_balanced, int32_t w_taint,
                   int32_t w_affinity, int32_t w_image);
void oracle_free(oracle *o);
/* Worker threads for the per-pod node loop (parallelize.Until chunking). */
void oracle_set_threads(oracle *o, int32_t threads);
/* PodTopologySpread score weight (default 2, the default profile's). */
void oracle_set_weight_spread(oracle *o, int32_t w);
/* InterPodAffinity score weight (2) and hardPodAffinityWeight (1). */
void oracle_set_weight_inter_pod_affinity(oracle *o, int32_t w, int32_t hard);
/* KubeSchedulerProfile.percentageOfNodesToScore (default 100; 0 = adaptive).
 * Below 100 each pod visits the node list from nextStartNodeIndex and stops
 * at numFeasibleNodesToFind feasible nodes (schedule_one.go; see oracle.cpp
 * window()).  Resets nextStartNodeIndex to 0. */
void oracle_set_percentage(oracle *o, int32_t pct);
uint64_t oracle_next_start(const oracle *o); /* nextStartNodeIndex */
/* schedule_one.go#numFeasibleNodesToFind */
int64_t oracle_num_feasible_nodes_to_find(int32_t pct, int64_t num_all_nodes);

int32_t oracle_nodes_upsert(oracle *o, const ks_node *nodes, const uint32_t *slots, uint32_t n);
int32_t oracle_nodes_delete(oracle *o, const uint32_t *slots, uint32_t n);
int32_t oracle_pods_add(oracle *o, const ks_pod *pods, const uint32_t *slots, uint32_t n);
int32_t oracle_pods_remove(oracle *o, const ks_pod *pods, const uint32_t *slots, uint32_t n);

/* Sequential schedulePod + assume for each pod in order. */
int32_t oracle_schedule(oracle *o, const ks_pod *pods, uint32_t n, ks_result *out);
/* Per-plugin scores of one pod on every slot against the current cache. */
int32_t oracle_plugin_scores(oracle *o, const ks_pod *pod, ks_node_score *out);
int32_t oracle_node_states(oracle *o, const uint32_t *slots, uint32_t n, ks_node_state *out);

/* Shard decomposition helpers (multi-rank protocol emulation on CPU).
 * prescore over slots [lo, hi): feasible count, per-plugin first-failure
 * counts and the normalising plugins' (max raw, count at max) over feasible
 * nodes.  best: highest packed key ((TotalScore+1)<<32 | ~slot) over the
 * shard's feasible nodes given the global maxima.  commit: AssumePod. */
typedef struct {
  uint32_t feasible;
  uint32_t fail_counts[KS_NUM_FAIL_COUNTS]; /* + KS_FAIL_PREFILTER_RESULT */
  int64_t taint_max, affinity_max;
  uint32_t taint_count, affinity_count;
  int32_t error; /* 1 if the pod's PreScore would fail (preferred-term parse error) */
  int32_t _pad;
} oracle_shard_prescore;
int32_t oracle_shard_prescore_run(oracle *o, const ks_pod *pod, uint32_t lo, uint32_t hi,
                                  oracle_shard_prescore *out);
uint64_t oracle_shard_best(oracle *o, const ks_pod *pod, uint32_t lo, uint32_t hi,
                           int64_t taint_max, int64_t affinity_max);
int32_t oracle_commit(oracle *o, const ks_pod *pod, uint32_t slot);

/* Scalar plugin arithmetic for known-answer tests. */
double oracle_go_log(double x); /* Go math.Log (topologyNormalizingWeight) */
int64_t oracle_least_allocated(int64_t alloc_cpu, int64_t alloc_mem, int64_t node_nz_cpu,
                               int64_t node_nz_mem, int64_t pod_nz_cpu, int64_t pod_nz_mem);
int64_t oracle_balanced_allocation(int64_t alloc_cpu, int64_t alloc_mem, int64_t node_req_cpu,
                                   int64_t node_req_mem, int64_t pod_req_cpu, int64_t pod_req_mem);
/* PodRequests: out[0..3] = req cpu, req mem, non-zero cpu, non-zero mem. */
int32_t oracle_pod_requests(const ks_pod *pod, int64_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
