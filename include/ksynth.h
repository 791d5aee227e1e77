/*
 * ksynth.h — seeded synthetic kwok-shaped clusters and pod streams
 * (libksynth.so).  Workload generator only: it is not on the hot path and
 * computes no scheduling result.
 *
 * Shapes follow the reference's own generators:
 *   nodes: kwok/make_nodes/main.go:116-182 (32 CPU, 256Gi, 32 pods,
 *          taint kwok.x-k8s.io/node=fake:NoSchedule, kwok labels)
 *   pods:  kwok/make_pods/main.go:119-172 (3 tolerations, busybox container)
 * with the request / heterogeneity / label distributions of SURVEY.md §8(d)
 * (configs C1..C5 of BASELINE.json).
 */
#ifndef KSYNTH_H
#define KSYNTH_H

#include <stdint.h>
#include "ksched.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
  KSYNTH_KWOK = 1,   /* C1: homogeneous kwok nodes                        */
  KSYNTH_HETERO = 2, /* C2/C3: heterogeneous shapes (+ prefill separately) */
  KSYNTH_LABELED = 4, /* C4: C2 shapes + zone/instance-type/pool/feature/gpu labels and taints */
  KSYNTH_ZONED = 8    /* C2 shapes + topology.kubernetes.io/zone (32 zones); prefill pods carry
                         app labels (PodTopologySpread workloads) */
};

typedef struct ksynth ksynth; /* owns every array and string it returns */

/* Nodes 0..n-1 of cluster `kind` (slot i = node i). */
ksynth *ksynth_nodes(int32_t kind, uint32_t n, uint64_t seed);
/* Pod stream of `kind`: KSYNTH_KWOK/HETERO = resource-only pods,
 * KSYNTH_LABELED = pods with selectors / affinity / tolerations (C4). */
ksynth *ksynth_pods(int32_t kind, uint32_t n, uint64_t seed);
/* Prefill for an n-node cluster of `kind`: pods bound to nodes so that node
 * i carries a seeded fraction in [0, max_fill) of its CPU.  Pods come with
 * their target slot (ksynth_slots). */
ksynth *ksynth_prefill(int32_t kind, uint32_t n_nodes, uint64_t nodes_seed, uint64_t seed,
                       double max_fill);
/* Pods that request nothing (kwok/make_pods/main.go:138-148 best-effort busybox). */
ksynth *ksynth_besteffort_pods(uint32_t n);
/* Deployment-shaped pods with topology spread constraints: pod j belongs to
 * app-k (k drawn from n_apps), labels {app: app-k}, C1 requests, kwok
 * tolerations; half carry PodTopologySpread's system defaults (hostname
 * maxSkew 3 + zone maxSkew 5, ScheduleAnyway, spread_defaulted), half their
 * own [zone maxSkew 1 DoNotSchedule, hostname maxSkew 1 ScheduleAnyway], all
 * selecting app=app-k. */
ksynth *ksynth_spread_pods(uint32_t n, uint32_t n_apps, uint64_t seed);
/* Deployment replicas under PodTopologySpread's system defaults: pod j is
 * replica j % replicas of deployment deploy-(j / replicas); a deployment's
 * pods are identical (labels {app: deploy-k}, one C1 request draw per
 * deployment, kwok tolerations, hostname maxSkew 3 + zone maxSkew 5
 * ScheduleAnyway selecting app=deploy-k, spread_defaulted). */
ksynth *ksynth_deploy_pods(uint32_t n, uint32_t replicas, uint64_t seed);
// The same deployments under their own constraints: zone maxSkew 1
// DoNotSchedule + hostname maxSkew 1 ScheduleAnyway.
ksynth *ksynth_deploy_dns_pods(uint32_t n, uint32_t replicas, uint64_t seed);
// InterPodAffinity deployment pods (ksynth.cpp): alternately required hostname
// anti-affinity + preferred zone affinity to the own app, and preferred
// hostname anti-affinity + required zone affinity to the next app.
ksynth *ksynth_affinity_pods(uint32_t n, uint32_t n_apps, uint64_t seed);

const ks_node *ksynth_node_array(const ksynth *s, uint32_t *n);
const ks_pod *ksynth_pod_array(const ksynth *s, uint32_t *n);
const uint32_t *ksynth_slots(const ksynth *s, uint32_t *n);
void ksynth_free(ksynth *s);

/* FNV-1a 64 over a byte range (fixture digests). */
uint64_t ksynth_fnv64(const void *data, uint64_t len, uint64_t seed);

#ifdef __cplusplus
}
#endif

#endif
