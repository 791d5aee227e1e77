/* ksgather.h — cross-host candidate gather.
 *
 * Within a host the shards of one node's GPUs are merged by RCCL (ksched.h
 * ks_comm_*): the host's result for a pod is ONE (node, TotalScore) pair.
 * Across hosts the reference's gRPC contract stays: every member sends its
 * int32 score to the pod's gatherer (PodService.CollectScore,
 * dist-scheduler/proto/pod.proto:25-35, grpc_server.go:116-127), which records
 * the scores and answers each sender whether its node won.  This library is
 * the gatherer's state machine and the member-side routing, as C ABI:
 *
 *   ksg_record_and_wait  ScoreEvaluator.RecordAndWait + fire
 *                        (pkg/scoreevaluator/scoreevaluator.go:45-126)
 *   ksg_target_index     SchedulerSet.GetTargetForScoring: FNV-1 32 of
 *                        "namespace/name" modulo the sorted member list
 *                        (pkg/schedulerset/schedulerset.go:107-143)
 *
 * The wire side (gRPC server and client of PodService.CollectScore) is
 * ksched/relay.py.  Host code only: no GPU, no torch.
 */
#ifndef KSGATHER_H
#define KSGATHER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ksg_evaluator ksg_evaluator;

/* Ties at the highest score: the reference picks uniformly at random among
 * the first 100 tied scores in arrival order (rand.Intn).  The deterministic
 * modes pick among them the lexicographically smallest node name, or the
 * lowest global node index of ksg_set_node_order -- the rule every host
 * applies to its own nodes (lowest slot), so a multi-host run ends as one
 * unsharded scheduler would. */
enum { KSG_TIE_RANDOM = 0, KSG_TIE_LOWEST_NAME = 1, KSG_TIE_LOWEST_INDEX = 2 };

/* members: scores that complete a pod (SchedulerSet.GetMemberCountNoRelays,
 * read when a pod's first score arrives); delay_ms: how long a pod waits for
 * missing members after its first score (the reference: 5 s,
 * grpc_server.go:135).  NULL on bad arguments. */
ksg_evaluator *ksg_open(uint32_t members, uint32_t delay_ms, int32_t tie_mode, uint64_t seed);
/* Fires every pending evaluation (its waiters return with the scores recorded
 * so far), wakes ksg_next_fired, waits until no thread is inside a call on
 * `ev`, then frees it.  Calls arriving after it started return -1; the caller
 * guarantees that no call STARTS after ksg_close returns (the handle is then
 * gone): a wrapper that cannot -- threads that may still be about to call --
 * uses ksg_shutdown first, waits for its own callers, then ksg_close. */
void ksg_close(ksg_evaluator *ev);
/* The first half of ksg_close: every later call returns -1 (ksg_next_fired
 * still reports evaluations fired before), every pending evaluation fires and
 * its waiters return; nothing is freed.  Idempotent. */
void ksg_shutdown(ksg_evaluator *ev);
/* KSG_TIE_LOWEST_INDEX: names[i] is the node of global index i (the hosts'
 * node slots laid end to end); a name not listed sorts after every listed one. */
void ksg_set_node_order(ksg_evaluator *ev, const char *const *names, uint32_t n);
/* Membership changed (relay tree): applies to pods whose first score arrives later. */
void ksg_set_members(ksg_evaluator *ev, uint32_t members);

/* Record one member's score for `key` ("namespace/name") and block until the
 * pod fires: when `members` scores have arrived (the last arrival fires it) or
 * delay_ms after its first score.  The winner -- highest score, ties as
 * tie_mode -- is copied to winner (NUL-terminated, truncated to winner_cap)
 * and *winner_score.  A score arriving after its pod fired starts a new
 * evaluation of that key (as the reference does).  Returns 1 when node_name
 * won (the CollectScore permit), 0 when it did not, -1 on bad arguments. */
int32_t ksg_record_and_wait(ksg_evaluator *ev, const char *key, const char *node_name, int32_t score,
                            char *winner, uint32_t winner_cap, int32_t *winner_score);

/* Non-blocking form for event-driven servers: record the score; returns 1 / 0
 * (permit or not) when this score fired the evaluation, 2 when it is still
 * pending (*eval_id names the evaluation; ksg_next_fired reports it once it
 * fires), -1 on bad arguments or after ksg_close began. */
int32_t ksg_record(ksg_evaluator *ev, const char *key, const char *node_name, int32_t score, uint64_t *eval_id,
                   char *winner, uint32_t winner_cap, int32_t *winner_score);
/* Wait up to timeout_ms for the next fired evaluation that has ksg_record
 * callers pending (firing evaluations whose delay expired meanwhile): 1 with
 * *eval_id and its winner, 0 on timeout, -1 once ksg_close began and nothing
 * is left to report.  One thread drives it for a whole server. */
int32_t ksg_next_fired(ksg_evaluator *ev, uint32_t timeout_ms, uint64_t *eval_id, char *winner, uint32_t winner_cap,
                       int32_t *winner_score);

/* Pods recorded and not fired yet (diagnostics / tests). */
uint32_t ksg_pending(ksg_evaluator *ev);

/* FNV-1 32-bit hash (Go hash/fnv New32) of n bytes. */
uint32_t ksg_fnv1_32(const char *data, uint32_t n);

/* Index into `members` of the gatherer for `key`: members sorted as
 * SchedulerSet.sortMembers (the leader first, then relay pods -- names with
 * the "dist-scheduler-relay" prefix -- then the rest, by name), FNV-1 32 of
 * key modulo the count.  leader may be NULL.  Returns UINT32_MAX for n = 0. */
uint32_t ksg_target_index(const char *key, const char *const *members, uint32_t n, const char *leader);

#ifdef __cplusplus
}
#endif

#endif /* KSGATHER_H */
