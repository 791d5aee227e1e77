"""ctypes mirror of include/ksched.h and include/ksynth.h.

Struct layouts must match the C headers byte for byte; tests/test_abi.py checks
sizes and that every declared symbol is exported by the built libraries.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_DIR = Path(__file__).resolve().parent / "lib"
# KSCHED_LIB_DIR selects a diagnostic libksched build (e.g. lib/stamps)
KSCHED_DIR = Path(os.environ.get("KSCHED_LIB_DIR", LIB_DIR))
# KSCHED_HOST_LIB_DIR selects builds of the host-only libraries (libksynth,
# libksgather), e.g. lib/asan (make sanitize)
HOST_DIR = Path(os.environ.get("KSCHED_HOST_LIB_DIR", LIB_DIR))

c_char_p = C.c_char_p


class KsLabel(C.Structure):
    _fields_ = [("key", c_char_p), ("value", c_char_p)]


class KsTaint(C.Structure):
    _fields_ = [("key", c_char_p), ("value", c_char_p), ("effect", C.c_int32), ("_pad", C.c_int32)]


class KsToleration(C.Structure):
    _fields_ = [("key", c_char_p), ("value", c_char_p), ("op", C.c_int32), ("effect", C.c_int32)]


class KsResource(C.Structure):
    _fields_ = [("name", c_char_p), ("value", C.c_int64)]


class KsImage(C.Structure):
    _fields_ = [("name", c_char_p), ("size_bytes", C.c_int64)]


class KsNode(C.Structure):
    _fields_ = [
        ("name", c_char_p),
        ("alloc_milli_cpu", C.c_int64),
        ("alloc_memory", C.c_int64),
        ("alloc_pods", C.c_int64),
        ("labels", C.POINTER(KsLabel)),
        ("taints", C.POINTER(KsTaint)),
        ("n_labels", C.c_uint32),
        ("n_taints", C.c_uint32),
        ("unschedulable", C.c_uint32),
        ("n_images", C.c_uint32),
        ("images", C.POINTER(KsImage)),
        ("extended", C.POINTER(KsResource)),
        ("n_extended", C.c_uint32),
        ("_pad", C.c_uint32),
    ]


class KsContainer(C.Structure):
    _fields_ = [
        ("milli_cpu", C.c_int64),
        ("memory", C.c_int64),
        ("flags", C.c_uint32),
        ("restart_always", C.c_uint32),
        ("image", c_char_p),
        ("extended", C.POINTER(KsResource)),
        ("n_extended", C.c_uint32),
        ("_pad", C.c_uint32),
    ]


class KsRequirement(C.Structure):
    _fields_ = [
        ("key", c_char_p),
        ("values", C.POINTER(c_char_p)),
        ("n_values", C.c_uint32),
        ("op", C.c_int32),
    ]


class KsTerm(C.Structure):
    _fields_ = [
        ("match_expressions", C.POINTER(KsRequirement)),
        ("match_fields", C.POINTER(KsRequirement)),
        ("n_expressions", C.c_uint32),
        ("n_fields", C.c_uint32),
    ]


class KsPreferredTerm(C.Structure):
    _fields_ = [("preference", KsTerm), ("weight", C.c_int32), ("_pad", C.c_int32)]


class KsLabelSelector(C.Structure):
    _fields_ = [
        ("match_labels", C.POINTER(KsLabel)),
        ("match_expressions", C.POINTER(KsRequirement)),
        ("n_match_labels", C.c_uint32),
        ("n_match_expressions", C.c_uint32),
        ("is_nil", C.c_uint32),
        ("_pad", C.c_uint32),
    ]


class KsSpreadConstraint(C.Structure):
    _fields_ = [
        ("topology_key", c_char_p),
        ("selector", KsLabelSelector),
        ("match_label_keys", C.POINTER(c_char_p)),
        ("n_match_label_keys", C.c_uint32),
        ("max_skew", C.c_int32),
        ("when_unsatisfiable", C.c_int32),
        ("min_domains", C.c_int32),
        ("node_affinity_policy", C.c_int32),
        ("node_taints_policy", C.c_int32),
    ]


class KsPodAffinityTerm(C.Structure):
    _fields_ = [
        ("selector", KsLabelSelector),
        ("namespace_selector", KsLabelSelector),
        ("namespaces", C.POINTER(c_char_p)),
        ("topology_key", c_char_p),
        ("n_namespaces", C.c_uint32),
        ("kind", C.c_int32),
        ("weight", C.c_int32),
        ("_pad", C.c_int32),
    ]


class KsPod(C.Structure):
    _fields_ = [
        ("ns", c_char_p),
        ("name", c_char_p),
        ("containers", C.POINTER(KsContainer)),
        ("init_containers", C.POINTER(KsContainer)),
        ("tolerations", C.POINTER(KsToleration)),
        ("node_selector", C.POINTER(KsLabel)),
        ("required_terms", C.POINTER(KsTerm)),
        ("preferred", C.POINTER(KsPreferredTerm)),
        ("node_name", c_char_p),
        ("overhead_milli_cpu", C.c_int64),
        ("overhead_memory", C.c_int64),
        ("n_containers", C.c_uint32),
        ("n_init_containers", C.c_uint32),
        ("n_tolerations", C.c_uint32),
        ("n_node_selector", C.c_uint32),
        ("n_required_terms", C.c_uint32),
        ("has_required", C.c_uint32),
        ("n_preferred", C.c_uint32),
        ("has_preferred", C.c_uint32),
        ("has_overhead", C.c_uint32),
        ("unmodelled", C.c_uint32),
        ("labels", C.POINTER(KsLabel)),
        ("spread", C.POINTER(KsSpreadConstraint)),
        ("n_labels", C.c_uint32),
        ("n_spread", C.c_uint32),
        ("spread_defaulted", C.c_uint32),
        ("_pad2", C.c_uint32),
        ("affinity_terms", C.POINTER(KsPodAffinityTerm)),
        ("namespace_labels", C.POINTER(KsLabel)),
        ("n_affinity_terms", C.c_uint32),
        ("n_namespace_labels", C.c_uint32),
    ]


NUM_FILTER_PLUGINS = 7
NUM_FAIL_COUNTS = 8  # + KS_FAIL_PREFILTER_RESULT
# ks_status codes and ks_event kinds (include/ksched.h)
KS_OK, KS_ERR_INVALID, KS_ERR_DEVICE, KS_ERR_CAPACITY, KS_ERR_UNSUPPORTED, KS_ERR_RANGE = 0, 1, 2, 3, 4, 5
KS_ERR_NOT_FOUND, KS_ERR_COMM, KS_ERR_STALE = 6, 7, 8
# KS_UNMODELLED_* pod feature bits
UNMODELLED = {"host_ports": 1, "topology_spread": 2, "pod_affinity": 4, "volumes": 8, "nominated_node": 16,
              "resource_claims": 32}
KS_EV_POD_ADD, KS_EV_POD_REMOVE, KS_EV_NODE_UPSERT, KS_EV_NODE_DELETE = 0, 1, 2, 3


class KsNodeInfo(C.Structure):
    _fields_ = [
        ("slot", C.c_uint32),
        ("deleted", C.c_uint32),
        ("generation", C.c_int64),
        ("node", C.POINTER(KsNode)),
    ]


class KsEvent(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("slot", C.c_uint32),
        ("pod", C.POINTER(KsPod)),
        ("node", C.POINTER(KsNode)),
    ]


class KsResult(C.Structure):
    _fields_ = [
        ("node_index", C.c_int32),
        ("status", C.c_int32),
        ("total_score", C.c_int64),
        ("feasible_nodes", C.c_uint32),
        ("evaluated_nodes", C.c_uint32),
        ("fail_counts", C.c_uint32 * NUM_FAIL_COUNTS),
        ("flags", C.c_uint32),
        ("_pad", C.c_uint32),
    ]


class KsNodeScore(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("least_allocated", C.c_int32),
        ("balanced_allocation", C.c_int32),
        ("taint_raw", C.c_int32),
        ("taint_score", C.c_int32),
        ("affinity_raw", C.c_int32),
        ("affinity_score", C.c_int32),
        ("image_locality", C.c_int32),
        ("spread_raw", C.c_int32),
        ("spread_score", C.c_int32),
        ("affinity_pod_raw", C.c_int32),
        ("affinity_pod_score", C.c_int32),
        ("total_score", C.c_int64),
    ]


class KsNodeState(C.Structure):
    _fields_ = [
        ("alloc_milli_cpu", C.c_int64),
        ("alloc_memory", C.c_int64),
        ("req_milli_cpu", C.c_int64),
        ("req_memory", C.c_int64),
        ("nonzero_milli_cpu", C.c_int64),
        ("nonzero_memory", C.c_int64),
        ("alloc_pods", C.c_int32),
        ("pod_count", C.c_int32),
    ]


class KsConfig(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("node_capacity", C.c_uint32),
        ("pods_per_round", C.c_uint32),
        ("topk", C.c_uint32),
        ("nodes_per_lane", C.c_uint32),
        ("world_size", C.c_uint32),
        ("rank", C.c_uint32),
        ("virtual_shards", C.c_uint32),
        ("weight_fit", C.c_int32),
        ("weight_balanced", C.c_int32),
        ("weight_taint", C.c_int32),
        ("weight_affinity", C.c_int32),
        ("weight_image", C.c_int32),
        ("percentage_of_nodes_to_score", C.c_int32),
        ("weight_topology_spread", C.c_int32),
        ("weight_inter_pod_affinity", C.c_int32),
        ("hard_pod_affinity_weight", C.c_int32),
        # execution options (include/ksched.h): none changes a result
        ("resolve_mode", C.c_uint32),
        ("resolve_par_max_passes", C.c_uint32),
        ("resolve_serial_rounds", C.c_uint32),
        ("dedup_identical_pods", C.c_uint32),
        ("early_fix", C.c_uint32),
        ("tuple_guess", C.c_uint32),
        ("ext_nodes_per_lane", C.c_uint32),
        ("sweep_pairs", C.c_uint32),
        ("sweep_pairs_ext", C.c_uint32),
        ("resolve_cus", C.c_uint32),
        ("side_cus", C.c_uint32),
        ("value_sync", C.c_uint32),
        ("sync_timeout_ms", C.c_uint32),
        ("spread_replica_runs", C.c_uint32),
    ]


RESOLVE_AUTO, RESOLVE_SERIAL, RESOLVE_PARALLEL = 0, 1, 2
OPTION_FIELDS = ("resolve_mode", "resolve_par_max_passes", "resolve_serial_rounds", "dedup_identical_pods", "early_fix",
                 "tuple_guess", "ext_nodes_per_lane", "sweep_pairs", "sweep_pairs_ext", "resolve_cus", "side_cus",
                 "value_sync", "sync_timeout_ms", "spread_replica_runs")


class KsStats(C.Structure):
    _fields_ = [
        ("rounds", C.c_uint64),
        ("pods_resolved", C.c_uint64),
        ("pods_scheduled", C.c_uint64),
        ("sweep_launches", C.c_uint64),
        ("sweep_ms", C.c_double),
        ("sweep_evals", C.c_uint64),
        ("resolve_ms", C.c_double),
        ("resolve_launches", C.c_uint64),
        ("spread_ms", C.c_double),
        ("spread_pods_timed", C.c_uint64),
        ("spread_pods", C.c_uint64),
        ("replica_runs", C.c_uint64),
        ("replica_pods", C.c_uint64),
        ("replica_ms", C.c_double),
        ("classes_inflight", C.c_uint64),
        ("late_class_pods", C.c_uint64),
    ]


# sizes from the C headers (checked in tests/test_abi.py against offsetof via the compiler)
EXPECTED_SIZES = {
    "ks_label": 16, "ks_taint": 24, "ks_toleration": 24, "ks_node": 88, "ks_container": 48,
    "ks_resource": 16, "ks_image": 16,
    "ks_requirement": 24, "ks_term": 24, "ks_preferred_term": 32, "ks_pod": 184, "ks_event": 24, "ks_result": 64,
    "ks_node_score": 56, "ks_node_state": 56, "ks_config": 124, "ks_pod_affinity_term": 96, "ks_stats": 112, "ks_label_selector": 32,
    "ks_spread_constraint": 72,
}
STRUCTS = {
    "ks_label": KsLabel, "ks_taint": KsTaint, "ks_toleration": KsToleration, "ks_node": KsNode,
    "ks_container": KsContainer, "ks_requirement": KsRequirement, "ks_term": KsTerm,
    "ks_preferred_term": KsPreferredTerm, "ks_pod": KsPod, "ks_event": KsEvent, "ks_node_info": KsNodeInfo, "ks_result": KsResult,
    "ks_node_score": KsNodeScore, "ks_node_state": KsNodeState, "ks_config": KsConfig,
    "ks_stats": KsStats, "ks_label_selector": KsLabelSelector, "ks_spread_constraint": KsSpreadConstraint,
    "ks_resource": KsResource, "ks_image": KsImage, "ks_pod_affinity_term": KsPodAffinityTerm,
}

KSCHED_SYMBOLS = [
    "ks_config_default", "ks_open", "ks_close", "ks_last_error", "ks_abi_version", "ks_nodes_upsert",
    "ks_nodes_upsert_each",
    "ks_nodes_delete", "ks_pods_add", "ks_pods_remove", "ks_events_apply", "ks_schedule", "ks_batch_prepare", "ks_batch_run",
    "ks_batch_results", "ks_batch_free", "ks_batch_submit", "ks_batch_wait", "ks_pods_check", "ks_plugin_scores", "ks_node_states", "ks_comm_unique_id", "ks_comm_init_local", "ks_snapshot_update",
    "ks_comm_init", "ks_comm_allreduce_max", "ks_get_stats", "ks_reset_stats", "ks_set_timing",
    "ks_debug_counters", "ks_debug_set_profile", "ks_debug_resolve_profile", "ks_debug_round_record", "ks_set_sync_timeout", "ks_debug_stall", "ks_batch_marks",
    "ks_debug_runs_started", "ks_next_start_index",
]
KSGATHER_SYMBOLS = [
    "ksg_open", "ksg_close", "ksg_set_members", "ksg_record_and_wait", "ksg_pending", "ksg_fnv1_32", "ksg_target_index",
    "ksg_record", "ksg_next_fired", "ksg_set_node_order", "ksg_shutdown",
]
KSYNTH_SYMBOLS = [
    "ksynth_nodes", "ksynth_pods", "ksynth_prefill", "ksynth_besteffort_pods", "ksynth_spread_pods", "ksynth_deploy_pods", "ksynth_deploy_dns_pods", "ksynth_affinity_pods", "ksynth_node_array",
    "ksynth_pod_array", "ksynth_slots", "ksynth_free", "ksynth_fnv64",
]


class KschedError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"ksched status {status}: {msg}")
        self.status = status


def _load(name: str, where: Path = LIB_DIR) -> C.CDLL:
    path = where / name
    if not path.exists():
        raise ImportError(
            f"{path} is missing: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')"
        )
    return C.CDLL(str(path), mode=os.RTLD_NOW | os.RTLD_GLOBAL)


_ksched = None
_ksynth = None


def ksched_lib() -> C.CDLL:
    """libksched.so with argtypes declared.  Raises ImportError when absent."""
    global _ksched
    if _ksched is not None:
        return _ksched
    L = _load("libksched.so", KSCHED_DIR)
    P = C.POINTER
    vp = C.c_void_p
    L.ks_config_default.argtypes = [P(KsConfig)]
    L.ks_config_default.restype = None
    L.ks_open.argtypes = [P(KsConfig), P(vp)]
    L.ks_close.argtypes = [vp]
    L.ks_close.restype = None
    L.ks_last_error.argtypes = [vp]
    L.ks_last_error.restype = c_char_p
    L.ks_abi_version.restype = C.c_int32
    L.ks_nodes_upsert.argtypes = [vp, P(KsNode), P(C.c_uint32), C.c_uint32]
    L.ks_nodes_upsert_each.argtypes = [vp, P(KsNode), P(C.c_uint32), C.c_uint32, P(C.c_int32)]
    L.ks_nodes_delete.argtypes = [vp, P(C.c_uint32), C.c_uint32]
    L.ks_pods_add.argtypes = [vp, P(KsPod), P(C.c_uint32), C.c_uint32]
    L.ks_pods_remove.argtypes = [vp, P(KsPod), P(C.c_uint32), C.c_uint32]
    L.ks_events_apply.argtypes = [vp, P(KsEvent), C.c_uint32]
    L.ks_snapshot_update.argtypes = [vp, P(KsNodeInfo), C.c_uint32, P(C.c_int64), P(C.c_uint32)]
    L.ks_schedule.argtypes = [vp, P(KsPod), C.c_uint32, P(KsResult)]
    L.ks_batch_prepare.argtypes = [vp, P(KsPod), C.c_uint32, P(vp)]
    L.ks_batch_run.argtypes = [vp, vp]
    L.ks_batch_results.argtypes = [vp, vp, P(KsResult)]
    L.ks_batch_free.argtypes = [vp, vp]
    L.ks_batch_free.restype = None
    L.ks_batch_submit.argtypes = [vp, vp]
    L.ks_batch_wait.argtypes = [vp, vp]
    L.ks_pods_check.argtypes = [vp, P(KsPod), C.c_uint32, P(C.c_int32)]
    L.ks_plugin_scores.argtypes = [vp, P(KsPod), P(KsNodeScore)]
    L.ks_node_states.argtypes = [vp, P(C.c_uint32), C.c_uint32, P(KsNodeState)]
    L.ks_comm_unique_id.argtypes = [P(C.c_uint8)]
    L.ks_comm_init.argtypes = [vp, P(C.c_uint8)]
    L.ks_debug_round_record.argtypes = [vp, C.c_uint32, P(C.c_uint64)]
    L.ks_comm_init_local.argtypes = [P(vp), C.c_uint32]
    L.ks_comm_allreduce_max.argtypes = [vp, P(C.c_double), C.c_uint32]
    L.ks_get_stats.argtypes = [vp, P(KsStats)]
    L.ks_reset_stats.argtypes = [vp]
    L.ks_set_timing.argtypes = [vp, C.c_int32]
    L.ks_debug_counters.argtypes = [vp, P(C.c_uint64)]
    L.ks_debug_set_profile.argtypes = [vp, C.c_int32]
    L.ks_debug_resolve_profile.argtypes = [vp, P(C.c_uint64)]
    L.ks_set_sync_timeout.argtypes = [vp, C.c_uint32]
    L.ks_debug_stall.argtypes = [vp, C.c_uint32, C.c_uint32]
    L.ks_debug_runs_started.argtypes = [vp, P(C.c_uint64)]
    L.ks_next_start_index.argtypes = [vp, P(C.c_uint64)]
    L.ks_batch_marks.argtypes = [vp, vp, P(C.c_uint8)]
    for f in KSCHED_SYMBOLS:
        fn = getattr(L, f)
        if fn.restype is C.c_int and f not in ("ks_abi_version",):
            fn.restype = C.c_int32
    _ksched = L
    return L


def ksynth_lib() -> C.CDLL:
    global _ksynth
    if _ksynth is not None:
        return _ksynth
    L = _load("libksynth.so", HOST_DIR)
    vp = C.c_void_p
    P = C.POINTER
    L.ksynth_nodes.argtypes = [C.c_int32, C.c_uint32, C.c_uint64]
    L.ksynth_nodes.restype = vp
    L.ksynth_pods.argtypes = [C.c_int32, C.c_uint32, C.c_uint64]
    L.ksynth_pods.restype = vp
    L.ksynth_prefill.argtypes = [C.c_int32, C.c_uint32, C.c_uint64, C.c_uint64, C.c_double]
    L.ksynth_prefill.restype = vp
    L.ksynth_besteffort_pods.argtypes = [C.c_uint32]
    L.ksynth_besteffort_pods.restype = vp
    L.ksynth_spread_pods.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
    L.ksynth_spread_pods.restype = vp
    L.ksynth_affinity_pods.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
    L.ksynth_deploy_pods.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
    L.ksynth_deploy_pods.restype = vp
    L.ksynth_deploy_dns_pods.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
    L.ksynth_deploy_dns_pods.restype = vp
    L.ksynth_affinity_pods.restype = vp
    L.ksynth_node_array.argtypes = [vp, P(C.c_uint32)]
    L.ksynth_node_array.restype = P(KsNode)
    L.ksynth_pod_array.argtypes = [vp, P(C.c_uint32)]
    L.ksynth_pod_array.restype = P(KsPod)
    L.ksynth_slots.argtypes = [vp, P(C.c_uint32)]
    L.ksynth_slots.restype = P(C.c_uint32)
    L.ksynth_free.argtypes = [vp]
    L.ksynth_free.restype = None
    L.ksynth_fnv64.argtypes = [vp, C.c_uint64, C.c_uint64]
    L.ksynth_fnv64.restype = C.c_uint64
    _ksynth = L
    return L


_ksgather = None


def ksgather_lib() -> C.CDLL:
    """libksgather.so: the cross-host gather (include/ksgather.h); host code only."""
    global _ksgather
    if _ksgather is not None:
        return _ksgather
    L = _load("libksgather.so", HOST_DIR)
    vp = C.c_void_p
    P = C.POINTER
    L.ksg_open.argtypes = [C.c_uint32, C.c_uint32, C.c_int32, C.c_uint64]
    L.ksg_open.restype = vp
    L.ksg_close.argtypes = [vp]
    L.ksg_close.restype = None
    L.ksg_shutdown.argtypes = [vp]
    L.ksg_shutdown.restype = None
    L.ksg_set_members.argtypes = [vp, C.c_uint32]
    L.ksg_set_members.restype = None
    L.ksg_record_and_wait.argtypes = [vp, C.c_char_p, C.c_char_p, C.c_int32, C.c_char_p, C.c_uint32, P(C.c_int32)]
    L.ksg_record_and_wait.restype = C.c_int32
    L.ksg_record.argtypes = [vp, C.c_char_p, C.c_char_p, C.c_int32, P(C.c_uint64), C.c_char_p, C.c_uint32,
                             P(C.c_int32)]
    L.ksg_record.restype = C.c_int32
    L.ksg_next_fired.argtypes = [vp, C.c_uint32, P(C.c_uint64), C.c_char_p, C.c_uint32, P(C.c_int32)]
    L.ksg_next_fired.restype = C.c_int32
    L.ksg_set_node_order.argtypes = [vp, P(C.c_char_p), C.c_uint32]
    L.ksg_set_node_order.restype = None
    L.ksg_pending.argtypes = [vp]
    L.ksg_pending.restype = C.c_uint32
    L.ksg_fnv1_32.argtypes = [C.c_char_p, C.c_uint32]
    L.ksg_fnv1_32.restype = C.c_uint32
    L.ksg_target_index.argtypes = [C.c_char_p, P(C.c_char_p), C.c_uint32, C.c_char_p]
    L.ksg_target_index.restype = C.c_uint32
    _ksgather = L
    return L
