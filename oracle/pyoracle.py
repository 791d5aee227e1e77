"""ctypes binding of liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline (see oracle/oracle.h:
PARITY UNPINNED).
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "k8s-1m_amd"))
from ksched import _abi  # noqa: E402  (struct definitions only)

# ORACLE_LIB: another build of the same source (oracle/_build/asan: make sanitize)
LIB = Path(os.environ.get("ORACLE_LIB", ROOT / "oracle" / "_build" / "liboracle.so"))


class ShardPrescore(C.Structure):
    _fields_ = [
        ("feasible", C.c_uint32),
        ("fail_counts", C.c_uint32 * 8),
        ("taint_max", C.c_int64),
        ("affinity_max", C.c_int64),
        ("taint_count", C.c_uint32),
        ("affinity_count", C.c_uint32),
        ("error", C.c_int32),
        ("_pad", C.c_int32),
    ]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB.exists():
        raise ImportError(f"{LIB} missing: run `make -C oracle`")
    L = C.CDLL(str(LIB))
    vp, P = C.c_void_p, C.POINTER
    L.oracle_new.argtypes = [C.c_uint32] + [C.c_int32] * 5
    L.oracle_new.restype = vp
    L.oracle_free.argtypes = [vp]
    L.oracle_free.restype = None
    L.oracle_set_threads.argtypes = [vp, C.c_int32]
    L.oracle_set_threads.restype = None
    L.oracle_set_weight_spread.argtypes = [vp, C.c_int32]
    L.oracle_set_weight_spread.restype = None
    L.oracle_set_weight_inter_pod_affinity.argtypes = [vp, C.c_int32, C.c_int32]
    L.oracle_set_weight_inter_pod_affinity.restype = None
    L.oracle_set_percentage.argtypes = [vp, C.c_int32]
    L.oracle_set_percentage.restype = None
    L.oracle_next_start.argtypes = [vp]
    L.oracle_next_start.restype = C.c_uint64
    L.oracle_num_feasible_nodes_to_find.argtypes = [C.c_int32, C.c_int64]
    L.oracle_num_feasible_nodes_to_find.restype = C.c_int64
    L.oracle_nodes_upsert.argtypes = [vp, P(_abi.KsNode), P(C.c_uint32), C.c_uint32]
    L.oracle_nodes_delete.argtypes = [vp, P(C.c_uint32), C.c_uint32]
    L.oracle_pods_add.argtypes = [vp, P(_abi.KsPod), P(C.c_uint32), C.c_uint32]
    L.oracle_pods_remove.argtypes = [vp, P(_abi.KsPod), P(C.c_uint32), C.c_uint32]
    L.oracle_schedule.argtypes = [vp, P(_abi.KsPod), C.c_uint32, P(_abi.KsResult)]
    L.oracle_plugin_scores.argtypes = [vp, P(_abi.KsPod), P(_abi.KsNodeScore)]
    L.oracle_node_states.argtypes = [vp, P(C.c_uint32), C.c_uint32, P(_abi.KsNodeState)]
    L.oracle_shard_prescore_run.argtypes = [vp, P(_abi.KsPod), C.c_uint32, C.c_uint32, P(ShardPrescore)]
    L.oracle_shard_best.argtypes = [vp, P(_abi.KsPod), C.c_uint32, C.c_uint32, C.c_int64, C.c_int64]
    L.oracle_shard_best.restype = C.c_uint64
    L.oracle_commit.argtypes = [vp, P(_abi.KsPod), C.c_uint32]
    for f in ("oracle_least_allocated", "oracle_balanced_allocation"):
        getattr(L, f).argtypes = [C.c_int64] * 6
        getattr(L, f).restype = C.c_int64
    L.oracle_go_log.argtypes = [C.c_double]
    L.oracle_go_log.restype = C.c_double
    L.oracle_pod_requests.argtypes = [P(_abi.KsPod), P(C.c_int64)]
    _lib = L
    return L


class Oracle:
    def __init__(self, capacity: int, weights=(1, 1, 3, 2, 1, 2), threads: int = 1, percentage: int = 100):
        self.L = lib()
        self.o = self.L.oracle_new(capacity, *weights[:5])
        if len(weights) > 5:
            self.L.oracle_set_weight_spread(self.o, weights[5])
        self.capacity = capacity
        if threads > 1:
            self.L.oracle_set_threads(self.o, threads)
        if percentage != 100:
            self.L.oracle_set_percentage(self.o, percentage)

    @property
    def next_start(self) -> int:
        """Scheduler.nextStartNodeIndex (percentageOfNodesToScore < 100)."""
        return int(self.L.oracle_next_start(self.o))

    def close(self):
        if self.o:
            self.L.oracle_free(self.o)
            self.o = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upsert(self, arr, slots, n):
        assert self.L.oracle_nodes_upsert(self.o, arr, slots, n) == 0

    def delete(self, slots, n):
        assert self.L.oracle_nodes_delete(self.o, slots, n) == 0

    def add_pods(self, arr, slots, n):
        assert self.L.oracle_pods_add(self.o, arr, slots, n) == 0

    def remove_pods(self, arr, slots, n):
        assert self.L.oracle_pods_remove(self.o, arr, slots, n) == 0

    def schedule(self, arr, n):
        out = (_abi.KsResult * max(1, n))()
        assert self.L.oracle_schedule(self.o, arr, n, out) == 0
        return out

    def plugin_scores(self, pod_ptr):
        out = (_abi.KsNodeScore * self.capacity)()
        assert self.L.oracle_plugin_scores(self.o, pod_ptr, out) == 0
        return out

    def node_states(self, slots):
        sl = (C.c_uint32 * max(1, len(slots)))(*slots)
        out = (_abi.KsNodeState * max(1, len(slots)))()
        assert self.L.oracle_node_states(self.o, sl, len(slots), out) == 0
        return list(out)[: len(slots)]

    def shard_prescore(self, pod_ptr, lo, hi):
        out = ShardPrescore()
        assert self.L.oracle_shard_prescore_run(self.o, pod_ptr, lo, hi, C.byref(out)) == 0
        return out

    def shard_best(self, pod_ptr, lo, hi, tt_max, na_max) -> int:
        return self.L.oracle_shard_best(self.o, pod_ptr, lo, hi, tt_max, na_max)

    def commit(self, pod_ptr, slot):
        assert self.L.oracle_commit(self.o, pod_ptr, slot) == 0
