"""Host-side mirror of the scheduler framework surface this path sits behind.

The reference calls the forked kube-scheduler's ``Scheduler.SchedulePod``
(upstream k8s.io/kubernetes v1.31.3 pkg/scheduler/schedule_one.go#schedulePod)
from ``ScheduleOne`` (dist-scheduler/cmd/dist-scheduler/scheduler.go:543) and
reads its outcome in two places:

* ``DistPermit.Permit`` reads ``framework.NodePluginScoresState`` from the
  CycleState and sends the chosen node's ``TotalScore`` as int32
  (dist-scheduler/pkg/distpermit/distpermit.go:51-72, :106);
* ``podScheduleFailure`` type-asserts ``*framework.FitError`` and reads
  ``Diagnosis.UnschedulablePlugins`` (scheduler.go:383-395).

``Scheduler`` below keeps those names, argument meanings and error behaviour:
``schedule_pod`` returns a ``ScheduleResult`` and writes
``NodePluginScoresState`` into the CycleState, or raises ``FitError``
(no feasible node) / ``FrameworkError`` (an Error status).  Every call goes to
libksched.so (HIP); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from enum import IntEnum
from typing import Dict, List, Optional, Sequence, Union

from . import _abi
from .objects import Arena, Node, Pod, nodes_array, pods_array

FILTER_PLUGINS = ["NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodeResourcesFit",
                  "PodTopologySpread", "InterPodAffinity"]
NODE_PLUGIN_SCORES_STATE_KEY = "NodePluginScores"  # fork: framework.NodePluginScoresStateKey
DEFAULT_WEIGHTS = {  # apis/config/v1 default plugin weights (v1.31)
    "NodeResourcesFit": 1,
    "NodeResourcesBalancedAllocation": 1,
    "TaintToleration": 3,
    "NodeAffinity": 2,
    "ImageLocality": 1,
    "PodTopologySpread": 2,
    "InterPodAffinity": 2,
}


class Code(IntEnum):  # framework.Code
    Success = 0
    Error = 1
    Unschedulable = 2
    UnschedulableAndUnresolvable = 3
    Wait = 4
    Skip = 5


@dataclass
class ScheduleResult:  # scheduler.ScheduleResult
    suggested_host: str
    evaluated_nodes: int
    feasible_nodes: int
    node_index: int = -1
    total_score: int = 0
    single_feasible: bool = False


@dataclass
class Diagnosis:  # framework.Diagnosis (NodeToStatus summarised per plugin)
    node_to_status: Dict[str, int] = field(default_factory=dict)
    unschedulable_plugins: set = field(default_factory=set)


class FitError(Exception):  # framework.FitError
    def __init__(self, pod: str, num_all_nodes: int, diagnosis: Diagnosis):
        self.pod = pod
        self.num_all_nodes = num_all_nodes
        self.diagnosis = diagnosis
        super().__init__(f"0/{num_all_nodes} nodes are available for pod {pod}: {diagnosis.node_to_status}")


class FrameworkError(Exception):
    """A plugin returned an Error status (e.g. NodeAffinity PreScore parse error)."""


@dataclass
class PluginScore:
    name: str
    score: int


@dataclass
class NodePluginScores:  # framework.NodePluginScores
    name: str
    scores: List[PluginScore]
    total_score: int


@dataclass
class NodePluginScoresState:  # fork-only framework.NodePluginScoresState
    node_plugin_scores: List[NodePluginScores]


class CycleState(dict):  # framework.CycleState (Read / Write)
    def write(self, key, value):
        self[key] = value

    def read(self, key):
        if key not in self:
            raise KeyError(f"{key} not found")
        return self[key]


def _check(lib, ctx, st: int):
    if st != 0:
        msg = lib.ks_last_error(ctx).decode() if ctx else "error"
        raise _abi.KschedError(st, msg)


class Scheduler:
    """One shard's scheduling core on one GPU (a ks_ctx)."""

    def __init__(self, node_capacity: int, *, device: int = 0, pods_per_round: int = 256, topk: int = 0,
                 nodes_per_lane: int = 4, world_size: int = 1, rank: int = 0, virtual_shards: int = 1,
                 weights: Optional[Dict[str, int]] = None, options: Optional[Dict[str, int]] = None,
                 percentage_of_nodes_to_score: int = 100):
        """options: ks_config execution options by field name (_abi.OPTION_FIELDS),
        e.g. {"resolve_mode": _abi.RESOLVE_SERIAL, "dedup_identical_pods": 0};
        none of them changes a result.  percentage_of_nodes_to_score: the
        profile's percentageOfNodesToScore (ksched.h; below 100 one shard only)."""
        self.lib = _abi.ksched_lib()
        cfg = _abi.KsConfig()
        self.lib.ks_config_default(C.byref(cfg))
        for k, v in (options or {}).items():
            if k not in _abi.OPTION_FIELDS:
                raise ValueError(f"unknown ks_config option {k}")
            setattr(cfg, k, int(v))
        cfg.device = device
        cfg.node_capacity = node_capacity
        cfg.pods_per_round = pods_per_round
        cfg.topk = topk
        cfg.nodes_per_lane = nodes_per_lane
        cfg.world_size = world_size
        cfg.rank = rank
        cfg.virtual_shards = virtual_shards
        w = dict(DEFAULT_WEIGHTS, **(weights or {}))
        cfg.weight_fit = w["NodeResourcesFit"]
        cfg.weight_balanced = w["NodeResourcesBalancedAllocation"]
        cfg.weight_taint = w["TaintToleration"]
        cfg.weight_affinity = w["NodeAffinity"]
        cfg.weight_image = w["ImageLocality"]
        cfg.weight_topology_spread = w["PodTopologySpread"]
        cfg.weight_inter_pod_affinity = w["InterPodAffinity"]
        cfg.hard_pod_affinity_weight = 1
        cfg.percentage_of_nodes_to_score = percentage_of_nodes_to_score
        self.weights = w
        self.capacity = node_capacity
        self.ctx = C.c_void_p()
        st = self.lib.ks_open(C.byref(cfg), C.byref(self.ctx))
        if st != 0:
            raise _abi.KschedError(st, "ks_open failed (no usable HIP device?)")
        self.names: Dict[int, str] = {}
        self.slots: Dict[str, int] = {}
        self.slot_gen: Dict[int, int] = {}  # last NodeInfo.Generation applied per slot (snapshot_update)

    def next_start_index(self) -> int:
        """Scheduler.nextStartNodeIndex (percentageOfNodesToScore < 100)."""
        v = C.c_uint64()
        _check(self.lib, self.ctx, self.lib.ks_next_start_index(self.ctx, C.byref(v)))
        return int(v.value)

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if self.ctx:
            self.lib.ks_close(self.ctx)
            self.ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _ok(self, st):
        _check(self.lib, self.ctx, st)

    # ------------------------------------------------- node cache (informer)
    def upsert_nodes(self, nodes: Sequence[Node], slots: Optional[Sequence[int]] = None):
        """AddNode / UpdateNode for k8s-shaped nodes; returns their slots."""
        if slots is None:
            slots = [self.slots.get(n.name, None) for n in nodes]
            free = (s for s in range(self.capacity) if s not in self.names)
            slots = [s if s is not None else next(free) for s in slots]
        a = Arena()
        arr, n = nodes_array(list(nodes), a)
        sl = (C.c_uint32 * max(1, n))(*slots)
        self._ok(self.lib.ks_nodes_upsert(self.ctx, arr, sl, n))
        for node, s in zip(nodes, slots):
            old = self.names.get(s)
            if old is not None:
                self.slots.pop(old, None)
            self.names[s] = node.name
            self.slots[node.name] = s
        return list(slots)

    def upsert_nodes_raw(self, arr, slots, n: int, names: Optional[Sequence[str]] = None):
        self._ok(self.lib.ks_nodes_upsert(self.ctx, arr, slots, n))

    def snapshot_update(self, items):
        """Cache.UpdateSnapshot: items = [(slot, generation, Node or None for
        RemoveNode)]; returns (snapshot generation, items applied).

        The slot -> name mirror follows what ks_snapshot_update applies, not
        every item it is handed: per slot only the highest generation above
        the slot's last applied one counts (stale or replayed items are
        skipped), deletions go first, and an upsert that renames a slot drops
        the old name's reverse entry."""
        a = Arena()
        live = [(sl, g, nd) for sl, g, nd in items]
        arr, _ = nodes_array([nd for _, _, nd in live if nd is not None], a) if any(
            nd is not None for _, _, nd in live) else (None, 0)
        infos = (_abi.KsNodeInfo * max(1, len(live)))()
        k = 0
        for i, (sl, g, nd) in enumerate(live):
            infos[i].slot, infos[i].generation = sl, g
            if nd is None:
                infos[i].deleted = 1
            else:
                infos[i].node = C.pointer(arr[k])
                k += 1
        # the items the library will apply (its filter, restated)
        best: Dict[int, int] = {}
        for i, (sl, g, nd) in enumerate(live):
            if g <= self.slot_gen.get(sl, -(1 << 63)):
                continue
            if sl not in best or live[best[sl]][1] < g:
                best[sl] = i
        order = sorted(best.values())
        gen, applied = C.c_int64(), C.c_uint32()
        try:
            self._ok(self.lib.ks_snapshot_update(self.ctx, infos, len(live), C.byref(gen), C.byref(applied)))
        except _abi.KschedError as e:
            if "deletions were applied" in str(e):  # the upserts failed after the deletions went in
                self._mirror_snapshot([i for i in order if live[i][2] is None], live)
            raise
        self._mirror_snapshot(order, live)
        return gen.value, applied.value

    def _mirror_snapshot(self, order, live):
        for i in order:  # deletions first, as the library applies them
            sl, g, nd = live[i]
            if nd is None:
                old = self.names.pop(sl, None)
                if old is not None and self.slots.get(old) == sl:
                    self.slots.pop(old, None)
        for i in order:
            sl, g, nd = live[i]
            if nd is not None:
                old = self.names.get(sl)
                if old is not None and old != nd.name and self.slots.get(old) == sl:
                    self.slots.pop(old, None)
                self.names[sl] = nd.name
                self.slots[nd.name] = sl
        for i in order:
            self.slot_gen[live[i][0]] = live[i][1]

    def delete_nodes(self, names: Sequence[str]):
        slots = [self.slots[n] for n in names]
        sl = (C.c_uint32 * max(1, len(slots)))(*slots)
        self._ok(self.lib.ks_nodes_delete(self.ctx, sl, len(slots)))
        for n, s in zip(names, slots):
            self.slots.pop(n, None)
            self.names.pop(s, None)

    def delete_slots(self, slots: Sequence[int]):
        sl = (C.c_uint32 * max(1, len(slots)))(*slots)
        self._ok(self.lib.ks_nodes_delete(self.ctx, sl, len(slots)))
        for s in slots:
            n = self.names.pop(s, None)
            if n is not None:
                self.slots.pop(n, None)

    def _pods_event(self, fn, pods: Sequence[Pod], slots: Sequence[int]):
        a = Arena()
        arr, n = pods_array(list(pods), a)
        sl = (C.c_uint32 * max(1, n))(*slots)
        self._ok(fn(self.ctx, arr, sl, n))

    def add_pods(self, pods: Sequence[Pod], slots: Sequence[int]):
        """NodeInfo.AddPod for pods already bound to (or assumed on) nodes."""
        self._pods_event(self.lib.ks_pods_add, pods, slots)

    def remove_pods(self, pods: Sequence[Pod], slots: Sequence[int]):
        """NodeInfo.RemovePod (pod deleted / ForgetPod)."""
        self._pods_event(self.lib.ks_pods_remove, pods, slots)

    # --------------------------------------------------------- scheduling
    def _results(self, raw, n) -> List[Union[ScheduleResult, FitError, FrameworkError]]:
        out = []
        for i in range(n):
            r = raw[i]
            if r.status == 0:
                out.append(ScheduleResult(self.names.get(r.node_index, str(r.node_index)), r.evaluated_nodes,
                                          r.feasible_nodes, r.node_index, r.total_score, bool(r.flags & 1)))
            elif r.status == 1:
                counts = {FILTER_PLUGINS[k]: int(r.fail_counts[k]) for k in range(7) if r.fail_counts[k]}
                out.append(FitError(f"pod#{i}", r.evaluated_nodes, Diagnosis(counts, set(counts))))
            else:
                out.append(FrameworkError(f"pod#{i}: plugin Error status"))
        return out

    def schedule_pods(self, pods: Sequence[Pod]):
        """Sequential schedulePod + assume for each pod, in queue order."""
        a = Arena()
        arr, n = pods_array(list(pods), a)
        raw = (_abi.KsResult * max(1, n))()
        self._ok(self.lib.ks_schedule(self.ctx, arr, n, raw))
        return self._results(raw, n)

    def schedule_raw(self, arr, n: int):
        raw = (_abi.KsResult * max(1, n))()
        self._ok(self.lib.ks_schedule(self.ctx, arr, n, raw))
        return raw

    def schedule_pod(self, state: CycleState, pod: Pod) -> ScheduleResult:
        """The ``SchedulePod`` hook: schedule one pod, assume it, write NodePluginScoresState."""
        res = self.schedule_pods([pod])[0]
        if isinstance(res, Exception):
            raise res
        state.write(NODE_PLUGIN_SCORES_STATE_KEY, NodePluginScoresState(
            [NodePluginScores(res.suggested_host, [], res.total_score)]))
        return res

    def plugin_scores(self, pod: Pod) -> List[_abi.KsNodeScore]:
        a = Arena()
        arr, _ = pods_array([pod], a)
        out = (_abi.KsNodeScore * self.capacity)()
        self._ok(self.lib.ks_plugin_scores(self.ctx, arr, out))
        return list(out)

    def node_states(self, slots: Sequence[int]) -> List[_abi.KsNodeState]:
        sl = (C.c_uint32 * max(1, len(slots)))(*slots)
        out = (_abi.KsNodeState * max(1, len(slots)))()
        self._ok(self.lib.ks_node_states(self.ctx, sl, len(slots), out))
        return list(out)[: len(slots)]

    # ---------------------------------------------------------- batches
    def prepare(self, arr, n: int):
        b = C.c_void_p()
        self._ok(self.lib.ks_batch_prepare(self.ctx, arr, n, C.byref(b)))
        return b

    def run(self, batch):
        self._ok(self.lib.ks_batch_run(self.ctx, batch))

    def results(self, batch, n: int):
        raw = (_abi.KsResult * max(1, n))()
        self._ok(self.lib.ks_batch_results(self.ctx, batch, raw))
        return raw

    def marks(self, batch, n: int) -> bytes:
        """Per-pod round marks of a finished batch (ks_batch_marks: KS_MARK_* bits)."""
        out = (C.c_uint8 * max(1, n))()
        self._ok(self.lib.ks_batch_marks(self.ctx, batch, out))
        return bytes(out)[:n]

    def free(self, batch):
        self.lib.ks_batch_free(self.ctx, batch)

    # ---------------------------------------------------------- measurement
    def set_timing(self, on: bool):
        self._ok(self.lib.ks_set_timing(self.ctx, 1 if on else 0))

    def stats(self) -> _abi.KsStats:
        s = _abi.KsStats()
        self._ok(self.lib.ks_get_stats(self.ctx, C.byref(s)))
        return s

    def reset_stats(self):
        self._ok(self.lib.ks_reset_stats(self.ctx))

    # ---------------------------------------------------------- multi-GPU
    @staticmethod
    def comm_unique_id() -> bytes:
        lib = _abi.ksched_lib()
        buf = (C.c_uint8 * 128)()
        st = lib.ks_comm_unique_id(buf)
        if st != 0:
            raise _abi.KschedError(st, "ncclGetUniqueId failed")
        return bytes(buf)

    def comm_init(self, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._ok(self.lib.ks_comm_init(self.ctx, buf))

    @staticmethod
    def comm_init_local(scheds: Sequence["Scheduler"]):
        """In-process communicator over contexts of this process (rank r =
        scheds[r]; one GPU may hold them all): the multi-rank path without
        RCCL, for tests.  Each rank must then be driven from its own thread."""
        lib = _abi.ksched_lib()
        arr = (C.c_void_p * len(scheds))(*[s.ctx.value for s in scheds])
        st = lib.ks_comm_init_local(arr, len(scheds))
        if st != 0:
            raise _abi.KschedError(st, lib.ks_last_error(scheds[0].ctx).decode())

    def allreduce_max(self, values):
        """Element-wise max over ranks (RCCL); doubles as a barrier."""
        arr = (C.c_double * max(1, len(values)))(*values)
        self._ok(self.lib.ks_comm_allreduce_max(self.ctx, arr, len(values)))
        return list(arr)[: len(values)]


def results_to_arrays(raw, n: int):
    """(node_index[int32], total_score[int64], status[int32], feasible[uint32]) numpy views."""
    import numpy as np

    buf = np.frombuffer(C.string_at(C.addressof(raw), n * C.sizeof(_abi.KsResult)), dtype=np.uint8)
    dt = np.dtype([("node_index", "<i4"), ("status", "<i4"), ("total_score", "<i8"), ("feasible", "<u4"),
                   ("evaluated", "<u4"), ("fail", "<u4", (8,)), ("flags", "<u4"), ("_pad", "<u4")])
    return buf.view(dt)
