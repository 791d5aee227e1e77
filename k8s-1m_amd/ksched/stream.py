"""C5 driver: a bursty pod stream with a seeded event log
between bursts, applied identically to any number of targets (libksched
contexts here; tests/stream.py adds the checker's target).

Between bursts, in log order (the informer events the reference's cache would
see, dist-scheduler/cmd/dist-scheduler/scheduler.go:200-228 -> upstream
internal/cache AddPod/RemovePod/UpdateNode/RemoveNode/AddNode):

  1. pod deletes   : a fraction of the bound pods (NodeInfo.RemovePod: frees
                     Requested / NonZeroRequested / the pod slot);
  2. node updates  : a fraction of the live nodes get a new shape (allocatable,
                     labels, taints) and keep their pods (UpdateNode);
  3. node deletes  : a fraction of the live nodes leave (RemoveNode); their
                     pods leave with them;
  4. node adds     : as many fresh nodes join, into the freed slots (AddNode).

The event log is a function of the seeds and of the burst results, which every
target must agree on before the log is generated (the tests assert it).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from ksched import _abi, synth


@dataclass
class Rates:
    pod_delete: float = 0.05
    node_update: float = 0.001
    node_delete: float = 0.0001


class GpuTarget:
    def __init__(self, s):
        self.s = s

    def _ok(self, st):
        assert st == 0, self.s.lib.ks_last_error(self.s.ctx)

    def upsert(self, arr, slots, n):
        self._ok(self.s.lib.ks_nodes_upsert(self.s.ctx, arr, slots, n))

    def delete(self, slots, n):
        self._ok(self.s.lib.ks_nodes_delete(self.s.ctx, slots, n))

    def add_pods(self, arr, slots, n):
        self._ok(self.s.lib.ks_pods_add(self.s.ctx, arr, slots, n))

    def remove_pods(self, arr, slots, n):
        self._ok(self.s.lib.ks_pods_remove(self.s.ctx, arr, slots, n))

    def apply_events(self, ev, n):
        self._ok(self.s.lib.ks_events_apply(self.s.ctx, ev, n))

    def schedule(self, arr, n):
        return self.s.schedule_raw(arr, n)

    def states(self, slots):
        return self.s.node_states(slots)


def _rows(src, T, idx):
    """numpy rows (bytes) of the T structs src[idx] (src: a ctypes array or pointer)."""
    idx = np.asarray(idx, dtype=np.int64)
    if not len(idx):
        return np.zeros((0, C.sizeof(T)), dtype=np.uint8)
    sz = C.sizeof(T)
    base = C.cast(src, C.c_void_p).value
    view = np.ctypeslib.as_array((C.c_uint8 * (sz * (int(idx.max()) + 1))).from_address(base)).reshape(-1, sz)
    return view[idx]


def _from_rows(rows, T):
    """ctypes array of T holding `rows` (a struct copy: pointers into the owners' memory stay valid)."""
    out = (T * max(1, len(rows)))()
    if len(rows):
        C.memmove(out, np.ascontiguousarray(rows).ctypes.data, rows.size)
    return out


def _gather(src, idx, T):
    """ctypes array of T copied from src[idx] (structs keep their pointers into src's owner)."""
    return _from_rows(_rows(src, T, idx), T)


def _u32(a):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return (C.c_uint32 * max(1, len(a)))(*a.tolist())


class BurstStream:
    """Seeded C5 stream: `n_bursts` bursts of `burst` pods on an `n_nodes` cluster.

    seeds = (nodes, pods, events); replacement / added node shapes come from a
    second node synth of the same kind (seed nodes + 1000)."""

    def __init__(self, kind, n_nodes, n_bursts, burst, seeds=(6, 7, 8), rates=Rates(), prefill=None):
        self.kind, self.n, self.n_bursts, self.burst = kind, n_nodes, n_bursts, burst
        self.nodes = synth.nodes(kind, n_nodes, seeds[0])
        self.pods = synth.pods(kind, n_bursts * burst, seeds[1])
        self.rng = np.random.default_rng(seeds[2])
        self.rates = rates
        n_pool = max(16, int(n_nodes * (rates.node_update + rates.node_delete) * n_bursts * 2) + 16)
        self.pool = synth.nodes(kind, n_pool, seeds[0] + 1000)
        self.pool_next = 0
        self.prefill = synth.prefill(kind, n_nodes, seeds[0], prefill, 0.5) if prefill is not None else None
        # bound pods: stream index (or -1 - prefill index) -> slot
        self.bound_pod = np.zeros(0, dtype=np.int64)
        self.bound_slot = np.zeros(0, dtype=np.int64)
        self.node_src = np.arange(n_nodes, dtype=np.int64)  # >= 0: self.nodes index, < 0: -1 - pool index
        # pool-derived nodes as actually upserted: node names are unique cluster-wide
        # (an update keeps the slot's name, an added node gets a fresh one)
        self.slot_node = {}
        self._names = []
        self.n_added = 0
        if self.prefill is not None:
            pf_slots = np.ctypeslib.as_array(self.prefill.slot_ptr, shape=(self.prefill.n_pods,)).astype(np.int64)
            self.bound_pod = -1 - np.arange(self.prefill.n_pods, dtype=np.int64)
            self.bound_slot = pf_slots.copy()

    # ---------------------------------------------------------------- setup
    def setup(self, targets):
        slots = synth.slot_array(self.n)
        for t in targets:
            t.upsert(self.nodes.nodes, slots, self.n)
            if self.prefill is not None:
                t.add_pods(self.prefill.pods, self.prefill.slot_ptr, self.prefill.n_pods)

    def burst_pods(self, b):
        return self.pods.pods_at(b * self.burst), self.burst

    def record(self, b, results):
        """Bind the scheduled pods of burst b (AssumePod -> bound)."""
        r = np.frombuffer(C.string_at(C.addressof(results), self.burst * C.sizeof(_abi.KsResult)),
                          dtype=np.dtype([("node_index", "<i4"), ("status", "<i4"), ("rest", f"V{C.sizeof(_abi.KsResult) - 8}")]))
        ok = np.nonzero(r["status"] == 0)[0]
        self.bound_pod = np.concatenate([self.bound_pod, b * self.burst + ok])
        self.bound_slot = np.concatenate([self.bound_slot, r["node_index"][ok].astype(np.int64)])

    # ---------------------------------------------------------------- events
    def _pod_struct_array(self, pods_idx):
        """ks_pod array of stream pods (index >= 0) and prefill pods (-1 - index), in order."""
        pods_idx = np.asarray(pods_idx, dtype=np.int64)
        rows = np.zeros((len(pods_idx), C.sizeof(_abi.KsPod)), dtype=np.uint8)
        own = pods_idx >= 0
        if own.any():
            rows[own] = _rows(self.pods.pods, _abi.KsPod, pods_idx[own])
        if (~own).any():
            rows[~own] = _rows(self.prefill.pods, _abi.KsPod, -1 - pods_idx[~own])
        return _from_rows(rows, _abi.KsPod)

    def make_events(self):
        """The event log after a burst (a list of (op, payload) in log order)."""
        ev = []
        nb = len(self.bound_pod)
        k = int(round(nb * self.rates.pod_delete))
        if k:
            pick = np.sort(self.rng.choice(nb, size=k, replace=False))
            ev.append(("remove_pods", (self.bound_pod[pick].copy(), self.bound_slot[pick].copy())))
            keep = np.ones(nb, dtype=bool)
            keep[pick] = False
            self.bound_pod, self.bound_slot = self.bound_pod[keep], self.bound_slot[keep]
        ku = int(round(self.n * self.rates.node_update))
        if ku:
            slots = np.sort(self.rng.choice(self.n, size=ku, replace=False))
            src = self._take_pool(ku)
            ev.append(("update_nodes", (slots, src)))
            self.node_src[slots] = -1 - src
        kd = int(round(self.n * self.rates.node_delete))
        if kd:
            slots = np.sort(self.rng.choice(self.n, size=kd, replace=False))
            ev.append(("delete_nodes", slots))
            gone = np.isin(self.bound_slot, slots)
            self.bound_pod, self.bound_slot = self.bound_pod[~gone], self.bound_slot[~gone]
            src = self._take_pool(kd)
            ev.append(("add_nodes", (slots, src)))
            self.node_src[slots] = -1 - src
        return ev

    def _take_pool(self, k):
        if self.pool_next + k > self.pool.n_nodes:
            raise RuntimeError("replacement node pool exhausted")
        src = np.arange(self.pool_next, self.pool_next + k, dtype=np.int64)
        self.pool_next += k
        return src

    def marshal(self, events):
        """The event log as ready-to-call ABI arrays (host-side marshalling, kept
        out of bench.py's timed region): a list of (op, arrays..., count)."""
        out = []
        for op, payload in events:
            if op == "remove_pods":
                pods_idx, slots = payload
                out.append((op, self._pod_struct_array(pods_idx), _u32(slots), len(slots)))
            elif op in ("update_nodes", "add_nodes"):
                slots, src = payload
                out.append((op, self._named(op, slots, src), _u32(slots), len(slots)))
            elif op == "delete_nodes":
                out.append((op, None, _u32(payload), len(payload)))
            else:
                raise ValueError(op)
        return out

    @staticmethod
    def event_log(ops):
        """The marshalled log as one ks_event array for ks_events_apply (the
        ordered delta feed): (array, count, keep-alive of the payloads)."""
        n = sum(o[3] for o in ops)
        ev = (_abi.KsEvent * max(1, n))()
        kinds = {"remove_pods": 1, "update_nodes": 2, "add_nodes": 2, "delete_nodes": 3}
        i = 0
        for op, arr, sl, m in ops:
            k = kinds[op]
            T = _abi.KsPod if k == 1 else _abi.KsNode
            for j in range(m):
                e = ev[i]
                e.kind = k
                e.slot = sl[j]
                if k == 1:
                    e.pod = C.cast(C.addressof(arr) + j * C.sizeof(T), C.POINTER(T))
                elif k == 2:
                    e.node = C.cast(C.addressof(arr) + j * C.sizeof(T), C.POINTER(T))
                i += 1
        return ev, n, ops

    @staticmethod
    def apply_marshalled(ops, targets):
        for op, arr, sl, n in ops:
            for t in targets:
                if op == "remove_pods":
                    t.remove_pods(arr, sl, n)
                elif op == "delete_nodes":
                    t.delete(sl, n)
                else:
                    t.upsert(arr, sl, n)

    def apply(self, events, targets):
        self.apply_marshalled(self.marshal(events), targets)

    def _slot_name(self, slot):
        if slot in self.slot_node:
            return self.slot_node[slot].name
        return self.nodes.nodes[int(slot)].name

    def _named(self, op, slots, src):
        """Pool nodes renamed: an update keeps the slot's node name, an add gets a new unique name."""
        arr = (_abi.KsNode * max(1, len(slots)))()
        for j, (slot, i) in enumerate(zip(slots.tolist(), src.tolist())):
            arr[j] = self.pool.nodes[i]
            if op == "update_nodes":
                name = self._slot_name(slot)
            else:
                name = f"added-node-{self.n_added}".encode()
                self.n_added += 1
            buf = C.create_string_buffer(name)  # kept alive with the stream
            self._names.append(buf)
            arr[j].name = C.cast(buf, C.c_char_p)
        for j, slot in enumerate(slots.tolist()):
            nd = _abi.KsNode()
            C.pointer(nd)[0] = arr[j]
            self.slot_node[slot] = nd
        return arr

    # ----------------------------------------------------------- rebuild
    def rebuild(self, target):
        """Load the stream's current cluster into a FRESH target from scratch:
        the live nodes, then every bound pod at its slot (checksum property)."""
        slots = np.arange(self.n)
        orig = self.node_src >= 0
        if orig.any():
            target.upsert(_gather(self.nodes.nodes, self.node_src[orig], _abi.KsNode), _u32(slots[orig]),
                          int(orig.sum()))
        if (~orig).any():
            rest = slots[~orig]
            arr = (_abi.KsNode * len(rest))()
            for j, slot in enumerate(rest.tolist()):
                arr[j] = self.slot_node[slot]
            target.upsert(arr, _u32(rest), len(rest))
        if len(self.bound_pod):
            target.add_pods(self._pod_struct_array(self.bound_pod), _u32(self.bound_slot), len(self.bound_pod))
