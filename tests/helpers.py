"""Shared comparison helpers for parity tests (oracle vs libksched)."""
import ctypes as C
import threading

import numpy as np

from ksched import _abi

RES_DT = np.dtype([("node_index", "<i4"), ("status", "<i4"), ("total_score", "<i8"), ("feasible", "<u4"),
                   ("evaluated", "<u4"), ("fail", "<u4", (8,)), ("flags", "<u4"), ("_pad", "<u4")])


def res_array(raw, n):
    return np.frombuffer(C.string_at(C.addressof(raw), n * C.sizeof(_abi.KsResult)), dtype=RES_DT).copy()


def assert_results_equal(got, want, n, what=""):
    g, w = res_array(got, n), res_array(want, n)
    if not np.array_equal(g, w):
        bad = np.nonzero(g != w)[0]
        i = int(bad[0])
        raise AssertionError(
            f"{what}: {len(bad)}/{n} results differ; first at pod {i}: got {g[i]} want {w[i]}")


def state_array(states):
    return np.array([(s.alloc_milli_cpu, s.alloc_memory, s.req_milli_cpu, s.req_memory, s.nonzero_milli_cpu,
                      s.nonzero_memory, s.alloc_pods, s.pod_count) for s in states], dtype=np.int64)


def scores_array(scores):
    return np.array([(s.status, s.least_allocated, s.balanced_allocation, s.taint_raw, s.taint_score,
                      s.affinity_raw, s.affinity_score, s.image_locality, s.spread_raw, s.spread_score,
                      s.affinity_pod_raw, s.affinity_pod_score, s.total_score) for s in scores],
                    dtype=np.int64)


STATE_DT = np.dtype([("alloc_cpu", "<i8"), ("alloc_mem", "<i8"), ("req_cpu", "<i8"), ("req_mem", "<i8"),
                     ("nz_cpu", "<i8"), ("nz_mem", "<i8"), ("alloc_pods", "<i4"), ("pod_count", "<i4")])


def states_np(fn, ctx, n):
    """All n slots' ks_node_state via ks_node_states / oracle_node_states(ctx, slots, n, out), as numpy."""
    slots = np.arange(n, dtype=np.uint32)
    out = (_abi.KsNodeState * max(1, n))()
    st = fn(ctx, slots.ctypes.data_as(C.POINTER(C.c_uint32)), n, out)
    assert st == 0, f"node_states failed ({st})"
    return np.frombuffer(C.string_at(C.addressof(out), n * C.sizeof(_abi.KsNodeState)), dtype=STATE_DT).copy()


class OracleTarget:
    """The C++ oracle (oracle/pyoracle.py) behind the C5 stream driver's target
    interface (ksched.stream.GpuTarget): the stream replays against both."""

    def __init__(self, o):
        self.o = o
        for name in ("upsert", "delete", "add_pods", "remove_pods", "schedule"):
            setattr(self, name, getattr(o, name))

    def states(self, slots):
        return self.o.node_states(slots)


def on_threads(fns):
    """Run the callables on threads and return their results (libksched's and
    the oracle's ctypes calls release the GIL, so per-rank setup runs side by
    side); the first error is raised."""
    out, errs = [None] * len(fns), []

    def go(i):
        try:
            out[i] = fns[i]()
        except Exception as e:  # noqa: BLE001 -- re-raised below
            errs.append(e)

    th = [threading.Thread(target=go, args=(i,)) for i in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return out


class Background:
    """One callable on a thread, its result fetched later (the oracle's 1M-node
    setup overlaps the GPU work)."""

    def __init__(self, fn):
        self._out, self._err = [], []

        def run():
            try:
                self._out.append(fn())
            except Exception as e:  # noqa: BLE001 -- re-raised by get()
                self._err.append(e)
        self._t = threading.Thread(target=run)
        self._t.start()

    def get(self):
        self._t.join()
        if self._err:
            raise self._err[0]
        return self._out[0]
