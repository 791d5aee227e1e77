"""Identical pods of a round swept once (RoundArgs::cls).

Resource-only batches whose pods repeat byte-identical descriptors (the
reference's own benchmark pods are all alike: kwok/make_pods/main.go:138-148
creates request-less pods from one template) sweep, merge, gather and patch
each class once per round window; every pod of the class reads that record.
Parity: bit-exact results and node states against the CPU oracle, and against
the same library with the deduplication switched off (dedup_identical_pods = 0), over
duplicate densities from "every pod alike" to a few repeats, round geometries
with early stops (short lists) and wasted speculative rounds, virtual shards,
and calls split so that classes straddle round windows.
"""
import ctypes as C
import os
import random

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array, states_np
from ksched import Scheduler, _abi, synth

pytestmark = pytest.mark.gpu


def repeated(src, idx):
    """A pod array whose pod j is a copy of src's pod idx[j]."""
    arr = (_abi.KsPod * len(idx))()
    for j, i in enumerate(idx):
        arr[j] = src.pods[i]
    return arr


def run_pair(ns, n, pods, m, splits=1, dedup=True, opts=None, **kw):
    """libksched results + node states for `pods`, with or without dedup
    (ks_config execution options)."""
    s = Scheduler(n, options=dict(opts or {}, dedup_identical_pods=1 if dedup else 0), **kw)
    try:
        s.upsert_nodes_raw(ns.nodes, synth.slot_array(n), n)
        bounds = np.linspace(0, m, splits + 1).astype(int)
        out = []
        for b0, b1 in zip(bounds, bounds[1:]):
            k = int(b1 - b0)
            ptr = C.cast(C.addressof(pods) + int(b0) * C.sizeof(_abi.KsPod), C.POINTER(_abi.KsPod))
            out.append(res_array(s.schedule_raw(ptr, k), k))
        return np.concatenate(out), states_np(s.lib.ks_node_states, s.ctx, n)
    finally:
        s.close()


def oracle_run(ns, n, pods, m):
    o = pyoracle.Oracle(n)
    o.upsert(ns.nodes, synth.slot_array(n), n)
    ptr = C.cast(C.addressof(pods), C.POINTER(_abi.KsPod))
    got = res_array(o.schedule(ptr, m), m)
    return got, states_np(o.L.oracle_node_states, o.o, n)


E = {"tuple_guess": 0}   # plain normaliser guesses: FIX re-sweeps happen
M = {"early_fix": 0}     # normaliser maxima measured by the merge
CASES = [
    # node kind, pod kind, nodes, pods, distinct shapes, P, K, virtual shards, splits, options
    (synth.KWOK, synth.HETERO, 2000, 3000, 1, 256, 256, 1, 1, None),   # every pod alike (the published workload)
    (synth.KWOK, synth.HETERO, 1500, 2000, 3, 64, 16, 2, 3, None),     # short lists: rounds stop early
    (synth.HETERO, synth.HETERO, 3000, 2500, 8, 256, 256, 1, 2, None),
    (synth.HETERO, synth.HETERO, 2048, 1800, 40, 100, 64, 3, 1, None),
    (synth.HETERO, synth.HETERO, 700, 1200, 2, 256, 8, 1, 4, None),    # lists of 8: wasted speculative rounds
    # labeled pods (EXT batches: taints, selectors, affinity, normalisation)
    (synth.LABELED, synth.LABELED, 3000, 2000, 12, 256, 256, 1, 2, None),
    (synth.LABELED, synth.LABELED, 2048, 1500, 30, 128, 64, 2, 1, E),
    (synth.LABELED, synth.LABELED, 2500, 1500, 6, 256, 256, 1, 1, M),
    (synth.LABELED, synth.LABELED, 1200, 1000, 4, 64, 16, 1, 3, E),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_dedup_equals_oracle_and_undeduplicated(case):
    kn, kp, n, m, shapes, P, K, shards, splits, opts = CASES[case]
    ns = synth.nodes(kn, n, 31 + case)
    src = synth.pods(kp, max(shapes, 1), 41 + case)
    r = random.Random(case)
    idx = [r.randrange(shapes) for _ in range(m)]
    pods = repeated(src, idx)
    kw = dict(pods_per_round=P, topk=K, virtual_shards=shards)
    got, gst = run_pair(ns, n, pods, m, splits, True, opts, **kw)
    ref, rst = run_pair(ns, n, pods, m, splits, False, opts, **kw)
    want, wst = oracle_run(ns, n, pods, m)
    what = f"case {CASES[case]}"
    assert_results_equal_np(got, want, f"{what} dedup vs oracle")
    assert_results_equal_np(ref, want, f"{what} no dedup vs oracle")
    assert np.array_equal(gst, wst), f"{what}: node states differ from the oracle"
    assert np.array_equal(gst, rst), f"{what}: node states differ with / without dedup"


def assert_results_equal_np(g, w, what):
    if not np.array_equal(g, w):
        bad = np.nonzero(g != w)[0]
        i = int(bad[0])
        raise AssertionError(f"{what}: {len(bad)}/{len(g)} results differ; first at pod {i}: got {g[i]} want {w[i]}")


def test_besteffort_stream_vs_oracle():
    # ksynth's request-less pods (the bench's kwok-be line) on prefilled kwok nodes
    n, m = 4000, 6000
    ns = synth.nodes(synth.KWOK, n, 5)
    ps = synth.besteffort_pods(m)
    pf = synth.prefill(synth.KWOK, n, 5, 6, 0.4)
    o = pyoracle.Oracle(n)
    o.upsert(ns.nodes, synth.slot_array(n), n)
    o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
    with Scheduler(n) as s:
        s.upsert_nodes_raw(ns.nodes, synth.slot_array(n), n)
        assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0, s.lib.ks_last_error(s.ctx)
        assert_results_equal(s.schedule_raw(ps.pods, m), o.schedule(ps.pods, m), m, "best-effort stream")
        assert np.array_equal(states_np(s.lib.ks_node_states, s.ctx, n),
                              states_np(o.L.oracle_node_states, o.o, n))
