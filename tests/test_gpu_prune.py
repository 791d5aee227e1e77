"""Pruned sweeps and node relayouts at test sizes.

At the default pilot size (64 blocks per shard) only clusters of a few
hundred thousand nodes prune, so these cases open their contexts with
KS_PRUNE_PILOT=2: every round sweeps two pilot blocks, takes each pod's
threshold from their lists and skips scoring in blocks whose TotalScore bound
is below it.  Results, node states and the relayouts the node-event streams
trigger must leave every result bit-exact against the oracle.
"""
import os

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array, states_np
from ksched import Scheduler, synth

pytestmark = pytest.mark.gpu


def open_pruned(cap, pilot="2", kt=None, **cfg):
    env = {"KS_PRUNE_PILOT": pilot}
    if kt is not None:
        env["KS_PRUNE_KT"] = str(kt)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Scheduler(cap, **cfg)  # switches are read when the context opens
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def run_case(kind, n, m, seeds=(1, 2), prefill=True, calls=3, pilot="2", kt=None, **cfg):
    ns = synth.nodes(kind, n, seeds[0])
    ps = synth.pods(kind, m, seeds[1])
    slots = synth.slot_array(n)
    s = open_pruned(n, pilot, kt, **cfg)
    o = pyoracle.Oracle(n, threads=8)
    s.upsert_nodes_raw(ns.nodes, slots, n)
    o.upsert(ns.nodes, slots, n)
    if prefill:
        pf = synth.prefill(kind, n, seeds[0], 3, 0.5)
        assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
        o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
    cuts = [m * i // calls for i in range(calls + 1)]
    for i in range(calls):
        a, b = cuts[i], cuts[i + 1]
        assert_results_equal(s.schedule_raw(ps.pods_at(a), b - a), o.schedule(ps.pods_at(a), b - a), b - a,
                             f"call {i}")
    assert np.array_equal(states_np(s.lib.ks_node_states, s.ctx, n), states_np(o.L.oracle_node_states, o.o, n))
    st = s.stats()
    s.close()
    o.close()
    return st


def test_hetero_pruned():
    st = run_case(synth.HETERO, 30000, 4000)
    assert st.relayouts >= 1
    assert st.prune_pruned > 0 and st.prune_pairs > 0


@pytest.mark.parametrize("kt", [1, 8, 64])
def test_threshold_ranks(kt):
    # kt = 1: lists are cut right below the best pilot key (short lists, early round ends)
    run_case(synth.HETERO, 20000, 3000, seeds=(3, 4), pilot="4", kt=kt)


def test_labeled_pruned():
    # EXT sweep: Filter with label programs and normaliser maxima still measured in pruned blocks
    st = run_case(synth.LABELED, 20000, 2500, seeds=(4, 5))
    assert st.prune_pruned > 0


@pytest.mark.parametrize("P,K", [(64, 8), (256, 512), (1, 1)])
def test_round_shapes_pruned(P, K):
    run_case(synth.HETERO, 12000, 1500, seeds=(6, 7), pods_per_round=P, topk=K)


def test_kwok_ties_pruned():
    # identical nodes bound equal to their keys: nothing may be pruned wrongly at ties
    run_case(synth.KWOK, 16000, 5000, prefill=False, topk=512)


@pytest.mark.parametrize("shards", [2, 3])
def test_virtual_shards_pruned(shards):
    run_case(synth.LABELED, 24000, 1500, seeds=(8, 9), virtual_shards=shards)


@pytest.mark.parametrize("npl", [2, 8])
def test_nodes_per_lane_pruned(npl):
    run_case(synth.HETERO, 24000, 1500, seeds=(10, 11), nodes_per_lane=npl)


def test_relayout_after_events():
    # node deletes / re-adds and pod removals between batches trigger relayouts;
    # results stay exact across them
    n = 20000
    ns = synth.nodes(synth.HETERO, n, 12)
    slots = synth.slot_array(n)
    s = open_pruned(n)
    o = pyoracle.Oracle(n, threads=8)
    s.upsert_nodes_raw(ns.nodes, slots, n)
    o.upsert(ns.nodes, slots, n)
    rng = np.random.default_rng(5)
    for b in range(4):
        ps = synth.pods(synth.HETERO, 1500, 20 + b)
        got = s.schedule_raw(ps.pods, 1500)
        want = o.schedule(ps.pods, 1500)
        assert_results_equal(got, want, 1500, f"batch {b}")
        # remove some of this batch's pods and delete / re-add 2 % of the nodes
        r = res_array(got, 1500)
        idx = [int(i) for i in np.nonzero(r["status"] == 0)[0][::3]]
        import ctypes as C
        from ksched import _abi
        arr = (_abi.KsPod * len(idx))(*[ps.pods[i] for i in idx])
        sl = (C.c_uint32 * len(idx))(*[int(r["node_index"][i]) for i in idx])
        assert s.lib.ks_pods_remove(s.ctx, arr, sl, len(idx)) == 0
        o.remove_pods(arr, sl, len(idx))
        dele = sorted(set(int(x) for x in rng.choice(n, n // 50, replace=False)))
        dsl = (C.c_uint32 * len(dele))(*dele)
        assert s.lib.ks_nodes_delete(s.ctx, dsl, len(dele)) == 0
        o.delete(dsl, len(dele))
        ptr = C.cast(ns.nodes, C.POINTER(_abi.KsNode))
        re = (_abi.KsNode * len(dele))(*[ptr[i] for i in dele])
        assert s.lib.ks_nodes_upsert(s.ctx, re, dsl, len(dele)) == 0
        o.upsert(re, dsl, len(dele))
    assert np.array_equal(states_np(s.lib.ks_node_states, s.ctx, n), states_np(o.L.oracle_node_states, o.o, n))
    assert s.stats().relayouts >= 2
    s.close()
    o.close()
