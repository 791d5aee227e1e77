"""libksched (HIP) on the hand-built scenarios: bit-exact vs the oracle and
meeting the scenario expectations; plus the per-plugin score dump."""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array, scores_array, states_np
from ksched import Scheduler, _abi
from ksched.objects import Arena, nodes_array, pods_array
from scenarios import SCENARIOS, check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(SCENARIOS))
@pytest.mark.parametrize("P", [256, 2])
def test_scenario_gpu(name, P):
    nodes, pods, exp = SCENARIOS[name]()
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    slots = (C.c_uint32 * n)(*range(n))
    o = pyoracle.Oracle(n)
    o.upsert(na, slots, n)
    want = o.schedule(pa, m)
    with Scheduler(n, pods_per_round=P) as s:
        s.upsert_nodes_raw(na, slots, n)
        got = s.schedule_raw(pa, m)
    assert_results_equal(got, want, m, name)
    check(res_array(got, m), exp)


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_scenario_plugin_scores(name):
    nodes, pods, _ = SCENARIOS[name]()
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    slots = (C.c_uint32 * n)(*range(n))
    o = pyoracle.Oracle(n)
    o.upsert(na, slots, n)
    with Scheduler(n) as s:
        s.upsert_nodes_raw(na, slots, n)
        for j in range(m):
            p = C.cast(C.addressof(pa.contents) + j * C.sizeof(_abi.KsPod), C.POINTER(_abi.KsPod))
            out = (_abi.KsNodeScore * n)()
            assert s.lib.ks_plugin_scores(s.ctx, p, out) == 0
            assert np.array_equal(scores_array(out), scores_array(o.plugin_scores(p))), (name, j)


def test_allocatable_range_enforced():
    # the exact truncated LeastAllocated needs allocatable < 2^44
    from scenarios import node

    a = Arena()
    for cpu, mem, ok in [((1 << 44) - 1, (1 << 44) - 1, True), (1 << 44, 1, False), (1, 1 << 44, False)]:
        na, n = nodes_array([node("x", cpu=cpu, mem=mem)], a)
        with Scheduler(1) as s:
            st = s.lib.ks_nodes_upsert(s.ctx, na, (C.c_uint32 * 1)(0), 1)
            assert (st == 0) == ok, (cpu, mem, st)
            if not ok:
                assert st == _abi.KS_ERR_RANGE if hasattr(_abi, "KS_ERR_RANGE") else st == 5


def test_upsert_rejects_duplicate_names_atomically():
    # metadata.name is unique; a rejected call leaves the cache unchanged
    from scenarios import node

    a = Arena()
    na, n = nodes_array([node("a"), node("b")], a)
    with Scheduler(4) as s:
        assert s.lib.ks_nodes_upsert(s.ctx, na, (C.c_uint32 * 2)(0, 1), 2) == 0
        dup, _ = nodes_array([node("c", cpu=1000), node("a", cpu=1000)], a)
        assert s.lib.ks_nodes_upsert(s.ctx, dup, (C.c_uint32 * 2)(2, 3), 2) == 1  # KS_ERR_INVALID
        st = s.node_states([0, 1, 2, 3])
        assert [x.pod_count for x in st] == [0, 0, -1, -1]
        same, _ = nodes_array([node("a", cpu=1000)], a)  # an update keeps the name on its slot
        assert s.lib.ks_nodes_upsert(s.ctx, same, (C.c_uint32 * 1)(0), 1) == 0
        assert s.node_states([0])[0].alloc_milli_cpu == 1000


@pytest.mark.parametrize("tuple_guess,fixes", [("0", 3), ("1", 2)])
def test_wrong_normaliser_guess_is_reswept(tuple_guess, fixes, monkeypatch):
    # normalizer_guess_wrong: with the simple guesses (worst prefer-taint word,
    # sum of the preferred weights the pod's nodeSelector does not rule out)
    # pods x, pref and pref-one-feasible are scored with a wrong max first
    # (pref-one-feasible's NodeAffinity guess is right -- its zone=z2 term is
    # ruled out by nodeSelector zone=z1 -- but its TaintToleration guess is
    # not) and the FIX-mode sweep must run for exactly those; the node-tuple
    # guesses (tuple_guess, default) get pref-one-feasible right, and x and
    # pref stay wrong (their worst node fails on resources, which tuples do
    # not see)
    nodes, pods, exp = SCENARIOS["normalizer_guess_wrong"]()
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    slots = (C.c_uint32 * n)(*range(n))
    o = pyoracle.Oracle(n)
    o.upsert(na, slots, n)
    want = o.schedule(pa, m)
    with Scheduler(n, options={"tuple_guess": int(tuple_guess)}) as s:
        s.upsert_nodes_raw(na, slots, n)
        got = s.schedule_raw(pa, m)
        dbg = (C.c_uint64 * 16)()
        assert s.lib.ks_debug_counters(s.ctx, dbg) == 0
    assert_results_equal(got, want, m, "normalizer_guess_wrong")
    check(res_array(got, m), exp)
    assert dbg[4] == fixes, list(dbg)


def test_event_log_mixed_kinds_in_order():
    # one ks_events_apply log mixing every kind, with order dependence (a pod
    # added to a node that is deleted, re-added and updated in the same log)
    # equals the oracle applying the same events one call at a time
    from scenarios import node, pod

    Gi = 1 << 30
    a = Arena()
    na, n = nodes_array([node(f"n{i}") for i in range(6)], a)
    fresh, _ = nodes_array([node("new2", cpu=8000, mem=16 * Gi), node("n3", cpu=64000, pods=110)], a)
    pa, _ = pods_array([pod("p1", cpu=1500, mem=2 * Gi), pod("p2", cpu=300), pod("be")], a)
    slots = (C.c_uint32 * n)(*range(n))
    o = pyoracle.Oracle(n)
    o.upsert(na, slots, n)
    log = [  # (kind, slot, pod index, node index)
        (_abi.KS_EV_POD_ADD, 1, 0, None), (_abi.KS_EV_POD_ADD, 2, 1, None), (_abi.KS_EV_POD_ADD, 2, 2, None),
        (_abi.KS_EV_NODE_DELETE, 2, None, None), (_abi.KS_EV_NODE_UPSERT, 2, None, 0),
        (_abi.KS_EV_POD_ADD, 2, 0, None), (_abi.KS_EV_POD_REMOVE, 1, 0, None),
        (_abi.KS_EV_NODE_UPSERT, 3, None, 1), (_abi.KS_EV_POD_ADD, 3, 2, None), (_abi.KS_EV_POD_ADD, 3, 2, None),
    ]
    ev = (_abi.KsEvent * len(log))()
    for i, (k, sl, pi, ni) in enumerate(log):
        ev[i].kind, ev[i].slot = k, sl
        if pi is not None:
            ev[i].pod = C.pointer(pa[pi])
        if ni is not None:
            ev[i].node = C.pointer(fresh[ni])
        one = (C.c_uint32 * 1)(sl)
        if k == _abi.KS_EV_POD_ADD:
            o.add_pods(C.pointer(pa[pi]), one, 1)
        elif k == _abi.KS_EV_POD_REMOVE:
            o.remove_pods(C.pointer(pa[pi]), one, 1)
        elif k == _abi.KS_EV_NODE_UPSERT:
            o.upsert(C.pointer(fresh[ni]), one, 1)
        else:
            o.delete(one, 1)
    with Scheduler(n) as s:
        s.upsert_nodes_raw(na, slots, n)
        assert s.lib.ks_events_apply(s.ctx, ev, len(log)) == 0, s.lib.ks_last_error(s.ctx)
        got = states_np(s.lib.ks_node_states, s.ctx, n)
        want = states_np(o.L.oracle_node_states, o.o, n)
        assert np.array_equal(got, want), (got, want)
        bad = (_abi.KsEvent * 1)()
        bad[0].kind = 7
        assert s.lib.ks_events_apply(s.ctx, bad, 1) == _abi.KS_ERR_INVALID
        assert b"unknown kind" in s.lib.ks_last_error(s.ctx)


@pytest.mark.parametrize("early", ["1", "0"])
def test_fix_list_spans_several_groups(early, monkeypatch):
    # More than 128 pods of one 256-pod round carry a preferred term no node
    # matches: their guessed NodeAffinity max (the term weight) is wrong (the
    # measured max is 0), so the compacted FIX list spans 3+ groups of MAX_PG.
    # Interleaved with pods whose guess is right, and with a PreferNoSchedule
    # taint so TaintToleration normalises too.  early_fix = 0 runs the FIX
    # sweep behind the merge (the multi-rank order) on one rank.
    from ksched.objects import NodeSelectorRequirement as R, NodeSelectorTerm as T, \
        PreferredSchedulingTerm as PT, Taint
    from scenarios import node, pod

    Gi = 1 << 30
    nodes = [node(f"n{i}", cpu=(8 + 8 * (i % 5)) * 1000, mem=(32 << (i % 4)) * Gi,
                  labels={"zone": f"z{i % 3}", "disk": "ssd" if i % 4 == 0 else "hdd"},
                  taints=[Taint("spot", "true", "PreferNoSchedule")] if i % 7 == 0 else [])
             for i in range(300)]
    pods = []
    flagged = 0
    for j in range(600):
        if j % 5 != 0:  # preferred term matching nothing: guess = weight, true max = 0
            pref = [PT(1 + j % 90, T([R("gpu", "Exists")]))]
            flagged += 1
        else:  # matches some feasible node: the guess (sum of weights) is right
            pref = [PT(10, T([R("disk", "In", ["ssd"])]))]
        pods.append(pod(f"p{j}", cpu=100 + 37 * (j % 23), mem=(1 + j % 7) * Gi // 4, preferred=pref))
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    slots = (C.c_uint32 * n)(*range(n))
    o = pyoracle.Oracle(n)
    o.upsert(na, slots, n)
    want = o.schedule(pa, m)
    # simple guesses (tuple_guess 0): every no-match term is guessed wrong
    with Scheduler(n, pods_per_round=256, options={"early_fix": int(early), "tuple_guess": 0}) as s:
        s.upsert_nodes_raw(na, slots, n)
        got = s.schedule_raw(pa, m)
        dbg = (C.c_uint64 * 16)()
        assert s.lib.ks_debug_counters(s.ctx, dbg) == 0
    assert_results_equal(got, want, m, f"fix groups (early={early})")
    # every flagged pod is re-swept at least once (a pod of a stopped round may be re-swept again)
    assert dbg[4] >= flagged, (list(dbg), flagged)
