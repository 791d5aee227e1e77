"""The in-order commit of the round kernels, for
resource-only and for label / taint rounds: the parallel proposal / verify
kernel (ksched_resolve.hip), the
serial kernel, and the automatic hand-over between them, each bit-exact
against the CPU oracle's one-pod-at-a-time scheduling and against each other.

The cases target what makes the parallel commit hard:
* BalancedAllocation rising after a commit (a node becomes MORE attractive for
  the next pods once one pod lands on it), so a node taken earlier in the
  round wins again -- inside one chunk and across chunks;
* identical nodes and identical pods (the kwok shape): every pod piles onto
  the same few nodes, the deferred-acceptance proposals are wrong for most
  pods and AUTO hands the rounds to the serial kernel;
* short candidate lists (K = 1, 8, 16): lists run out and rounds stop early;
* zero-request pods (Fit never fails on resources, LeastAllocated uses the
  non-zero defaults) and pod-count limits (Fit fails once a node is full, the
  feasible counts change mid-round);
* several schedule calls, so node state carried between batches is checked.
Oracle: oracle/oracle.cpp (parity unpinned).
"""
import ctypes as C
import random

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array, states_np
from ksched import Scheduler, _abi, synth
from ksched.objects import Arena, nodes_array, pods_array
from scenarios import node, pod

pytestmark = pytest.mark.gpu

Gi = 1 << 30
MODES = {"auto": {"resolve_mode": _abi.RESOLVE_AUTO}, "serial": {"resolve_mode": _abi.RESOLVE_SERIAL},
         "parallel": {"resolve_mode": _abi.RESOLVE_PARALLEL},
         # AUTO with a low pass cap: every round that needs more than 2 passes
         # hands the next 3 rounds to the serial kernel
         "auto_cap": {"resolve_mode": _abi.RESOLVE_AUTO, "resolve_par_max_passes": 2, "resolve_serial_rounds": 3}}


def ba_rise_cluster(n, m, seed):
    """Nodes with CPU already half used and memory nearly free, pods that ask
    mostly for memory: each commit moves a node's memory fraction towards its
    CPU fraction, so its BalancedAllocation for the next such pod rises."""
    r = random.Random(seed)
    nodes, pre, pre_slots = [], [], []
    for i in range(n):
        cpu = r.choice([8, 16, 32]) * 1000
        mem = r.choice([32, 64, 128]) * Gi
        nodes.append(node(f"n{i}", cpu=cpu, mem=mem, pods=r.choice([8, 16, 110])))
        used = int(cpu * r.uniform(0.3, 0.7)) // 50 * 50
        pre.append(pod(f"pre{i}", cpu=used, mem=int(mem * r.uniform(0.0, 0.1)) // (1 << 20) << 20))
        pre_slots.append(i)
    pods = []
    for j in range(m):
        if r.random() < 0.15:
            pods.append(pod(f"be{j}"))  # no requests: non-zero defaults for LeastAllocated only
        else:
            pods.append(pod(f"p{j}", cpu=r.choice([50, 100, 200]), mem=r.choice([2, 4, 6, 8]) * Gi))
    return nodes, pre, pre_slots, pods


def pod_slice(pods_arr, b0):
    """Pointer to pods_arr[b0:] (pods_arr: a ctypes array or POINTER(KsPod))."""
    return C.cast(C.cast(pods_arr, C.c_void_p).value + int(b0) * C.sizeof(_abi.KsPod), C.POINTER(_abi.KsPod))


def run_modes(nodes_arr, n, pods_arr, m, pre=None, splits=1, modes=("auto", "serial", "parallel"), **kw):
    """Results + node states of every resolve mode and of the oracle."""
    slots = (C.c_uint32 * n)(*range(n))
    o = pyoracle.Oracle(n)
    o.upsert(nodes_arr, slots, n)
    if pre is not None:
        o.add_pods(*pre)
    bounds = np.linspace(0, m, splits + 1).astype(int)
    want = np.concatenate([res_array(o.schedule(pod_slice(pods_arr, b0), int(b1 - b0)), int(b1 - b0))
                           for b0, b1 in zip(bounds, bounds[1:])])
    wst = states_np(o.L.oracle_node_states, o.o, n)
    o.close()
    out = {}
    for mode in modes:
        with Scheduler(n, options=MODES[mode], **kw) as s:
            s.upsert_nodes_raw(nodes_arr, slots, n)
            if pre is not None:
                assert s.lib.ks_pods_add(s.ctx, *pre) == 0, s.lib.ks_last_error(s.ctx)
            got = []
            for b0, b1 in zip(bounds, bounds[1:]):
                k = int(b1 - b0)
                ptr = pod_slice(pods_arr, b0)
                got.append(res_array(s.schedule_raw(ptr, k), k))
            dbg = (C.c_uint64 * 16)()
            assert s.lib.ks_debug_counters(s.ctx, dbg) == 0
            out[mode] = (np.concatenate(got), states_np(s.lib.ks_node_states, s.ctx, n), list(dbg))
    return want, wst, out


def check_modes(want, wst, out, what):
    for mode, (got, st, _) in out.items():
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            i = int(bad[0])
            raise AssertionError(f"{what} [{mode}]: {len(bad)}/{len(want)} results differ; first at pod {i}: "
                                 f"got {got[i]} want {want[i]}")
        assert np.array_equal(st, wst), f"{what} [{mode}]: node states differ from the oracle"


@pytest.mark.parametrize("seed,n,m,P,K,splits", [
    (1, 300, 1200, 256, 256, 1),
    (2, 1000, 2000, 256, 64, 2),
    (3, 120, 900, 64, 16, 3),
    (4, 2000, 1500, 256, 8, 1),
    (5, 500, 1500, 100, 256, 2),
])
def test_balanced_allocation_rise(seed, n, m, P, K, splits):
    nodes, pre, pre_slots, pods = ba_rise_cluster(n, m, seed)
    a = Arena()
    na, _ = nodes_array(nodes, a)
    pa, _ = pods_array(pods, a)
    fa, nf = pods_array(pre, a)
    fs = (C.c_uint32 * nf)(*pre_slots)
    want, wst, out = run_modes(na, n, pa, m, pre=(fa, fs, nf), splits=splits, pods_per_round=P, topk=K)
    check_modes(want, wst, out, f"BA rise seed {seed}")
    # the workload does what it is for: some pods win a node an earlier pod of
    # the same round took (consecutive pods on one node)
    sched = want[want["status"] == 0]["node_index"]
    assert (sched[1:] == sched[:-1]).any()
    par_rounds = out["parallel"][2][13]
    assert par_rounds > 0, "the parallel kernel resolved no round"


@pytest.mark.parametrize("kind,pods,K", [("kwok", "besteffort", 256), ("kwok", "besteffort", 16), ("kwok", "c1", 512),
                                         ("kwok", "c1", 16), ("hetero", "c1", 256), ("hetero", "besteffort", 32)])
def test_synthetic_streams(kind, pods, K):
    n, m = 3000, 5000
    k = {"kwok": synth.KWOK, "hetero": synth.HETERO}[kind]
    ns = synth.nodes(k, n, 11)
    ps = synth.besteffort_pods(m) if pods == "besteffort" else synth.pods(synth.HETERO, m, 12)
    pf = synth.prefill(k, n, 11, 13, 0.4) if kind == "hetero" else None
    pre = (pf.pods, pf.slot_ptr, pf.n_pods) if pf is not None else None
    want, wst, out = run_modes(ns.nodes, n, ps.pods, m, pre=pre, splits=2, topk=K,
                               modes=("auto", "serial", "parallel", "auto_cap"))
    check_modes(want, wst, out, f"{kind}/{pods}/K={K}")
    # counters: [0] rounds, [12] parallel passes, [13] rounds the parallel
    # kernel resolved, [15] of those in one step (one class of request-less pods)
    par, cap = out["parallel"][2], out["auto_cap"][2]
    if pods == "besteffort":
        assert par[15] > 0, f"no round of identical request-less pods resolved in one step: {par}"
    assert par[13] == par[0], f"RESOLVE_PARALLEL left rounds to the serial kernel: {par}"
    if par[12] > 2 * par[0]:
        # some round needed more than 2 passes: the capped AUTO handed later rounds to the serial kernel
        assert cap[13] < cap[0], f"AUTO never handed a round to the serial kernel: {cap}"


def test_pod_count_limits_mid_round():
    # small pods per node: nodes fill up inside a round, so feasible counts and
    # Fit failure counts change between consecutive pods
    r = random.Random(7)
    nodes = [node(f"n{i}", cpu=64000, mem=256 * Gi, pods=r.choice([1, 2, 3])) for i in range(400)]
    pods = [pod(f"p{j}", cpu=r.choice([None, 100, 500]), mem=r.choice([None, Gi])) for j in range(1100)]
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    want, wst, out = run_modes(na, n, pa, m, splits=1)
    check_modes(want, wst, out, "pod-count limits")
    assert (want["status"] == 1).any(), "no pod ran out of nodes"


@pytest.mark.parametrize("shards", [1, 3])
def test_parallel_vs_serial_fuzz(shards):
    # random node / pod shapes, virtual shards, uneven splits: the two kernels
    # and the oracle agree on every field
    for seed in range(4):
        r = random.Random(100 * shards + seed)
        n = r.choice([97, 640, 1500])
        m = r.choice([300, 1000])
        nodes = [node(f"n{i}", cpu=r.choice([2, 4, 8, 16, 64]) * 1000, mem=r.choice([4, 16, 64, 256]) * Gi,
                      pods=r.choice([4, 16, 110])) for i in range(n)]
        pods = [pod(f"p{j}", cpu=r.choice([None, 0, 50, 250, 1000, 3000]),
                    mem=r.choice([None, 0, Gi // 4, Gi, 3 * Gi])) for j in range(m)]
        a = Arena()
        na, _ = nodes_array(nodes, a)
        pa, _ = pods_array(pods, a)
        P = r.choice([32, 128, 256])
        want, wst, out = run_modes(na, n, pa, m, splits=r.randrange(1, 4), modes=("serial", "parallel"),
                                   pods_per_round=P, topk=r.choice([P, 8, 64]), virtual_shards=shards)
        check_modes(want, wst, out, f"fuzz seed {seed} shards {shards}")


@pytest.mark.parametrize("K,P,shards,splits", [(256, 256, 1, 2), (16, 256, 1, 1), (64, 100, 3, 3), (512, 256, 1, 1)])
def test_labeled_streams_every_mode(K, P, shards, splits):
    # label / taint rounds (EXT: NodeAffinity required + preferred terms,
    # nodeSelectors, hard and PreferNoSchedule taints with their tolerations,
    # TaintToleration / NodeAffinity normalisation, FIX re-sweeps) through the
    # parallel commit, the serial kernel and the hand-over between them
    n, m = 4000, 3000
    ns = synth.nodes(synth.LABELED, n, 21)
    ps = synth.pods(synth.LABELED, m, 22)
    pf = synth.prefill(synth.LABELED, n, 21, 23, 0.5)
    want, wst, out = run_modes(ns.nodes, n, ps.pods, m, pre=(pf.pods, pf.slot_ptr, pf.n_pods), splits=splits,
                               modes=("auto", "serial", "parallel", "auto_cap"), pods_per_round=P, topk=K,
                               virtual_shards=shards)
    check_modes(want, wst, out, f"labeled K={K} P={P} shards={shards}")
    par = out["parallel"][2]
    assert par[0] > 0 and par[13] == par[0], f"RESOLVE_PARALLEL left label / taint rounds to the serial kernel: {par}"
    assert out["auto"][2][13] > 0, f"AUTO resolved no label / taint round in parallel: {out['auto'][2]}"
    assert (want["status"] == 0).any() and (want["status"] == 1).any()


def test_labeled_normaliser_edges_every_mode():
    # every pod normalises TaintToleration (PreferNoSchedule taints of 0-3
    # keys on every node) and most NodeAffinity (preferred terms), the nodes
    # at the taint max hold one pod each, and a few pods carry a nodeName or a
    # metadata.name PreFilterResult: normaliser drops stop rounds inside a
    # chunk of the parallel commit
    from ksched.objects import (NodeSelectorRequirement as Req, NodeSelectorTerm as Term,
                                PreferredSchedulingTerm as Pref, Taint)
    r = random.Random(31)
    keys = ["a", "b", "c"]
    nodes = []
    for i in range(700):
        tk = r.sample(keys, r.choice([0, 1, 1, 2, 3]))
        nodes.append(node(f"n{i}", cpu=r.choice([4, 8, 16]) * 1000, mem=r.choice([8, 16, 32]) * Gi,
                          pods=1 if len(tk) == 3 else r.choice([2, 3, 9]),
                          labels={"zone": f"z{i % 5}", "tier": r.choice(["a", "b"])},
                          taints=[Taint(k, "x", "PreferNoSchedule") for k in tk]))
    pods = []
    for j in range(1600):
        kw = {}
        if r.random() < 0.6:
            kw["preferred"] = [Pref(r.choice([1, 5, 20]), Term([Req("zone", "In", [f"z{r.randrange(5)}"])])),
                               Pref(r.choice([1, 3]), Term([Req("tier", "In", [r.choice(["a", "b"])])]))]
        if r.random() < 0.2:
            kw["node_selector"] = {"tier": r.choice(["a", "b"])}
        u = r.random()
        if u < 0.01:
            kw["node_name"] = f"n{r.randrange(700)}"
        elif u < 0.02:
            names = [f"n{r.randrange(700)}" for _ in range(3)]
            kw["required_terms"] = [Term(match_fields=[Req("metadata.name", "In", names)])]
        pods.append(pod(f"p{j}", cpu=r.choice([100, 500, 1000]), mem=r.choice([1, 2]) * Gi, **kw))
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    want, wst, out = run_modes(na, n, pa, m, splits=2, modes=("auto", "serial", "parallel"), pods_per_round=256,
                               topk=64)
    check_modes(want, wst, out, "labeled normaliser edges")
    par = out["parallel"][2]
    assert par[0] > 0 and par[13] == par[0], f"parallel commit counters {par}"


@pytest.mark.parametrize("mode", ["auto", "serial", "parallel"])
def test_normaliser_max_drops_mid_round(mode):
    # TaintToleration normalises by the max raw (untolerated PreferNoSchedule
    # taints) over the FEASIBLE nodes.  The only nodes at the max (two taints)
    # hold one pod each, and the round's first pods are steered onto them by
    # a nodeSelector: once they are full the max over feasible nodes drops
    # 2 -> 1 and every later pod's TaintToleration score changes on every
    # node.  The round must stop there and the rest be swept again, in the
    # serial and in the parallel commit.
    from ksched.objects import Taint
    p = lambda k: Taint(k, "true", "PreferNoSchedule")  # noqa: E731
    nodes = ([node(f"max{i}", pods=1, labels={"special": "yes"}, taints=[p("s"), p("t")]) for i in range(2)] +
             [node(f"one{i}", taints=[p("s")]) for i in range(30)] + [node(f"zero{i}") for i in range(30)])
    pods = ([pod(f"steer{i}", cpu=500, mem=Gi, node_selector={"special": "yes"}) for i in range(2)] +
            [pod(f"p{j}", cpu=250 * (1 + j % 4), mem=Gi) for j in range(120)])
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    want, wst, out = run_modes(na, n, pa, m, modes=(mode,), pods_per_round=256, topk=64)
    check_modes(want, wst, out, f"normaliser drop [{mode}]")
    assert sorted(want["node_index"][:2]) == [0, 1], "the steered pods did not fill the max nodes"
    rounds = out[mode][2][0]
    assert rounds >= 2, f"one round resolved all {m} pods: the normaliser drop did not stop it ({out[mode][2]})"


@pytest.mark.parametrize("K", [256, 8])
def test_identical_requestless_pods_fill_nodes(K):
    # one class of request-less pods (the one-step path): nodes hold 1-3 pods,
    # so nodes fill up inside a round (Fit losses change every later pod's
    # feasible count); with K = 8 the list runs out and rounds stop early
    r = random.Random(11)
    nodes = [node(f"n{i}", cpu=r.choice([4, 8, 16]) * 1000, mem=r.choice([8, 16]) * Gi, pods=r.choice([1, 2, 3]))
             for i in range(400)]
    pods = [pod(f"b{j}") for j in range(1000)]
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    want, wst, out = run_modes(na, n, pa, m, splits=2, modes=("auto", "serial"), topk=K)
    check_modes(want, wst, out, f"identical request-less pods K={K}")
    assert out["auto"][2][15] > 0, "the one-step path never ran"
    assert (want["status"] == 1).any(), "the cluster never filled up"


@pytest.mark.parametrize("shape", ["balanced", "ba_rise"])
def test_identical_pods_with_requests(shape):
    # one class of pods WITH requests (a deployment's replicas): the one-step
    # path applies only when every listed node's key sequence is
    # non-increasing.  "balanced": pods in the nodes' cpu:memory ratio on
    # empty nodes keep BalancedAllocation at 100, so it must apply;
    # "ba_rise": memory-heavy pods on nodes whose CPU is half used raise
    # BalancedAllocation, so those rounds fall back to the passes.  Both
    # bit-exact against the oracle.
    r = random.Random(23)
    if shape == "balanced":
        nodes = [node(f"n{i}", cpu=16000 * k, mem=64 * Gi * k, pods=110) for i, k in
                 enumerate(r.choice([1, 2, 4]) for _ in range(600))]
        pre = None
        pods = [pod(f"d{j}", cpu=500, mem=2 * Gi) for j in range(1500)]
    else:
        nodes, prepods, pre_slots, _ = ba_rise_cluster(600, 0, 23)
        pods = [pod(f"d{j}", cpu=100, mem=4 * Gi) for j in range(1500)]
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    if shape == "ba_rise":
        fa, nf = pods_array(prepods, a)
        pre = (fa, (C.c_uint32 * nf)(*pre_slots), nf)
    want, wst, out = run_modes(na, n, pa, m, pre=pre, splits=2, modes=("auto", "serial", "parallel"))
    check_modes(want, wst, out, f"identical pods with requests ({shape})")
    onestep = out["parallel"][2][15]
    if shape == "balanced":
        assert onestep > 0, f"the one-step path never ran: {out['parallel'][2]}"
