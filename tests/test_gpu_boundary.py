"""The drop-in boundary's admission rules and its asynchronous form.

* Pods carrying a feature whose plugin ksched does not model are refused with
  KS_ERR_UNSUPPORTED (ks_pods_check names each, ks_batch_prepare fails), never
  scheduled approximately: host ports (NodePorts), topology spread the caller
  could not express, pod (anti-)affinity (InterPodAffinity), volumes, a
  nominated node, resource claims; any batch while a bound pod carries pod
  (anti-)affinity; percentageOfNodesToScore below 100 with more than one shard
  at ks_open (below 100 on one shard runs the window pass).
* A batch that resolved node names goes stale when the node set changes.
* ks_batch_submit / ks_batch_wait give the results of sequential ks_batch_run
  calls, with the next batch compiled while the previous one runs.
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array
from ksched import Scheduler, _abi, synth
from ksched.objects import Arena, NodeSelectorRequirement as R, NodeSelectorTerm as T, nodes_array, pods_array
from scenarios import node, pod

pytestmark = pytest.mark.gpu


def small_cluster(s, n=8, images=None):
    a = Arena()
    nodes = [node(f"n{i}") for i in range(n)]
    if images:
        for i, im in images.items():
            nodes[i].images = list(im)
    na, _ = nodes_array(nodes, a)
    assert s.lib.ks_nodes_upsert(s.ctx, na, (C.c_uint32 * n)(*range(n)), n) == 0
    return a


@pytest.mark.parametrize("feature", sorted(_abi.UNMODELLED))
def test_unmodelled_feature_is_refused(feature):
    with Scheduler(8) as s:
        a = small_cluster(s)
        pods = [pod("ok", cpu=100), pod("x", cpu=100, unmodelled=[feature]), pod("ok2")]
        pa, m = pods_array(pods, a)
        st = (C.c_int32 * m)()
        assert s.lib.ks_pods_check(s.ctx, pa, m, st) == _abi.KS_ERR_UNSUPPORTED
        assert list(st) == [0, _abi.KS_ERR_UNSUPPORTED, 0]
        assert b"pod 1" in s.lib.ks_last_error(s.ctx)
        out = (_abi.KsResult * m)()
        assert s.lib.ks_schedule(s.ctx, pa, m, out) == _abi.KS_ERR_UNSUPPORTED
        # nothing was committed by the refused call
        assert all(x.pod_count == 0 for x in s.node_states(list(range(8))))


def test_image_on_a_node_is_admitted():
    # ImageLocality is modelled (one-pod path): pods whose images nodes report are admitted
    with Scheduler(8) as s:
        a = small_cluster(s, images={3: [("busybox", 5 << 20), ("registry.k8s.io/pause:3.9", 1 << 20)]})
        from ksched.objects import Container, Pod
        tag = Pod("tag", containers=[Container({"cpu": 100}, image="busybox:latest")])
        pa, m = pods_array([tag], a)
        st = (C.c_int32 * m)()
        assert s.lib.ks_pods_check(s.ctx, pa, m, st) == 0


def test_bound_pod_with_pod_affinity_blocks_batches_until_removed():
    with Scheduler(8) as s:
        a = small_cluster(s)
        bound, _ = pods_array([pod("anti", cpu=100, unmodelled=["pod_affinity"])], a)
        pa, m = pods_array([pod("p", cpu=100)], a)
        st = (C.c_int32 * 1)()
        assert s.lib.ks_pods_check(s.ctx, pa, 1, st) == 0
        assert s.lib.ks_pods_add(s.ctx, bound, (C.c_uint32 * 1)(2), 1) == 0
        assert s.lib.ks_pods_check(s.ctx, pa, 1, st) == _abi.KS_ERR_UNSUPPORTED
        assert b"InterPodAffinity" in s.lib.ks_last_error(s.ctx)
        assert s.lib.ks_pods_remove(s.ctx, bound, (C.c_uint32 * 1)(2), 1) == 0
        assert s.lib.ks_pods_check(s.ctx, pa, 1, st) == 0


# below 100: the window pass on one shard (tests/test_gpu_pct.py);
# with more than one shard refused
@pytest.mark.parametrize("pct,shards,status", [(100, 1, 0), (5, 1, 0), (0, 1, 0), (5, 2, _abi.KS_ERR_UNSUPPORTED),
                                               (101, 1, _abi.KS_ERR_INVALID), (-1, 1, _abi.KS_ERR_INVALID)])
def test_percentage_of_nodes_to_score(pct, shards, status):
    lib = _abi.ksched_lib()
    cfg = _abi.KsConfig()
    lib.ks_config_default(C.byref(cfg))
    assert cfg.percentage_of_nodes_to_score == 100
    cfg.node_capacity = 16
    cfg.virtual_shards = shards
    cfg.percentage_of_nodes_to_score = pct
    ctx = C.c_void_p()
    assert lib.ks_open(C.byref(cfg), C.byref(ctx)) == status
    if status == 0:
        lib.ks_close(ctx)


def test_batch_naming_nodes_goes_stale_when_nodes_change():
    with Scheduler(16) as s:
        a = small_cluster(s)
        named, _ = pods_array([pod("by-name", cpu=100, node_name="n3")], a)
        plain, _ = pods_array([pod("plain", cpu=100)], a)
        b1, b2 = s.prepare(named, 1), s.prepare(plain, 1)
        na, _ = nodes_array([node("n8")], a)
        assert s.lib.ks_nodes_upsert(s.ctx, na, (C.c_uint32 * 1)(8), 1) == 0  # a new node name
        assert s.lib.ks_batch_run(s.ctx, b1) == _abi.KS_ERR_STALE
        assert s.lib.ks_batch_run(s.ctx, b2) == 0  # no name resolved: still valid
        s.free(b1)
        s.free(b2)


def test_prefilter_counts_nodes_outside_the_result():
    with Scheduler(8) as s:
        a = small_cluster(s)
        p = pod("named", cpu=100, required_terms=[T(match_fields=[R("metadata.name", "In", ["n5", "zz"])])])
        pa, _ = pods_array([p], a)
        r = res_array(s.schedule_raw(pa, 1), 1)[0]
        # both values enter the PreFilterResult; Filter rejects the two-value
        # term (parse error), so n5 fails NodeAffinity and 7 nodes are prefiltered
        assert r["status"] == 1 and list(r["fail"]) == [0, 0, 0, 1, 0, 0, 0, 7]


def test_async_submit_equals_sequential_runs():
    n, per, nb = 20_000, 3_000, 5
    nodes = synth.nodes(synth.LABELED, n, 1)
    pf = synth.prefill(synth.LABELED, n, 1, 3, 0.5)
    pods = synth.pods(synth.LABELED, per * nb, 2)
    out = []
    for mode in ("sync", "async"):
        s = Scheduler(n)
        s.upsert_nodes_raw(nodes.nodes, synth.slot_array(n), n)
        assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
        res = []
        if mode == "sync":
            for k in range(nb):
                b = s.prepare(pods.pods_at(k * per), per)
                s.run(b)
                res.append(res_array(s.results(b, per), per))
                s.free(b)
        else:
            # compile batch k+1 while batch k runs; two in flight at a time
            b = s.prepare(pods.pods_at(0), per)
            assert s.lib.ks_batch_submit(s.ctx, b) == 0
            for k in range(nb):
                nxt = None
                if k + 1 < nb:
                    nxt = s.prepare(pods.pods_at((k + 1) * per), per)
                    assert s.lib.ks_batch_submit(s.ctx, nxt) == 0
                assert s.lib.ks_batch_wait(s.ctx, b) == 0, s.lib.ks_last_error(s.ctx)
                res.append(res_array(s.results(b, per), per))
                s.free(b)
                b = nxt
        out.append(np.concatenate(res))
        s.close()
    assert np.array_equal(out[0], out[1])
    # and the oracle agrees on the first batch
    o = pyoracle.Oracle(n, threads=16)
    o.upsert(nodes.nodes, synth.slot_array(n), n)
    o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
    want = res_array(o.schedule(pods.pods, 600), 600)
    assert np.array_equal(out[1][:600], want)


def test_batch_pool_reuses_buffers_and_results_survive_other_runs():
    with Scheduler(64) as s:
        a = small_cluster(s, n=64)
        pa, m = pods_array([pod(f"p{i}", cpu=100 + i) for i in range(40)], a)
        b1 = s.prepare(pa, m)
        s.run(b1)
        r1 = res_array(s.results(b1, m), m)
        b2 = s.prepare(pa, 20)  # a second batch while b1 is held
        s.run(b2)
        assert np.array_equal(res_array(s.results(b1, m), m), r1)  # b1's results unchanged
        s.free(b2)
        b3 = s.prepare(pa, 10)  # reuses b2's buffers
        assert b3.value == b2.value
        s.free(b3)
        s.free(b1)


def test_label_dictionary_reclaim_streams_beyond_256_bits():
    # Batches over time use 480 distinct nodeSelector pairs (the label words
    # hold 256 bits): the dictionary restarts empty when a batch cannot get
    # its bits, nodes are re-encoded, and every batch still equals the oracle
    from ksched.objects import Taint
    n = 1200
    nodes = [node(f"n{i}", cpu=8000 + 1000 * (i % 9), labels={"k": f"v{i % 480}", "z": f"z{i % 7}"},
                  taints=[Taint("t", "x", "NoSchedule")] if i % 11 == 0 else [])
             for i in range(n)]
    a = Arena()
    na, _ = nodes_array(nodes, a)
    slots = (C.c_uint32 * n)(*range(n))
    o = pyoracle.Oracle(n)
    o.upsert(na, slots, n)
    with Scheduler(n) as s:
        s.upsert_nodes_raw(na, slots, n)
        for b in range(8):
            pods = [pod(f"p{b}-{j}", cpu=100 + j, node_selector={"k": f"v{(b * 60 + j) % 480}"},
                        required_terms=[T([R("z", "NotIn", [f"z{(b + j) % 7}"])])] if j % 3 == 0 else None)
                    for j in range(60)]
            pa, m = pods_array(pods, a)
            assert_results_equal(s.schedule_raw(pa, m), o.schedule(pa, m), m, f"batch {b}")
        dbg = (C.c_uint64 * 16)()
        assert s.lib.ks_debug_counters(s.ctx, dbg) == 0
        assert dbg[5] >= 1, list(dbg)  # the label dictionary was reclaimed


def test_taint_dictionary_rebuild_after_churn():
    # 100 distinct NoSchedule taints over the cluster's life, at most 12 live:
    # the 64-bit taint words are rebuilt from the present nodes
    from ksched.objects import Taint, Toleration
    n = 40
    a = Arena()
    o = pyoracle.Oracle(n)
    with Scheduler(n) as s:
        slots = (C.c_uint32 * n)(*range(n))
        for gen in range(10):
            nodes = [node(f"n{i}", taints=[Taint(f"t{gen * 10 + i % 12}", "", "NoSchedule")] if i % 3 else [])
                     for i in range(n)]
            na, _ = nodes_array(nodes, a)
            assert s.lib.ks_nodes_upsert(s.ctx, na, slots, n) == 0, s.lib.ks_last_error(s.ctx)
            o.upsert(na, slots, n)
            pods = [pod(f"p{gen}-{j}", cpu=200, tolerations=[Toleration(f"t{gen * 10 + j % 12}", "Exists")])
                    for j in range(30)]
            pa, m = pods_array(pods, a)
            assert_results_equal(s.schedule_raw(pa, m), o.schedule(pa, m), m, f"generation {gen}")
        dbg = (C.c_uint64 * 16)()
        assert s.lib.ks_debug_counters(s.ctx, dbg) == 0
        assert dbg[6] >= 1, list(dbg)


def test_node_range_errors_fail_their_own_item_only():
    # ks_nodes_upsert_each: a node whose memory allocatable is >= 2^44
    # (LeastAllocated's exact-floor bound) fails alone with
    # KS_ERR_RANGE; the others -- a 20 TiB ephemeral-storage node among them,
    # which only Fit compares, in exact int64 -- are applied and scheduled
    # bit-exact against the oracle holding the same nodes.  ks_nodes_upsert
    # applies nothing from the same call.
    from ksched.objects import Container, Node, Pod

    Gi, Ti = 1 << 30, 1 << 40
    nodes = [Node(f"n{i}", {"cpu": 16000, "memory": 64 * Gi, "pods": 110}, {}, [], False) for i in range(6)]
    nodes[3] = Node("n3", {"cpu": 16000, "memory": 1 << 45, "pods": 110}, {}, [], False)
    nodes[5] = Node("n5", {"cpu": 16000, "memory": 64 * Gi, "pods": 110}, {}, [], False,
                    extended={"ephemeral-storage": 20 * Ti})
    a = Arena()
    na, n = nodes_array(nodes, a)
    slots = (C.c_uint32 * n)(*range(n))
    with Scheduler(n) as s:
        assert s.lib.ks_nodes_upsert(s.ctx, na, slots, n) == 5  # KS_ERR_RANGE: the whole call refused
        st = s.node_states(list(range(n)))
        assert all(x.pod_count == -1 for x in st), "ks_nodes_upsert applied part of a refused call"
        status = (C.c_int32 * n)()
        assert s.lib.ks_nodes_upsert_each(s.ctx, na, slots, n, status) == 5
        assert list(status) == [0, 0, 0, 5, 0, 0]
        pods = [Pod(f"p{j}", containers=[Container({"cpu": 500, "memory": Gi, "ephemeral-storage": 6 * Ti
                                                    if j % 3 == 0 else 0})]) for j in range(12)]
        pa, m = pods_array(pods, a)
        got = s.schedule_raw(pa, m)
    keep = [i for i in range(n) if i != 3]
    ka, nk = nodes_array([nodes[i] for i in keep], a)
    o = pyoracle.Oracle(n)
    o.upsert(ka, (C.c_uint32 * nk)(*keep), nk)
    want = o.schedule(pa, m)
    assert_results_equal(got, want, m, "per-item upsert")
    r = res_array(got, m)
    assert (r["node_index"][[0, 3, 6]] == 5).all()  # 6 TiB each: only the 20 TiB node has it
    assert r["status"][9] == 1  # 3 x 6 TiB taken: 2 TiB left on the only ephemeral-storage node


def test_upsert_refuses_negative_extended_before_applying():
    # ks_nodes_upsert validates the whole call before it writes anything: one
    # good node plus one with a negative extended allocatable leaves the good
    # node absent (include/ksched.h, ks_nodes_upsert)
    from ksched.objects import Node

    Gi = 1 << 30
    nodes = [Node("good", {"cpu": 16000, "memory": 64 * Gi, "pods": 110}, {}, [], False,
                  extended={"example.com/gpu": 4}),
             Node("bad", {"cpu": 16000, "memory": 64 * Gi, "pods": 110}, {}, [], False,
                  extended={"example.com/gpu": -1})]
    a = Arena()
    na, n = nodes_array(nodes, a)
    with Scheduler(4) as s:
        assert s.lib.ks_nodes_upsert(s.ctx, na, (C.c_uint32 * n)(0, 1), n) == 5  # KS_ERR_RANGE
        assert all(x.pod_count == -1 for x in s.node_states([0, 1])), "refused call applied its good node"
        # the per-item form applies the good one only
        status = (C.c_int32 * n)()
        assert s.lib.ks_nodes_upsert_each(s.ctx, na, (C.c_uint32 * n)(0, 1), n, status) == 5
        assert list(status) == [0, 5]
        st = s.node_states([0, 1])
        assert st[0].pod_count == 0 and st[1].pod_count == -1


def test_upsert_each_name_moves_only_with_its_slot():
    # ks_nodes_upsert_each judges node-name moves against the items it
    # accepts: a rejected item for slot 0 (which holds "n1") cannot vacate
    # the name, so the item renaming slot 1 to "n1" is rejected on its own and
    # the unrelated item is still applied (per-item contract)
    from ksched.objects import Node

    Gi = 1 << 30
    res = {"cpu": 16000, "memory": 64 * Gi, "pods": 110}
    a = Arena()
    with Scheduler(4) as s:
        na, n = nodes_array([Node("n1", res, {}, [], False), Node("n2", res, {}, [], False)], a)
        assert s.lib.ks_nodes_upsert(s.ctx, na, (C.c_uint32 * n)(0, 1), n) == 0
        items = [Node("renamed", {"cpu": 16000, "memory": 1 << 45, "pods": 110}, {}, [], False),  # out of range
                 Node("n1", res, {}, [], False),                                                  # slot 1 -> "n1"
                 Node("n3", res, {}, [], False)]                                                  # slot 2: new
        na, n = nodes_array(items, a)
        status = (C.c_int32 * n)()
        rc = s.lib.ks_nodes_upsert_each(s.ctx, na, (C.c_uint32 * n)(0, 1, 2), n, status)
        assert rc != 0 and list(status)[:2] == [5, 1] and status[2] == 0, list(status)
        st = s.node_states([0, 1, 2])
        assert all(x.pod_count == 0 for x in st), "the valid item was not applied"
