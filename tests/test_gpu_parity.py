"""GPU parity: libksched (HIP, gfx950) vs the CPU oracle on identical inputs.

Bit-exact on every field of every result (chosen slot, TotalScore, status,
feasible / evaluated counts, per-plugin first-failure counts) and on the node
resource state after the stream.  Oracle: oracle/oracle.cpp (parity unpinned:
upstream v1.31.3 restated).
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array, scores_array, state_array
from ksched import Scheduler, synth

pytestmark = pytest.mark.gpu


def run_both(kind_nodes, n_nodes, kind_pods, n_pods, seeds=(1, 2), prefill=None, cap=None, **cfg):
    cap = cap or n_nodes
    ns = synth.nodes(kind_nodes, n_nodes, seeds[0])
    ps = synth.pods(kind_pods, n_pods, seeds[1])
    slots = synth.slot_array(n_nodes)
    o = pyoracle.Oracle(cap)
    o.upsert(ns.nodes, slots, n_nodes)
    s = Scheduler(cap, **cfg)
    s.upsert_nodes_raw(ns.nodes, slots, n_nodes)
    if prefill is not None:
        pf = synth.prefill(kind_nodes, n_nodes, seeds[0], prefill, 0.5)
        o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
        assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0, s.lib.ks_last_error(s.ctx)
    want = o.schedule(ps.pods, n_pods)
    got = s.schedule_raw(ps.pods, n_pods)
    all_slots = list(range(cap))
    st_w = state_array(o.node_states(all_slots))
    st_g = state_array(s.node_states(all_slots))
    return s, o, got, want, st_g, st_w, (ns, ps)


def check(got, want, n, st_g, st_w, what):
    assert_results_equal(got, want, n, what)
    assert np.array_equal(st_g, st_w), f"{what}: node state differs"


def test_c1_kwok_homogeneous():
    # C1 shape: kwok nodes (all identical: maximal ties), resource-only pods
    s, o, got, want, sg, sw, _ = run_both(synth.KWOK, 1000, synth.KWOK, 4000)
    check(got, want, 4000, sg, sw, "C1")
    r = res_array(got, 4000)
    assert (r["status"] == 0).all()
    s.close()


def test_hetero_prefilled():
    s, o, got, want, sg, sw, _ = run_both(synth.HETERO, 3000, synth.HETERO, 3000, prefill=3)
    check(got, want, 3000, sg, sw, "C2-small")
    s.close()


def test_labeled_taints_affinity():
    s, o, got, want, sg, sw, _ = run_both(synth.LABELED, 2000, synth.LABELED, 3000, seeds=(4, 5))
    check(got, want, 3000, sg, sw, "C4-small")
    r = res_array(got, 3000)
    assert (r["status"] == 1).any() and (r["status"] == 0).any()
    s.close()


@pytest.mark.parametrize("P,K", [(16, 4), (64, 8), (1, 1), (256, 256), (200, 256), (256, 512), (128, 300)])
def test_round_shapes(P, K):
    # tiny candidate lists force early round ends; results must not change
    s, o, got, want, sg, sw, _ = run_both(synth.HETERO, 1500, synth.HETERO, 2000, prefill=7,
                                          pods_per_round=P, topk=K)
    check(got, want, 2000, sg, sw, f"P={P} K={K}")
    s.close()


@pytest.mark.parametrize("K", [256, 512])
def test_labeled_long_lists(K):
    # EXT resolve with both halves of every list wave's 128 entries in use
    s, o, got, want, sg, sw, _ = run_both(synth.LABELED, 2500, synth.LABELED, 2500, seeds=(14, 15), topk=K)
    check(got, want, 2500, sg, sw, f"labeled K={K}")
    s.close()


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_virtual_shards(shards):
    # the sharded path (per-shard sweep + cross-shard merge) equals one shard
    s, o, got, want, sg, sw, _ = run_both(synth.LABELED, 1800, synth.LABELED, 1500, seeds=(8, 9),
                                          virtual_shards=shards)
    check(got, want, 1500, sg, sw, f"shards={shards}")
    s.close()


@pytest.mark.parametrize("npl", [2, 8])
def test_nodes_per_lane(npl):
    s, o, got, want, sg, sw, _ = run_both(synth.HETERO, 2500, synth.HETERO, 1000, prefill=11, nodes_per_lane=npl)
    check(got, want, 1000, sg, sw, f"npl={npl}")
    s.close()


def test_plugin_scores_dump():
    n = 1500
    ns = synth.nodes(synth.LABELED, n, 21)
    ps = synth.pods(synth.LABELED, 64, 22)
    slots = synth.slot_array(n)
    o = pyoracle.Oracle(n)
    o.upsert(ns.nodes, slots, n)
    s = Scheduler(n)
    s.upsert_nodes_raw(ns.nodes, slots, n)
    pf = synth.prefill(synth.LABELED, n, 21, 23, 0.5)
    o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
    assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
    for j in range(64):
        p = ps.pods_at(j)
        want = scores_array(o.plugin_scores(p))
        out = (type(o.plugin_scores(p)[0]) * n)()
        assert s.lib.ks_plugin_scores(s.ctx, p, out) == 0
        got = scores_array(out)
        bad = np.nonzero((got != want).any(1))[0]
        assert len(bad) == 0, (f"pod {j}: {len(bad)} nodes differ; " + "; ".join(
            f"node {i}: got {got[i].tolist()} want {want[i].tolist()}" for i in bad[:4]))
    s.close()


def test_capacity_with_empty_slots_and_deletes():
    # capacity larger than the node count; some nodes deleted mid-stream
    cap, n = 2600, 2000
    ns = synth.nodes(synth.HETERO, n, 31)
    ps = synth.pods(synth.HETERO, 2000, 32)
    slots = (C.c_uint32 * n)(*[i * 7 % cap for i in range(n)])  # scattered, distinct slots
    o = pyoracle.Oracle(cap)
    o.upsert(ns.nodes, slots, n)
    s = Scheduler(cap, pods_per_round=128)
    s.upsert_nodes_raw(ns.nodes, slots, n)
    want1 = o.schedule(ps.pods, 1000)
    got1 = s.schedule_raw(ps.pods, 1000)
    assert_results_equal(got1, want1, 1000, "before delete")
    dels = (C.c_uint32 * 50)(*[slots[i] for i in range(0, 500, 10)])
    o.delete(dels, 50)
    assert s.lib.ks_nodes_delete(s.ctx, dels, 50) == 0
    rest = ps.pods_at(1000)
    want2 = o.schedule(rest, 1000)
    got2 = s.schedule_raw(rest, 1000)
    assert_results_equal(got2, want2, 1000, "after delete")
    s.close()


def test_duplicate_slots_in_one_upsert():
    # one call naming a slot several times: events apply in order (last state wins)
    cap, n = 300, 1200
    ns = synth.nodes(synth.LABELED, n, 51)
    ps = synth.pods(synth.LABELED, 800, 52)
    slots = (C.c_uint32 * n)(*[(i * 37) % cap for i in range(n)])
    o = pyoracle.Oracle(cap)
    o.upsert(ns.nodes, slots, n)
    s = Scheduler(cap, pods_per_round=64)
    s.upsert_nodes_raw(ns.nodes, slots, n)
    assert_results_equal(s.schedule_raw(ps.pods, 800), o.schedule(ps.pods, 800), 800, "dup slots")
    assert np.array_equal(state_array(s.node_states(list(range(cap)))), state_array(o.node_states(list(range(cap)))))
    s.close()


def test_cluster_fills_up():
    # far more pods than capacity: the tail is unschedulable (FitError with diagnosis)
    n = 64
    ns = synth.nodes(synth.KWOK, n, 41)
    ps = synth.pods(synth.KWOK, 3000, 42)
    slots = synth.slot_array(n)
    o = pyoracle.Oracle(n)
    o.upsert(ns.nodes, slots, n)
    s = Scheduler(n, pods_per_round=64)
    s.upsert_nodes_raw(ns.nodes, slots, n)
    want = o.schedule(ps.pods, 3000)
    got = s.schedule_raw(ps.pods, 3000)
    assert_results_equal(got, want, 3000, "fill-up")
    r = res_array(got, 3000)
    assert (r["status"] == 1).sum() > 500
    s.close()


def test_empty_cluster():
    s = Scheduler(100)
    ps = synth.pods(synth.KWOK, 10, 1)
    got = res_array(s.schedule_raw(ps.pods, 10), 10)
    assert (got["status"] == 1).all() and (got["evaluated"] == 0).all() and (got["node_index"] == -1).all()
    s.close()


def test_rccl_single_rank_path():
    # the RCCL code path (all-reduce of normalisation maxima, all-gather of shard
    # records, allreduce_max barrier) with a one-rank communicator
    n = 1500
    ns = synth.nodes(synth.LABELED, n, 61)
    ps = synth.pods(synth.LABELED, 1200, 62)
    slots = synth.slot_array(n)
    o = pyoracle.Oracle(n)
    o.upsert(ns.nodes, slots, n)
    s = Scheduler(n, world_size=1, rank=0)
    s.comm_init(Scheduler.comm_unique_id())
    s.upsert_nodes_raw(ns.nodes, slots, n)
    assert_results_equal(s.schedule_raw(ps.pods, 1200), o.schedule(ps.pods, 1200), 1200, "rccl 1 rank")
    assert s.allreduce_max([1.5, -2.0]) == [1.5, -2.0]
    s.close()
