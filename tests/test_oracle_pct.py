"""percentageOfNodesToScore < 100 in the CPU oracle: numFeasibleNodesToFind
and the rotating nextStartNodeIndex window (upstream v1.31.3
pkg/scheduler/schedule_one.go#numFeasibleNodesToFind, findNodesThatFitPod,
findNodesThatPassFilters; restated sequentially in oracle.cpp window()).
The expectations are derived by hand from those functions (parity unpinned:
the reference holds no vectors for them)."""
import pytest

import pyoracle
from helpers import res_array
from ksched.objects import (Arena, Container, Node, NodeSelectorRequirement, NodeSelectorTerm, Pod, nodes_array,
                            pods_array)

Gi = 1 << 30


@pytest.mark.parametrize("pct,n,want", [
    (5, 50, 50), (100, 99, 99), (0, 99, 99),       # fewer than minFeasibleNodesToFind: all
    (5, 1000, 100), (50, 150, 100),                # below the 100-node floor
    (5, 5000, 250), (5, 1_000_000, 50_000), (10, 1234, 123), (100, 1234, 1234),
    (0, 1000, 420),                                # adaptive: 50 - 1000/125 = 42 %
    (0, 100, 100), (0, 6000, 300), (0, 1_000_000, 50_000),  # adaptive floor 5 %
])
def test_num_feasible_nodes_to_find(pct, n, want):
    assert pyoracle.lib().oracle_num_feasible_nodes_to_find(pct, n) == want


def cluster(n, unsched=lambda i: False):
    return [Node(f"h{i}", {"cpu": 4000, "memory": 8 * Gi, "pods": 110}, {"kubernetes.io/hostname": f"h{i}"},
                 unschedulable=unsched(i)) for i in range(n)]


def run(nodes, pods, pct, o=None, a=None):
    a = a or Arena()
    if o is None:
        o = pyoracle.Oracle(len(nodes), percentage=pct)
        na, n = nodes_array(nodes, a)
        o.upsert(na, (pyoracle.C.c_uint32 * n)(*range(n)), n)
    pa, m = pods_array(pods, a)
    return res_array(o.schedule(pa, m), m), o


def pods(k, j0=0):
    return [Pod(f"p{j0 + j}", containers=[Container({"cpu": 100, "memory": 256 << 20})]) for j in range(k)]


def test_rotation_identical_nodes():
    # 1000 equal nodes, pct 10: k = 100 and the 101st feasible node stops the
    # visit, so each pod processes 100 nodes and the next one starts after them
    r, o = run(cluster(1000), pods(10), 10)
    assert list(r["node_index"]) == [100 * j for j in range(10)]  # equal scores: lowest slot of the window
    assert (r["feasible"] == 100).all() and (r["evaluated"] == 100).all()
    assert o.next_start == 0  # 10 x 100 processed, modulo 1000
    r, o = run(None, pods(1, 10), 10, o)
    assert r["node_index"][0] == 1  # window [0, 100) again; slot 0 now holds a pod
    assert o.next_start == 100


def test_rotation_skips_infeasible():
    # every third node unschedulable: the 101st feasible node is at index 151,
    # so 151 nodes are processed (100 feasible, 51 NodeUnschedulable)
    r, o = run(cluster(300, lambda i: i % 3 == 0), pods(2), 5)
    assert r["node_index"][0] == 1
    assert (r["feasible"][0], r["evaluated"][0], r["fail"][0][0]) == (100, 151, 51)
    # the second window starts at the node that stopped the first (151); it
    # holds the 100 feasible nodes of 151..299 and ends at node 1 (0 is not
    # feasible): 150 processed
    assert r["node_index"][1] == 151 and r["evaluated"][1] == 150
    assert o.next_start == (151 + 150) % 300


def test_rotation_wraps_and_all_feasible_below_k():
    # 150 nodes, 80 feasible: fewer than k + 1 = 101, every node is processed
    # and nextStartNodeIndex comes back to where it was
    r, o = run(cluster(150, lambda i: i >= 80), pods(3), 5)
    assert (r["feasible"] == [80, 80, 80]).all() and (r["evaluated"] == 150).all()
    assert o.next_start == 0


def test_window_wraps_round_the_list():
    # 200 nodes, pct 50: k = 100; the second pod starts at 100 and its window
    # is [100, 200); the third wraps to [0, 100) where slot 0 is taken
    r, o = run(cluster(200), pods(3), 50)
    assert list(r["node_index"][:2]) == [0, 100]
    assert r["node_index"][2] == 1 and o.next_start == 100


def test_deleted_nodes_shrink_the_list():
    a = Arena()
    nodes = cluster(400)
    r, o = run(nodes, pods(3), 25, a=a)  # k = 100: windows at 0, 100, 200
    assert list(r["node_index"]) == [0, 100, 200] and o.next_start == 300
    o.delete((pyoracle.C.c_uint32 * 150)(*range(250, 400)), 150)  # 250 nodes left; 300 % 250 = 50
    r, o = run(None, pods(1, 3), 25, o, a)
    assert r["node_index"][0] == 50  # the window starts at list index 300 % 250 = 50
    assert o.next_start == (300 + 100) % 250


def test_prefilter_result_nodes_are_not_visited():
    # a pod naming two nodes (NodeAffinity PreFilterResult): the list is those
    # two (fewer than 100: all processed); the other nodes keep their
    # PreFilterResult status; nextStartNodeIndex moves by the two processed
    names = [NodeSelectorTerm(match_fields=[NodeSelectorRequirement("metadata.name", "In", [h])]) for h in ("h5", "h7")]
    p = [Pod("named", containers=[Container({"cpu": 100})], required_terms=names)]
    r, o = run(cluster(300), p, 5)
    assert r["node_index"][0] == 5 and r["feasible"][0] == 2 and r["evaluated"][0] == 300
    assert r["fail"][0][7] == 298  # KS_FAIL_PREFILTER_RESULT
    assert o.next_start == 2


def test_pct_100_keeps_every_result():
    nodes = cluster(500, lambda i: i % 7 == 0)
    r100, o = run(nodes, pods(20), 100)
    rdef, _ = run(nodes, pods(20), 100, None)
    assert (r100 == rdef).all() and (r100["evaluated"] == 500).all() and o.next_start == 0
