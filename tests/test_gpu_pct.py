"""percentageOfNodesToScore < 100 on the GPU: the probe
filter pass, the window kernel and the pass over the window against the
oracle's sequential restatement (oracle.cpp window(); upstream v1.31.3
schedule_one.go#numFeasibleNodesToFind / findNodesThatPassFilters, SURVEY.md
A5; the reference deploys pct 5 at terraform/kubernetes/dist-scheduler.tf:562).
Bit-exact on every result field (feasible and evaluated counts included), on
every node's state and on nextStartNodeIndex after each batch.  Parity
unpinned (no reference vectors): the oracle window is pinned by the
hand-derived KATs of tests/test_oracle_pct.py."""
import random

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array
from ksched import Scheduler
from ksched.objects import (Container, Node, NodeSelectorRequirement, NodeSelectorTerm, Pod, PreferredSchedulingTerm,
                            Taint, Toleration)
from spread_cases import HOST, ZONE
from test_gpu_spread import Pair, rand_ipa_pod, rand_nodes, rand_res_nodes, rand_res_pod

pytestmark = pytest.mark.gpu

Gi, Mi = 1 << 30, 1 << 20


class PctPair(Pair):
    def __init__(self, n, pct, **cfg):
        self.n = n
        from ksched.objects import Arena
        self.a = Arena()
        self.s = Scheduler(n, percentage_of_nodes_to_score=pct, **cfg)
        self.o = pyoracle.Oracle(n, percentage=pct)

    def check_start(self, what=""):
        assert self.s.next_start_index() == self.o.next_start, what


def rand_pct_pod(rng, j):
    r = rng.random()
    if r < 0.45:  # spread / InterPodAffinity / selectors / tolerations / plain
        return rand_ipa_pod(rng, j, frac=0.25, spread_frac=0.35)
    req = {"cpu": rng.randrange(1, 30) * 50, "memory": rng.randrange(1, 48) * 64 * Mi}
    kw = {}
    if r < 0.65:  # NodeAffinity preferred terms: the normaliser's maximum over the window's feasible nodes
        kw["preferred"] = [PreferredSchedulingTerm(rng.randint(1, 100), NodeSelectorTerm(
            [NodeSelectorRequirement("disk", "In", ["ssd"])])), PreferredSchedulingTerm(rng.randint(1, 100),
            NodeSelectorTerm([NodeSelectorRequirement("rack", "In", [f"r{rng.randrange(8)}"])]))]
    elif r < 0.72:  # a NodeAffinity PreFilterResult: the list is the named nodes
        kw["required_terms"] = [NodeSelectorTerm(match_fields=[NodeSelectorRequirement("metadata.name", "In", [h])])
                                for h in rng.sample([f"h{i}" for i in range(40)], rng.randint(1, 4))]
    elif r < 0.8:
        kw["tolerations"] = [Toleration("ded", "Equal", "x", "NoSchedule")]
    return Pod(f"q{j}", containers=[Container(req)], labels={"app": f"a{rng.randrange(4)}"}, **kw)


def soft_taints(rng, nodes):
    for nd in nodes:
        if rng.random() < 0.2:  # TaintToleration's normaliser (PreferNoSchedule counts)
            nd.taints = nd.taints + [Taint("soft", "y", "PreferNoSchedule")]
    return nodes


@pytest.mark.parametrize("seed,n,zones,pct", [(81, 300, 3, 5), (82, 1500, 12, 5), (83, 1500, 8, 50),
                                              (84, 5000, 20, 0), (85, 700, 5, 30)])
def test_pct_random_stream(seed, n, zones, pct):
    rng = random.Random(seed)
    x = PctPair(n, pct)
    x.upsert(soft_taints(rng, rand_nodes(rng, n, zones)), list(range(n)))
    pre = [rand_ipa_pod(rng, 10_000 + j, frac=0.1, spread_frac=0.0) for j in range(n // 3)]
    for p in pre:
        p.affinity_terms = [t for t in p.affinity_terms if t.kind != "anti-affinity"]
    x.add(pre, [rng.randrange(n) for _ in pre])
    for b in range(4):
        pods = [rand_pct_pod(rng, b * 1000 + j) for j in range(90)]
        r = x.schedule(pods, f"seed {seed} pct {pct} batch {b}")
        x.states_equal(f"seed {seed} batch {b}")
        x.check_start(f"seed {seed} batch {b}")
        if b == 0 and n >= 1000 and pct:
            assert (r["evaluated"] < n).any()  # windows shorter than the list were taken
        # deleted and re-added nodes between batches: the list shrinks and grows
        slots = rng.sample(range(n), 4)
        x.delete(slots[:2])
        x.upsert(rand_nodes(rng, 1, zones, slot0=n + 10 * b), [slots[0]])
    x.close()


def test_pct_windows_through_full_nodes():
    # nodes fill after one or two pods: windows grow past the full nodes and
    # the last pods find fewer than k + 1 feasible (every node processed)
    rng = random.Random(86)
    n = 400
    x = PctPair(n, 10)
    nodes = [Node(f"h{i}", {"cpu": 1000, "memory": 4 * Gi, "pods": rng.choice([1, 2])},
                  {HOST: f"h{i}", ZONE: f"z{i % 4}"}) for i in range(n)]
    x.upsert(nodes, list(range(n)))
    pods = [Pod(f"f{j}", containers=[Container({"cpu": 300, "memory": 256 * Mi})]) for j in range(700)]
    r = x.schedule(pods, "fill")
    x.states_equal("fill")
    x.check_start("fill")
    assert (r["status"] == 1).any() and (r["evaluated"] == n).any() and (r["evaluated"] < n).any()
    x.close()


def test_pct_images_and_extended_resources():
    # ImageLocality (image states over the present nodes) and extended /
    # ephemeral resources on the one-pod chain with the window
    rng = random.Random(88)
    n = 1200
    x = PctPair(n, 10)
    x.upsert(rand_res_nodes(rng, n), list(range(n)))
    for b in range(3):
        pods = [rand_res_pod(rng, b * 1000 + j) for j in range(80)]
        x.schedule(pods, f"res batch {b}")
        x.states_equal(f"res batch {b}")
        x.check_start(f"res batch {b}")
    x.close()


def test_pct_batches_in_flight():
    # ks_batch_submit with the next batch compiled while one runs: the window
    # state (nextStartNodeIndex) lives on the device and carries from batch to
    # batch in submission order; results equal the oracle's sequential ones
    from ksched.objects import pods_array
    rng = random.Random(89)
    n = 2000
    x = PctPair(n, 5)
    x.upsert(soft_taints(rng, rand_nodes(rng, n, 8)), list(range(n)))
    batches = [[rand_pct_pod(rng, b * 1000 + j) for j in range(120)] for b in range(4)]
    arrs = [pods_array(p, x.a) for p in batches]
    want = [x.o.schedule(pa, m) for pa, m in arrs]
    s = x.s
    hs = []
    for pa, m in arrs:
        h = s.prepare(pa, m)
        assert s.lib.ks_batch_submit(s.ctx, h) == 0, s.lib.ks_last_error(s.ctx)
        hs.append(h)
    for h, (pa, m), w, b in zip(hs, arrs, want, range(4)):
        assert s.lib.ks_batch_wait(s.ctx, h) == 0, s.lib.ks_last_error(s.ctx)
        assert_results_equal(s.results(h, m), w, m, f"in-flight batch {b}")
        s.free(h)
    x.states_equal("in flight")
    x.check_start("in flight")
    x.close()


def test_pct_100_is_the_default_path():
    # pct 100 keeps the round kernels: results equal the pct-100 oracle and
    # nextStartNodeIndex stays 0
    rng = random.Random(87)
    n = 600
    x = PctPair(n, 100)
    x.upsert(rand_nodes(rng, n, 4), list(range(n)))
    pods = [rand_pct_pod(rng, j) for j in range(200)]
    x.schedule(pods, "pct 100")
    x.states_equal("pct 100")
    assert x.s.next_start_index() == 0 and x.o.next_start == 0
    assert int(x.s.stats().spread_pods) < len(pods)  # plain pods stayed on the rounds
    x.close()


def test_pct_refused_with_shards():
    from ksched import _abi
    with pytest.raises(_abi.KschedError):
        Scheduler(64, virtual_shards=2, percentage_of_nodes_to_score=5)
    with pytest.raises(_abi.KschedError):
        Scheduler(64, percentage_of_nodes_to_score=101)
