"""The C++ oracle's percentageOfNodesToScore window against a second,
independent restatement in plain Python (CPU; parity unpinned: neither is the
reference, but they are written separately from upstream v1.31.3's text).

Resource-only pods on untainted, unlabelled nodes, so the profile reduces to
NodeResourcesFit (filter + LeastAllocated), BalancedAllocation and a constant
TaintToleration 3 x 100 (every raw score 0, DefaultNormalizeScore(reverse)
gives 100):

* schedule_one.go#numFeasibleNodesToFind / findNodesThatFitPod /
  findNodesThatPassFilters with one worker: visit from nextStartNodeIndex %
  len(nodes), stop at the (k+1)-th feasible node, nextStartNodeIndex +=
  processed;
* noderesources/fit.go#fitsRequest; least_allocated.go#leastRequestedScore
  and resource_allocation.go (NonZeroRequested, 100m / 200Mi defaults for
  missing requests); balanced_allocation.go (float64 fractions, std = |f0 -
  f1| / 2);
* selectHost: the highest TotalScore, the lowest slot among ties (ksched's
  deterministic tie-break)."""
import random

import pytest

import pyoracle
from helpers import res_array
from ksched.objects import Arena, Container, Node, Pod, nodes_array, pods_array

Mi, Gi = 1 << 20, 1 << 30
DEF_CPU, DEF_MEM = 100, 200 * Mi


def num_to_find(pct, n):
    if n < 100:
        return n
    p = pct if pct else max(50 - n // 125, 5)
    return max(n * p // 100, 100)


class PyNode:
    def __init__(self, cpu, mem, pods):
        self.ac, self.am, self.ap = cpu, mem, pods
        self.rc = self.rm = self.zc = self.zm = self.np = 0


def requests(pod):
    c = pod.containers[0].requests
    rc, rm = c.get("cpu", 0), c.get("memory", 0)
    zc = c["cpu"] if "cpu" in c else DEF_CPU
    zm = c["memory"] if "memory" in c else DEF_MEM
    return rc, rm, zc, zm


def fits(nd, rc, rm):
    if nd.np + 1 > nd.ap:
        return False
    if rc == 0 and rm == 0:
        return True
    return not ((rc > 0 and rc > nd.ac - nd.rc) or (rm > 0 and rm > nd.am - nd.rm))


def least(req, cap):
    if cap == 0 or req > cap:
        return 0
    return (cap - req) * 100 // cap


def score(nd, rc, rm, zc, zm):
    la_num, la_w = 0, 0
    for cap, req in ((nd.ac, nd.zc + zc), (nd.am, nd.zm + zm)):
        if cap:
            la_num += least(req, cap)
            la_w += 1
    la = la_num // la_w if la_w else 0
    fr = [min(1.0, float(req) / float(cap)) for cap, req in ((nd.ac, nd.rc + rc), (nd.am, nd.rm + rm)) if cap]
    std = abs((fr[0] - fr[1]) / 2) if len(fr) == 2 else 0.0
    ba = int((1 - std) * 100)
    return la + ba + 3 * 100


def py_schedule(nodes, pods, pct):
    nxt, out = 0, []
    n = len(nodes)
    for pod in pods:
        rc, rm, zc, zm = requests(pod)
        k = num_to_find(pct, n)
        s = nxt % n
        feas, processed = [], n
        for j in range(n):
            i = (s + j) % n
            if fits(nodes[i], rc, rm):
                if len(feas) == k:
                    processed = j
                    break
                feas.append(i)
        nxt = (nxt + processed) % n
        if not feas:
            out.append((-1, 0, processed))
            continue
        best = max(feas, key=lambda i: (score(nodes[i], rc, rm, zc, zm), -i))
        nd = nodes[best]
        nd.rc += rc
        nd.rm += rm
        nd.zc += zc
        nd.zm += zm
        nd.np += 1
        out.append((best, len(feas), processed))
    return out, nxt


@pytest.mark.parametrize("seed", range(12))
def test_window_matches_python_restatement(seed):
    rng = random.Random(500 + seed)
    n = rng.choice([60, 150, 320])
    pct = rng.choice([0, 3, 5, 20, 50, 100])
    spec = [(rng.choice([1000, 2000, 4000, 0]), rng.choice([2, 4, 8]) * Gi, rng.choice([1, 3, 110])) for _ in range(n)]
    nodes = [Node(f"n{i}", {"cpu": c, "memory": m, "pods": p}) for i, (c, m, p) in enumerate(spec)]
    pods = []
    for j in range(rng.choice([40, 150])):
        r = rng.random()
        req = {} if r < 0.15 else ({"cpu": rng.randrange(1, 20) * 100} if r < 0.3 else
                                   {"cpu": rng.randrange(1, 20) * 100, "memory": rng.randrange(1, 16) * 128 * Mi})
        pods.append(Pod(f"p{j}", containers=[Container(req)]))
    a = Arena()
    o = pyoracle.Oracle(n, percentage=pct)
    na, _ = nodes_array(nodes, a)
    o.upsert(na, (pyoracle.C.c_uint32 * n)(*range(n)), n)
    pa, m = pods_array(pods, a)
    got = res_array(o.schedule(pa, m), m)
    want, nxt = py_schedule([PyNode(*t) for t in spec], pods, pct)
    for j, (node, feas, processed) in enumerate(want):
        g = got[j]
        assert (int(g["node_index"]), int(g["feasible"]), int(g["evaluated"])) == (node, feas, processed), \
            (seed, n, pct, j, g, (node, feas, processed))
    assert o.next_start == (nxt if pct != 100 else 0)
