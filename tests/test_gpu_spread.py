"""PodTopologySpread on the GPU (ksched_spread.hip) against the oracle's
restatement of upstream v1.31.3 podtopologyspread and the hand-derived cases
of tests/spread_cases.py: results, per-plugin score dumps and node states
bit for bit; mixed batches (spread pods between round-kernel segments);
selector-class counts kept through ks_pods_add / remove, node upserts and
deletes, and pods the round kernels bind."""
import ctypes as C
import random

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array, scores_array, states_np
from ksched import Scheduler, _abi
from ksched.objects import (Arena, Container, LabelSelector, LabelSelectorRequirement, Node, Pod, Taint,
                            Toleration, TopologySpreadConstraint as TSC, nodes_array, pods_array,
                            system_default_spread)
from scenarios import check
from spread_cases import CASES, HOST, ZONE

pytestmark = pytest.mark.gpu

Gi, Mi = 1 << 30, 1 << 20


def u32(xs):
    return (C.c_uint32 * max(1, len(xs)))(*xs)


def pod_ptr(arr, j):
    return C.cast(C.addressof(arr.contents) + j * C.sizeof(_abi.KsPod), C.POINTER(_abi.KsPod))


class Pair:
    """libksched and the oracle fed the same cache events."""

    def __init__(self, n, **cfg):
        self.n = n
        self.a = Arena()
        self.s = Scheduler(n, **cfg)
        self.o = pyoracle.Oracle(n)

    def upsert(self, nodes, slots):
        na, k = nodes_array(nodes, self.a)
        self.s.upsert_nodes_raw(na, u32(slots), k)
        self.o.upsert(na, u32(slots), k)

    def delete(self, slots):
        assert self.s.lib.ks_nodes_delete(self.s.ctx, u32(slots), len(slots)) == 0
        self.o.delete(u32(slots), len(slots))

    def add(self, pods, slots, sign=1):
        if not pods:
            return
        pa, k = pods_array(pods, self.a)
        fn = self.s.lib.ks_pods_add if sign > 0 else self.s.lib.ks_pods_remove
        assert fn(self.s.ctx, pa, u32(slots), k) == 0, self.s.lib.ks_last_error(self.s.ctx)
        (self.o.add_pods if sign > 0 else self.o.remove_pods)(pa, u32(slots), k)

    def schedule(self, pods, what=""):
        pa, m = pods_array(pods, self.a)
        want = self.o.schedule(pa, m)
        got = self.s.schedule_raw(pa, m)
        assert_results_equal(got, want, m, what)
        return res_array(got, m)

    def dump_equal(self, pod, what=""):
        pa, _ = pods_array([pod], self.a)
        out = (_abi.KsNodeScore * self.n)()
        assert self.s.lib.ks_plugin_scores(self.s.ctx, pa, out) == 0, self.s.lib.ks_last_error(self.s.ctx)
        g, w = scores_array(out), scores_array(self.o.plugin_scores(pa))
        assert np.array_equal(g, w), (what, np.nonzero((g != w).any(axis=1))[0][:5])
        return out

    def states_equal(self, what=""):
        g = states_np(self.s.lib.ks_node_states, self.s.ctx, self.n)
        w = states_np(self.o.L.oracle_node_states, self.o.o, self.n)
        assert np.array_equal(g, w), what

    def close(self):
        self.s.close()
        self.o.close()


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("P", [256, 2])
def test_spread_case_gpu(name, P):
    nodes, bound, pods, exp, dumps = CASES[name]()
    x = Pair(len(nodes), pods_per_round=P)
    x.upsert(nodes, list(range(len(nodes))))
    x.add([p for p, _ in bound], [s for _, s in bound])
    for j, p in enumerate(pods):
        if j in dumps:
            out = x.dump_equal(p, f"{name} dump {j}")
            assert [(out[i].spread_raw, out[i].spread_score) for i in range(len(nodes))] == dumps[j]
    r = x.schedule(pods, name)  # one batch: spread pods in order, each against the previous commits
    check(r, exp)
    x.states_equal(name)
    x.close()


# ------------------------------------------------------------ random streams

APPS = ["web", "api", "db", "cache"]
NSS = ["default", "other"]


def rand_nodes(rng, n, zones, slot0=0, nozone=0.05):
    out = []
    for i in range(n):
        lab = {HOST: f"h{slot0 + i}", "rack": f"r{rng.randrange(8)}"}
        if rng.random() > nozone:
            lab[ZONE] = f"z{rng.randrange(zones)}"
        if rng.random() < 0.3:
            lab["disk"] = "ssd"
        taints = [Taint("ded", "x")] if rng.random() < 0.05 else []
        out.append(Node(f"h{slot0 + i}", {"cpu": rng.choice([4000, 8000, 16000]),
                                          "memory": rng.choice([8, 16, 32]) * Gi, "pods": rng.choice([8, 32, 110])},
                        lab, taints))
    return out


def rand_selector(rng):
    r = rng.random()
    if r < 0.05:
        return None
    if r < 0.1:
        return LabelSelector()
    if r < 0.7:
        return LabelSelector({"app": rng.choice(APPS)})
    tier = LabelSelectorRequirement("tier", "NotIn", ["gold"]) if rng.random() < 0.5 else \
        LabelSelectorRequirement("tier", "DoesNotExist")
    return LabelSelector(match_expressions=[LabelSelectorRequirement("app", "In", rng.sample(APPS, 2)), tier])


def rand_pod(rng, j, spread_frac=0.6):
    labels = {"app": rng.choice(APPS)}
    if rng.random() < 0.3:
        labels["tier"] = "gold"
    if rng.random() < 0.5:
        labels["rev"] = str(rng.randrange(3))
    kw = {}
    if rng.random() < 0.15:
        kw["node_selector"] = {"disk": "ssd"}
    if rng.random() < 0.1:
        kw["tolerations"] = [Toleration("ded", "Equal", "x", "NoSchedule")]
    spread, defaulted = [], False
    if rng.random() < spread_frac:
        r = rng.random()
        if r < 0.25:
            spread, defaulted = system_default_spread(LabelSelector({"app": labels["app"]})), True
        else:
            used = set()
            for _ in range(rng.randint(1, 3)):
                key = rng.choice([ZONE, HOST, "rack"])
                when = rng.choice(["DoNotSchedule", "ScheduleAnyway"])
                if (key, when) in used:
                    continue
                used.add((key, when))
                spread.append(TSC(rng.randint(1, 3), key, when, rand_selector(rng),
                                  min_domains=rng.choice([None, None, 2, 40]) if when == "DoNotSchedule" else None,
                                  node_affinity_policy=rng.choice([None, "Honor", "Ignore"]),
                                  node_taints_policy=rng.choice([None, "Honor", "Ignore"]),
                                  match_label_keys=["rev"] if rng.random() < 0.2 else []))
    req = {} if rng.random() < 0.1 else {"cpu": rng.randrange(1, 40) * 50, "memory": rng.randrange(1, 64) * 64 * Mi}
    return Pod(f"p{j}", namespace=rng.choice(NSS), containers=[Container(req)], labels=labels,
               topology_spread=spread, spread_defaulted=defaulted, **kw)


@pytest.mark.parametrize("seed,n,zones,P", [(1, 300, 3, 256), (2, 1000, 12, 64), (3, 2500, 40, 256), (4, 700, 5, 2)])
def test_spread_random_stream(seed, n, zones, P):
    rng = random.Random(seed)
    x = Pair(n, pods_per_round=P)
    x.upsert(rand_nodes(rng, n, zones), list(range(n)))
    pre = [rand_pod(rng, 10_000 + j, spread_frac=0.0) for j in range(n // 2)]
    live = [(p, rng.randrange(n)) for p in pre]  # bound pods still on their node
    x.add([p for p, _ in live], [s for _, s in live])
    for b in range(4):
        pods = [rand_pod(rng, b * 1000 + j) for j in range(120)]
        x.schedule(pods, f"seed {seed} batch {b}")
        x.states_equal(f"seed {seed} batch {b}")
        # cache churn between batches: removals, relabelled / deleted / re-added nodes
        rng.shuffle(live)
        gone, live = live[:5], live[5:]
        x.add([p for p, _ in gone], [s for _, s in gone], sign=-1)
        slots = rng.sample(range(n), 3)
        live = [(p, s) for p, s in live if s != slots[0]]  # their pods leave with the deleted node
        x.upsert(rand_nodes(rng, 3, zones, slot0=n + 10 * b), slots)
        x.delete([slots[0]])
        x.upsert(rand_nodes(rng, 1, zones, slot0=n + 10 * b + 5), [slots[0]])
        p = rand_pod(rng, 99_000 + b, spread_frac=1.0)
        x.dump_equal(p, f"seed {seed} dump {b}")
    x.close()


def test_spread_bound_pod_removal_and_mixed_batch():
    rng = random.Random(7)
    n = 400
    x = Pair(n)
    x.upsert(rand_nodes(rng, n, 6, nozone=0.0), list(range(n)))
    bound = [Pod(f"b{j}", containers=[Container({"cpu": 100})], labels={"app": "web"}) for j in range(200)]
    slots = [rng.randrange(n) for _ in bound]
    x.add(bound, slots)
    c = [TSC(1, ZONE, "DoNotSchedule", LabelSelector({"app": "web"}))]
    web = lambda j: Pod(f"w{j}", containers=[Container({"cpu": 100})], labels={"app": "web"}, topology_spread=c)
    plain = lambda j: Pod(f"q{j}", containers=[Container({"cpu": 100})], labels={"app": "web"})
    # spread pods between round-kernel segments whose pods the spread selector counts
    pods = [plain(j) for j in range(300)] + [web(j) for j in range(20)] + [plain(300 + j) for j in range(300)] + \
           [web(20 + j) for j in range(20)]
    x.schedule(pods, "mixed")
    x.states_equal("mixed")
    x.add(bound[:100], slots[:100], sign=-1)  # removals lower the zone counts
    x.schedule([web(100 + j) for j in range(30)], "after removal")
    x.states_equal("after removal")
    x.close()


def test_spread_refusals():
    s = Scheduler(8)
    a = Arena()
    na, k = nodes_array([Node("n", {"cpu": 1000, "memory": Gi, "pods": 8}, {ZONE: "a"})], a)
    s.upsert_nodes_raw(na, u32([0]), k)
    bad = [
        [TSC(0, ZONE)],                                     # maxSkew < 1
        [TSC(1, ZONE), TSC(2, ZONE)],                       # duplicate {topologyKey, whenUnsatisfiable}
        [TSC(1, ZONE, "ScheduleAnyway", min_domains=2)],    # minDomains with ScheduleAnyway
        [TSC(1, ZONE, "DoNotSchedule", LabelSelector({"bad key!": "x"}))],
        [TSC(1, ZONE, "DoNotSchedule", LabelSelector(match_expressions=[LabelSelectorRequirement("a", "In")]))],
        [TSC(1, f"k{i}") for i in range(9)],                # more than MAX_SPREAD
    ]
    pods = [Pod(f"p{i}", topology_spread=c) for i, c in enumerate(bad)]
    pa, m = pods_array(pods, a)
    st = (C.c_int32 * m)()
    s.lib.ks_pods_check(s.ctx, pa, m, st)
    assert list(st) == [_abi.KS_ERR_UNSUPPORTED] * m
    ok = Pod("fine", topology_spread=[TSC(1, ZONE, "DoNotSchedule", LabelSelector({"app": "x"}))])
    pa, m = pods_array([ok], a)
    assert s.lib.ks_pods_check(s.ctx, pa, 1, st) == 0
    s.close()


def test_spread_1k_nodes_many_pods_same_deployment():
    # a deployment's replicas with the system defaults (hostname 3, zone 5):
    # every pod's scores depend on all earlier ones
    rng = random.Random(11)
    n = 1000
    x = Pair(n)
    x.upsert(rand_nodes(rng, n, 8), list(range(n)))
    sel = LabelSelector({"app": "web"})
    pods = [Pod(f"r{j}", containers=[Container({"cpu": 250, "memory": 256 * Mi})], labels={"app": "web"},
                topology_spread=system_default_spread(sel), spread_defaulted=True) for j in range(1500)]
    r = x.schedule(pods, "replicas")
    assert (r["status"] == 0).all()
    x.states_equal("replicas")
    x.close()


# ------------------------------------------- extended resources, ImageLocality

@pytest.mark.parametrize("name", sorted(__import__("solo_cases").CASES))
@pytest.mark.parametrize("P", [256, 2])
def test_solo_case_gpu(name, P):
    from solo_cases import CASES as SOLO
    nodes, bound, pods, exp, dumps = SOLO[name]()
    x = Pair(len(nodes), pods_per_round=P)
    x.upsert(nodes, list(range(len(nodes))))
    x.add([p for p, _ in bound], [s for _, s in bound])
    for j, p in enumerate(pods):
        if j in dumps:
            out = x.dump_equal(p, f"{name} dump {j}")
            assert [out[i].image_locality for i in range(len(nodes))] == dumps[j]
    r = x.schedule(pods, name)
    check(r, exp)
    x.states_equal(name)
    x.close()


IMAGES = [(f"reg.example/app{i}:v{i % 3}", (20 + 97 * i) << 20) for i in range(12)]
XRES = ["nvidia.com/gpu", "ephemeral-storage", "hugepages-2Mi", "example.com/nic"]


def rand_res_nodes(rng, n, slot0=0):
    out = rand_nodes(rng, n, 6, slot0)
    for nd in out:
        if rng.random() < 0.5:
            nd.extended["nvidia.com/gpu"] = rng.choice([1, 2, 4, 8])
        if rng.random() < 0.6:
            nd.extended["ephemeral-storage"] = rng.choice([50, 100, 200]) * Gi
        if rng.random() < 0.2:
            nd.extended["hugepages-2Mi"] = rng.choice([256, 1024]) * Mi
        if rng.random() < 0.1:
            nd.extended["example.com/nic"] = rng.randint(1, 4)
        nd.images = rng.sample(IMAGES, rng.randint(0, 5))
    return out


def rand_res_pod(rng, j):
    p = rand_pod(rng, j, spread_frac=0.25)
    c = p.containers[0]
    if rng.random() < 0.3:
        c.requests["nvidia.com/gpu"] = rng.choice([0, 1, 2, 4])
    if rng.random() < 0.3:
        c.requests["ephemeral-storage"] = rng.choice([1, 10, 40]) * Gi
    if rng.random() < 0.05:
        c.requests["hugepages-2Mi"] = 256 * Mi
    if rng.random() < 0.05:
        c.requests["example.com/nic"] = 1
    if rng.random() < 0.5:
        c.image = rng.choice(IMAGES)[0] if rng.random() < 0.8 else "unknown/img"
    if rng.random() < 0.1:
        p.init_containers = [Container({"nvidia.com/gpu": rng.choice([1, 8])}, image=rng.choice(IMAGES)[0])]
    return p


@pytest.mark.parametrize("seed,n,P", [(21, 400, 256), (22, 1500, 64)])
def test_resources_images_random_stream(seed, n, P):
    rng = random.Random(seed)
    x = Pair(n, pods_per_round=P)
    x.upsert(rand_res_nodes(rng, n), list(range(n)))
    pre = [rand_res_pod(rng, 50_000 + j) for j in range(n // 3)]
    for p in pre:
        p.topology_spread = []
    live = [(p, rng.randrange(n)) for p in pre]
    x.add([p for p, _ in live], [s for _, s in live])
    for b in range(3):
        pods = [rand_res_pod(rng, b * 1000 + j) for j in range(150)]
        x.schedule(pods, f"seed {seed} batch {b}")
        x.states_equal(f"seed {seed} batch {b}")
        rng.shuffle(live)
        gone, live = live[:5], live[5:]
        x.add([p for p, _ in gone], [s for _, s in gone], sign=-1)
        slots = rng.sample(range(n), 3)
        live = [(p, s) for p, s in live if s != slots[1]]
        x.upsert(rand_res_nodes(rng, 3, slot0=n + 10 * b), slots)  # new images / allocatable
        x.delete([slots[1]])
        x.dump_equal(rand_res_pod(rng, 90_000 + b), f"seed {seed} dump {b}")
    x.close()


# ------------------------------------------------------------ InterPodAffinity

@pytest.mark.parametrize("name", sorted(__import__("ipa_cases").CASES))
@pytest.mark.parametrize("P", [256, 2])
def test_ipa_case_gpu(name, P):
    from ipa_cases import CASES as IPA
    nodes, bound, pods, exp, dumps = IPA[name]()
    x = Pair(len(nodes), pods_per_round=P)
    x.upsert(nodes, list(range(len(nodes))))
    x.add([p for p, _ in bound], [s for _, s in bound])
    for j, p in enumerate(pods):
        if j in dumps:
            out = x.dump_equal(p, f"{name} dump {j}")
            assert [(out[i].affinity_pod_raw, out[i].affinity_pod_score) for i in range(len(nodes))] == dumps[j]
    r = x.schedule(pods, name)
    check(r, exp)
    x.states_equal(name)
    x.close()


def rand_term(rng, kinds=("affinity", "anti-affinity", "preferred-affinity", "preferred-anti-affinity")):
    from ksched.objects import PodAffinityTerm
    kind = rng.choice(kinds)
    r = rng.random()
    ns, nsel = [], None
    if r < 0.15:
        ns = rng.sample(NSS, rng.randint(1, 2))
    elif r < 0.25:
        nsel = LabelSelector({"team": "blue"}) if rng.random() < 0.7 else LabelSelector()
    sel = rand_selector(rng) if rng.random() < 0.5 else LabelSelector({"app": rng.choice(APPS)})
    return PodAffinityTerm(rng.choice([ZONE, HOST, "rack"]), sel, ns, nsel, kind,
                           rng.randint(1, 100) if kind.startswith("preferred") else 0)


def rand_ipa_pod(rng, j, frac=0.5, spread_frac=0.2):
    p = rand_pod(rng, j, spread_frac=spread_frac)
    if p.namespace == "other":
        p.namespace_labels = {"team": "blue"}
    if rng.random() < frac:
        p.affinity_terms = [rand_term(rng) for _ in range(rng.randint(1, 3))]
    return p


@pytest.mark.parametrize("seed,n,zones,P", [(31, 300, 3, 256), (32, 1200, 10, 64), (33, 600, 4, 2)])
def test_ipa_random_stream(seed, n, zones, P):
    rng = random.Random(seed)
    x = Pair(n, pods_per_round=P)
    x.upsert(rand_nodes(rng, n, zones), list(range(n)))
    pre = [rand_ipa_pod(rng, 10_000 + j, frac=0.15, spread_frac=0.0) for j in range(n // 3)]
    for p in pre:
        # bound pods: anti-affinity only in rare, narrow terms so most incoming pods stay schedulable
        p.affinity_terms = [t for t in p.affinity_terms if t.kind != "anti-affinity" or rng.random() < 0.3]
    live = [(p, rng.randrange(n)) for p in pre]
    x.add([p for p, _ in live], [s for _, s in live])
    for b in range(4):
        pods = [rand_ipa_pod(rng, b * 1000 + j, frac=0.3) for j in range(100)]
        x.schedule(pods, f"seed {seed} batch {b}")
        x.states_equal(f"seed {seed} batch {b}")
        rng.shuffle(live)
        gone, live = live[:6], live[6:]
        x.add([p for p, _ in gone], [s for _, s in gone], sign=-1)
        slots = rng.sample(range(n), 3)
        live = [(p, s) for p, s in live if s != slots[0]]
        x.upsert(rand_nodes(rng, 3, zones, slot0=n + 10 * b), slots)
        x.delete([slots[0]])
        x.upsert(rand_nodes(rng, 1, zones, slot0=n + 10 * b + 5), [slots[0]])
        extra = [rand_ipa_pod(rng, 70_000 + 10 * b + k, frac=0.8, spread_frac=0.0) for k in range(3)]
        es = [rng.randrange(n) for _ in extra]
        x.add(extra, es)  # new term classes between batches
        live += list(zip(extra, es))
        x.dump_equal(rand_ipa_pod(rng, 99_000 + b, frac=1.0), f"seed {seed} dump {b}")
        x.dump_equal(rand_ipa_pod(rng, 98_000 + b, frac=0.0, spread_frac=0.0), f"seed {seed} plain dump {b}")
    x.close()


def test_ipa_deployment_anti_affinity_replicas():
    # a deployment with hostname anti-affinity to itself and zone preferred
    # affinity: every replica lands on a fresh node until none is left
    rng = random.Random(41)
    n = 300
    x = Pair(n)
    x.upsert(rand_nodes(rng, n, 6, nozone=0.0), list(range(n)))
    from ksched.objects import PodAffinityTerm as T
    sel = LabelSelector({"app": "web"})
    terms = [T(HOST, sel, kind="anti-affinity"), T(ZONE, sel, kind="preferred-affinity", weight=10)]
    pods = [Pod(f"r{j}", containers=[Container({"cpu": 100, "memory": 64 * Mi})], labels={"app": "web"},
                affinity_terms=terms) for j in range(n + 20)]
    r = x.schedule(pods, "replicas")
    ok = r["status"] == 0
    assert ok[:n - 30].all() and not ok[n:].any()
    assert len(set(r["node_index"][ok].tolist())) == int(ok.sum())  # one per node
    x.states_equal("replicas")
    x.close()


def test_ipa_refusals():
    from ksched.objects import PodAffinityTerm as T
    s = Scheduler(8)
    a = Arena()
    na, k = nodes_array([Node("n", {"cpu": 1000, "memory": Gi, "pods": 8}, {ZONE: "a"})], a)
    s.upsert_nodes_raw(na, u32([0]), k)
    bad = [
        [T("", LabelSelector({"app": "x"}))],                                       # empty topology key
        [T(ZONE, LabelSelector({"bad key!": "x"}))],                                 # selector parse error
        [T(ZONE, LabelSelector({"app": "x"}), kind="preferred-affinity", weight=0)],  # weight out of range
        [T(ZONE, LabelSelector({"app": "x"}), namespace_selector=LabelSelector(
            match_expressions=[LabelSelectorRequirement("a", "In")]))],              # namespace selector error
        [T(ZONE, LabelSelector({"app": f"x{i}"}), kind="anti-affinity") for i in range(70)],  # > MAX_AFF
    ]
    pods = [Pod(f"p{i}", affinity_terms=t) for i, t in enumerate(bad)]
    pa, m = pods_array(pods, a)
    st = (C.c_int32 * m)()
    s.lib.ks_pods_check(s.ctx, pa, m, st)
    assert list(st) == [_abi.KS_ERR_UNSUPPORTED] * m
    ok = Pod("fine", affinity_terms=[T(ZONE, LabelSelector({"app": "x"}), kind="anti-affinity")])
    pa, m = pods_array([ok], a)
    assert s.lib.ks_pods_check(s.ctx, pa, 1, st) == 0
    s.close()


def test_ipa_shared_hostname_values():
    # two nodes carrying the same hostname label value form one topology
    # domain: per-node counts no longer stand for domain sums (AF_NODE off),
    # before and after the relabel that makes the values shared
    from ksched.objects import PodAffinityTerm as T
    rng = random.Random(51)
    n = 64
    x = Pair(n)
    nodes = rand_nodes(rng, n, 4, nozone=0.0)
    x.upsert(nodes, list(range(n)))
    sel = LabelSelector({"app": "web"})
    anti = [T(HOST, sel, kind="anti-affinity"), T(HOST, sel, kind="preferred-anti-affinity", weight=7)]
    mk = lambda j: Pod(f"w{j}", containers=[Container({"cpu": 100})], labels={"app": "web"}, affinity_terms=anti)
    x.schedule([mk(j) for j in range(20)], "unique hostnames")
    x.states_equal("unique")
    dup = rand_nodes(rng, 2, 4, slot0=1000, nozone=0.0)
    for d in dup:
        d.labels[HOST] = "shared"
    x.upsert(dup, [40, 41])
    x.schedule([mk(100 + j) for j in range(40)], "shared hostname")
    x.states_equal("shared")
    x.dump_equal(mk(999), "shared dump")
    x.close()
