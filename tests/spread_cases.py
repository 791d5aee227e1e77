"""PodTopologySpread cases with outcomes derived by hand from upstream v1.31.3
pkg/scheduler/framework/plugins/podtopologyspread (filtering.go#Filter,
calPreFilterState, minMatchNum; scoring.go#initPreScoreState, PreScore, Score,
NormalizeScore, topologyNormalizingWeight = math.Log(size + 2)).

Every case is (nodes, bound, pods, exp, dumps):
  bound: [(pod, slot)] bound before scheduling (ks_pods_add / oracle_pods_add)
  exp:   per scheduled pod, as tests/scenarios.py#check
  dumps: {pod index: [(spread_raw, spread_score) per node]} from the plugin
         score dump of that pod against the cache before it is scheduled
Used by test_oracle_spread.py (CPU oracle) and test_gpu_spread.py (libksched
against the oracle and these expectations).
"""
import math

from ksched.objects import (Container, LabelSelector, LabelSelectorRequirement, Node, Pod, Taint,
                            TopologySpreadConstraint as TSC, system_default_spread)
from scenarios import SPREAD

Gi = 1 << 30
Mi = 1 << 20
ZONE, HOST = "topology.kubernetes.io/zone", "kubernetes.io/hostname"
WEB = LabelSelector({"app": "web"})


def node(name, zone=None, labels=None, taints=None):
    lab = {HOST: name}
    if zone is not None:
        lab[ZONE] = zone
    lab.update(labels or {})
    return Node(name, {"cpu": 4000, "memory": 8 * Gi, "pods": 110}, lab, list(taints or []))


def pod(name, labels=None, spread=None, ns="default", defaulted=False, **kw):
    return Pod(name, namespace=ns, containers=[Container({"cpu": 100, "memory": 100 * Mi})],
               labels=dict(labels if labels is not None else {"app": "web"}), topology_spread=list(spread or []),
               spread_defaulted=defaulted, **kw)


def four_nodes(extra=None):
    # zones a, a, b, c; matching pods: 2 on n0, 1 on n2
    nodes = [node("n0", "a"), node("n1", "a"), node("n2", "b"), node("n3", "c")] + list(extra or [])
    bound = [(pod("b0"), 0), (pod("b1"), 0), (pod("b2"), 2)]
    return nodes, bound


CASES = {}


def case(fn):
    CASES[fn.__name__] = fn
    return fn


@case
def zone_do_not_schedule():
    nodes, bound = four_nodes()
    c = [TSC(1, ZONE, "DoNotSchedule", WEB)]
    pods = [pod("p0", spread=c), pod("p1", spread=c), pod("p2", spread=c)]
    exp = [
        # counts a=2 b=1 c=0, min 0: a 2+1-0 > 1, b 1+1 > 1, c ok
        dict(node=3, feasible=1, fails={SPREAD: 3}),
        # a=2 b=1 c=1, min 1: a fails, b / c ok; equal scores -> lowest slot
        dict(node=2, feasible=2, fails={SPREAD: 2}),
        # a=2 b=2 c=1, min 1: only c
        dict(node=3, feasible=1, fails={SPREAD: 3}),
    ]
    return nodes, bound, pods, exp, {}


@case
def min_domains():
    nodes = [node("n0", "a"), node("n1", "a"), node("n2", "b"), node("n3", "c")]
    bound = [(pod("b0"), 0), (pod("b1"), 2), (pod("b2"), 3)]  # a=1 b=1 c=1
    pods = [pod("p0", spread=[TSC(1, ZONE, "DoNotSchedule", WEB)]),
            pod("p1", spread=[TSC(1, ZONE, "DoNotSchedule", WEB, min_domains=4)])]
    exp = [
        dict(node=1, feasible=4),  # skew 1 everywhere; n1 has no pod -> best LeastAllocated
        # after p0 on n1: a=2 b=1 c=1; 3 domains < minDomains 4 -> min 0: every skew >= 2
        dict(node=None, status=1, feasible=0, fails={SPREAD: 4}),
    ]
    return nodes, bound, pods, exp, {}


@case
def missing_key_unresolvable():
    nodes, bound = four_nodes([node("n4")])  # n4 has no zone label
    pods = [pod("p0", spread=[TSC(2, ZONE, "DoNotSchedule", WEB)])]
    # min 0: a 2+1 > 2 fails, b 1+1 ok, c ok, n4 lacks the key
    exp = [dict(node=3, feasible=2, fails={SPREAD: 3})]
    return nodes, bound, pods, exp, {}


@case
def zone_schedule_anyway():
    nodes, bound = four_nodes()
    pods = [pod("p0", spread=[TSC(1, ZONE, "ScheduleAnyway", WEB)])]
    w = math.log(3 + 2)  # three zones among the filtered nodes
    raw = [round(2 * w), round(2 * w), round(1 * w), 0]  # 3, 3, 2, 0
    mn, mx = min(raw), max(raw)
    score = [100 * (mx + mn - r) // mx for r in raw]  # 0, 0, 33, 100
    exp = [dict(node=3, feasible=4)]
    return nodes, bound, pods, exp, {0: list(zip(raw, score))}


@case
def hostname_schedule_anyway():
    nodes, bound = four_nodes()
    pods = [pod("p0", spread=[TSC(1, HOST, "ScheduleAnyway", WEB)])]
    w = math.log(4 + 2)  # four filtered nodes, none ignored
    raw = [round(2 * w), 0, round(w), 0]  # 4, 0, 2, 0
    score = [100 * (4 + 0 - r) // 4 for r in raw]  # 0, 100, 50, 100
    exp = [dict(node=1, feasible=4)]
    return nodes, bound, pods, exp, {0: list(zip(raw, score))}


@case
def system_defaults_keep_unlabelled_nodes():
    # spread_defaulted: requireAllTopologies = false, so n4 (no zone) is scored:
    # its zone is "" for topoSize and it gets no zone term
    nodes, bound = four_nodes([node("n4")])
    pods = [pod("p0", spread=system_default_spread(WEB), defaulted=True)]
    wz, wh = math.log(4 + 2), math.log(5 + 2)  # zones a, b, c, ""; five hosts
    raw = [round(2 * wh + 2 + 2 * wz + 4), round(0 + 2 + 2 * wz + 4), round(wh + 2 + wz + 4),
           round(0 + 2 + 0 + 4), round(0 + 2)]  # 13, 10, 10, 6, 2
    mn, mx = min(raw), max(raw)
    score = [100 * (mx + mn - r) // mx for r in raw]
    exp = [dict(node=4, feasible=5)]
    return nodes, bound, pods, exp, {0: list(zip(raw, score))}


@case
def own_constraints_ignore_unlabelled_nodes():
    # the pod's own ScheduleAnyway constraints: n4 lacks the zone key -> ignored
    # (score 0), the others normalise among themselves
    nodes, bound = four_nodes([node("n4")])
    pods = [pod("p0", spread=[TSC(1, ZONE, "ScheduleAnyway", WEB)])]
    w = math.log(3 + 2)
    raw = [round(2 * w), round(2 * w), round(w), 0]
    score = [100 * (3 - r) // 3 for r in raw] + [0]
    exp = [dict(node=3, feasible=5)]
    return nodes, bound, pods, exp, {0: list(zip(raw + [0], score))}


@case
def namespaces_are_separate():
    nodes, bound = four_nodes()
    bound += [(pod("o0", ns="other"), 3), (pod("o1", ns="other"), 3)]
    pods = [pod("p0", spread=[TSC(1, ZONE, "DoNotSchedule", WEB)]),
            pod("q0", ns="other", spread=[TSC(1, ZONE, "DoNotSchedule", WEB)])]
    exp = [dict(node=3, feasible=1),  # other-namespace pods on n3 do not count
           # ns other: a=0 b=0 c=2 (n3 now also holds p0, a default-namespace pod) -> min 0, c fails
           dict(node=1, feasible=3, fails={SPREAD: 1})]
    return nodes, bound, pods, exp, {}


@case
def node_affinity_policy():
    extra = {"disk": "ssd"}
    nodes = [node("n0", "a", extra), node("n1", "a", extra), node("n2", "b", extra), node("n3", "c")]
    bound = [(pod("b0"), 0), (pod("b1"), 0), (pod("b2"), 2)]
    honor = pod("honor", spread=[TSC(1, ZONE, "DoNotSchedule", WEB)], node_selector=extra)
    ignore = pod("ignore", spread=[TSC(1, ZONE, "DoNotSchedule", WEB, node_affinity_policy="Ignore")],
                 node_selector=extra)
    # Honor: zone c (no ssd node) is not a domain -> min = b = 1: a fails, b ok
    # Ignore: c counts with 0 -> min 0: a and b fail, n3 fails NodeAffinity
    exp = [dict(node=2, feasible=1), dict(node=None, status=1, feasible=0)]
    return nodes, bound, [honor, ignore], exp, {}


@case
def node_taints_policy():
    nodes = [node("n0", "a"), node("n1", "a"), node("n2", "b"), node("n3", "c", taints=[Taint("k", "v")])]
    bound = [(pod("b0"), 0), (pod("b1"), 0), (pod("b2"), 2)]
    honor = pod("honor", spread=[TSC(1, ZONE, "DoNotSchedule", WEB, node_taints_policy="Honor")])
    ignore = pod("ignore", spread=[TSC(1, ZONE, "DoNotSchedule", WEB)])
    # Honor: tainted n3's zone is not a domain -> min 1 -> n2; Ignore (default): min 0, nothing fits
    exp = [dict(node=2, feasible=1), dict(node=None, status=1, feasible=0)]
    return nodes, bound, [honor, ignore], exp, {}


@case
def match_label_keys():
    nodes = [node("n0", "a"), node("n1", "a"), node("n2", "b"), node("n3", "c")]
    bound = [(pod("b0", {"app": "web", "rev": "1"}), 0), (pod("b1", {"app": "web", "rev": "1"}), 0),
             (pod("b2", {"app": "web", "rev": "2"}), 2)]
    c = [TSC(1, ZONE, "DoNotSchedule", WEB, match_label_keys=["rev"])]
    pods = [pod("p0", {"app": "web", "rev": "2"}, spread=c)]
    # only rev=2 counts: a=0 b=1 c=0, min 0 -> b fails; n1 / n3 hold no pod -> n1
    exp = [dict(node=1, feasible=3, fails={SPREAD: 1})]
    return nodes, bound, pods, exp, {}


@case
def nil_and_empty_selectors():
    nodes, bound = four_nodes()
    pods = [pod("nil", spread=[TSC(1, ZONE, "DoNotSchedule", None)]),           # counts 0, no self match
            pod("empty", spread=[TSC(1, ZONE, "DoNotSchedule", LabelSelector())]),  # Empty(): 0, self 1
            pod("other", labels={"app": "db"}, spread=[TSC(1, ZONE, "DoNotSchedule", WEB)])]  # no self match
    exp = [dict(node=1, feasible=4), dict(node=3, feasible=4),
           # nil landed on n1, empty on n3 (both app=web): a=3 b=1 c=1, min 1, no self match -> a fails
           dict(node=2, feasible=2, fails={SPREAD: 2})]
    return nodes, bound, pods, exp, {}


@case
def expressions_and_mixed_constraints():
    nodes, bound = four_nodes()
    sel = LabelSelector(match_expressions=[LabelSelectorRequirement("app", "In", ["web", "api"]),
                                           LabelSelectorRequirement("tier", "DoesNotExist")])
    pods = [pod("p0", spread=[TSC(2, ZONE, "DoNotSchedule", sel), TSC(1, HOST, "ScheduleAnyway", sel)]),
            pod("p1", labels={"app": "api"}, spread=[TSC(1, ZONE, "DoNotSchedule", sel),
                                                     TSC(1, HOST, "ScheduleAnyway", sel)])]
    # p0: zone min 0, maxSkew 2: a 3 > 2 fails; b, c ok; hostname scores n2 (1 pod) below n3 (0)
    # p1 (after p0 on n3): a=2 b=1 c=1, min 1: a fails (2), b and c ok (skew 1)
    exp = [dict(node=3, feasible=2, fails={SPREAD: 2}), dict(node=2, feasible=2, fails={SPREAD: 2})]
    return nodes, bound, pods, exp, {}
