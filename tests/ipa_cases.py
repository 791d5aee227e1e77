"""InterPodAffinity cases with outcomes derived by hand from upstream v1.31.3
pkg/scheduler/framework/plugins/interpodaffinity (filtering.go#PreFilter /
Filter: satisfyPodAffinity, satisfyPodAntiAffinity,
satisfyExistingPodsAntiAffinity; scoring.go#PreScore / Score /
NormalizeScore with hardPodAffinityWeight 1).  Same shape as
tests/spread_cases.py: (nodes, bound, pods, exp, dumps) with dumps
{pod: [(affinity_pod_raw, affinity_pod_score) per node]}.
"""
from ksched.objects import LabelSelector, PodAffinityTerm as T
from scenarios import POD_AFFINITY
from spread_cases import HOST, ZONE, node, pod

WEB, DB = LabelSelector({"app": "web"}), LabelSelector({"app": "db"})


def cluster():
    # zones a, a, b, c; web pods: 2 on n0, 1 on n2
    nodes = [node("n0", "a"), node("n1", "a"), node("n2", "b"), node("n3", "c")]
    return nodes, [(pod("w0"), 0), (pod("w1"), 0), (pod("w2"), 2)]


CASES = {}


def case(fn):
    CASES[fn.__name__] = fn
    return fn


@case
def required_anti_affinity_hostname():
    nodes, bound = cluster()
    t = [T(HOST, WEB, kind="anti-affinity")]
    pods = [pod("p0", affinity_terms=t), pod("p1", affinity_terms=t), pod("p2", affinity_terms=t)]
    exp = [dict(node=1, feasible=2, fails={POD_AFFINITY: 2}),   # n0, n2 hold web pods
           dict(node=3, feasible=1, fails={POD_AFFINITY: 3}),
           dict(node=None, status=1, feasible=0, fails={POD_AFFINITY: 4})]
    return nodes, bound, pods, exp, {}


@case
def required_anti_affinity_zone():
    nodes, bound = cluster()
    t = [T(ZONE, WEB, kind="anti-affinity")]
    pods = [pod("p0", affinity_terms=t), pod("p1", affinity_terms=t)]
    exp = [dict(node=3, feasible=1, fails={POD_AFFINITY: 3}), dict(node=None, status=1, feasible=0)]
    return nodes, bound, pods, exp, {}


@case
def existing_pods_anti_affinity():
    nodes, bound = cluster()
    # a db pod on n1 refuses web pods on its host; another in zone b refuses them zone-wide
    bound += [(pod("db0", {"app": "db"}, affinity_terms=[T(HOST, WEB, kind="anti-affinity")]), 1),
              (pod("db1", {"app": "db"}, affinity_terms=[T(ZONE, WEB, kind="anti-affinity")]), 2)]
    pods = [pod("web"), pod("api", {"app": "api"})]
    exp = [dict(node=3, feasible=2, fails={POD_AFFINITY: 2}),  # n1 (host) and n2 (zone b) refuse
           dict(node=1, feasible=4)]                            # not selected: every node
    return nodes, bound, pods, exp, {}


@case
def required_affinity():
    nodes, bound = cluster()
    bound += [(pod("db", {"app": "db"}), 2)]
    nodes.append(node("n4"))  # no zone label: fails every zone term
    pods = [pod("front", {"app": "front"}, affinity_terms=[T(ZONE, DB)]),
            # no pod anywhere matches: the first of a series that selects itself passes ...
            pod("cache0", {"app": "cache"}, affinity_terms=[T(ZONE, LabelSelector({"app": "cache"}))]),
            # ... one that does not select itself does not
            pod("lonely", {"app": "x"}, affinity_terms=[T(ZONE, LabelSelector({"app": "y"}))])]
    exp = [dict(node=2, feasible=1, fails={POD_AFFINITY: 4}),
           dict(node=1, feasible=4, fails={POD_AFFINITY: 1}),   # n4 lacks the key; n1 and n3 hold no pod
           dict(node=None, status=1, feasible=0, fails={POD_AFFINITY: 5})]
    return nodes, bound, pods, exp, {}


@case
def preferred_affinity_scores():
    nodes, bound = cluster()
    pods = [pod("p0", affinity_terms=[T(ZONE, WEB, kind="preferred-affinity", weight=50)])]
    raw = [100, 100, 50, 0]  # topologyScore[zone]: a = 2 x 50, b = 1 x 50
    score = [100, 100, 50, 0]
    exp = [dict(node=1, feasible=4)]
    return nodes, bound, pods, exp, {0: list(zip(raw, score))}


@case
def preferred_anti_affinity_scores():
    nodes, bound = cluster()
    pods = [pod("p0", affinity_terms=[T(HOST, WEB, kind="preferred-anti-affinity", weight=100)])]
    raw = [-200, 0, -100, 0]
    score = [0, 100, 50, 100]  # 100 * (s - min) / (max - min)
    exp = [dict(node=1, feasible=4)]
    return nodes, bound, pods, exp, {0: list(zip(raw, score))}


@case
def existing_pods_terms_score():
    nodes, bound = cluster()
    bound += [(pod("cache", {"app": "cache"},
                   affinity_terms=[T(HOST, WEB, kind="preferred-affinity", weight=30)]), 3),
              (pod("sidecar", {"app": "sc"}, affinity_terms=[T(ZONE, WEB)]), 2)]  # required: hard weight 1
    pods = [pod("web")]
    raw = [0, 0, 1, 30]
    score = [0, 0, int(100 * (1 / 30)), 100]  # float64 then int64: 3
    exp = [dict(node=3, feasible=4)]
    return nodes, bound, pods, exp, {0: list(zip(raw, score))}


@case
def namespaces_and_selectors():
    nodes, bound = cluster()
    bound += [(pod("o0", ns="other", namespace_labels={"team": "blue"}), 3)]
    pods = [
        # the term's namespace defaults to the pod's own ("default"): the web pod in "other" does not count
        pod("d", affinity_terms=[T(HOST, WEB, kind="anti-affinity")]),
        # namespaces lists "other": only n3 holds a matching pod
        pod("o", affinity_terms=[T(HOST, WEB, namespaces=["other"], kind="anti-affinity")]),
        # a namespace selector matching team=blue namespaces
        pod("s", affinity_terms=[T(HOST, WEB, namespace_selector=LabelSelector({"team": "blue"}),
                                   kind="anti-affinity")]),
        # an empty namespace selector selects every namespace
        pod("all", affinity_terms=[T(HOST, WEB, namespace_selector=LabelSelector(), kind="anti-affinity")]),
    ]
    exp = [dict(node=1, feasible=2, fails={POD_AFFINITY: 2}),  # n0, n2 (default-ns web pods)
           # n3 (o0), and n1: "d" landed there and its own anti-affinity term
           # (default namespace, app=web) refuses "o" (existing pods' anti-affinity)
           dict(node=2, feasible=2, fails={POD_AFFINITY: 2}),
           dict(node=0, feasible=2, fails={POD_AFFINITY: 2}),  # n3 (team=blue) and n1 ("d")
           dict(node=None, status=1, feasible=0)]
    return nodes, bound, pods, exp, {}
