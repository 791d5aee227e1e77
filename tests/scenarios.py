"""Hand-built k8s-shaped scenarios with expected outcomes derived from upstream
v1.31.3 plugin semantics.  Used by
test_oracle_semantics.py (CPU oracle) and test_gpu_semantics.py (libksched vs
the oracle vs these expectations)."""
from ksched.objects import (Container, Node, NodeSelectorRequirement as Req, NodeSelectorTerm as Term, Pod,
                            PreferredSchedulingTerm as Pref, Taint, Toleration)

Gi = 1 << 30
UNSCHED, NAME, TAINT, AFFINITY, FIT, SPREAD, POD_AFFINITY, PREFILTER = range(8)


def node(name, cpu=32000, mem=256 * Gi, pods=32, labels=None, taints=None, unschedulable=False):
    return Node(name, {"cpu": cpu, "memory": mem, "pods": pods}, dict(labels or {}), list(taints or []),
                unschedulable)


def pod(name, cpu=None, mem=None, **kw):
    req = {}
    if cpu is not None:
        req["cpu"] = cpu
    if mem is not None:
        req["memory"] = mem
    return Pod(name, containers=[Container(req)], **kw)


# Each scenario: (nodes, pods, expectations); expectation per pod: dict with any of
# node (slot or None), status (0 ok / 1 unschedulable / 2 error), feasible, fails {plugin: n}, score.
SCENARIOS = {}


def scenario(fn):
    SCENARIOS[fn.__name__] = fn
    return fn


@scenario
def taints_filter():
    nodes = [node("a", taints=[Taint("k", "v", "NoSchedule")]), node("b", taints=[Taint("x", "", "NoExecute")]),
             node("c")]
    pods = [
        pod("none"),                                                            # only c
        pod("eq", tolerations=[Toleration("k", "Equal", "v", "NoSchedule")]),    # a, c -> a (slot 0)
        pod("eq-wrong-value", tolerations=[Toleration("k", "Equal", "w", "NoSchedule")]),
        pod("eff-mismatch", tolerations=[Toleration("k", "Exists", "", "NoExecute")]),
        pod("all", tolerations=[Toleration("", "Exists", "", "")]),             # everything
        pod("bad-op", tolerations=[Toleration("k", "Maybe", "v", "")]),
        pod("noexec", tolerations=[Toleration("x", "Exists", "", "NoExecute")]),  # b, c -> b
    ]
    exp = [
        dict(node=2, feasible=1, fails={TAINT: 2}),
        dict(node=0, feasible=2, fails={TAINT: 1}),
        dict(node=2, feasible=1),
        dict(node=2, feasible=1),
        dict(node=0, feasible=3),
        dict(node=2, feasible=1),
        dict(node=1, feasible=2),
    ]
    return nodes, pods, exp


@scenario
def prefer_taints_normalize():
    p = lambda k: Taint(k, "true", "PreferNoSchedule")  # noqa: E731
    nodes = [node("two", taints=[p("s"), p("t")]), node("one", taints=[p("s")]), node("zero")]
    # TT raw 2/1/0, max 2 -> 0/50/100; totals differ by 3*50
    pods = [pod("x", cpu=1000, mem=Gi), pod("tol-s", cpu=1000, mem=Gi,
                                               tolerations=[Toleration("s", "Exists", "", "PreferNoSchedule")]),
            pod("tol-all-effects", cpu=1000, mem=Gi, tolerations=[Toleration("", "Exists", "", "")])]
    exp = [dict(node=2), dict(node=1), dict(node=0)]
    return nodes, pods, exp


@scenario
def normalizer_guess_wrong():
    # The sweep scores normalising plugins with a guessed max raw (the worst
    # prefer-taint word present / the sum of preferred weights); here the node
    # carrying the worst word is infeasible and the preferred terms exclude
    # each other, so the measured max differs and the pods are re-swept.
    p = lambda k: Taint(k, "true", "PreferNoSchedule")  # noqa: E731
    T = lambda *reqs: Term(list(reqs))  # noqa: E731
    nodes = [node("two", taints=[p("s"), p("t"), Taint("h", "", "NoSchedule")], labels={"zone": "z0"}),
             node("one", taints=[p("s")], labels={"zone": "z1"}), node("zero", labels={"zone": "z2"}),
             node("full", pods=0, taints=[p("s"), p("t")])]
    pods = [
        pod("x", cpu=1000, mem=Gi),                                               # guess 2, max 1 -> zero
        pod("tol-h", cpu=1000, mem=Gi, tolerations=[Toleration("h", "Exists", "", "NoSchedule")]),  # max 2
        pod("pref", cpu=1000, mem=Gi, tolerations=[Toleration("s", "Exists", "", "PreferNoSchedule")],
            preferred=[Pref(10, T(Req("zone", "In", ["z1"]))), Pref(20, T(Req("zone", "In", ["z2"])))]),
        pod("pref-one-feasible", cpu=1000, mem=Gi, node_selector={"zone": "z1"},
            preferred=[Pref(10, T(Req("zone", "In", ["z1"]))), Pref(20, T(Req("zone", "In", ["z2"])))]),
        pod("none-feasible", cpu=10 ** 9, mem=Gi),
    ]
    exp = [dict(node=2, feasible=2), dict(node=2, feasible=3), dict(node=2, feasible=2),
           dict(node=1, feasible=1, single=True), dict(status=1, node=None, feasible=0)]
    return nodes, pods, exp


@scenario
def unschedulable_nodes():
    nodes = [node("cordoned", unschedulable=True), node("ok")]
    pods = [pod("x"), pod("tol", tolerations=[Toleration("node.kubernetes.io/unschedulable", "Exists", "",
                                                          "NoSchedule")]),
            pod("tol-wrong-effect", tolerations=[Toleration("node.kubernetes.io/unschedulable", "Exists", "",
                                                            "NoExecute")])]
    exp = [dict(node=1, fails={UNSCHED: 1}), dict(node=0, feasible=2), dict(node=1, fails={UNSCHED: 1})]
    return nodes, pods, exp


@scenario
def node_name():
    nodes = [node("n0"), node("n1"), node("n2", taints=[Taint("k", "v", "NoSchedule")])]
    pods = [pod("pin", node_name="n1"), pod("pin-tainted", node_name="n2"), pod("pin-missing", node_name="zz")]
    exp = [dict(node=1, feasible=1, fails={NAME: 2}),
           dict(node=None, status=1, fails={NAME: 2, TAINT: 1}),
           dict(node=None, status=1, fails={NAME: 3})]
    return nodes, pods, exp


@scenario
def node_affinity_operators():
    nodes = [node("a", labels={"zone": "z1", "gpus": "8", "ssd": ""}),
             node("b", labels={"zone": "z2", "gpus": "2"}),
             node("c", labels={"zone": "z1", "gpus": "many"}),
             node("d", labels={})]
    T = lambda *reqs, fields=(): Term(list(reqs), list(fields))  # noqa: E731
    pods = [
        pod("sel", node_selector={"zone": "z1"}),                                   # a, c
        pod("in", required_terms=[T(Req("zone", "In", ["z2", "z9"]))]),             # b
        pod("notin", required_terms=[T(Req("zone", "NotIn", ["z1"]))]),             # b, d (absent key passes)
        pod("exists", required_terms=[T(Req("ssd", "Exists"))]),                    # a
        pod("dne", required_terms=[T(Req("ssd", "DoesNotExist"))]),                 # b, c, d
        pod("gt", required_terms=[T(Req("gpus", "Gt", ["4"]))]),                    # a ("many" fails parse)
        pod("lt", required_terms=[T(Req("gpus", "Lt", ["4"]))]),                    # b
        pod("gt-bad-value", required_terms=[T(Req("gpus", "Gt", ["four"]))]),       # parse error: none
        pod("gt-neg-value", required_terms=[T(Req("gpus", "Gt", ["-1"]))]),         # "-1" invalid label value
        pod("or-terms", required_terms=[T(Req("zone", "In", ["z2"])), T(Req("ssd", "Exists"))]),  # a, b
        pod("bad-term-or", required_terms=[T(Req("gpus", "Gt", ["x"])), T(Req("zone", "In", ["z2"]))]),  # b
        pod("nil-terms", required_terms=[]),                                        # required set, no terms: none
        pod("empty-term", required_terms=[T(), T(Req("zone", "In", ["z2"]))]),      # empty term skipped: b
        pod("fields", required_terms=[T(fields=[Req("metadata.name", "In", ["c"])])]),  # c
        pod("fields-notin", required_terms=[T(fields=[Req("metadata.name", "NotIn", ["c"])])]),  # a, b, d
        pod("fields-bad", required_terms=[T(fields=[Req("metadata.name", "In", ["a", "b"])])]),  # 2 values: none
        pod("bad-key", required_terms=[T(Req("bad key!", "Exists"))]),              # invalid key: none
        pod("sel-and-aff", node_selector={"zone": "z1"}, required_terms=[T(Req("gpus", "Lt", ["10"]))]),  # a
        pod("in-empty-values", required_terms=[T(Req("zone", "In", []))]),          # parse error: none
    ]
    exp = [dict(node=0, feasible=2, fails={AFFINITY: 2}), dict(node=1, feasible=1), dict(node=1, feasible=2),
           dict(node=0, feasible=1), dict(node=1, feasible=3), dict(node=0, feasible=1), dict(node=1, feasible=1),
           dict(status=1, fails={AFFINITY: 4}), dict(status=1), dict(node=0, feasible=2), dict(node=1, feasible=1),
           dict(status=1), dict(node=1, feasible=1), dict(node=2, feasible=1), dict(node=3, feasible=3),
           dict(status=1), dict(status=1), dict(node=0, feasible=1), dict(status=1)]
    return nodes, pods, exp


@scenario
def preferred_affinity():
    nodes = [node("a", labels={"zone": "z1"}), node("b", labels={"zone": "z2", "fast": "1"}),
             node("c", labels={"zone": "z3", "fast": "1"})]
    T = lambda *reqs: Term(list(reqs))  # noqa: E731
    pods = [
        pod("pref-z2", preferred=[Pref(50, T(Req("zone", "In", ["z2"])))]),                       # b
        pod("pref-fast-z3", preferred=[Pref(10, T(Req("fast", "Exists"))), Pref(20, T(Req("zone", "In", ["z3"])))]),
        pod("pref-zero-weight", preferred=[Pref(0, T(Req("zone", "In", ["z3"])))]),                 # a (tie)
        pod("pref-empty-list", preferred=[]),                                                       # a
        pod("pref-parse-error", preferred=[Pref(5, T(Req("zone", "Gt", ["x"])))]),                   # Error
        pod("pref-error-single", node_name="c", preferred=[Pref(5, T(Req("zone", "Gt", ["x"])))]),    # 1 feasible
    ]
    exp = [dict(node=1), dict(node=2), dict(node=0), dict(node=0), dict(status=2, feasible=3),
           dict(node=2, feasible=1)]
    return nodes, pods, exp


@scenario
def fit_limits():
    nodes = [node("tiny", cpu=1000, mem=Gi, pods=1), node("big", cpu=4000, mem=8 * Gi, pods=2)]
    pods = [
        pod("fits-tiny", cpu=900, mem=Gi // 2),      # LA prefers big; goes to big (more free)
        pod("too-big", cpu=5000, mem=Gi),            # insufficient cpu everywhere
        pod("too-much-mem", cpu=10, mem=16 * Gi),    # insufficient memory everywhere
        pod("be-1"),                                  # best effort: only pod-count matters
        pod("be-2"),                                  # tiny: 1 pod max; big now has 2 -> tiny
        pod("be-3"),                                  # no pod slots anywhere
        pod("zero-explicit", cpu=0, mem=0),           # explicit zero: still needs a pod slot
    ]
    exp = [dict(node=1, feasible=2), dict(status=1, fails={FIT: 2}), dict(status=1, fails={FIT: 2}),
           dict(node=None), dict(node=None), dict(status=1, fails={FIT: 2}), dict(status=1)]
    return nodes, pods, exp


@scenario
def single_feasible_flag():
    nodes = [node("a", taints=[Taint("k", "", "NoSchedule")]), node("b")]
    pods = [pod("x", cpu=100, mem=Gi)]
    exp = [dict(node=1, feasible=1, single=True)]
    return nodes, pods, exp


@scenario
def ties_lowest_slot():
    nodes = [node(f"n{i}") for i in range(7)]
    pods = [pod("be", ) for _ in range(9)]
    # identical empty nodes: LeastAllocated (cpu) of a best-effort pod stays 99 until a node holds
    # 3 of them (32000 - 400 -> 98), so pods fill slots in order, three at a time
    exp = [dict(node=i // 3) for i in range(9)]
    return nodes, pods, exp


@scenario
def extreme_allocatable():
    # capacities at the exact-arithmetic limit (allocatable < 2^44), tiny and zero
    # capacities (a zero-allocatable resource is skipped by both scorers), and
    # requests that make (cap - req) * 100 / cap an exact integer
    big = (1 << 44) - 1
    nodes = [node("max", cpu=big, mem=big, pods=110), node("tiny", cpu=1, mem=1, pods=110),
             node("nocpu", cpu=0, mem=64 * Gi, pods=110), node("nomem", cpu=32000, mem=0, pods=110),
             node("none", cpu=0, mem=0, pods=110), node("odd", cpu=99991, mem=3 * Gi + 7, pods=110)]
    pods = [pod("be"), pod("zero", cpu=0, mem=0), pod("exact", cpu=320, mem=Gi),
            pod("half-max", cpu=big // 2, mem=big // 2 + 1), pod("p1", cpu=1, mem=1),
            pod("p3", cpu=99991 // 100, mem=(3 * Gi + 7) // 100), pod("cpu-only", cpu=1600)]
    pods += [pod(f"f{i}", cpu=37 * i + 1, mem=(i + 1) * 64 * 1024 * 1024) for i in range(24)]
    return nodes, pods, []


@scenario
def wide_label_dictionary():
    # ~200 label-pair bits: the label programs span all four 64-bit words of a
    # node's bitset (the widest EXT sweep variant), in required and preferred terms
    vals = [f"r{v}" for v in range(200)]
    racks = ["r0", "r40", "r80", "r120", "r160", "r199"]
    nodes = [node(f"n{i}", labels={"rack": racks[i], "row": f"w{i}"}) for i in range(6)]
    T = lambda *reqs: Term(list(reqs))  # noqa: E731
    pods = [
        pod("in-many", required_terms=[T(Req("rack", "In", vals))]),                          # all
        pod("in-high", required_terms=[T(Req("rack", "In", vals[120:]))]),                    # 3, 4, 5
        pod("notin-high", required_terms=[T(Req("rack", "NotIn", vals[160:]))]),              # 0-3
        pod("sel-r199", node_selector={"rack": "r199"}),                                       # 5
        pod("r80-or-w5", required_terms=[T(Req("rack", "In", ["r80"])), T(Req("row", "In", ["w5"]))]),  # 2, 5
        pod("row-and-notin-low", required_terms=[T(Req("row", "Exists"), Req("rack", "NotIn", vals[:120]))]),
        pod("pref-r199", preferred=[Pref(50, T(Req("rack", "In", ["r199"])))]),               # 5 (normalised)
    ]
    # best-effort pods keep LeastAllocated at 99 for a node's first three, so
    # ties fall to the lowest feasible slot
    exp = [dict(node=0, feasible=6), dict(node=3, feasible=3, fails={AFFINITY: 3}), dict(node=0, feasible=4),
           dict(node=5, feasible=1, fails={AFFINITY: 5}), dict(node=2, feasible=2), dict(node=3, feasible=3),
           dict(node=5, feasible=6)]
    return nodes, pods, exp


@scenario
def prefilter_result():
    # NodeAffinity.PreFilter (upstream v1.31 nodeaffinity#PreFilter) with required
    # terms that all name nodes via matchFields metadata.name In: only the union of
    # the per-term name intersections is evaluated; every other node is
    # UnschedulableAndUnresolvable "filtered out by the prefilter result" with no
    # plugin blamed (fail_counts[7]); an empty union rejects every node at
    # NodeAffinity.  The PreFilter reads RAW values: a name-In requirement with two
    # values puts both names in the result, although Filter rejects that term
    # (parse error: one value required).
    nodes = [node(f"n{i}", taints=[Taint("t", "", "NoSchedule")] if i == 3 else [],
                  unschedulable=(i == 4), labels={"zone": "a" if i % 2 else "b"}) for i in range(8)]
    F = lambda *names: Req("metadata.name", "In", list(names))  # noqa: E731
    pods = [
        pod("one", required_terms=[Term(match_fields=[F("n2")])]),
        pod("two-terms", required_terms=[Term(match_fields=[F("n5")]), Term(match_fields=[F("n1")])]),
        # tainted / unschedulable named nodes fail their Filter plugins; the rest are prefiltered
        pod("named-bad", required_terms=[Term(match_fields=[F("n3")]), Term(match_fields=[F("n4")])]),
        pod("conflict", required_terms=[Term(match_fields=[F("n1"), F("n2")])]),
        pod("absent", required_terms=[Term(match_fields=[F("nope")])]),
        # one term without a name field: every node stays eligible (no PreFilterResult)
        pod("mixed", required_terms=[Term(match_fields=[F("n6")]),
                                     Term(match_expressions=[Req("zone", "In", ["a"])])]),
        # two values: PreFilterResult {n6, n7}; the term itself never matches (parse error)
        pod("two-values", required_terms=[Term(match_fields=[F("n6", "n7")])]),
        # intersection within a term, label expression on top
        pod("intersect", required_terms=[Term(match_expressions=[Req("zone", "In", ["a"])],
                                              match_fields=[F("n7"), F("n7")])]),
    ]
    exp = [
        dict(node=2, feasible=1, fails={PREFILTER: 7}, single=True),
        dict(node=1, feasible=2, fails={PREFILTER: 6}),
        dict(node=None, status=1, feasible=0, fails={TAINT: 1, UNSCHED: 1, PREFILTER: 6}),
        dict(node=None, status=1, feasible=0, fails={AFFINITY: 8, PREFILTER: 0}),
        dict(node=None, status=1, feasible=0, fails={PREFILTER: 8}),
        dict(node=1, fails={PREFILTER: 0}),
        dict(node=None, status=1, feasible=0, fails={AFFINITY: 2, PREFILTER: 6}),
        dict(node=7, feasible=1, fails={PREFILTER: 7}),
    ]
    return nodes, pods, exp


@scenario
def ba_float_boundary():
    # a 21760m / explicit-0-memory pod on an empty 32-core
    # node has BalancedAllocation (1 - 0.34) * 100 = 65.99999999999999 -> 65 in
    # Go's float64 (66 in exact arithmetic).  Node 0 (40 cores / 64 Gi, first
    # filled to 5250m / 2 Gi by pod 0) then totals 431 = node 1's; the tie
    # goes to slot 0.  A score off by one at node 1 would pick node 1: this pins
    # the sweep's binary32 fast path's hand-off to binary64 next to integers.
    nodes = [node("b", cpu=40000, mem=64 * Gi), node("a", cpu=32000, mem=256 * Gi)]
    pods = [pod("fill", cpu=5250, mem=2 * Gi), pod("kat", cpu=21760, mem=0)]
    exp = [dict(node=0, feasible=2), dict(node=0, feasible=2, score=431)]
    return nodes, pods, exp


def check(results, exp):
    """results: structured numpy array (tests.helpers.RES_DT)."""
    for i, e in enumerate(exp):
        r = results[i]
        if "node" in e and e["node"] is not None:
            assert r["node_index"] == e["node"], (i, r, e)
        if "status" in e:
            assert r["status"] == e["status"], (i, r, e)
        elif e.get("node", 0) is not None and "node" in e:
            assert r["status"] == 0, (i, r, e)
        if "feasible" in e:
            assert r["feasible"] == e["feasible"], (i, r, e)
        for k, v in e.get("fails", {}).items():
            assert r["fail"][k] == v, (i, k, r, e)
        if "score" in e:
            assert r["total_score"] == e["score"], (i, r, e)
        if e.get("single"):
            assert r["flags"] & 1, (i, r)
