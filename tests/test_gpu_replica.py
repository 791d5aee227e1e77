"""Replica runs of the spread path (ksched_spread.hip replica_*):
runs of identical pods whose constraints are all ScheduleAnyway -- deployment
replicas under the system default constraints -- scheduled by one filter pass
and one workgroup per run.  Results and node states against the oracle
(upstream v1.31.3 podtopologyspread restated in oracle.cpp) bit for bit, and
the device counters show which path ran."""
import ctypes as C
import random
import time

import pytest

from ksched.objects import (Container, LabelSelector, Node, NodeSelectorRequirement, NodeSelectorTerm, Pod,
                            PreferredSchedulingTerm, Taint, Toleration, TopologySpreadConstraint as TSC,
                            system_default_spread)
from spread_cases import HOST, ZONE
from test_gpu_spread import Pair, rand_nodes

pytestmark = pytest.mark.gpu

Gi, Mi = 1 << 30, 1 << 20
RUN_MIN_PODS = 4  # ksched_kernels.hpp


def replicas(app, n, req, variant="defaults", j0=0, **kw):
    """n identical pods of one deployment (only the names differ)."""
    sel = LabelSelector({"app": app})
    spread, defaulted = [], False
    if variant == "defaults":
        spread, defaulted = system_default_spread(sel), True
    elif variant == "own":  # the pod's own constraints: requireAllTopologies
        spread = [TSC(2, ZONE, "ScheduleAnyway", sel), TSC(1, HOST, "ScheduleAnyway", sel)]
    elif variant == "host":
        spread = [TSC(1, HOST, "ScheduleAnyway", sel)]
    elif variant == "rack":
        spread = [TSC(2, "rack", "ScheduleAnyway", sel)]
    elif variant == "other-selector":  # the selector does not count the pods themselves
        spread = system_default_spread(LabelSelector({"app": "other"}))
    elif variant == "policies":
        spread = [TSC(3, HOST, "ScheduleAnyway", sel, node_taints_policy="Honor"),
                  TSC(5, ZONE, "ScheduleAnyway", sel, node_affinity_policy="Honor", node_taints_policy="Honor")]
    elif variant == "dns":  # DoNotSchedule on the zone (the run's filter follows the counts)
        spread = [TSC(1, ZONE, "DoNotSchedule", sel)]
    elif variant == "dns-host":  # ... with a ScheduleAnyway hostname term
        spread = [TSC(1, ZONE, "DoNotSchedule", sel), TSC(2, HOST, "ScheduleAnyway", sel)]
    elif variant == "dns-rack":
        spread = [TSC(2, "rack", "DoNotSchedule", sel), TSC(1, HOST, "ScheduleAnyway", sel)]
    elif variant == "dns-min":  # minDomains above the domain count: global minimum 0
        spread = [TSC(3, ZONE, "DoNotSchedule", sel, min_domains=40)]
    elif variant == "dns-other":  # the selector does not count the pods themselves
        spread = [TSC(1, ZONE, "DoNotSchedule", LabelSelector({"app": "other"})), TSC(1, HOST, "ScheduleAnyway", sel)]
    elif variant == "dns-policies":
        spread = [TSC(2, ZONE, "DoNotSchedule", sel, node_affinity_policy="Honor", node_taints_policy="Honor")]
    else:
        raise ValueError(variant)
    return [Pod(f"{app}-{j0 + j}", containers=[Container(req)], labels={"app": app}, topology_spread=spread,
                spread_defaulted=defaulted, **kw) for j in range(n)]


def counters(x):
    st = x.s.stats()
    return int(st.replica_runs), int(st.replica_pods)


def prefill(x, rng, n, apps, k):
    bound = [Pod(f"b{j}", containers=[Container({"cpu": 100, "memory": 128 * Mi})],
                 labels={"app": rng.choice(apps)}) for j in range(k)]
    x.add(bound, [rng.randrange(n) for _ in bound])


@pytest.mark.parametrize("seed,n,zones", [(41, 600, 4), (42, 1500, 24), (43, 300, 2)])
def test_replica_deployments(seed, n, zones):
    # deployments of 1-300 replicas, every variant of program the runs model,
    # between plain pods and DoNotSchedule spread pods that split the sequences
    rng = random.Random(seed)
    x = Pair(n)
    x.upsert(rand_nodes(rng, n, zones), list(range(n)))
    apps = [f"app{k}" for k in range(6)]
    prefill(x, rng, n, apps, n)
    ssd = {"disk": "ssd"}
    pref = [PreferredSchedulingTerm(20, NodeSelectorTerm([NodeSelectorRequirement("disk", "In", ["ssd"])]))]
    tol = [Toleration("ded", "Equal", "x", "NoSchedule")]
    variants = [("defaults", {}), ("own", {}), ("host", {}), ("rack", {}), ("other-selector", {}),
                ("defaults", {"node_selector": ssd}), ("policies", {"tolerations": tol}),
                ("defaults", {"preferred": pref}), ("policies", {"node_selector": ssd, "tolerations": tol})]
    j = 0
    for b in range(3):
        pods = []
        for v, kw in variants:
            app = rng.choice(apps)
            req = {"cpu": rng.randrange(1, 20) * 50, "memory": rng.randrange(1, 32) * 64 * Mi}
            k = rng.choice([1, 3, 4, 37, 120, 300])
            pods += replicas(app, k, req, v, j0=j, **kw)
            j += k
            if rng.random() < 0.5:  # a plain pod (round kernels) or a DoNotSchedule one between deployments
                dns = [TSC(1, ZONE, "DoNotSchedule", LabelSelector({"app": app}))] if rng.random() < 0.5 else []
                pods.append(Pod(f"x{j}", containers=[Container({"cpu": 100})], labels={"app": app},
                                topology_spread=dns))
                j += 1
        x.schedule(pods, f"seed {seed} batch {b}")
        x.states_equal(f"seed {seed} batch {b}")
    runs, done = counters(x)
    assert runs > 0 and done > 0
    x.close()


DNS_VARIANTS = ["dns", "dns-host", "dns-rack", "dns-min", "dns-other", "dns-policies"]


@pytest.mark.parametrize("seed,n,zones,fill", [(71, 600, 4, False), (72, 1500, 24, False), (73, 300, 3, True),
                                               (74, 900, 7, True)])
def test_replica_dns_deployments(seed, n, zones, fill):
    # DoNotSchedule on a non-hostname key in replica runs: the start's skew
    # (prefilled matching pods) blocks domains, placements unblock them (the
    # minimum moves), nodes lacking the key are never candidates; with fill
    # the nodes run out of pods so runs end at Fit losses and the last pods
    # fail the spread filter or find no node
    rng = random.Random(seed)
    x = Pair(n)
    nodes = rand_nodes(rng, n, zones)
    if fill:
        for nd in nodes:
            nd.allocatable["pods"] = rng.choice([1, 2, 4])
    x.upsert(nodes, list(range(n)))
    apps = [f"app{k}" for k in range(4)] + ["other"]
    prefill(x, rng, n, apps, n // 2)
    ssd = {"disk": "ssd"}
    tol = [Toleration("ded", "Equal", "x", "NoSchedule")]
    j = 0
    for b in range(3):
        pods = []
        for v in DNS_VARIANTS:
            kw = rng.choice([{}, {}, {"node_selector": ssd}, {"tolerations": tol}])
            app = rng.choice(apps[:4])
            req = {"cpu": rng.randrange(1, 20) * 50, "memory": rng.randrange(1, 32) * 64 * Mi}
            k = rng.choice([3, 5, 37, 120, 300])
            pods += replicas(app, k, req, v, j0=j, **kw)
            j += k
        x.schedule(pods, f"seed {seed} batch {b}")
        x.states_equal(f"seed {seed} batch {b}")
    runs, done = counters(x)
    assert runs > 0 and done > 0
    x.close()


@pytest.mark.parametrize("replicas_on", [1, 0])
def test_replica_fit_losses_and_unschedulable(replicas_on):
    # nodes fill after a few pods: runs end at every Fit loss (and fall back to
    # the chain when they end short); the last replicas find no node at all
    rng = random.Random(44)
    n = 150
    x = Pair(n, options={"spread_replica_runs": replicas_on})
    nodes = [Node(f"h{i}", {"cpu": 1000, "memory": 4 * Gi, "pods": rng.choice([2, 3, 5])},
                  {HOST: f"h{i}", ZONE: f"z{i % 3}"}) for i in range(n)]
    x.upsert(nodes, list(range(n)))
    pods = replicas("web", 700, {"cpu": 300, "memory": 256 * Mi})
    r = x.schedule(pods, "fill")
    assert (r["status"] == 0).any() and (r["status"] == 1).any()
    x.states_equal("fill")
    runs, done = counters(x)
    assert (done > 0) == bool(replicas_on)
    x.close()


def test_replica_touched_cap():
    # more distinct nodes than one run may take (RUN_TOUCHED): several runs
    rng = random.Random(45)
    n = 2600
    x = Pair(n)
    x.upsert(rand_nodes(rng, n, 10, nozone=0.0), list(range(n)))
    pods = replicas("web", 2200, {"cpu": 100, "memory": 64 * Mi}, "host")
    r = x.schedule(pods, "touched cap")
    assert (r["status"] == 0).all()
    x.states_equal("touched cap")
    runs, done = counters(x)
    assert runs >= 3 and done == 2200
    x.close()


def test_replica_refused_runs():
    # more (domain, hostname count) groups than a run holds, and a hostname
    # count beyond the key's range: the per-pod chain schedules them
    n = 1300
    x = Pair(n)
    nodes = [Node(f"h{i}", {"cpu": 64000, "memory": 256 * Gi, "pods": 400}, {HOST: f"h{i}", ZONE: f"z{i % 4}",
                                                                            "rack": f"r{i}"}) for i in range(n)]
    x.upsert(nodes, list(range(n)))
    x.schedule(replicas("web", 40, {"cpu": 100}, "rack"), "groups")
    x.states_equal("groups")
    assert counters(x) == (0, 0)
    many = [Pod(f"b{j}", containers=[Container({"cpu": 10})], labels={"app": "api"}) for j in range(300)]
    x.add(many, [7] * len(many))
    x.schedule(replicas("api", 30, {"cpu": 100}), "hostname count")
    x.states_equal("hostname count")
    assert counters(x) == (0, 0)
    x.schedule(replicas("db", 30, {"cpu": 100}), "runs again")  # other pods: counts 0, runs
    x.states_equal("runs again")
    assert counters(x)[1] == 30
    x.close()


def test_replica_short_sequences_and_taints():
    # sequences shorter than RUN_MIN_PODS take the chain; normalised
    # TaintToleration (PreferNoSchedule) and ImageLocality-free pods
    rng = random.Random(46)
    n = 500
    x = Pair(n)
    nodes = rand_nodes(rng, n, 5)
    for i in range(0, n, 7):
        nodes[i].taints = [Taint("soft", "y", "PreferNoSchedule")]
    x.upsert(nodes, list(range(n)))
    prefill(x, rng, n, ["web"], 200)
    pods = replicas("web", RUN_MIN_PODS - 1, {"cpu": 150}) + replicas("web", RUN_MIN_PODS, {"cpu": 200}, j0=10) + \
        replicas("web", 64, {"cpu": 250, "memory": Gi}, j0=20)
    x.schedule(pods, "short")
    x.states_equal("short")
    assert counters(x)[1] == RUN_MIN_PODS + 64
    x.close()


def test_class_created_while_a_batch_runs():
    # ks_batch_prepare creates a new deployment's selector class while the
    # batch before it still runs (ABI 6, no drain).  Batch A binds plain pods
    # labelled app=late, which no class selects yet; its rounds are held back
    # 0.3 s (ks_debug_stall), so it is in flight while batch B compiles.  B
    # holds the replicas of a deployment selecting app=late and of a fresh
    # one.  A's pods are counted into B's class when A ends
    # (ks_stats.late_class_pods); results and node states equal the oracle's.
    from helpers import assert_results_equal, res_array
    from ksched.objects import pods_array
    rng = random.Random(61)
    n = 1200
    x = Pair(n)
    x.upsert(rand_nodes(rng, n, 6), list(range(n)))
    x.schedule(replicas("warm", 1, {"cpu": 100}), "columns")  # topology columns exist
    plain = [Pod(f"late-{j}", containers=[Container({"cpu": 100, "memory": 64 * Mi})], labels={"app": "late"})
             for j in range(300)]
    deps = replicas("late", 48, {"cpu": 250, "memory": 256 * Mi}, j0=1000) + \
        replicas("fresh", 24, {"cpu": 300, "memory": 128 * Mi})
    pa, ma = pods_array(plain, x.a)
    pb, mb = pods_array(deps, x.a)
    want_a, want_b = x.o.schedule(pa, ma), x.o.schedule(pb, mb)
    s = x.s
    s.reset_stats()
    assert s.lib.ks_debug_stall(s.ctx, 0, 300_000) == 0
    ba = s.prepare(pa, ma)
    started = C.c_uint64()
    assert s.lib.ks_debug_runs_started(s.ctx, C.byref(started)) == 0
    runs0 = started.value
    assert s.lib.ks_batch_submit(s.ctx, ba) == 0, s.lib.ks_last_error(s.ctx)
    # wait until the worker has taken A's class masks (its run started); A
    # then waits in its held-back round
    deadline = time.monotonic() + 30
    while started.value == runs0:
        assert time.monotonic() < deadline, "batch A's run never started"
        time.sleep(0.001)
        assert s.lib.ks_debug_runs_started(s.ctx, C.byref(started)) == 0
    bb = s.prepare(pb, mb)  # A is in flight: the classes are created without a drain
    assert s.lib.ks_batch_submit(s.ctx, bb) == 0, s.lib.ks_last_error(s.ctx)
    for b, m, want, what in ((ba, ma, want_a, "batch in flight"), (bb, mb, want_b, "new classes")):
        assert s.lib.ks_batch_wait(s.ctx, b) == 0, s.lib.ks_last_error(s.ctx)
        assert_results_equal(s.results(b, m), want, m, what)
        s.free(b)
    st = s.stats()
    bound_a = int((res_array(want_a, ma)["status"] == 0).sum())
    assert bound_a > 0 and st.classes_inflight == 2 and st.late_class_pods == bound_a, \
        (bound_a, st.classes_inflight, st.late_class_pods)
    x.states_equal("late class counts")
    x.close()
