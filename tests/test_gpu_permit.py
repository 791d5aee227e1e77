"""Permit rejection and the cross-host gather, end to end (SURVEY.md §8(b),
§8(f) F3).

In the reference every shard schedules (and assumes) every pod; DistPermit
sends the shard's (node, TotalScore) to the pod's gatherer and only the
winner's permit passes (dist-scheduler/pkg/distpermit/distpermit.go:51-121).
Every losing shard's schedulingCycle then runs Unreserve + Cache.ForgetPod, so
the pod leaves that shard's cache (scheduler.go:386-389).  With ksched the
assume is the device commit of ks_schedule, and the shim's Unreserve hook
calls ks_pods_remove.

* test_forget_rejected_pods_vs_oracle: schedule a batch, forget a seeded 7/8
  of its scheduled pods (what the losing shards do), schedule the next batch;
  results and node tables equal an oracle that did the same.
* test_hosts_gather_equals_unsharded: four hosts, each a ksched context over
  its own quarter of the nodes, send every pod's (node name, score) over gRPC
  PodService.CollectScore to a gatherer (ksched/relay.py + libksgather,
  lowest-global-index ties); losing hosts forget the pod.  Every pod's winner
  and TotalScore equal the unsharded oracle's, and every host's node table
  equals the oracle's rows for its nodes.
Oracle: oracle/oracle.cpp (parity unpinned).
"""
import ctypes as C
import random
import threading

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array, states_np
from ksched import Scheduler, _abi, relay, synth

pytestmark = pytest.mark.gpu


def subset(ptr, idx, T=_abi.KsPod):
    out = (T * max(1, len(idx)))()
    for j, i in enumerate(idx):
        out[j] = ptr[int(i)]
    return out


def u32(a):
    a = [int(x) for x in a]
    return (C.c_uint32 * max(1, len(a)))(*a)


@pytest.mark.parametrize("kind", [synth.HETERO, synth.LABELED])
def test_forget_rejected_pods_vs_oracle(kind):
    n, m = 4000, 1500
    ns = synth.nodes(kind, n, 31)
    slots = synth.slot_array(n)
    ps = synth.pods(kind, 3 * m, 32)
    s = Scheduler(n, pods_per_round=256)
    o = pyoracle.Oracle(n)
    try:
        for t in (s, o):
            (t.upsert_nodes_raw if t is s else t.upsert)(ns.nodes, slots, n)
        rng = random.Random(33)
        for b in range(3):
            arr = ps.pods_at(b * m)
            got, want = s.schedule_raw(arr, m), o.schedule(arr, m)
            assert_results_equal(got, want, m, f"batch {b}")
            r = res_array(got, m)
            placed = np.nonzero(r["status"] == 0)[0]
            lost = sorted(rng.sample(list(placed), (7 * len(placed)) // 8))  # the losing shards' pods
            pods, sl = subset(arr, lost), u32(r["node_index"][lost])
            assert s.lib.ks_pods_remove(s.ctx, pods, sl, len(lost)) == 0, s.lib.ks_last_error(s.ctx)
            o.remove_pods(pods, sl, len(lost))
            assert np.array_equal(states_np(s.lib.ks_node_states, s.ctx, n),
                                  states_np(o.L.oracle_node_states, o.o, n)), f"node tables after forgetting batch {b}"
    finally:
        s.close()
        o.close()


def test_hosts_gather_equals_unsharded():
    H, n, m = 4, 3000, 240
    per = n // H
    ns = synth.nodes(synth.HETERO, n, 41)
    pf = synth.prefill(synth.HETERO, n, 41, 42, 0.5)
    ps = synth.pods(synth.HETERO, m, 43)
    names = [ns.nodes[i].name.decode() for i in range(n)]
    pf_slot = [pf.slot_ptr[i] for i in range(pf.n_pods)]
    hosts = []
    o = pyoracle.Oracle(n)
    o.upsert(ns.nodes, synth.slot_array(n), n)
    o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
    ev = relay.ScoreEvaluator(members=H, delay_s=30, tie=relay.TIE_LOWEST_INDEX)
    ev.set_node_order(names)  # global index = the unsharded slot
    srv = relay.CollectScoreServer(ev).start()
    try:
        for h in range(H):  # host h: global slots [h per, (h + 1) per) as local slots 0..per-1
            s = Scheduler(per)
            s.upsert_nodes_raw(subset(ns.nodes, range(h * per, (h + 1) * per), _abi.KsNode),
                               synth.slot_array(per), per)
            mine = [i for i in range(pf.n_pods) if h * per <= pf_slot[i] < (h + 1) * per]
            assert s.lib.ks_pods_add(s.ctx, subset(pf.pods, mine), u32(pf_slot[i] - h * per for i in mine),
                                     len(mine)) == 0
            hosts.append(s)
        want = res_array(o.schedule(ps.pods, m), m)
        cli = relay.ScoreClient(srv.address)
        for i in range(m):
            pod = ps.pods_at(i)
            res = [res_array(s.schedule_raw(pod, 1), 1)[0] for s in hosts]
            pay = [("", 0) if r["status"] != 0 else (names[h * per + int(r["node_index"])], int(r["total_score"]))
                   for h, r in enumerate(res)]
            permits = [None] * H

            def send(h):
                permits[h] = cli.send_score(f"pod-{i}", "default", *pay[h])

            th = [threading.Thread(target=send, args=(h,)) for h in range(H)]
            for t in th:
                t.start()
            for t in th:
                t.join(30)
            won = [h for h in range(H) if permits[h]]
            for h in range(H):  # every host assumed its own choice: the losers forget it (Unreserve)
                if res[h]["status"] == 0 and h not in won:
                    assert hosts[h].lib.ks_pods_remove(hosts[h].ctx, pod, u32([res[h]["node_index"]]), 1) == 0
            if want[i]["status"] != 0:
                assert not won and all(r["status"] != 0 for r in res), f"pod {i}: unsharded found no node"
                continue
            assert len(won) == 1, f"pod {i}: permits {permits}"
            h = won[0]
            assert h * per + int(res[h]["node_index"]) == int(want[i]["node_index"]), f"pod {i}: winner node"
            assert int(res[h]["total_score"]) == int(want[i]["total_score"]), f"pod {i}: TotalScore"
        ow = states_np(o.L.oracle_node_states, o.o, n)
        for h, s in enumerate(hosts):
            assert np.array_equal(states_np(s.lib.ks_node_states, s.ctx, per), ow[h * per:(h + 1) * per]), \
                f"host {h}: node table"
        assert (want["status"] == 0).all()
    finally:
        srv.stop()
        ev.close()
        for s in hosts:
            s.close()
        o.close()
