"""F3: cross-host gather (include/ksgather.h, ksched/relay.py) on CPU.

The gatherer's state machine against scoreevaluator.go's behaviour (fire when
every member has scored or after the delay, highest score, ties among the
first 100, late scores start a new evaluation), the member-side gatherer
choice (FNV-1 32 over "namespace/name" modulo the sorted member list,
schedulerset.go:107-143), and PodService.CollectScore end to end over gRPC on
127.0.0.1 with the reference's message layout.
"""
import threading
import time

import pytest

from ksched import relay


def run_parallel(fns):
    out = [None] * len(fns)

    def go(i, f):
        out[i] = f()

    th = [threading.Thread(target=go, args=(i, f)) for i, f in enumerate(fns)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    return out


def test_fires_when_all_members_scored():
    ev = relay.ScoreEvaluator(members=4, delay_s=30, tie=relay.TIE_LOWEST_NAME)
    t0 = time.time()
    res = run_parallel([lambda n=n, s=s: ev.record_and_wait("ns/p", n, s)
                        for n, s in (("node-a", 410), ("node-b", 455), ("node-c", 0), ("node-d", 300))])
    assert time.time() - t0 < 5  # did not wait for the delay
    assert [r[0] for r in res] == [False, True, False, False]
    assert all(r[1:] == ("node-b", 455) for r in res)
    assert ev.pending() == 0
    ev.close()


def test_fires_after_delay_with_missing_member():
    ev = relay.ScoreEvaluator(members=3, delay_s=0.3, tie=relay.TIE_LOWEST_NAME)
    t0 = time.time()
    res = run_parallel([lambda: ev.record_and_wait("ns/q", "n1", 200), lambda: ev.record_and_wait("ns/q", "n2", 350)])
    dt = time.time() - t0
    assert 0.25 <= dt < 3
    assert [r[0] for r in res] == [False, True]
    ev.close()


def test_ties_deterministic_lowest_name():
    ev = relay.ScoreEvaluator(members=3, delay_s=30, tie=relay.TIE_LOWEST_NAME)
    res = run_parallel([lambda n=n: ev.record_and_wait("ns/t", n, 500) for n in ("zeta", "alpha", "mid")])
    assert [r[0] for r in res] == [False, True, False]
    ev.close()


def test_ties_random_among_tied():
    wins = {"a": 0, "b": 0, "c": 0}
    for i in range(60):
        ev = relay.ScoreEvaluator(members=4, delay_s=30, tie=relay.TIE_RANDOM, seed=i)
        res = run_parallel([lambda n=n, s=s: ev.record_and_wait(f"ns/r{i}", n, s)
                            for n, s in (("a", 7), ("b", 7), ("c", 7), ("d", 3))])
        assert sum(r[0] for r in res) == 1 and not res[3][0]
        wins[res[0][1]] += 1
        ev.close()
    assert all(v > 5 for v in wins.values()), wins


def test_only_zero_scores_and_late_score():
    ev = relay.ScoreEvaluator(members=2, delay_s=30, tie=relay.TIE_LOWEST_NAME)
    res = run_parallel([lambda: ev.record_and_wait("ns/z", "", 0), lambda: ev.record_and_wait("ns/z", "", 0)])
    assert all(r[1:] == ("", 0) for r in res)
    # a score arriving after its pod fired starts a new evaluation (scoreevaluator.go:48-52)
    ev.set_members(1)
    permit, w, s = ev.record_and_wait("ns/z", "late-node", 90)
    assert (permit, w, s) == (True, "late-node", 90)
    ev.close()


def test_fnv1_and_target_index():
    lib = relay._abi.ksgather_lib()
    # FNV-1 32 known answers (Go hash/fnv New32): "" -> offset basis, "a" -> 0x050c5d7e
    assert lib.ksg_fnv1_32(b"", 0) == 0x811C9DC5
    assert lib.ksg_fnv1_32(b"a", 1) == 0x050C5D7E
    members = ["dist-scheduler-7", "dist-scheduler-relay-1", "dist-scheduler-2", "leader-0", "dist-scheduler-relay-0"]
    order = ["leader-0", "dist-scheduler-relay-0", "dist-scheduler-relay-1", "dist-scheduler-2", "dist-scheduler-7"]
    for key in ("default/pod-1", "ns/x", "kube-system/coredns-abc"):
        h = lib.ksg_fnv1_32(key.encode(), len(key)) % len(members)
        assert members[relay.target_index(key, members, "leader-0")] == order[h]
    assert relay.target_index("ns/x", ["only"]) == 0


class Result:  # ks_result fields host_score reads
    def __init__(self, status, node_index, total_score):
        self.status, self.node_index, self.total_score = status, node_index, total_score


def test_collect_score_over_grpc():
    ev = relay.ScoreEvaluator(members=3, delay_s=20, tie=relay.TIE_LOWEST_NAME)
    srv = relay.CollectScoreServer(ev).start()
    try:
        names = ["node-%d" % i for i in range(8)]
        hosts = [Result(0, 3, 412), Result(0, 6, 498), Result(1, -1, 0)]  # the third host has no candidate
        payloads = [relay.host_score(r, names) for r in hosts]
        assert payloads[2] == ("", 0)
        cli = relay.ScoreClient(srv.address)
        res = run_parallel([lambda n=n, s=s: cli.send_score("web-0", "default", n, s) for n, s in payloads])
        assert res == [False, True, False]
        # the wire bytes are pod.proto's: field numbers 1-4, int32 score
        b = relay.SchedulingScore(podName="p", namespace="n", nodeName="x", score=7).SerializeToString()
        assert b == b"\x0a\x01p\x12\x01n\x1a\x01x\x20\x07"
        assert relay.ScheduleResponse(permit=True).SerializeToString() == b"\x08\x01"
    finally:
        srv.stop()
        ev.close()


@pytest.mark.parametrize("pods", [50, 200])
def test_many_pods_concurrently(pods):
    # the default server: far more pods in flight than the former thread pool's
    # 64 workers, none of them waiting for the 20-s delay
    ev = relay.ScoreEvaluator(members=2, delay_s=20, tie=relay.TIE_LOWEST_NAME)
    srv = relay.CollectScoreServer(ev).start()
    t0 = time.time()
    try:
        cli = relay.ScoreClient(srv.address)
        fns = []
        for p in range(pods):
            fns.append(lambda p=p: cli.send_score(f"pod-{p}", "ns", f"a{p}", 100 + p % 3))
            fns.append(lambda p=p: cli.send_score(f"pod-{p}", "ns", f"b{p}", 101))
        res = run_parallel(fns)
        for p in range(pods):
            a, b = res[2 * p], res[2 * p + 1]
            assert a + b == 1
            assert a == (100 + p % 3 >= 101)  # ties: the lowest name (a...) wins
        assert ev.pending() == 0
        assert time.time() - t0 < 15, "pods waited for the delay: RPCs were queued"
    finally:
        srv.stop()
        ev.close()


def test_delay_fires_pending_async_records():
    # a member never answers: the server's fired thread fires the pod at its delay
    ev = relay.ScoreEvaluator(members=3, delay_s=0.4, tie=relay.TIE_LOWEST_NAME)
    srv = relay.CollectScoreServer(ev).start()
    try:
        cli = relay.ScoreClient(srv.address)
        t0 = time.time()
        res = run_parallel([lambda: cli.send_score("slow", "ns", "n1", 300), lambda: cli.send_score("slow", "ns", "n2", 200)])
        assert res == [True, False] and 0.3 <= time.time() - t0 < 5
    finally:
        srv.stop()
        ev.close()


def test_ties_lowest_global_index():
    # KSG_TIE_LOWEST_INDEX: ties go to the lowest global node index, the rule
    # each host applies to its own slots, whatever the names
    ev = relay.ScoreEvaluator(members=3, delay_s=30, tie=relay.TIE_LOWEST_INDEX)
    ev.set_node_order(["zz-node", "mm-node", "aa-node"])
    res = run_parallel([lambda n=n: ev.record_and_wait("ns/i", n, 500) for n in ("aa-node", "zz-node", "mm-node")])
    assert [r[0] for r in res] == [False, True, False]
    res = run_parallel([lambda n=n: ev.record_and_wait("ns/j", n, 500) for n in ("unlisted", "aa-node", "b")])
    assert [r[0] for r in res] == [False, True, False]  # listed names before unlisted ones
    ev.close()


def test_close_releases_waiters():
    # ksg_close fires every pending pod and frees the evaluator only after
    # every waiter has returned (no waiter touches freed memory)
    ev = relay.ScoreEvaluator(members=5, delay_s=60, tie=relay.TIE_LOWEST_NAME)
    out = []
    th = [threading.Thread(target=lambda n=n: out.append(ev.record_and_wait("ns/c", f"n{n}", 10 + n)))
          for n in range(3)]
    for t in th:
        t.start()
    deadline = time.time() + 10
    while ev.pending() == 0 and time.time() < deadline:
        time.sleep(0.01)
    time.sleep(0.1)
    t0 = time.time()
    ev.close()
    for t in th:
        t.join(5)
    assert time.time() - t0 < 5 and len(out) == 3
    assert sorted(o[0] for o in out) == [False, False, True]
    assert all(o[1:] == ("n2", 12) for o in out)


def test_close_evaluator_while_rpcs_are_parked():
    # ScoreEvaluator.close() with CollectScore RPCs parked on an unfired pod
    # (one member never scores): close fires the pod with the scores recorded
    # so far and the server answers every parked sender before it stops; the
    # evaluator is freed only after no server thread is inside a call on it
    ev = relay.ScoreEvaluator(members=3, delay_s=60, tie=relay.TIE_LOWEST_NAME)
    srv = relay.CollectScoreServer(ev).start()
    cli = relay.ScoreClient(srv.address)
    out = [None, None]

    def send(i, node, score):
        out[i] = cli.send_score("parked", "ns", node, score, timeout=20)

    th = [threading.Thread(target=send, args=(0, "n1", 400)), threading.Thread(target=send, args=(1, "n2", 300))]
    for t in th:
        t.start()
    deadline = time.time() + 10
    while ev.pending() == 0 and time.time() < deadline:
        time.sleep(0.01)
    time.sleep(0.2)
    t0 = time.time()
    ev.close()  # fires "ns/parked": n1 wins
    for t in th:
        t.join(15)
    srv.stop()
    assert out == [True, False] and time.time() - t0 < 10


def test_close_evaluator_races_async_records():
    # ksg_record calls racing ksg_close: each either records (and is reported
    # or answered) or is refused; none touches the evaluator after it is freed
    for _ in range(20):
        ev = relay.ScoreEvaluator(members=4, delay_s=30, tie=relay.TIE_LOWEST_NAME)
        stop = threading.Event()

        def spam(k):
            i = 0
            while not stop.is_set() and i < 200:
                try:
                    ev.record(f"ns/p{k}-{i}", f"n{k}", 10 + i % 7)
                except ValueError:  # refused: the evaluator is closing / closed
                    return
                i += 1

        th = [threading.Thread(target=spam, args=(k,)) for k in range(4)]
        for t in th:
            t.start()
        time.sleep(0.002)
        ev.close()
        stop.set()
        for t in th:
            t.join(10)
        assert not any(t.is_alive() for t in th)


def test_start_reports_a_bind_failure():
    # an address gRPC cannot bind: start() raises instead of returning a
    # server with port 0 and no loop
    ev = relay.ScoreEvaluator(members=1, delay_s=1, tie=relay.TIE_LOWEST_NAME)
    try:
        with pytest.raises(Exception):
            relay.CollectScoreServer(ev, address="256.256.256.256:70000").start()
    finally:
        ev.close()
