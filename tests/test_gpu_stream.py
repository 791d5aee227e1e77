"""C5 on the GPU: bursty pod streams with incremental cache
updates between bursts (pod deletes, node updates, node deletes + adds).

* small streams: libksched vs the CPU oracle, bit-exact on every result of
  every burst and on the final node state;
* the full C5 stream (1M nodes, 100 bursts x 100k pods, bench.py's path):
  the oracle replays every decision and event log and schedules windows of
  pods itself over early, middle and last bursts; the node tables are equal
  after 10M pods; the incrementally updated device cache equals a cache
  rebuilt from scratch, both schedule the next burst identically, and its
  first pods equal the oracle.
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array, states_np
from ksched import Scheduler, synth
from helpers import OracleTarget
from ksched.stream import BurstStream, GpuTarget, Rates

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,P", [(synth.HETERO, 256), (synth.LABELED, 128), (synth.KWOK, 64)])
def test_c5_stream_vs_oracle(kind, P):
    n, bursts, burst = 2500, 6, 800
    st = BurstStream(kind, n, bursts, burst, rates=Rates(0.05, 0.02, 0.01), prefill=3)
    s = Scheduler(n, pods_per_round=P)
    g, o = GpuTarget(s), OracleTarget(pyoracle.Oracle(n))
    st.setup([g, o])
    for b in range(bursts):
        arr, m = st.burst_pods(b)
        got, want = g.schedule(arr, m), o.schedule(arr, m)
        assert_results_equal(got, want, m, f"burst {b}")
        st.record(b, want)
        st.apply(st.make_events(), [g, o])
    sg = states_np(s.lib.ks_node_states, s.ctx, n)
    sw = states_np(o.o.L.oracle_node_states, o.o.o, n)
    assert np.array_equal(sg, sw)
    s.close()


# C5 check windows: burst -> first pods of 32-pod windows the oracle schedules
# itself (early, middle and last bursts; burst starts, ends and offsets that
# are not round-aligned): 17 windows = 544 pods
C5_WINDOWS = {0: (0, 40_961, 99_968), 1: (0, 77_777), 2: (5_003,), 33: (12_345, 61_003),
              50: (0, 50_021, 99_968), 66: (31_337,), 75: (70_001,), 98: (88_001,), 99: (0, 49_999, 99_968)}
C5_WLEN = 32


class _BurstPods:
    """pods / pods_at of one burst of a BurstStream (the replay's view)."""

    def __init__(self, st, b):
        self.base = b * st.burst
        self.st = st
        self.pods = st.pods.pods_at(self.base)

    def pods_at(self, i):
        return self.st.pods.pods_at(self.base + i)


def test_c5_full_stream_replay():
    # configs[4] at its full length, as bench.py --workload c5 runs it
    # (run_c5: the same seeded BurstStream, ks_batch_prepare + ks_batch_run per
    # burst, the burst's watch-event log through ks_events_apply): 1M nodes,
    # 100 bursts x 100k pods = 10M pods, C5 rates (5 % of bound pods deleted,
    # 0.1 % node updates, 0.01 % node deletes + adds per burst).
    # * The oracle replays every decision and applies the same logs (per-kind
    #   calls), one burst behind on a thread of its own, and schedules 544 pods
    #   itself in windows over early, middle and last bursts: bit-exact.
    # * After the last burst the 1M-node tables are equal (every commit and
    #   every event of 10M pods booked identically).
    # * A cache rebuilt from scratch from the live nodes and bound pods equals
    #   the incremental one, and both schedule a further burst identically;
    #   its first pods equal the oracle's.
    import queue
    import threading

    from test_gpu_fullsize import replay_check

    n, bursts, burst = 1_000_000, 100, 100_000
    st = BurstStream(synth.HETERO, n, bursts + 1, burst, prefill=3)
    s = Scheduler(n)
    g = GpuTarget(s)
    o = pyoracle.Oracle(n, threads=16)
    ot = OracleTarget(o)
    st.setup([g, ot])
    work, errors, checked = queue.Queue(maxsize=3), [], [0]

    def oracle_side():
        while True:
            item = work.get()
            if item is None:
                return
            if errors:
                continue
            b, res, ops = item
            try:
                checked[0] += replay_check(o, _BurstPods(st, b), res, burst, windows=C5_WINDOWS.get(b, ()),
                                           wlen=C5_WLEN)
                st.apply_marshalled(ops, [ot])
            except BaseException as e:  # noqa: BLE001 -- re-raised on the test thread
                errors.append(e)

    th = threading.Thread(target=oracle_side, daemon=True)
    th.start()
    scheduled = 0
    try:
        for b in range(bursts):
            arr, m = st.burst_pods(b)
            batch = s.prepare(arr, m)
            s.run(batch)
            res = s.results(batch, m)
            s.free(batch)
            scheduled += int((res_array(res, m)["status"] == 0).sum())
            st.record(b, res)
            ops = st.marshal(st.make_events())
            ev, ne, _keep = st.event_log(ops)
            assert ne > 0
            g.apply_events(ev, ne)
            work.put((b, res, ops))
            if errors:
                break
    finally:
        work.put(None)
        th.join()
    if errors:
        raise errors[0]
    assert checked[0] == C5_WLEN * sum(len(w) for w in C5_WINDOWS.values()) >= 512
    assert scheduled > 0.99 * bursts * burst
    a = states_np(s.lib.ks_node_states, s.ctx, n)
    assert np.array_equal(a, states_np(o.L.oracle_node_states, o.o, n)), "node tables differ after 10M pods"
    # conservation: pods counted on the nodes = the stream's bound pods
    assert a["pod_count"][a["pod_count"] >= 0].sum() == len(st.bound_pod)
    fresh = Scheduler(n)
    st.rebuild(GpuTarget(fresh))
    assert np.array_equal(a, states_np(fresh.lib.ks_node_states, fresh.ctx, n)), "incremental != rebuilt cache"
    arr, m = st.burst_pods(bursts)
    got = s.schedule_raw(arr, m)
    assert_results_equal(got, fresh.schedule_raw(arr, m), m, "incremental vs rebuilt cache")
    fresh.close()
    k = 32
    assert_results_equal(got, o.schedule(arr, k), k, "after 10M pods: incremental cache vs oracle")
    s.close()
    o.close()


def test_event_log_equals_separate_calls():
    # ks_events_apply (one ordered log per burst) leaves the same cache as the
    # per-kind calls, burst after burst, and later bursts schedule identically
    n, bursts, burst = 100_000, 3, 20_000
    st = BurstStream(synth.HETERO, n, bursts + 1, burst, rates=Rates(0.05, 0.01, 0.002))
    a, b = Scheduler(n), Scheduler(n)
    ga, gb = GpuTarget(a), GpuTarget(b)
    st.setup([ga, gb])
    for k in range(bursts):
        arr, m = st.burst_pods(k)
        ra, rb = ga.schedule(arr, m), gb.schedule(arr, m)
        assert_results_equal(ra, rb, m, f"burst {k}")
        st.record(k, ra)
        ops = st.marshal(st.make_events())
        st.apply_marshalled(ops, [ga])
        ev, ne, keep = st.event_log(ops)
        assert ne > 0
        gb.apply_events(ev, ne)
    sa = states_np(a.lib.ks_node_states, a.ctx, n)
    assert np.array_equal(sa, states_np(b.lib.ks_node_states, b.ctx, n))
    arr, m = st.burst_pods(bursts)
    assert_results_equal(a.schedule_raw(arr, m), b.schedule_raw(arr, m), m, "after the logs")
    a.close()
    b.close()


def test_c2_batched_equals_sequential():
    # configs[1] shape (100k nodes): the in-order batched commit (P = 256) equals
    # one-pod-at-a-time scheduling (P = 1) on the same device, for 20k pods,
    # and the oracle on the first 1,000
    n, m = 100_000, 20_000
    ns = synth.nodes(synth.HETERO, n, 1)
    pf = synth.prefill(synth.HETERO, n, 1, 3, 0.5)
    ps = synth.pods(synth.HETERO, m, 2)
    out = []
    for P, K in ((256, 256), (1, 1)):
        s = Scheduler(n, pods_per_round=P, topk=K)
        s.upsert_nodes_raw(ns.nodes, synth.slot_array(n), n)
        assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
        out.append(s.schedule_raw(ps.pods, m))
        s.close()
    assert_results_equal(out[0], out[1], m, "P=256 vs P=1")
    o = pyoracle.Oracle(n, threads=16)
    o.upsert(ns.nodes, synth.slot_array(n), n)
    o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
    assert_results_equal(out[0], o.schedule(ps.pods, 1000), 1000, "vs oracle")
