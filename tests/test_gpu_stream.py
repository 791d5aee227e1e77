"""C5 on the GPU: bursty pod streams with incremental cache
updates between bursts (pod deletes, node updates, node deletes + adds).

* small streams: libksched vs the CPU oracle, bit-exact on every result of
  every burst and on the final node state;
* the full 1M-node C5 shape: the incrementally updated device cache equals a
  cache rebuilt from scratch from the live nodes and bound pods, both schedule
  the next burst identically, and the first pods of that burst equal the
  oracle on the same 1M-node state.
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


def test_c5_1m_incremental_equals_rebuild():
    n, bursts, burst = 1_000_000, 3, 100_000
    st = BurstStream(synth.HETERO, n, bursts + 1, burst)  # C5 rates: 5 % pods, 0.1 % / 0.01 % nodes
    s = Scheduler(n)
    g = GpuTarget(s)
    st.setup([g])
    for b in range(bursts):
        arr, m = st.burst_pods(b)
        res = g.schedule(arr, m)
        r = res_array(res, m)
        assert (r["status"] == 0).all()
        st.record(b, res)
        st.apply(st.make_events(), [g])
    fresh = Scheduler(n)
    st.rebuild(GpuTarget(fresh))
    a = states_np(s.lib.ks_node_states, s.ctx, n)
    assert np.array_equal(a, states_np(fresh.lib.ks_node_states, fresh.ctx, n))
    # conservation: Requested summed over nodes = Σ requests of the bound pods
    assert a["pod_count"][a["pod_count"] >= 0].sum() == len(st.bound_pod)
    arr, m = st.burst_pods(bursts)
    got = s.schedule_raw(arr, m)
    assert_results_equal(got, fresh.schedule_raw(arr, m), m, "incremental vs rebuilt cache")
    fresh.close()
    # the first pods of the next burst against the oracle on the same 1M-node state
    o = OracleTarget(pyoracle.Oracle(n, threads=16))
    st.rebuild(o)
    k = 48
    assert_results_equal(got, o.schedule(arr, k), k, "1M-node C5 state vs oracle")
    s.close()


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
