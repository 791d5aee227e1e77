"""C5 event stream on the CPU oracle (no GPU): the event log applied
incrementally between bursts leaves the same cache as a cluster rebuilt from
scratch out of the live nodes and the bound pods (checksum-of-state property),
and both caches schedule the next burst identically."""
import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, state_array
from ksched import synth
from helpers import OracleTarget
from ksched.stream import BurstStream, Rates

RATES = Rates(pod_delete=0.05, node_update=0.02, node_delete=0.01)


@pytest.mark.parametrize("kind", [synth.HETERO, synth.LABELED])
def test_events_equal_rebuild(kind):
    n, bursts, burst = 1500, 4, 600
    st = BurstStream(kind, n, bursts + 1, burst, rates=RATES, prefill=3)
    o = OracleTarget(pyoracle.Oracle(n))
    st.setup([o])
    for b in range(bursts):
        arr, m = st.burst_pods(b)
        res = o.schedule(arr, m)
        st.record(b, res)
        st.apply(st.make_events(), [o])
    fresh = OracleTarget(pyoracle.Oracle(n))
    st.rebuild(fresh)
    slots = list(range(n))
    assert np.array_equal(state_array(o.states(slots)), state_array(fresh.states(slots)))
    arr, m = st.burst_pods(bursts)
    assert_results_equal(o.schedule(arr, m), fresh.schedule(arr, m), m, "after rebuild")


def test_event_log_is_seeded():
    a = BurstStream(synth.HETERO, 500, 2, 100, rates=RATES)
    b = BurstStream(synth.HETERO, 500, 2, 100, rates=RATES)
    for s in (a, b):
        o = OracleTarget(pyoracle.Oracle(500))
        s.setup([o])
        s.record(0, o.schedule(*s.burst_pods(0)))
    ea, eb = a.make_events(), b.make_events()
    assert [e[0] for e in ea] == [e[0] for e in eb] == ["remove_pods", "update_nodes", "delete_nodes", "add_nodes"]
    for (_, pa), (_, pb) in zip(ea, eb):
        pa = pa if isinstance(pa, tuple) else (pa,)
        pb = pb if isinstance(pb, tuple) else (pb,)
        for x, y in zip(pa, pb):
            assert np.array_equal(x, y)
