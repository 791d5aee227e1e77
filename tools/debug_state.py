"""Diagnostic: schedule a kwok stream on the GPU and on the oracle and report
node states that differ (slot, field, GPU vs oracle, pods the results put
there).  python tools/debug_state.py [nodes] [pods] [pods_per_round]"""
import sys

import numpy as np

sys.path.insert(0, "k8s-1m_amd")
sys.path.insert(0, "oracle")
sys.path.insert(0, "tests")
import pyoracle  # noqa: E402
from helpers import res_array  # noqa: E402
from ksched import Scheduler, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
P = int(sys.argv[3]) if len(sys.argv) > 3 else 256
nodes = synth.nodes(synth.KWOK, n, 1)
pods = synth.pods(synth.KWOK, m, 2)
slots = synth.slot_array(n)
with Scheduler(n, pods_per_round=P) as s:
    s.upsert_nodes_raw(nodes.nodes, slots, n)
    got = res_array(s.schedule_raw(pods.pods, m), m)
    gs = s.node_states(list(range(n)))
o = pyoracle.Oracle(n)
o.upsert(nodes.nodes, slots, n)
want = res_array(o.schedule(pods.pods, m), m)
ws = o.node_states(list(range(n)))
print("results equal:", np.array_equal(got, want))
f = lambda x: (x.req_milli_cpu, x.req_memory, x.nonzero_milli_cpu, x.nonzero_memory, x.pod_count)  # noqa: E731
bad = [i for i in range(n) if f(gs[i]) != f(ws[i])]
print("slots differing:", len(bad))
for i in bad[:12]:
    on = np.nonzero(want["node_index"] == i)[0]
    print(f"slot {i}: gpu {f(gs[i])} oracle {f(ws[i])} pods->slot {len(on)} first {on[:6].tolist()} last {on[-3:].tolist()}")
