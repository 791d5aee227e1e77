"""Reproduce a C5 stream divergence and dump the first differing node (GPU)."""
import ctypes as C
import sys

sys.path[:0] = ["k8s-1m_amd", "oracle", "tests"]
import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
from helpers import res_array, scores_array  # noqa: E402
from ksched import Scheduler, _abi, synth  # noqa: E402
from stream import BurstStream, GpuTarget, OracleTarget, Rates  # noqa: E402

kind, P = synth.LABELED, 128
n, bursts, burst = 2500, 6, 800
st = BurstStream(kind, n, bursts, burst, rates=Rates(0.05, 0.02, 0.01), prefill=3)
s = Scheduler(n, pods_per_round=P)
g, o = GpuTarget(s), OracleTarget(pyoracle.Oracle(n))
st.setup([g, o])


def dump_node(nd):
    labs = {nd.labels[i].key.decode(): nd.labels[i].value.decode() for i in range(nd.n_labels)}
    taints = [(nd.taints[i].key.decode(), (nd.taints[i].value or b"").decode(), nd.taints[i].effect)
              for i in range(nd.n_taints)]
    return f"name={nd.name.decode()} labels={labs} taints={taints} unsched={nd.unschedulable}"


for b in range(bursts):
    arr, m = st.burst_pods(b)
    got, want = g.schedule(arr, m), o.schedule(arr, m)
    rg, rw = res_array(got, m), res_array(want, m)
    bad = np.nonzero(rg != rw)[0]
    if len(bad):
        i = int(bad[0])
        print(f"burst {b}: {len(bad)} differ, first pod {i}: got {rg[i]} want {rw[i]}")
        # replay: fresh targets at the state before pod i of this burst
        # (schedule the burst prefix on both, then dump plugin scores of pod i)
        p = C.cast(C.addressof(arr.contents) + i * C.sizeof(_abi.KsPod), C.POINTER(_abi.KsPod))
        break
    st.record(b, want)
    st.apply(st.make_events(), [g, o])
else:
    print("no divergence")
    sys.exit(0)

# rebuild both at the start of burst b, schedule pods < i, dump pod i
g2, o2 = GpuTarget(Scheduler(n, pods_per_round=P)), OracleTarget(pyoracle.Oracle(n))
for t in (g2, o2):
    st.rebuild(t)
if i:
    ra, rb = res_array(g2.schedule(arr, i), i), res_array(o2.schedule(arr, i), i)
    print("prefix equal:", np.array_equal(ra, rb))
out = (_abi.KsNodeScore * n)()
assert g2.s.lib.ks_plugin_scores(g2.s.ctx, p, out) == 0
sg = scores_array(out)
sw = scores_array(o2.o.plugin_scores(p))
d = np.nonzero((sg != sw).any(1))[0]
print("nodes differing in plugin scores:", d[:10])
pod = p.contents
print("pod:", pod.name.decode(), "nsel", {pod.node_selector[k].key.decode(): pod.node_selector[k].value.decode()
                                        for k in range(pod.n_node_selector)})
for t in range(pod.n_required_terms):
    term = pod.required_terms[t]
    for e in range(term.n_expressions):
        r = term.match_expressions[e]
        print("  term", t, r.key.decode(), r.op, [r.values[v].decode() for v in range(r.n_values)])
for j in d[:4]:
    src = st.node_src[j]
    nd = st.nodes.nodes[int(src)] if src >= 0 else st.pool.nodes[int(-1 - src)]
    print(f"slot {j} src {src}: gpu {sg[j].tolist()} oracle {sw[j].tolist()}")
    print("   ", dump_node(nd))
