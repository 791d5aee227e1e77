import sys, ctypes as C
sys.path[:0] = ['k8s-1m_amd', 'oracle', 'tests']
import numpy as np
import pyoracle
from helpers import scores_array, res_array
from ksched import Scheduler, synth, _abi
n = 1500
ns = synth.nodes(synth.LABELED, n, 21); ps = synth.pods(synth.LABELED, 64, 22)
slots = synth.slot_array(n)
o = pyoracle.Oracle(n); o.upsert(ns.nodes, slots, n)
s = Scheduler(n); s.upsert_nodes_raw(ns.nodes, slots, n)
pf = synth.prefill(synth.LABELED, n, 21, 23, 0.5)
o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
print('prefill pods', pf.n_pods)
sg = np.array([(x.req_milli_cpu, x.req_memory, x.pod_count) for x in s.node_states(list(range(n)))])
sw = np.array([(x.req_milli_cpu, x.req_memory, x.pod_count) for x in o.node_states(list(range(n)))])
print('state equal', np.array_equal(sg, sw), sg[:3].tolist(), sw[:3].tolist())
for j in range(4):
    p = ps.pods_at(j)
    want = scores_array(o.plugin_scores(p))
    out = (_abi.KsNodeScore * n)()
    assert s.lib.ks_plugin_scores(s.ctx, p, out) == 0
    got = scores_array(out)
    bad = np.nonzero((got != want).any(1))[0]
    print('pod', j, 'nbad', len(bad), 'first', bad[:5])
    for i in bad[:4]:
        print('  node', i, 'got', got[i].tolist(), 'want', want[i].tolist())
    print('  status hist got', np.unique(got[:, 0], return_counts=True), 'want', np.unique(want[:, 0], return_counts=True))
# schedule pod 2 alone
r = res_array(s.schedule_raw(ps.pods_at(2), 1), 1); w = res_array(o.schedule(ps.pods_at(2), 1), 1)
print('sched got', r, '\nsched want', w)
