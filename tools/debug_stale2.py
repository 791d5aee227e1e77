import sys, ctypes as C, time
sys.path[:0] = ['k8s-1m_amd', 'oracle', 'tests']
import numpy as np
import pyoracle
from helpers import scores_array
from ksched import Scheduler, synth, _abi
hip = C.CDLL('libamdhip64.so')
n = 1500
ns = synth.nodes(synth.LABELED, n, 21); ps = synth.pods(synth.LABELED, 64, 22)
slots = synth.slot_array(n)
o = pyoracle.Oracle(n); o.upsert(ns.nodes, slots, n)
s = Scheduler(n); s.upsert_nodes_raw(ns.nodes, slots, n)
pf = synth.prefill(synth.LABELED, n, 21, 23, 0.5)
o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
for variant in ['test_loop', 'sleep', 'gpu_first', 'test_loop2']:
    bad = []
    for j in range(64):
        p = ps.pods_at(j)
        if variant == 'gpu_first':
            out = (_abi.KsNodeScore * n)()
            assert s.lib.ks_plugin_scores(s.ctx, p, out) == 0
            want = scores_array(o.plugin_scores(p))
        else:
            want = scores_array(o.plugin_scores(p))
            if variant == 'sleep':
                time.sleep(0.002)
            out = (type(o.plugin_scores(p)[0]) * n)()
            assert s.lib.ks_plugin_scores(s.ctx, p, out) == 0
        got = scores_array(out)
        if not np.array_equal(got, want):
            bad.append(j)
    print(variant, 'bad', len(bad), bad[:12], flush=True)
