"""Experiment: ks_plugin_scores mismatches after buffer address reuse."""
import sys, ctypes as C, os
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
wants = [scores_array(o.plugin_scores(ps.pods_at(j))) for j in range(64)]
keep = []
for variant in ['plain', 'devsync', 'noreuse', 'plain2']:
    bad = []
    for j in range(64):
        if variant == 'devsync':
            hip.hipDeviceSynchronize()
        if variant == 'noreuse':
            p = C.c_void_p(); hip.hipMalloc(C.byref(p), C.c_size_t(1 << 16)); keep.append(p)
        out = (_abi.KsNodeScore * n)()
        assert s.lib.ks_plugin_scores(s.ctx, ps.pods_at(j), out) == 0
        got = scores_array(out)
        if not np.array_equal(got, wants[j]):
            bad.append(j)
    print(variant, 'bad pods', len(bad), bad[:10], flush=True)
