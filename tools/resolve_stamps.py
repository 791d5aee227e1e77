"""Per-phase cycle breakdown of the resolve kernel (diagnostic KS_STAMPS build).

KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/stamps python tools/resolve_stamps.py [nodes] [pods] [hetero|labeled]
Per-role work / barrier-wait cycles per pod; the stamps' own cost inflates absolute times.
"""
import ctypes as C
import os
import sys

sys.path.insert(0, "k8s-1m_amd")
from ksched import Scheduler, synth  # noqa: E402

nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
npods = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
kind = {"hetero": synth.HETERO, "labeled": synth.LABELED}[sys.argv[3] if len(sys.argv) > 3 else "hetero"]
s = Scheduler(nodes, pods_per_round=256)
ns = synth.nodes(kind, nodes, 1)
s.upsert_nodes_raw(ns.nodes, synth.slot_array(nodes), nodes)
pf = synth.prefill(kind, nodes, 1, 3, 0.5)
assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
ps = synth.pods(kind, npods, 2)
b = s.prepare(ps.pods, npods)
s.run(b)
k = (C.c_uint64 * 16)()
assert s.lib.ks_debug_counters(s.ctx, k) == 0
# decider and eval wave: cycles of work and barrier wait per iteration (pod);
# decider sub-phases: LDS loads, reductions, decision + result, commit
pods = max(1, k[1])
print(f"lib={os.environ.get('KSCHED_LIB_DIR', 'default')} rounds={k[0]} pods={k[1]}")
for i, nm in enumerate(["decider", "eval"]):
    print(f"  {nm:9s} work {k[8 + 2 * i] / pods:8.0f} cyc/pod   wait {k[9 + 2 * i] / pods:8.0f} cyc/pod")
for i, nm in enumerate(["loads", "reductions", "decision", "commit"]):
    print(f"    decider {nm:11s} {k[12 + i] / pods:8.0f} cyc/pod")
