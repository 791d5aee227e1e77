#!/usr/bin/env python3
"""Diagnostic: candidate-list quality of sharded vs unsharded sweeps at 1M nodes.

For S in (1, 8) virtual shards on one GPU: one 256-pod round's merged records
(ks_debug_round_record: bound, key count, keys) and the round counters of a
32768-pod batch (rounds resolved, speculated rounds wasted)."""
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "k8s-1m_amd"))
from ksched import Scheduler, synth  # noqa: E402

N = 1_000_000
nodes = synth.nodes(synth.HETERO, N, 1)
pre = synth.prefill(synth.HETERO, N, 1, 3, 0.5)
pods = synth.pods(synth.HETERO, 256 + 32768, 2)
for arg in sys.argv[1:] or ["1", "8"]:
    S, npl = (int(x) for x in (arg.split(":") + ["4"])[:2])  # shards[:nodes per lane]
    s = Scheduler(N, virtual_shards=S, nodes_per_lane=npl)
    s.upsert_nodes_raw(nodes.nodes, synth.slot_array(N), N)
    assert s.lib.ks_pods_add(s.ctx, pre.pods, pre.slot_ptr, pre.n_pods) == 0
    s.schedule_raw(pods.pods, 256)
    rec = (C.c_uint64 * (2 + 256))()
    rows = []
    for p in range(0, 256, 32):
        assert s.lib.ks_debug_round_record(s.ctx, p, rec) == 0
        bound, nk = rec[0], rec[1]
        keys = [rec[2 + i] for i in range(nk)]
        above = sum(1 for k in keys if k > bound)
        rows.append({"pod": p, "bound_score": (bound >> 32) - 1 if bound else None, "nkeys": nk,
                     "top_score": (keys[0] >> 32) - 1 if keys else None,
                     "last_score": (keys[-1] >> 32) - 1 if keys else None, "keys_above_bound": above})
    dbg0 = (C.c_uint64 * 16)()
    s.lib.ks_debug_counters(s.ctx, dbg0)
    s.schedule_raw(pods.pods_at(256), 32768)
    dbg = (C.c_uint64 * 16)()
    s.lib.ks_debug_counters(s.ctx, dbg)
    print(json.dumps({"shards": S, "npl": npl, "rounds": dbg[0] - dbg0[0], "wasted": dbg[3] - dbg0[3], "records": rows}),
          flush=True)
    s.close()
