#!/usr/bin/env python3
"""Diagnostic: where the end-to-end step time goes (1 GPU, C3 shape).

Modes over the same number of 32768-pod steps:
  resident   prepare all batches first, then time ks_batch_run only
  serial     prepare -> run -> results per step (no overlap)
  pipelined  the bench's headline loop (prepare k+1 while k runs), with the
             time each call takes on the main thread
"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "k8s-1m_amd"))
from ksched import Scheduler, _abi, synth  # noqa: E402

N, B, STEPS = 1_000_000, 32768, 6
s = Scheduler(N)
nodes = synth.nodes(synth.HETERO, N, 1)
s.upsert_nodes_raw(nodes.nodes, synth.slot_array(N), N)
pre = synth.prefill(synth.HETERO, N, 1, 3, 0.5)
assert s.lib.ks_pods_add(s.ctx, pre.pods, pre.slot_ptr, pre.n_pods) == 0
pods = synth.pods(synth.HETERO, 4 * STEPS * B, 9)
lib, ctx = s.lib, s.ctx
out = (_abi.KsResult * B)()
off = 0


def take():
    global off
    p = pods.pods_at(off * B)
    off += 1
    return p


import os  # noqa: E402

res = {}
if os.environ.get("TIMING") == "1":
    s.set_timing(True)
# resident
bs = [s.prepare(take(), B) for _ in range(STEPS)]
t0 = time.perf_counter()
for b in bs:
    s.run(b)
res["resident_ms"] = 1e3 * (time.perf_counter() - t0) / STEPS
for b in bs:
    s.free(b)
# serial
tp = tr = 0.0
for _ in range(STEPS):
    t0 = time.perf_counter()
    b = s.prepare(take(), B)
    t1 = time.perf_counter()
    s.run(b)
    t2 = time.perf_counter()
    s.results(b, B)
    s.free(b)
    tp += t1 - t0
    tr += t2 - t1
res["serial_prepare_ms"] = 1e3 * tp / STEPS
res["serial_run_ms"] = 1e3 * tr / STEPS
# pipelined
acc = {"prepare": 0.0, "submit": 0.0, "wait": 0.0, "results": 0.0, "free": 0.0}
t_all = time.perf_counter()
cur = s.prepare(take(), B)
lib.ks_batch_submit(ctx, cur)
for k in range(STEPS):
    nxt = None
    if k + 1 < STEPS:
        t0 = time.perf_counter()
        nxt = s.prepare(take(), B)
        t1 = time.perf_counter()
        lib.ks_batch_submit(ctx, nxt)
        t2 = time.perf_counter()
        acc["prepare"] += t1 - t0
        acc["submit"] += t2 - t1
    t0 = time.perf_counter()
    assert lib.ks_batch_wait(ctx, cur) == 0
    t1 = time.perf_counter()
    lib.ks_batch_results(ctx, cur, out)
    t2 = time.perf_counter()
    s.free(cur)
    t3 = time.perf_counter()
    acc["wait"] += t1 - t0
    acc["results"] += t2 - t1
    acc["free"] += t3 - t2
    cur = nxt
res["pipelined_ms"] = 1e3 * (time.perf_counter() - t_all) / STEPS
res.update({f"pipelined_{k}_ms": round(1e3 * v / STEPS, 3) for k, v in acc.items()})
print(json.dumps({k: round(v, 3) for k, v in res.items()}), flush=True)
s.close()
