"""One multi-rank case of libksched on one GPU (run as a subprocess by
tests/test_gpu_multirank.py).

`world` contexts (rank r of world_size `world`, node slots sharded
contiguously) share an in-process communicator (ks_comm_init_local: the
RCCL collectives of the multi-rank path -- all-reduce(max) of the measured
normaliser maxima, all-gather of the shard records -- as device copies
ordered by stream events), each driven by its own host thread, exactly as
one process per GPU drives it.  Every rank's results and node states must
equal a one-rank context's and the CPU oracle's, bit for bit.

Prints one JSON line: {"ok": true, ...} or {"ok": false, "error": ...}.
"""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("k8s-1m_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
from helpers import res_array, state_array  # noqa: E402
from ksched import Scheduler, synth  # noqa: E402


def main(cfg):
    world, kind, n, m = cfg["world"], cfg["kind"], cfg["nodes"], cfg["pods"]
    P, K, calls = cfg.get("P", 256), cfg.get("K", 0), cfg.get("calls", 3)
    nodes = synth.nodes(kind, n, cfg.get("node_seed", 11))
    slots = synth.slot_array(n)
    if cfg.get("pods_kind") in ("spread", "affinity"):
        # one-pod-path pods (PodTopologySpread / InterPodAffinity) interleaved
        # with plain pods: run replicated on every rank over the whole table
        from test_gpu_fullsize import MixedStream
        gen = synth.spread_pods if cfg["pods_kind"] == "spread" else synth.affinity_pods
        keep = (gen(m // 2, 16, cfg.get("pod_seed", 12)), synth.pods(synth.HETERO, m - m // 2, 13))
        pods = MixedStream(keep[1], keep[0], 64)
    else:
        pods = synth.pods(kind, m, cfg.get("pod_seed", 12))
    pre = synth.prefill(kind, n, 1, 3, 0.5) if cfg.get("prefill") else None
    ranks = [Scheduler(n, device=0, pods_per_round=P, topk=K, world_size=world, rank=r) for r in range(world)]
    Scheduler.comm_init_local(ranks)
    one = Scheduler(n, device=0, pods_per_round=P, topk=K)
    for s in ranks + [one]:
        s.upsert_nodes_raw(nodes.nodes, slots, n)
        if pre is not None:
            assert s.lib.ks_pods_add(s.ctx, pre.pods, pre.slot_ptr, pre.n_pods) == 0, s.lib.ks_last_error(s.ctx)
    # the pod stream in `calls` ks_schedule calls (pipeline state across calls)
    cuts = [m * i // calls for i in range(calls + 1)]
    out = [[None] * calls for _ in range(world)]
    errs = []

    def drive(r):
        try:
            s = ranks[r]
            for i in range(calls):
                a, b = cuts[i], cuts[i + 1]
                out[r][i] = res_array(s.schedule_raw(pods.pods_at(a), b - a), b - a)
            s.allreduce_max([float(r)])  # host barrier through the group
        except Exception as e:  # noqa: BLE001 -- reported to the parent
            errs.append(f"rank {r}: {e!r}")

    th = [threading.Thread(target=drive, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    if any(t.is_alive() for t in th):
        return {"ok": False, "error": "a rank thread did not finish in 240 s"}
    if errs:
        return {"ok": False, "error": "; ".join(errs)}
    want_one = np.concatenate([res_array(one.schedule_raw(pods.pods_at(cuts[i]), cuts[i + 1] - cuts[i]),
                                         cuts[i + 1] - cuts[i]) for i in range(calls)])
    o = pyoracle.Oracle(n, threads=16)
    o.upsert(nodes.nodes, slots, n)
    if pre is not None:
        o.add_pods(pre.pods, pre.slot_ptr, pre.n_pods)
    want = res_array(o.schedule(pods.pods, m), m)
    if not np.array_equal(want_one, want):
        return {"ok": False, "error": "one-rank context differs from the oracle"}
    all_slots = list(range(n))
    st_w = state_array(o.node_states(all_slots))
    for r in range(world):
        got = np.concatenate(out[r])
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            i = int(bad[0])
            return {"ok": False, "error": f"rank {r}: {len(bad)}/{m} results differ; first pod {i}: "
                                          f"got {got[i]} want {want[i]}"}
        if not np.array_equal(state_array(ranks[r].node_states(all_slots)), st_w):
            return {"ok": False, "error": f"rank {r}: node state differs from the oracle"}
    dbg = (__import__("ctypes").c_uint64 * 16)()
    ranks[0].lib.ks_debug_counters(ranks[0].ctx, dbg)
    res = {"ok": True, "scheduled": int((want["status"] == 0).sum()), "rounds": int(dbg[0]),
           "reswept": int(dbg[4]), "wasted": int(dbg[3])}
    for s in ranks + [one]:
        s.close()
    o.close()
    return res


if __name__ == "__main__":
    print(json.dumps(main(json.loads(sys.argv[1]))), flush=True)
