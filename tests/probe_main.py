"""Parity run of a few fuzz geometries on the race-probe build of libksched
(KSCHED_LIB_DIR=k8s-1m_amd/ksched/lib/probe, `make probe`): the resolve
kernel's non-decider waves read the loop's done word late in the last
iterations, which is the window in which the pre-fix single done word let a
wave leave the loop one barrier early.  Run as a child process by
tests/test_gpu_stall.py (the library directory is chosen when ksched loads).

Prints one line per case and "probe ok" at the end; exits non-zero on the
first difference from the oracle (test infrastructure: oracle/ is the checker).
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "k8s-1m_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]

import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
from helpers import assert_results_equal, state_array  # noqa: E402
from ksched import Scheduler, synth  # noqa: E402
from test_gpu_fuzz import case  # noqa: E402


def run(seed):
    c = case(seed)
    n, m = c["n_nodes"], c["n_pods"]
    ns = synth.nodes(c["kn"], n, 3 * seed + 1)
    ps = synth.pods(c["kp"], m, 3 * seed + 2)
    slots = synth.slot_array(n)
    o = pyoracle.Oracle(n)
    o.upsert(ns.nodes, slots, n)
    # the serial commit kernel (the one whose loop exit the probe build delays)
    s = Scheduler(n, pods_per_round=c["P"], topk=c["K"], nodes_per_lane=c["npl"], virtual_shards=c["shards"],
                  options={"resolve_mode": 1})
    try:
        s.lib.ks_set_sync_timeout(s.ctx, 20000)
        s.upsert_nodes_raw(ns.nodes, slots, n)
        if c["prefill"] is not None:
            pf = synth.prefill(c["kn"], n, 3 * seed + 1, c["prefill"], 0.5)
            o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
            assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0, s.lib.ks_last_error(s.ctx)
        half = m // 2
        for b0, b1 in ((0, half), (half, m)):
            k = b1 - b0
            want = o.schedule(ps.pods_at(b0), k)
            got = s.schedule_raw(ps.pods_at(b0), k)
            assert_results_equal(got, want, k, f"probe case {seed} pods [{b0}, {b1})")
            assert np.array_equal(state_array(s.node_states(list(range(n)))),
                                  state_array(o.node_states(list(range(n))))), f"probe case {seed}: node state"
    finally:
        s.close()
    print(f"case {seed} ok: {c}", flush=True)


if __name__ == "__main__":
    assert "probe" in os.environ.get("KSCHED_LIB_DIR", ""), "run with KSCHED_LIB_DIR=.../lib/probe"
    for seed in [int(a) for a in sys.argv[1:]] or [5, 0, 3]:
        run(seed)
    print("probe ok", flush=True)
