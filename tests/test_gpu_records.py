"""The fused sweep's own per-node scores vs the oracle.

ks_plugin_scores checks every plugin through a separate dump kernel; the
timed sweep only emits packed keys.  Here a batch of at most pods_per_round
pods is scheduled in one round, and for each pod the merged candidate record
the sweep (+ merge, + FIX re-sweep for normalising plugins) produced
(ks_debug_round_record) must list exactly the highest packed keys
((TotalScore + 1) << 32 | ~slot) the oracle's NodePluginScores give against
the round-start state, with a bound at least every unlisted feasible key and
the same feasible count.  That checks the sweep's fused TotalScore of every
listed node -- dozens to hundreds per pod -- not only the chosen one.
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from helpers import res_array, scores_array
from ksched import Scheduler, synth

pytestmark = pytest.mark.gpu


def oracle_keys(o, pod_ptr):
    sc = scores_array(o.plugin_scores(pod_ptr))
    feas = np.nonzero(sc[:, 0] == -1)[0]
    keys = ((sc[feas, -1].astype(np.uint64) + np.uint64(1)) << np.uint64(32)) | (
        np.uint64(0xFFFFFFFF) - feas.astype(np.uint64))
    return np.sort(keys)[::-1], len(feas)


@pytest.mark.parametrize("kind,seeds,vshards", [(synth.HETERO, (1, 2), 1), (synth.LABELED, (4, 5), 1),
                                                 (synth.LABELED, (6, 7), 3), (synth.KWOK, (8, 9), 1)])
def test_round_records_match_oracle(kind, seeds, vshards):
    n, m, K = 100000, 32, 256  # ~100 sweep blocks: lists long enough that round 0 resolves every pod
    ns = synth.nodes(kind, n, seeds[0])
    ps = synth.pods(kind, m, seeds[1])
    slots = synth.slot_array(n)
    o = pyoracle.Oracle(n, threads=16)
    o.upsert(ns.nodes, slots, n)
    s = Scheduler(n, pods_per_round=256, topk=K, virtual_shards=vshards)
    s.upsert_nodes_raw(ns.nodes, slots, n)
    if kind != synth.KWOK:
        pf = synth.prefill(kind, n, seeds[0], 3, 0.5)
        o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
        assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
    want = [oracle_keys(o, ps.pods_at(i)) for i in range(m)]  # round-start state
    r = res_array(s.schedule_raw(ps.pods, m), m)
    dbg = (C.c_uint64 * 16)()
    s.lib.ks_debug_counters(s.ctx, dbg)
    # one round resolved every pod: the parity-0 records are round 0's, swept
    # against the round-start state (a re-sweep would overwrite them)
    assert dbg[0] == 1, f"{dbg[0]} rounds: round 0 stopped early and its records were re-swept"
    out = (C.c_uint64 * (2 + K))()
    listed = 0
    for i in range(m):
        assert s.lib.ks_debug_round_record(s.ctx, i, out) == 0, s.lib.ks_last_error(s.ctx)
        bound, nk = int(out[0]), int(out[1])
        got = np.array(out[2:2 + nk], dtype=np.uint64)
        keys, nfeas = want[i]
        assert int(r["feasible"][i]) == nfeas or r["status"][i] != 0
        assert nk <= len(keys)
        assert np.array_equal(got, keys[:nk]), f"pod {i}: listed keys differ from the oracle's top {nk}"
        if nk < len(keys):
            assert bound >= int(keys[nk]), f"pod {i}: bound below an unlisted feasible key"
        listed += nk
    assert listed >= m * 8, f"only {listed} keys listed over {m} pods"
    s.close()
    o.close()
