"""Seeded parity sweep: libksched (HIP, gfx950) vs the CPU oracle over mixed
workload shapes and round geometries.

Each case draws, from its own seed, a node kind and a pod kind (mixed kinds
included: resource-only pods on tainted / labeled nodes take the EXT filter
chain, labeled pods on unlabeled nodes fail NodeAffinity), a prefill, the round
geometry (P pods per round, top-K list length, nodes per lane, virtual shards)
and a split of the pod stream into several schedule calls, so that node state
carried across batches is checked as well.  Bit-exact on every result field and
on every node's resource state after each call.  Oracle: oracle/oracle.cpp
(parity unpinned); the case shapes follow the reference's own
knobs: pods per scheduling cycle (`ScheduleOne`, cmd/dist-scheduler/
scheduler.go:543) and shards (`SchedulerSet`).
"""
import random

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, state_array
from ksched import Scheduler, synth

pytestmark = pytest.mark.gpu

KINDS = (synth.KWOK, synth.HETERO, synth.LABELED)


def case(seed):
    r = random.Random(1000 + seed)
    P = r.choice([1, 7, 32, 100, 256])
    return dict(
        kn=r.choice(KINDS),
        kp=r.choice(KINDS),
        n_nodes=r.choice([65, 300, 1031, 2048]),
        n_pods=r.choice([200, 700, 1300]),
        prefill=r.choice([None, r.randrange(1, 100)]),
        P=P,
        K=r.choice([P, 1, 16, 64, 256]),
        npl=r.choice([2, 4, 8]),
        shards=r.choice([1, 1, 2, 5]),
        splits=r.randrange(1, 4),
    )


@pytest.mark.parametrize("seed", range(48))
def test_fuzz_parity(seed):
    c = case(seed)
    n, m = c["n_nodes"], c["n_pods"]
    ns = synth.nodes(c["kn"], n, 3 * seed + 1)
    ps = synth.pods(c["kp"], m, 3 * seed + 2)
    slots = synth.slot_array(n)
    o = pyoracle.Oracle(n)
    o.upsert(ns.nodes, slots, n)
    s = Scheduler(n, pods_per_round=c["P"], topk=c["K"], nodes_per_lane=c["npl"], virtual_shards=c["shards"])
    s.upsert_nodes_raw(ns.nodes, slots, n)
    if c["prefill"] is not None:
        pf = synth.prefill(c["kn"], n, 3 * seed + 1, c["prefill"], 0.5)
        o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
        assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0, s.lib.ks_last_error(s.ctx)
    cuts = sorted(random.Random(seed).sample(range(1, m), c["splits"] - 1)) if c["splits"] > 1 else []
    bounds = [0] + cuts + [m]
    all_slots = list(range(n))
    try:
        for b0, b1 in zip(bounds, bounds[1:]):
            k = b1 - b0
            want = o.schedule(ps.pods_at(b0), k)
            got = s.schedule_raw(ps.pods_at(b0), k)
            assert_results_equal(got, want, k, f"case {seed} {c} pods [{b0}, {b1})")
            assert np.array_equal(state_array(s.node_states(all_slots)), state_array(o.node_states(all_slots))), \
                f"case {seed} {c}: node state differs after pods [{b0}, {b1})"
    finally:
        s.close()


@pytest.mark.parametrize("kind", [synth.HETERO, synth.LABELED])
def test_mid_size(kind):
    # 50k prefilled nodes, 1500 pods over full rounds: the sweep grid at a size
    # where every lane of many blocks holds nodes and lists are well populated
    n, m = 50000, 1500
    ns = synth.nodes(kind, n, 71)
    ps = synth.pods(kind, m, 72)
    slots = synth.slot_array(n)
    o = pyoracle.Oracle(n, threads=16)  # the GPU box's CPU share
    o.upsert(ns.nodes, slots, n)
    s = Scheduler(n)
    s.upsert_nodes_raw(ns.nodes, slots, n)
    pf = synth.prefill(kind, n, 71, 73, 0.5)
    o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
    assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0, s.lib.ks_last_error(s.ctx)
    try:
        assert_results_equal(s.schedule_raw(ps.pods, m), o.schedule(ps.pods, m), m, f"50k kind={kind}")
        all_slots = list(range(n))
        assert np.array_equal(state_array(s.node_states(all_slots)), state_array(o.node_states(all_slots)))
    finally:
        s.close()
