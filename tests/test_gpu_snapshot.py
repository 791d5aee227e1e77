"""Generation-based snapshot updates (ks_snapshot_update: upstream
Cache.UpdateSnapshot, pkg/scheduler/internal/cache/cache.go).

A host cache stamps every node change with the next global generation (as
upstream's nextGeneration()); each cycle the shim hands ksched the cache's
NodeInfos -- here every live node plus tombstones of deleted ones, in a
shuffled order with replayed stale entries -- and only the items newer than
the snapshot change it.  The device cache must end equal to an oracle fed the
net changes directly, and the next batch must schedule bit-exact.
"""
import ctypes as C
import random

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, states_np
from ksched import Scheduler, _abi, synth

pytestmark = pytest.mark.gpu


def node_ptr(arr, i):
    return C.cast(C.addressof(arr.contents) + i * C.sizeof(_abi.KsNode), C.POINTER(_abi.KsNode))


@pytest.mark.parametrize("kind", [synth.HETERO, synth.LABELED])
def test_snapshot_generations_vs_oracle(kind):
    n, rounds = 3000, 5
    rng = random.Random(7)
    versions = [synth.nodes(kind, n, seed) for seed in (1, 21, 22)]  # node objects a slot can take
    s = Scheduler(n, pods_per_round=128)
    o = pyoracle.Oracle(n)
    gen = 0
    cache = {}  # slot -> (generation, version index or None for deleted)
    history = []  # every (slot, generation, version) ever published (stale replays come from here)

    def publish(slot, ver):
        nonlocal gen
        gen += 1
        cache[slot] = (gen, ver)
        history.append((slot, gen, ver))

    for slot in range(n):
        if rng.random() < 0.95:
            publish(slot, 0)
    pre = synth.prefill(kind, n, 1, 3, 0.3)
    applied_total = 0
    snap_gen = 0
    for r in range(rounds + 1):
        if r > 0:  # cache changes between cycles: updates, deletes, re-adds
            for slot in rng.sample(range(n), 150):
                g0, v0 = cache.get(slot, (0, None))
                if v0 is None:
                    publish(slot, rng.randrange(3))
                elif rng.random() < 0.3:
                    publish(slot, None)
                else:
                    publish(slot, rng.randrange(3))
        # the cache's NodeInfos (live + tombstones) and replayed stale entries
        items = [(sl, g, v) for sl, (g, v) in cache.items()] + rng.sample(history, min(len(history), 400))
        rng.shuffle(items)
        infos = (_abi.KsNodeInfo * len(items))()
        for i, (sl, g, v) in enumerate(items):
            infos[i].slot, infos[i].generation = sl, g
            if v is None:
                infos[i].deleted = 1
            else:
                infos[i].node = node_ptr(versions[v].nodes, sl)
        g_out, applied = C.c_int64(), C.c_uint32()
        assert s.lib.ks_snapshot_update(s.ctx, infos, len(items), C.byref(g_out), C.byref(applied)) == 0, \
            s.lib.ks_last_error(s.ctx)
        assert g_out.value == gen
        applied_total += applied.value
        # the oracle gets the net change since the previous cycle
        for sl, (g, v) in sorted(cache.items()):
            if g <= snap_gen:
                continue
            if v is None:
                if o.node_states([sl])[0].alloc_pods >= 0:
                    o.delete((C.c_uint32 * 1)(sl), 1)
            else:
                o.upsert(node_ptr(versions[v].nodes, sl), (C.c_uint32 * 1)(sl), 1)
        snap_gen = gen
        if r == 0:  # bound pods on the initial nodes (they stay through later upserts)
            keep = [i for i in range(pre.n_pods) if cache.get(pre.slot_ptr[i], (0, None))[1] is not None]
            arr = (_abi.KsPod * len(keep))(*[pre.pods[i] for i in keep])
            sl = (C.c_uint32 * len(keep))(*[pre.slot_ptr[i] for i in keep])
            assert s.lib.ks_pods_add(s.ctx, arr, sl, len(keep)) == 0, s.lib.ks_last_error(s.ctx)
            o.add_pods(arr, sl, len(keep))
        # replaying the same list changes nothing
        assert s.lib.ks_snapshot_update(s.ctx, infos, len(items), C.byref(g_out), C.byref(applied)) == 0
        assert applied.value == 0
        assert np.array_equal(states_np(s.lib.ks_node_states, s.ctx, n),
                              states_np(o.L.oracle_node_states, o.o, n)), f"cycle {r}: node state"
        ps = synth.pods(kind, 600, 100 + r)
        assert_results_equal(s.schedule_raw(ps.pods, 600), o.schedule(ps.pods, 600), 600, f"cycle {r}")
    assert applied_total > n
    s.close()
    o.close()


def test_snapshot_rejects_bad_items_without_change():
    s = Scheduler(16)
    ns = synth.nodes(synth.HETERO, 16, 1)
    infos = (_abi.KsNodeInfo * 2)()
    infos[0].slot, infos[0].generation, infos[0].node = 3, 5, node_ptr(ns.nodes, 3)
    infos[1].slot, infos[1].generation = 99, 6  # beyond capacity
    assert s.lib.ks_snapshot_update(s.ctx, infos, 2, None, None) != 0
    assert s.node_states([3])[0].pod_count < 0  # nothing applied (empty slot)
    infos[1].slot, infos[1].deleted = 4, 1  # deleting an empty slot is a no-op
    g, a = C.c_int64(), C.c_uint32()
    assert s.lib.ks_snapshot_update(s.ctx, infos, 2, C.byref(g), C.byref(a)) == 0
    assert (g.value, a.value) == (6, 2)
    assert s.node_states([3])[0].pod_count == 0 and s.node_states([3])[0].alloc_pods > 0
    s.close()


def test_scheduler_snapshot_mirror_follows_applied_items():
    # Scheduler.snapshot_update (the framework wrapper): shuffled NodeInfo lists
    # with stale replays, renames and tombstones; the slot <-> name mirror must
    # follow what the library applied, so results name the right node
    from ksched import Node, Pod
    from ksched.objects import Container

    n = 40
    rng = random.Random(11)
    s = Scheduler(n)
    gen = 0
    cache = {}    # slot -> (generation, version or None)
    history = []  # every published (slot, generation, version)

    def node(slot, ver):
        return Node(f"node-{slot}-v{ver}", {"cpu": 4000 + 1000 * ver, "memory": 8 << 30, "pods": 110})

    def publish(slot, ver):
        nonlocal gen
        gen += 1
        cache[slot] = (gen, ver)
        history.append((slot, gen, ver))

    for slot in range(n):
        publish(slot, 0)
    try:
        for cycle in range(8):
            if cycle:
                for slot in rng.sample(range(n), 12):
                    g0, v0 = cache[slot]
                    publish(slot, None if (v0 is not None and rng.random() < 0.3) else rng.randrange(1, 50))
            items = [(sl, g, v) for sl, (g, v) in cache.items()] + rng.sample(history, min(len(history), 30))
            rng.shuffle(items)
            s.snapshot_update([(sl, g, None if v is None else node(sl, v)) for sl, g, v in items])
            want = {sl: f"node-{sl}-v{v}" for sl, (g, v) in cache.items() if v is not None}
            assert s.names == want, f"cycle {cycle}: slot -> name mirror"
            assert s.slots == {nm: sl for sl, nm in want.items()}, f"cycle {cycle}: name -> slot mirror"
            # a pod only the largest live node fits reports that node's name
            big = max(want, key=lambda sl: (cache[sl][1], -sl))
            cpu = 4000 + 1000 * cache[big][1] - 1
            if sum(1 for sl in want if cache[sl][1] == cache[big][1]) == 1:
                res = s.schedule_pods([Pod(f"p{cycle}", containers=[Container({"cpu": cpu, "memory": 1 << 20})])])[0]
                assert res.suggested_host == want[big], (cycle, res, want[big])
                s.remove_pods([Pod(f"p{cycle}", containers=[Container({"cpu": cpu, "memory": 1 << 20})])], [big])
    finally:
        s.close()
