"""Parity at BASELINE.json's full sizes, on the exact paths the bench lines run.

A 1M-node oracle cannot schedule a 32,768-pod batch in test time (~20 pods/s
on 16 threads), so these tests use a REPLAY check: libksched schedules the
whole batch through the default configuration (P = K = 256, 4 nodes per lane,
pipelined rounds, early FIX for normalising plugins); the oracle then replays
the GPU's own decisions (NodeInfo.AddPod at the chosen slot) up to each check
window and schedules the window's pods itself.  Every window's results must be
bit-identical (node, TotalScore, feasible / evaluated counts, Diagnosis), so
each window proves the GPU's decisions correct given the state the GPU had
reached; windows sit in the first round, mid-batch at offsets that are not
round-aligned (pipelined rounds, patched lists, carried commits), and at the
end of the batch.  After the last window the oracle replays the remaining
decisions and the two node tables must be equal (commit bookkeeping of every
pod).

Workloads: C3 (1M heterogeneous, prefilled), C4 (1M labeled: EXT sweep, 2 nodes
per lane, early FIX with wrongly guessed normalisers asserted to occur), the
reference's own kwok shape with request-less pods (kwok/make_nodes/main.go:
126-181, kwok/make_pods/main.go:118-148), and the kwok line's C1-shaped pods.
"""
import ctypes as C
import os

import numpy as np
import pytest

import pyoracle
from helpers import Background, assert_results_equal, res_array, states_np
from ksched import Scheduler, _abi, synth
from ksched.stream import _gather

pytestmark = pytest.mark.gpu

N = 1_000_000
BATCH = 32_768
WLEN = 32
WINDOWS = (0, 5_003, 16_411, BATCH - WLEN)
ORACLE_THREADS = 16  # the GPU box's CPU share


def pod_subset(pods_ptr, idx):
    """Contiguous ks_pod array of pods_ptr[idx] (the structs keep their pointers)."""
    return _gather(pods_ptr, idx, _abi.KsPod)


def u32(a):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return (C.c_uint32 * max(1, len(a)))(*a.tolist())


def replay_check(o, pods, got, m, windows=WINDOWS, wlen=WLEN):
    """Replay the GPU's decisions into oracle `o` and check each window (see module doc)."""
    r = res_array(got, m)
    pos = 0
    checked = 0
    for w in sorted(windows):
        assert w >= pos
        idx = np.nonzero(r["status"][pos:w] == 0)[0] + pos
        if len(idx):
            o.add_pods(pod_subset(pods.pods, idx), u32(r["node_index"][idx]), len(idx))
        want = o.schedule(pods.pods_at(w), wlen)  # commits the window in the oracle
        sub = (_abi.KsResult * wlen).from_buffer_copy(
            C.string_at(C.addressof(got) + w * C.sizeof(_abi.KsResult), wlen * C.sizeof(_abi.KsResult)))
        assert_results_equal(sub, want, wlen, f"window at pod {w}")
        checked += wlen
        pos = w + wlen
    idx = np.nonzero(r["status"][pos:m] == 0)[0] + pos
    if len(idx):
        o.add_pods(pod_subset(pods.pods, idx), u32(r["node_index"][idx]), len(idx))
    return checked


MARK_FIX, MARK_ROUND_START, MARK_AFTER_WASTE = 1, 2, 4  # ks_batch_marks (include/ksched.h)


MIN_CHECKED = 512  # pods whose decision the oracle checks in each full-size test (replay windows)


def pick_windows(marks, m, wlen=WLEN, fixed=WINDOWS, per_kind=3, round_every=16, min_pods=MIN_CHECKED, seed=0):
    """The fixed windows; windows starting where the round machinery changed
    course (ks_batch_marks): the first pods re-swept with measured normaliser
    maxima (FIX) and the first pods of rounds that follow a wasted speculated
    round, up to `per_kind` of each spread over the batch; a window at the
    start of every `round_every`-th resolved round (where the parallel commit
    begins with an empty fixed prefix); then seeded random windows until at
    least `min_pods` pods are checked.  Non-overlapping."""
    mk = np.frombuffer(marks, dtype=np.uint8)
    cand = [(w, "fixed") for w in fixed]
    for bit, what in ((MARK_FIX, "fix"), (MARK_AFTER_WASTE, "after-waste")):
        idx = np.nonzero(mk & bit)[0]
        idx = idx[idx + wlen <= m]
        if len(idx):
            for j in np.unique(np.linspace(0, len(idx) - 1, min(per_kind, len(idx))).astype(int)):
                cand.append((int(idx[j]), what))
    starts = np.nonzero(mk & MARK_ROUND_START)[0]
    starts = starts[starts + wlen <= m]
    cand += [(int(w), "round-start") for w in starts[::round_every]]

    def take(cands):  # non-overlapping; the fixed windows first
        out = []
        for fixed_pass in (True, False):
            for w, what in sorted(cands):
                if (what == "fixed") == fixed_pass and all(w + wlen <= x or w >= x + wlen for x, _ in out):
                    out.append((w, what))
        return sorted(out)

    out = take(cand)
    rng = np.random.default_rng(1234 + seed)
    tries = 0
    while len(out) * wlen < min(min_pods, m) and tries < 1000:
        tries += 1
        w = int(rng.integers(0, m - wlen + 1))
        if all(w + wlen <= x or w >= x + wlen for x, _ in out):
            out = take(out + [(w, "random")])
    return out


def build_oracle(nodes, slots, pf):
    """The 1M-node cluster (and its prefill pods) in a fresh oracle."""
    o = pyoracle.Oracle(N, threads=ORACLE_THREADS)
    o.upsert(nodes.nodes, slots, N)
    if pf is not None:
        o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
    return o


def run_fullsize(kind, pods, prefill, *, opts=None, **cfg):
    nodes = synth.nodes(kind, N, 1)
    slots = synth.slot_array(N)
    pf = synth.prefill(kind, N, 1, 3, 0.5) if prefill else None
    oracle_job = Background(lambda: build_oracle(nodes, slots, pf))  # overlaps the GPU run
    s = Scheduler(N, options=opts, **cfg)
    s.upsert_nodes_raw(nodes.nodes, slots, N)
    if pf is not None:
        assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
    b = s.prepare(pods.pods, BATCH)
    s.run(b)
    got = s.results(b, BATCH)
    marks = s.marks(b, BATCH)
    s.free(b)
    dbg = (C.c_uint64 * 16)()
    assert s.lib.ks_debug_counters(s.ctx, dbg) == 0
    o = oracle_job.get()
    wins = pick_windows(marks, BATCH)
    checked = replay_check(o, pods, got, BATCH, windows=[w for w, _ in wins])
    assert checked >= MIN_CHECKED, f"only {checked} pods checked by the oracle"
    mk = np.frombuffer(marks, dtype=np.uint8)
    covered = np.zeros(BATCH, dtype=bool)
    for w, _ in wins:
        covered[w:w + WLEN] = True
    # a FIX re-sweep / a wasted round that happened is also checked
    for bit in (MARK_FIX, MARK_AFTER_WASTE):
        assert not (mk & bit).any() or (covered & ((mk & bit) != 0)).any(), f"no window on a pod marked {bit}"
    assert (mk & MARK_ROUND_START).sum() >= BATCH // 256
    sg = states_np(s.lib.ks_node_states, s.ctx, N)
    sw = states_np(o.L.oracle_node_states, o.o, N)
    assert np.array_equal(sg, sw), "node tables differ after replaying every decision"
    s.close()
    o.close()
    return res_array(got, BATCH), list(dbg)


C3_STEPS, C3_STEP = 20, 50_000  # BASELINE configs[2]: 1M pods; bench.py's headline step size


def bench_pipeline_replay(kind, n_nodes, steps, step, *, prefill=0.5, min_checked=MIN_CHECKED, opts=None):
    """A bench line exactly as bench.py runs it (run_batches / end_to_end):
    the cluster (nodes seed 1, prefill seed 3), the pod stream of seed 7,
    `steps` steps of `step` pods through ks_batch_prepare / ks_batch_submit /
    ks_batch_wait / ks_batch_results with bench.E2E_DEPTH batches in flight
    (batch k+1 compiled while k runs).  The oracle replays every decision and
    schedules >= min_checked of the pods itself in windows over the whole
    stream: the first pod of steps (where a batch hands the pipelined rounds
    to the next), round starts, FIX / after-waste marks and seeded random
    windows; then the node tables must be equal.  Returns the results and
    the debug counters."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench

    m = steps * step
    nodes = synth.nodes(kind, n_nodes, 1)
    slots = synth.slot_array(n_nodes)
    pf = synth.prefill(kind, n_nodes, 1, 3, prefill) if prefill > 0 else None
    pods = synth.pods(kind, m, 7)

    def build():
        o = pyoracle.Oracle(n_nodes, threads=ORACLE_THREADS)
        o.upsert(nodes.nodes, slots, n_nodes)
        if pf is not None:
            o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
        return o
    oracle_job = Background(build)  # overlaps the GPU run
    s = Scheduler(n_nodes, options=opts)
    s.upsert_nodes_raw(nodes.nodes, slots, n_nodes)
    if pf is not None:
        assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
    got = (_abi.KsResult * m)()
    marks = bytearray(m)
    inflight, nxt = [], 0
    for k in range(steps):
        while nxt < steps and len(inflight) < bench.E2E_DEPTH:
            b = s.prepare(pods.pods_at(nxt * step), step)
            assert s.lib.ks_batch_submit(s.ctx, b) == 0, s.lib.ks_last_error(s.ctx)
            inflight.append(b)
            nxt += 1
        cur = inflight.pop(0)
        assert s.lib.ks_batch_wait(s.ctx, cur) == 0, s.lib.ks_last_error(s.ctx)
        C.memmove(C.addressof(got) + k * step * C.sizeof(_abi.KsResult), s.results(cur, step),
                  step * C.sizeof(_abi.KsResult))
        marks[k * step:(k + 1) * step] = s.marks(cur, step)
        s.free(cur)
    dbg = (C.c_uint64 * 16)()
    assert s.lib.ks_debug_counters(s.ctx, dbg) == 0
    o = oracle_job.get()
    ks = sorted({0, 1, 2, steps // 2, steps - 1} & set(range(steps)))
    fixed = tuple(k * step for k in ks) + (m - WLEN,)
    wins = pick_windows(bytes(marks), m, fixed=fixed, per_kind=2, round_every=1000, min_pods=min_checked)
    checked = replay_check(o, pods, got, m, windows=[w for w, _ in wins])
    assert checked >= min_checked, f"only {checked} pods checked by the oracle"
    assert {w for w, _ in wins} >= set(fixed)
    mk = np.frombuffer(bytes(marks), dtype=np.uint8)
    covered = np.zeros(m, dtype=bool)
    for w, _ in wins:
        covered[w:w + WLEN] = True
    for bit in (MARK_FIX, MARK_AFTER_WASTE):  # a FIX re-sweep / a wasted round that happened is also checked
        assert not (mk & bit).any() or (covered & ((mk & bit) != 0)).any(), f"no window on a pod marked {bit}"
    sg = states_np(s.lib.ks_node_states, s.ctx, n_nodes)
    sw = states_np(o.L.oracle_node_states, o.o, n_nodes)
    assert np.array_equal(sg, sw), f"node tables differ after replaying all {m} decisions"
    s.close()
    o.close()
    return res_array(got, m), list(dbg)


def test_c3_bench_pipeline_1m_replay():
    # configs[2] as the headline runs it: 1M heterogeneous nodes, 20 steps of
    # 50,000 pods = 1M pods
    r, dbg = bench_pipeline_replay(synth.HETERO, N, C3_STEPS, C3_STEP)
    assert dbg[0] >= C3_STEPS * C3_STEP // 256
    assert (r["status"] == 0).all()


def test_c4_bench_pipeline_1m_replay():
    # configs[3] as `bench.py --kind labeled` runs it: 1M labeled nodes
    # (zones, instance types, pools, features, taints), labeled pods with
    # nodeSelectors, required / preferred node affinity and tolerations,
    # 10 steps of 50,000 pods = 500k pods with the default node-tuple
    # normaliser guesses; FIX re-sweeps and the parallel commit of label /
    # taint rounds at bench length
    r, dbg = bench_pipeline_replay(synth.LABELED, N, 10, 50_000)
    assert dbg[4] > 0, "no pod was re-swept with a measured normaliser (FIX path not exercised)"
    assert dbg[13] > 0, "the parallel commit resolved no label / taint round"
    assert (r["status"] == 0).mean() > 0.9


def test_c2_bench_pipeline_100k_replay():
    # configs[1] as the c2 line runs it (`bench.py --nodes 100000 --batch
    # 20000`): 100k heterogeneous nodes, 5 steps of 20,000 pods = 100k pods,
    # 2048 of them scheduled by the oracle itself
    r, dbg = bench_pipeline_replay(synth.HETERO, 100_000, 5, 20_000, min_checked=2048)
    assert (r["status"] == 0).mean() > 0.99


def test_c4_labeled_1m_replay_fix_behind_merge():
    # simple normaliser guesses (tuple_guess = 0), so that the FIX path runs
    # often, with the FIX sweep behind the merge on the side stream
    # (early_fix = 0, the multi-rank order) on one rank; the early FIX sweep
    # of the default configuration runs at bench length in
    # test_c4_bench_pipeline_1m_replay (asserting FIX re-sweeps), and the
    # default node-tuple guesses there too
    r, dbg = run_fullsize(synth.LABELED, synth.pods(synth.LABELED, BATCH, 2), prefill=True,
                          opts={"tuple_guess": 0, "early_fix": 0})
    assert dbg[4] > 0, "no pod was re-swept with a measured normaliser (FIX path not exercised)"
    assert (r["status"] == 0).mean() > 0.9


def test_kwok_1m_requestless_replay():
    # the reference's published workload shape: identical kwok nodes, busybox
    # pods with no requests (non-zero defaults 100m / 200Mi for LeastAllocated)
    r, dbg = run_fullsize(synth.KWOK, synth.besteffort_pods(BATCH), prefill=False)
    assert (r["status"] == 0).all()
    # identical nodes: ties everywhere, lowest slot wins; 3 pods per node before LeastAllocated drops
    assert r["node_index"][:6].tolist() == [0, 0, 0, 1, 1, 1]


def test_kwok_1m_c1_pods_replay():
    r, dbg = run_fullsize(synth.KWOK, synth.pods(synth.KWOK, BATCH, 2), prefill=False)
    assert (r["status"] == 0).all()


def test_kwok_1m_c1_pods_k512_replay():
    # the kwok bench geometry: 512 candidates per pod, so a round's lists
    # survive the previous round's commits to identical nodes
    r, dbg = run_fullsize(synth.KWOK, synth.pods(synth.KWOK, BATCH, 2), prefill=False, topk=512)
    assert (r["status"] == 0).all()
    # Under resolve AUTO a parallel-commit bail (dbg[14]) hands its whole
    # round to the serial kernel, so a bail wastes no speculative sweep: a
    # wasted round means the 512-entry lists did not survive the previous
    # round's commits (round 2's bound: at most 1 in 20)
    assert dbg[3] * 20 < dbg[0], f"wasted speculative rounds {dbg[3]} ({dbg[14]} AUTO hand-overs) of {dbg[0]}"


class MixedStream:
    """A ks_pod array interleaving two synthetic streams in blocks (pods_at / pods like synth.Synth)."""

    def __init__(self, a, b, block):
        self.keep = (a, b)
        out = []
        ia = ib = 0
        while ia < a.n_pods or ib < b.n_pods:
            for _ in range(block):
                if ia < a.n_pods:
                    out.append(a.pods[ia])
                    ia += 1
            for _ in range(block):
                if ib < b.n_pods:
                    out.append(b.pods[ib])
                    ib += 1
        self.n_pods = len(out)
        self.arr = (_abi.KsPod * self.n_pods)(*out)
        self.pods = C.cast(self.arr, C.POINTER(_abi.KsPod))

    def pods_at(self, start):
        return C.cast(C.addressof(self.arr) + start * C.sizeof(_abi.KsPod), C.POINTER(_abi.KsPod))


def test_spread_1m_replay():
    # the spread bench's cluster (1M nodes in 32 zones, prefill pods of 64 apps)
    # with deployment pods carrying PodTopologySpread constraints interleaved
    # with plain pods: spread path and round kernels alternate, class counts
    # follow both; the oracle replays every decision and checks three windows
    n_pods = 3072
    nodes = synth.nodes(synth.ZONED, N, 1)
    slots = synth.slot_array(N)
    pf = synth.prefill(synth.ZONED, N, 1, 3, 0.5)
    oracle_job = Background(lambda: build_oracle(nodes, slots, pf))  # overlaps the GPU run
    spread, plain = synth.spread_pods(n_pods // 2, 64, 5), synth.pods(synth.HETERO, n_pods // 2, 6)
    mixed = MixedStream(plain, spread, 128)
    s = Scheduler(N)
    s.upsert_nodes_raw(nodes.nodes, slots, N)
    assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
    b = s.prepare(mixed.pods, n_pods)
    s.run(b)
    got = s.results(b, n_pods)
    s.free(b)
    st = _abi.KsStats()
    assert s.lib.ks_get_stats(s.ctx, C.byref(st)) == 0
    assert st.spread_pods == n_pods // 2
    o = oracle_job.get()
    # windows straddle a plain -> spread boundary, sit inside a spread run, and end the batch
    replay_check(o, mixed, got, n_pods, windows=(124, 1400, n_pods - 6), wlen=6)
    sg = states_np(s.lib.ks_node_states, s.ctx, N)
    sw = states_np(o.L.oracle_node_states, o.o, N)
    assert np.array_equal(sg, sw), "node tables differ after replaying every decision"
    r = res_array(got, n_pods)
    assert (r["status"] == 0).mean() > 0.9
    s.close()
    o.close()


@pytest.mark.parametrize("dns", [False, True])
def test_deploy_1m_replay(dns):
    # the deploy bench's workload: deployments of 256 identical replicas under
    # the system default spread constraints (deploy-dns: zone DoNotSchedule +
    # hostname ScheduleAnyway) on the 1M-node zoned cluster, all in replica
    # runs; the oracle replays every decision and schedules
    # windows at a run's first pod, inside runs and at the end
    n_pods = 2048
    nodes = synth.nodes(synth.ZONED, N, 1)
    slots = synth.slot_array(N)
    pf = synth.prefill(synth.ZONED, N, 1, 3, 0.5)
    oracle_job = Background(lambda: build_oracle(nodes, slots, pf))  # overlaps the GPU run
    dep = (synth.deploy_dns_pods if dns else synth.deploy_pods)(n_pods, 256, 5)
    s = Scheduler(N)
    s.upsert_nodes_raw(nodes.nodes, slots, N)
    assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
    b = s.prepare(dep.pods, n_pods)
    s.run(b)
    got = s.results(b, n_pods)
    s.free(b)
    st = _abi.KsStats()
    assert s.lib.ks_get_stats(s.ctx, C.byref(st)) == 0
    assert st.replica_pods == n_pods and st.replica_runs >= n_pods // 256
    o = oracle_job.get()
    replay_check(o, dep, got, n_pods, windows=(0, 130, 512, 1201, n_pods - 4), wlen=4)
    sg = states_np(s.lib.ks_node_states, s.ctx, N)
    sw = states_np(o.L.oracle_node_states, o.o, N)
    assert np.array_equal(sg, sw), "node tables differ after replaying every decision"
    assert (res_array(got, n_pods)["status"] == 0).all()
    s.close()
    o.close()


def test_affinity_1m_replay():
    # the affinity bench's cluster with InterPodAffinity deployment pods
    # interleaved with plain pods: term classes of the batch's own pods
    # (required hostname anti-affinity) are counted by the commits and read by
    # later pods; the oracle replays every decision and checks three windows
    n_pods = 2048
    nodes = synth.nodes(synth.ZONED, N, 1)
    slots = synth.slot_array(N)
    pf = synth.prefill(synth.ZONED, N, 1, 3, 0.5)
    oracle_job = Background(lambda: build_oracle(nodes, slots, pf))  # overlaps the GPU run
    aff, plain = synth.affinity_pods(n_pods // 2, 16, 7), synth.pods(synth.HETERO, n_pods // 2, 8)
    mixed = MixedStream(plain, aff, 128)
    s = Scheduler(N)
    s.upsert_nodes_raw(nodes.nodes, slots, N)
    assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
    b = s.prepare(mixed.pods, n_pods)
    s.run(b)
    got = s.results(b, n_pods)
    s.free(b)
    st = _abi.KsStats()
    assert s.lib.ks_get_stats(s.ctx, C.byref(st)) == 0
    assert st.spread_pods == n_pods // 2
    o = oracle_job.get()
    replay_check(o, mixed, got, n_pods, windows=(124, 900, n_pods - 6), wlen=6)
    sg = states_np(s.lib.ks_node_states, s.ctx, N)
    sw = states_np(o.L.oracle_node_states, o.o, N)
    assert np.array_equal(sg, sw), "node tables differ after replaying every decision"
    r = res_array(got, n_pods)
    assert (r["status"] == 0).mean() > 0.9
    s.close()
    o.close()
