"""Full-size multi-rank case on one GPU (run as a subprocess by
tests/test_gpu_multirank.py): BASELINE.json's 1,000,000-node configurations
split over world_size ranks exactly as `bench.py --gpus 8` splits them
(rank r sweeps slots [r N / W, (r + 1) N / W), 125,000 nodes per rank at
W = 8; reference: the node shards of dist-scheduler/cmd/dist-scheduler/
scheduler.go:200-206), driven by one host thread per rank over the
in-process communicator (ks_comm_init_local: the RCCL all-gather of shard
records and all-reduce of normaliser maxima as device copies).

Checks, bit for bit:
  * every rank's results and node table equal rank 0's;
  * a one-rank context scheduling the same stream gives the same results and
    node table;
  * the oracle (test infrastructure) replays rank 0's decisions and checks
    windows of pods at fixed offsets and where the rounds changed course
    (FIX re-sweeps, rounds after a wasted speculated round: ks_batch_marks),
    then its node table equals the ranks' (test_gpu_fullsize.replay_check).

kinds: c3 (1M heterogeneous prefilled, resource-only pods), c4 (1M labeled:
EXT sweep, normaliser maxima all-reduced, multi-rank FIX path), c5 (a C5
burst, its event log through ks_events_apply on every rank, the next burst).
Prints one JSON line: {"ok": true, ...} or {"ok": false, "error": ...}.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("k8s-1m_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
from helpers import res_array, states_np  # noqa: E402
from ksched import Scheduler, synth  # noqa: E402
from helpers import Background, OracleTarget, on_threads  # noqa: E402
from ksched.stream import BurstStream, GpuTarget  # noqa: E402
from test_gpu_fullsize import MIN_CHECKED, pick_windows, replay_check  # noqa: E402

N = 1_000_000
BATCH = 32_768
ORACLE_THREADS = 16


class Fail(Exception):
    pass


def run_ranks(ranks, pods, m):
    """Every rank schedules pods[0:m] as one batch from its own thread."""
    out, marks, errs = [None] * len(ranks), [None] * len(ranks), []

    def drive(r):
        try:
            s = ranks[r]
            b = s.prepare(pods.pods, m)
            s.run(b)
            out[r] = s.results(b, m)
            marks[r] = s.marks(b, m)
            s.free(b)
        except Exception as e:  # noqa: BLE001 -- reported to the parent
            errs.append(f"rank {r}: {e!r}")

    th = [threading.Thread(target=drive, args=(r,)) for r in range(len(ranks))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    if any(t.is_alive() for t in th):
        raise Fail("a rank thread did not finish in 300 s")
    if errs:
        raise Fail("; ".join(errs))
    r0 = res_array(out[0], m)
    for r in range(1, len(ranks)):
        if not np.array_equal(res_array(out[r], m), r0):
            raise Fail(f"rank {r}: results differ from rank 0's")
    return out[0], marks[0]


def one_rank_setup(nodes, slots, pf, stream, npl):
    """A one-rank context holding the same cluster (built while the ranks run)."""
    s = Scheduler(N, nodes_per_lane=npl)
    t = GpuTarget(s)
    if stream is not None:
        stream.setup([t])
    else:
        s.upsert_nodes_raw(nodes.nodes, slots, N)
        if pf is not None:
            assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
    return s, t


def one_rank_run(s, t, bursts, events):
    """The ranks' stream on the one-rank context: results per burst, node table."""
    res = []
    for i, (pods, m) in enumerate(bursts):
        b = s.prepare(pods.pods, m)
        s.run(b)
        res.append(res_array(s.results(b, m), m))
        s.free(b)
        if i < len(events):
            ev, n, _keep = events[i]
            t.apply_events(ev, n)
    table = states_np(s.lib.ks_node_states, s.ctx, N)
    s.close()
    return res, table


class StreamPods:
    """Burst b of a BurstStream as a (pods, pods_at) object for replay_check."""

    def __init__(self, st, b):
        self.pods = st.burst_pods(b)[0]
        self._st, self._b = st, b

    def pods_at(self, i):
        return self._st.pods.pods_at(self._b * self._st.burst + i)


def main(cfg):
    world, kind = cfg["world"], cfg["kind"]
    t0 = time.time()
    stream = nodes = slots = pf = None
    m = BATCH
    if kind == "c5":
        stream = BurstStream(synth.HETERO, N, 2, BATCH)  # C5 rates: 5 % pods, 0.1 % / 0.01 % nodes
    elif kind == "spread":
        # the spread bench's cluster (1M nodes in 32 zones, prefill pods of 64
        # apps) with deployment pods carrying PodTopologySpread constraints
        # interleaved with plain pods: the one-pod path replicated on every rank
        from test_gpu_fullsize import MixedStream
        m = 3072
        nodes = synth.nodes(synth.ZONED, N, 1)
        slots = synth.slot_array(N)
        pf = synth.prefill(synth.ZONED, N, 1, 3, 0.5)
        keep = (synth.spread_pods(m // 2, 64, 5), synth.pods(synth.HETERO, m // 2, 6))
        pods = MixedStream(keep[1], keep[0], 128)
    else:
        k = synth.HETERO if kind == "c3" else synth.LABELED
        nodes = synth.nodes(k, N, 1)
        slots = synth.slot_array(N)
        pf = synth.prefill(k, N, 1, 3, 0.5)
        pods = synth.pods(k, BATCH, 2 if kind == "c3" else 7)
    npl = cfg.get("npl", 2)  # bench.py --gpus N > 1 lays the table out with 2 nodes per lane

    def build_oracle():  # the same cluster in the oracle, built while the GPU runs
        o = pyoracle.Oracle(N, threads=ORACLE_THREADS)
        ot = OracleTarget(o)
        if stream is not None:
            BurstStream(synth.HETERO, N, 2, BATCH).setup([ot])
        else:
            o.upsert(nodes.nodes, slots, N)
            o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
        return o, ot
    oracle_job = Background(build_oracle)
    one_job = Background(lambda: one_rank_setup(nodes, slots, pf, BurstStream(synth.HETERO, N, 2, BATCH)
                                                if stream is not None else None, npl))
    ranks = [Scheduler(N, world_size=world, rank=r, nodes_per_lane=npl) for r in range(world)]
    Scheduler.comm_init_local(ranks)
    targets = [GpuTarget(s) for s in ranks]

    def setup_rank(r):
        if stream is not None:
            stream.setup([targets[r]])
        else:
            s = ranks[r]
            s.upsert_nodes_raw(nodes.nodes, slots, N)
            assert s.lib.ks_pods_add(s.ctx, pf.pods, pf.slot_ptr, pf.n_pods) == 0
    on_threads([lambda r=r: setup_rank(r) for r in range(world)])
    setup_s = time.time() - t0
    # the stream: one batch (c3 / c4), or burst 0, its event log, burst 1 (c5)
    got, marks, events, bursts = [], [], [], []
    nb = 2 if stream is not None else 1
    for b in range(nb):
        if stream is not None:
            p = StreamPods(stream, b)
            bursts.append((p, BATCH))
        else:
            bursts.append((pods, m))
        res, mk = run_ranks(ranks, bursts[-1][0], m)
        got.append(res)
        marks.append(mk)
        if stream is not None and b + 1 < nb:
            stream.record(b, res)
            ops = stream.marshal(stream.make_events())
            ev = BurstStream.event_log(ops)
            events.append(ev)
            on_threads([lambda t=t: t.apply_events(ev[0], ev[1]) for t in targets])
    tables = [states_np(s.lib.ks_node_states, s.ctx, N) for s in ranks]
    for r in range(1, world):
        if not np.array_equal(tables[r], tables[0]):
            raise Fail(f"rank {r}: node table differs from rank 0's")
    dbg = (__import__("ctypes").c_uint64 * 16)()
    ranks[0].lib.ks_debug_counters(ranks[0].ctx, dbg)
    for s in ranks:
        s.close()
    run_s = time.time() - t0 - setup_s
    # one rank, same stream
    one, one_table = one_rank_run(*one_job.get(), bursts, events)
    for b in range(nb):
        if not np.array_equal(one[b], res_array(got[b], bursts[b][1])):
            raise Fail(f"burst {b}: the one-rank context's results differ from the ranks'")
    if not np.array_equal(one_table, tables[0]):
        raise Fail("the one-rank context's node table differs from the ranks'")
    # the oracle replays rank 0's decisions, checking windows
    o, ot = oracle_job.get()
    checked, kinds = 0, set()
    for b in range(nb):
        mb = bursts[b][1]
        if kind == "spread":  # windows straddle a plain -> spread boundary, sit in a spread run, end the batch
            wins, wlen = [(124, "fixed"), (1400, "fixed"), (mb - 6, "fixed")], 6
        else:
            wins, wlen = pick_windows(marks[b], mb, seed=b), 32
        kinds |= {what for _, what in wins}
        checked += replay_check(o, bursts[b][0], got[b], mb, windows=[w for w, _ in wins], wlen=wlen)
        if b < len(events):
            BurstStream.apply_marshalled(events[b][2], [ot])
    if kind != "spread" and checked < MIN_CHECKED * nb:
        raise Fail(f"only {checked} pods checked by the oracle over {nb} bursts")
    ow = states_np(o.L.oracle_node_states, o.o, N)
    if not np.array_equal(ow, tables[0]):
        raise Fail("node tables differ from the oracle's after replaying every decision")
    o.close()
    r0 = res_array(got[0], bursts[0][1])
    return {"ok": True, "kind": kind, "world": world, "npl": npl, "scheduled": int((r0["status"] == 0).sum()),
            "rounds": int(dbg[0]), "reswept": int(dbg[4]), "wasted": int(dbg[3]), "oracle_pods_checked": checked,
            "window_kinds": sorted(kinds), "setup_s": round(setup_s, 1), "ranks_s": round(run_s, 1),
            "total_s": round(time.time() - t0, 1)}


if __name__ == "__main__":
    try:
        res = main(json.loads(sys.argv[1]))
    except Fail as e:
        res = {"ok": False, "error": str(e)}
    print(json.dumps(res), flush=True)
