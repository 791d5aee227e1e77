#!/usr/bin/env python3
"""bench.py — pods scheduled/sec at 1M nodes (BASELINE.json metric) on MI355X.

Workload (BASELINE.json configs[2], "C3" of SURVEY.md §8(d)): a 1,000,000-node
kwok-shaped heterogeneous cluster (cpu 8-96 cores, memory 32-512 Gi, 32/110
pods, kwok NoSchedule taint; every node pre-filled with seeded pods to a
random 0-50% of its CPU), and a stream of resource-only pods (cpu 50-4000m,
memory 64Mi x 1..256, 10% best-effort, kwok tolerations).  Filter =
NodeUnschedulable/NodeName/TaintToleration/NodeAffinity/NodeResourcesFit,
Score = LeastAllocated + BalancedAllocation + TaintToleration (+ NodeAffinity
skipped, ImageLocality 0), percentageOfNodesToScore = 100, deterministic
lowest-slot tie-break, sequential-equivalent in-order commit.

A "step" schedules one batch of pods (default 32768) to completion against the
live cluster; inputs are resident in HBM before the timed region (the batch
is compiled and uploaded by ks_batch_prepare beforehand).  With --gpus N the
node slots are sharded across N ranks (one process per GPU, RCCL candidate
all-gather); every rank schedules the same pods, so `value` is the job's
pods/s (strong scaling: the cluster is fixed at 1M nodes).

--kind labeled is configs[3] (C4: label bitsets, nodeSelector / required and
preferred NodeAffinity, NoSchedule / NoExecute / PreferNoSchedule taints).
--workload c5 is configs[4] (C5): a step is one burst (default 100k pods)
scheduled to completion followed by the seeded watch-event log (5 % of the
bound pods deleted, 0.1 % node updates, 0.01 % node deletes + adds) applied
to the device cache through the C ABI; the timed region holds both, the
host-side generation and marshalling of the log do not (ksched/stream.py).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "k8s-1m_amd"))

B_NODE = 56  # algorithmic bytes per (pod, node) evaluation, resource-only
B_NODE_LABELED = 96  # ... with label / taint bitsets (C4)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# VALU issue peak in lane-ops/s: 256 CUs x 4 SIMD-32 x 32 lanes x 2.4 GHz
# (MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles; 32-bit
# rate -- binary64 instructions take twice as long, so the sweep's mix peaks lower)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=32768,
                    help="pods per step (each batch refills the round pipeline once)")
    ap.add_argument("--pods-per-round", type=int, default=256)
    ap.add_argument("--topk", type=int, default=0)
    ap.add_argument("--nodes-per-lane", type=int, default=4)
    ap.add_argument("--kind", default="hetero", choices=["hetero", "kwok", "labeled"])
    ap.add_argument("--workload", default="batch", choices=["batch", "c5"],
                    help="batch: one batch of --batch pods per step; c5: one burst + its event log per step")
    ap.add_argument("--burst", type=int, default=100_000, help="pods per burst (--workload c5)")
    ap.add_argument("--prefill", type=float, default=0.5)
    ap.add_argument("--cpu-pods", type=int, default=40, help="oracle sample size (pods), single thread")
    ap.add_argument("--cpu-threads", type=int, default=16, help="oracle threads for cpu_baseline (box CPU share)")
    ap.add_argument("--cpu-pods-mt", type=int, default=240, help="oracle sample size (pods), multi-thread")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-file", default=os.environ.get("KS_PMC_FILE", str(ROOT / "profiles" / "pmc_sweep.json")),
                    help="JSON with measured L2-fabric bytes per sweep launch (tools/pmc.sh + tools/pmc_summary.py)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # No torch in this process: torch bundles its own libamdhip64 / librccl
    # (ROCm 7.0) with the same sonames as the /opt/rocm 7.2 libraries
    # libksched links, and one process must not mix the two runtimes.  The
    # ranks rendezvous through a file on the node (RCCL unique id) and use the
    # scheduler's own RCCL communicator for barriers and the max-over-ranks time.
    from ksched import Scheduler, synth
    from ksched.framework import results_to_arrays

    kind = {"hetero": synth.HETERO, "kwok": synth.KWOK, "labeled": synth.LABELED}[args.kind]
    t_setup = time.time()
    sched = Scheduler(args.nodes, device=local_rank if world > 1 else 0, pods_per_round=args.pods_per_round,
                      topk=args.topk, nodes_per_lane=args.nodes_per_lane, world_size=world, rank=rank)
    if world > 1:
        sched.comm_init(exchange_unique_id(rank, world))
        if rank == 0:  # ncclCommInitRank returned: every rank has read the id
            uid_path(world).unlink(missing_ok=True)

    if args.workload == "c5":
        return run_c5(args, kind, sched, world, rank, t_setup)
    nodes = synth.nodes(kind, args.nodes, 1)
    slots = synth.slot_array(args.nodes)
    sched.upsert_nodes_raw(nodes.nodes, slots, args.nodes)
    pre = None
    if args.prefill > 0:
        pre = synth.prefill(kind, args.nodes, 1, 3, args.prefill)
        assert sched.lib.ks_pods_add(sched.ctx, pre.pods, pre.slot_ptr, pre.n_pods) == 0, \
            sched.lib.ks_last_error(sched.ctx)
    n_batches = args.warmup + args.steps
    pods = synth.pods(kind, n_batches * args.batch, 2)
    batches = [sched.prepare(pods.pods_at(b * args.batch), args.batch) for b in range(n_batches)]
    setup_s = time.time() - t_setup

    def barrier():
        if world > 1:
            sched.allreduce_max([0.0])  # RCCL all-reduce on the scheduler's stream

    def sync():
        pass  # ks_batch_run returns after hipStreamSynchronize on the scheduler stream

    for b in range(args.warmup):
        sched.run(batches[b])
    sched.reset_stats()
    sched.set_timing(True)
    barrier()
    sync()
    t0 = time.perf_counter()
    for b in range(args.warmup, n_batches):
        sched.run(batches[b])
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    sched.set_timing(False)
    if world > 1:
        elapsed = sched.allreduce_max([elapsed])[0]
    # scheduled fraction of the timed pods (sanity for the reader)
    scheduled = 0
    for b in range(args.warmup, n_batches):
        r = results_to_arrays(sched.results(batches[b], args.batch), args.batch)
        scheduled += int((r["status"] == 0).sum())

    pods_timed = args.steps * args.batch
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_pods > 0:
        cpu = cpu_baseline(args, kind, nodes, slots, pre, pods)
    line = report(args, sched, world, pods_timed, elapsed, scheduled, setup_s, cpu)
    for b in batches:
        sched.free(b)
    sched.close()
    if rank == 0:
        print(json.dumps(line), flush=True)


def run_c5(args, kind, sched, world, rank, t_setup):
    """configs[4] (C5): bursts scheduled to completion, each followed by its
    watch-event log applied in order through ks_events_apply.  Timed per step:
    the burst's ks_batch_run plus the log's ks_events_apply call; the log's
    generation (which needs the burst's bindings) and its marshalling to ABI
    structs run outside the timed region."""
    from ksched.framework import results_to_arrays
    from ksched.stream import BurstStream, GpuTarget

    n_bursts = args.warmup + args.steps
    stream = BurstStream(kind, args.nodes, n_bursts, args.burst, prefill=3)
    target = GpuTarget(sched)
    stream.setup([target])
    setup_s = time.time() - t_setup

    def barrier():
        if world > 1:
            sched.allreduce_max([0.0])

    t_run = t_ev = 0.0
    scheduled = n_events = 0
    for b in range(n_bursts):
        timed = b >= args.warmup
        if b == args.warmup:
            sched.reset_stats()
            sched.set_timing(True)
        arr, m = stream.burst_pods(b)
        batch = sched.prepare(arr, m)
        barrier()
        t0 = time.perf_counter()
        sched.run(batch)  # returns after the scheduler stream has drained
        barrier()
        dt = time.perf_counter() - t0
        res = sched.results(batch, m)
        if timed:
            t_run += dt
            r = results_to_arrays(res, m)
            scheduled += int((r["status"] == 0).sum())
        stream.record(b, res)
        sched.free(batch)
        # the API server's side (log generation, ABI structs) is untimed
        ev, ne, keep = stream.event_log(stream.marshal(stream.make_events()))
        barrier()
        t0 = time.perf_counter()
        target.apply_events(ev, ne)  # ks_events_apply: the ordered log, device work done on return
        barrier()
        dt = time.perf_counter() - t0
        del keep
        if timed:
            t_ev += dt
            n_events += ne
    sched.set_timing(False)
    elapsed = t_run + t_ev
    if world > 1:
        elapsed = sched.allreduce_max([elapsed])[0]
    pods_timed = args.steps * args.burst
    c5 = {"burst_ms_mean": round(1e3 * t_run / args.steps, 3), "events_ms_mean": round(1e3 * t_ev / args.steps, 3),
          "events_per_burst": round(n_events / args.steps, 1),
          "events_per_s": round(n_events / t_ev, 1) if t_ev else None,
          "bound_pods_after": int(len(stream.bound_pod))}
    line = report(args, sched, world, pods_timed, elapsed, scheduled, setup_s, None, c5=c5)
    sched.close()
    if rank == 0:
        print(json.dumps(line), flush=True)


WORKLOADS = {
    "hetero": "C3: {n} heterogeneous kwok-shaped nodes, prefill<{f:.0%} cpu, resource-only pods; "
              "Fit+LeastAllocated+BalancedAllocation+TaintToleration, pct=100, in-order commit",
    "kwok": "C1 shape at scale: {n} homogeneous kwok nodes, prefill<{f:.0%} cpu, resource-only pods; "
            "Fit+LeastAllocated+BalancedAllocation+TaintToleration, pct=100, in-order commit",
    "labeled": "C4: {n} nodes with label bitsets and NoSchedule/NoExecute/PreferNoSchedule taints, "
               "prefill<{f:.0%} cpu; pods with nodeSelector / required + preferred NodeAffinity / "
               "tolerations; all default Filter + Score plugins incl. TaintToleration and NodeAffinity "
               "normalisation, pct=100, in-order commit",
}


def report(args, sched, world, pods_timed, elapsed, scheduled, setup_s, cpu, c5=None):
    st = sched.stats()
    dbg = (C.c_uint64 * 16)()
    sched.lib.ks_debug_counters(sched.ctx, dbg)
    value = pods_timed / elapsed
    labeled = args.kind == "labeled"
    b_node = B_NODE_LABELED if labeled else B_NODE
    sweep_avg_ms = st.sweep_ms / max(1, st.sweep_launches)
    evals_per_launch = st.sweep_evals / max(1, st.sweep_launches)
    achieved = b_node * evals_per_launch / (sweep_avg_ms * 1e-3) / 1e9 if st.sweep_launches else None
    traffic, pmc = None, {}
    # the PMC file was measured on the default (C3) workload: used for C3 lines only
    if args.pmc_file and Path(args.pmc_file).exists() and args.kind == "hetero" and args.workload == "batch":
        pmc = json.loads(Path(args.pmc_file).read_text())
        traffic = pmc.get("hbm_bytes_per_sweep_launch")

    line = {
        "metric": "pods scheduled/sec at 1M nodes (1/2/4/8 GPU) + % of HBM roofline",
        "value": round(value, 1),
        "unit": "pods/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64+f64",
        "data": "synthetic (seeded kwok-shaped cluster and pod stream, libksynth)",
        "config": {
            "workload": WORKLOADS[args.kind].format(n=args.nodes, f=args.prefill),
            "nodes": args.nodes,
            "pods_per_step": args.burst if c5 else args.batch,
            "pods_per_round": args.pods_per_round,
            "topk": args.topk or args.pods_per_round,
            "parallelism": f"node-sharded x{world} (RCCL all-gather)" if world > 1 else "1 GPU",
            "node_evals_per_pod": args.nodes,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": traffic,
            "kernel": "ks::sweep_kernel",
            "bytes_per_eval": b_node,
            "evals_per_launch": int(evals_per_launch),
            "avg_launch_ms": round(sweep_avg_ms, 4),
            "traffic_source": (f"profiles/{Path(args.pmc_file).name} ({pmc.get('tag')}): 2 x FETCH_SIZE + WRITE_SIZE "
                               "per launch at the default config; L2 memory-side bytes (Infinity-Cache hits "
                               "included)") if traffic else None,
            "valu_lane_ops_per_eval": pmc.get("valu_lane_ops_per_eval"),
            # the sweep re-reads each node row once per pod group, not once per
            # pod, so its HBM fraction exceeds 1; the binding resource is VALU issue
            "valu": valu_roofline(pmc, evals_per_launch, sweep_avg_ms),
        },
        "cpu_baseline": cpu,
        "extra": {
            "rounds": int(st.rounds),
            "pods_per_round_resolved": round(pods_timed / max(1, st.rounds), 2),
            "resolve_ms_per_round": round(st.resolve_ms / max(1, st.resolve_launches), 4),
            "sweep_ms_total": round(st.sweep_ms, 3),
            "resolve_ms_total": round(st.resolve_ms, 3),
            "scheduled_fraction": round(scheduled / pods_timed, 4),
            "speculated_rounds_wasted": int(dbg[3]),  # since open (warmup included)
            "pods_reswept_wrong_norm_guess": int(dbg[4]),  # since open (warmup included)
            "node_evals_per_s": round(value * args.nodes, 1),
            "setup_s": round(setup_s, 2),
        },
    }
    if c5:
        line["config"]["workload"] = (
            f"C5: {args.nodes} heterogeneous nodes, prefill<50% cpu; bursts of {args.burst} resource-only pods, "
            "each followed by its watch-event log (5% bound-pod deletes, 0.1% node updates, 0.01% node "
            "deletes + adds) applied to the device cache; pct=100, in-order commit")
        line["config"]["bursts_timed"] = args.steps
        line["extra"].update(c5)
    return line




def valu_roofline(pmc, evals_per_launch, sweep_avg_ms):
    ops = pmc.get("valu_lane_ops_per_eval")
    if not ops or not sweep_avg_ms:
        return None
    achieved = ops * evals_per_launch / (sweep_avg_ms * 1e-3) / 1e12
    return {"achieved": round(achieved, 2), "peak": round(VALU_PEAK_TOPS, 2), "unit": "T lane-ops/s",
            "frac": round(achieved / VALU_PEAK_TOPS, 4),
            "source": "SQ_INSTS_VALU x 64 per evaluation from the PMC file; 32-bit issue-rate peak"}


def uid_path(world: int) -> Path:
    # Every local rank of one launch is a child of the same torchrun agent, so
    # the agent's pid (+ its restart count) names this launch alone: a file
    # left by an earlier launch on the same port is never read.
    key = "_".join([os.environ.get("TORCHELASTIC_RUN_ID", "run"), os.environ.get("MASTER_PORT", "0"),
                    str(os.getppid()), os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")]).replace("/", "_")
    return Path(os.environ.get("TMPDIR", "/tmp")) / f"ksched_uid_{key}_w{world}.bin"


def exchange_unique_id(rank: int, world: int) -> bytes:
    """Rank 0 publishes the RCCL unique id in a file every local rank reads."""
    from ksched import Scheduler

    path = uid_path(world)
    if rank == 0:
        tmp = path.with_suffix(".tmp")
        tmp.write_bytes(Scheduler.comm_unique_id())
        os.replace(tmp, path)
        return path.read_bytes()
    deadline = time.time() + 300
    while time.time() < deadline:
        if path.exists():
            data = path.read_bytes()
            if len(data) == 128:
                return data
        time.sleep(0.05)
    raise TimeoutError(f"rank {rank}: no RCCL unique id at {path}")


def cpu_baseline(args, kind, nodes, slots, pre, pods):
    """The CPU oracle (oracle/oracle.cpp, C++ restatement of upstream v1.31.3) on
    the same cluster, timed on a bounded pod sample, one host thread."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle

    o = pyoracle.Oracle(args.nodes)
    o.upsert(nodes.nodes, slots, args.nodes)
    if pre is not None:
        o.add_pods(pre.pods, pre.slot_ptr, pre.n_pods)
    # single thread: the first cpu_pods pods of the stream
    n1 = args.cpu_pods
    t0 = time.perf_counter()
    o.schedule(pods.pods, n1)
    dt1 = time.perf_counter() - t0
    o.close()
    # threads with parallelize.Until's chunking (oracle.cpp), on a fresh replica
    nt, n = max(1, args.cpu_threads), args.cpu_pods_mt
    o = pyoracle.Oracle(args.nodes, threads=nt)
    o.upsert(nodes.nodes, slots, args.nodes)
    if pre is not None:
        o.add_pods(pre.pods, pre.slot_ptr, pre.n_pods)
    t0 = time.perf_counter()
    o.schedule(pods.pods, n)
    dt = time.perf_counter() - t0
    o.close()
    return {"value": round(n / dt, 2), "unit": "pods/s", "cores": nt, "kind": "port",
            "sample": f"first {n} pods of the stream on the same {args.nodes}-node prefilled cluster "
                      f"({n * args.nodes:.2e} node evaluations, {dt:.1f} s), {nt} threads "
                      "(parallelize.Until chunking)",
            "single_thread": {"value": round(n1 / dt1, 2), "cores": 1,
                              "sample": f"first {n1} pods, {dt1:.1f} s"}}


if __name__ == "__main__":
    main()
