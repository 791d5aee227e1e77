#!/usr/bin/env python3
"""bench.py — pods scheduled/sec at 1M nodes (BASELINE.json metric) on MI355X.

Workload (default: BASELINE.json configs[2], "C3" of SURVEY.md §8(d)): a
1,000,000-node kwok-shaped heterogeneous cluster (cpu 8-96 cores, memory
32-512 Gi, 32/110 pods, kwok NoSchedule taint; every node pre-filled with
seeded pods to a random 0-50% of its CPU), and a stream of resource-only pods
(cpu 50-4000m, memory 64Mi x 1..256, 10% best-effort, kwok tolerations).
Filter = NodeUnschedulable/NodeName/TaintToleration/NodeAffinity/
NodeResourcesFit, Score = LeastAllocated + BalancedAllocation +
TaintToleration (+ NodeAffinity skipped, ImageLocality 0),
percentageOfNodesToScore = 100, deterministic lowest-slot tie-break,
sequential-equivalent in-order commit.

A "step" schedules one batch of pods (default 50,000: the driver's 20 steps
are configs[2]'s 1,000,000 pods) to completion against the
live cluster, through the whole boundary the cgo caller uses: `value` times
ks_batch_prepare (pod compile + H2D), ks_batch_submit / ks_batch_wait (every
round + D2H of the results) and ks_batch_results, pipelined so that compiling
batch k+1 overlaps running batch k.  Beside it the line reports:

* value_inputs_resident: the same number of steps with every batch compiled
  and uploaded before the timed region (ks_batch_run only: the device-side
  rate with inputs resident in HBM);
* latency: per-call wall time of ks_schedule (compile + upload + run +
  results) for 1-, 16- and 256-pod batches (p50 / p99), next to the
  reference's ScheduleOne latency (~560 us per pod per shard, README.adoc:786);
* roofline: the sweep kernel's VALU issue fraction (its binding resource) from
  the PMC file measured for this exact configuration and kernel source
  (profiles/pmc/<key>.json, tools/gpu.sh pmc), with the measured HBM traffic and
  its fraction of 8 TB/s beside it;
* cpu_baseline: the C++ oracle (a restatement of upstream kube-scheduler) on a
  bounded prefix of the same stream, on the box's CPU share.

--gpus N: one process per GPU.  Launched by torchrun (WORLD_SIZE set) each
rank runs directly; otherwise bench.py starts the N rank processes itself
(children get RANK / LOCAL_RANK / WORLD_SIZE; nothing touches the GPU before
they start).  Node slots are sharded across ranks (RCCL candidate
all-gather); every rank schedules the same pods, so `value` is the job's pods/s
(strong scaling: the cluster is fixed at 1M nodes).

--kind labeled is configs[3] (C4).  --kind kwok is the reference's own node
shape (kwok/make_nodes/main.go:126-181), with --pods besteffort its request-less
busybox pods (kwok/make_pods/main.go:118-148).  --workload c5 is configs[4]:
a step is one burst (default 100k pods) scheduled to completion followed by
the seeded watch-event log applied through ks_events_apply.
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "k8s-1m_amd"))

B_NODE = 56  # node-row bytes per (pod, node) evaluation, resource-only
B_NODE_LABELED = 96  # ... with label / taint bitsets (C4)
# PodTopologySpread path: node-table bytes the kernel chain reads / writes per
# (pod, node): prep 52 (slot, apods, taint / label / numeric
# words, 2 domain ids, 1 class count), filter 101 (slot, 56-B resource row,
# 32-B label / taint words, 2 domain ids, status), score 21 (status, domain
# ids, class count, raw score), select 101 (status, slot, resource row,
# label / taint words, raw score)
B_SPREAD_NODE = 275
# InterPodAffinity pods of --pods affinity on the same chain: prep 32 (slot,
# apods, domain id + count column of 3 records), filter 133 (slot, 56-B
# resource row, 32-B label / taint words, 3 domain ids + domain sums, status,
# packed parts, raw score), select 21 (status, slot, packed parts, raw score)
B_AFF_NODE = 186
# Replica runs of --pods deploy, per node per run: the filter
# pass (B_SPREAD_FILTER: slot, resource row, label / taint words, domain ids,
# class count, status, packed parts), the sort keys + positions written (12),
# read and written once by the radix sort (24), the sorted keys read by the
# group-start pass (8)
B_SPREAD_FILTER = 109
B_RUN_NODE = B_SPREAD_FILTER + 12 + 24 + 8
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# VALU issue peak of the sweep: 256 CUs x 4 SIMDs x 2.4 GHz SIMD cycles per
# second over the cycles ONE wave64 VALU instruction of the sweep's own mix
# occupies a SIMD.  That cost is measured, not assumed: tools/valu_issue.hip
# times every opcode of the sweep's pod loop at 4 waves per SIMD on MI355X
# (profiles/valu_issue.jsonl: the 32-bit add / logic / move class 2.3-2.5
# cycles, f64 arithmetic, conversions, compares, multiplies, DPP, readlane and
# VOP3 forms 4.2-4.4) and tools/valu_mix.py weights them by each kernel's loop
# mix (profiles/valu_mix.json: 4.08 cycles for the C3 kernel, 3.88 for C4's).
SIMD_CYCLES_PER_S = 256 * 4 * 2.4e9
VALU_CYCLES_FALLBACK = 4.0  # when valu_mix.json does not match the kernel sources
E2E_DEPTH = 2  # batches submitted ahead in the headline loop (compile of k+1 and k+2 overlaps run k)
REF_SCHEDULE_ONE_US = 560.0  # README.adoc:786 (per pod per shard, ~195 nodes evaluated)
KERNEL_SOURCES = ["k8s-1m_amd/csrc/ksched_kernels.hip", "k8s-1m_amd/csrc/ksched_eval.hpp", "k8s-1m_amd/csrc/ksched_dev.hpp",
                  "k8s-1m_amd/csrc/ksched_kernels.hpp", "k8s-1m_amd/csrc/ksched_util.hpp",
                  "k8s-1m_amd/csrc/ksched_instr.hpp", "k8s-1m_amd/csrc/ksched_resolve.hip",
                  "k8s-1m_amd/csrc/ksched_resolve_serial.hpp", "k8s-1m_amd/Makefile"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=50_000,
                    help="pods per step (each batch refills the round pipeline once)")
    ap.add_argument("--pods-per-round", type=int, default=256)
    ap.add_argument("--topk", type=int, default=0)
    ap.add_argument("--nodes-per-lane", type=int, default=None,
                    help="default 4 on one GPU; 2 when sharded over several GPUs (twice the sweep blocks per "
                         "shard: a shard's candidate lists hold up to 4 keys per block, and at tied top scores "
                         "a 125k-node shard's lists ran short with 4, DESIGN §6)")
    ap.add_argument("--kind", default="hetero", choices=["hetero", "kwok", "labeled", "zoned"])
    ap.add_argument("--pods", default="default", choices=["default", "besteffort", "spread", "deploy", "deploy-dns", "affinity"],
                    help="besteffort: request-less pods (kwok/make_pods/main.go:118-148); spread: "
                         "deployment pods with PodTopologySpread constraints (use with --kind zoned); deploy: "
                         "deployment replicas under the system default constraints (identical per deployment); deploy-dns: "
                         "the same deployments under zone maxSkew 1 DoNotSchedule + hostname ScheduleAnyway")
    ap.add_argument("--apps", type=int, default=64, help="deployments of the --pods spread stream")
    ap.add_argument("--pct", type=int, default=100,
                    help="percentageOfNodesToScore (100: every node; the reference's deployed profile uses 5, "
                         "terraform/kubernetes/dist-scheduler.tf:562): below 100 every pod takes the one-pod chain "
                         "with the window pass (DESIGN.md §5.8)")
    ap.add_argument("--replicas", type=int, default=256, help="replicas per deployment of the --pods deploy stream")
    ap.add_argument("--workload", default="batch", choices=["batch", "c5"],
                    help="batch: one batch of --batch pods per step; c5: one burst + its event log per step")
    ap.add_argument("--burst", type=int, default=100_000, help="pods per burst (--workload c5)")
    ap.add_argument("--prefill", type=float, default=None, help="max prefill fraction (default 0.5, kwok 0)")
    ap.add_argument("--no-resident", action="store_true",
                    help="skip the secondary inputs-resident pass (batches compiled + uploaded before timing)")
    ap.add_argument("--latency-calls", type=int, default=100, help="ks_schedule calls per latency batch size (0: skip)")
    ap.add_argument("--cpu-pods", type=int, default=48, help="oracle sample (pods), single thread (~4 s at 1M nodes)")
    ap.add_argument("--cpu-pods-mt", type=int, default=1000, help="oracle sample (pods), multi-thread (~10 s at 1M nodes on 16 threads)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch check only: spawn / join the ranks, exchange the rendezvous file, check "
                         "RANK / LOCAL_RANK / WORLD_SIZE, print one JSON line per rank; no GPU call")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="ks_config execution option (include/ksched.h), e.g. resolve_mode=1; none changes a result")
    ap.add_argument("--resolve-profile", action="store_true",
                    help="phase clocks of the parallel commit during the inputs-resident pass (diagnostic)")
    ap.add_argument("--pmc-dir", default=str(ROOT / "profiles" / "pmc"),
                    help="per-configuration PMC summaries (tools/gpu.sh pmc + tools/pmc_summary.py)")
    a = ap.parse_args()
    if a.nodes_per_lane is None:
        a.nodes_per_lane = 2 if a.gpus > 1 else 4
    if a.prefill is None:
        a.prefill = 0.0 if a.kind == "kwok" else 0.5
    if a.pods in ("spread", "deploy", "deploy-dns", "affinity") or a.pct != 100:  # one-pod path: smaller steps
        if a.batch == 50_000:
            a.batch = 2048
        a.cpu_pods = min(a.cpu_pods, 4)
        a.cpu_pods_mt = min(a.cpu_pods_mt, 16)
        a.latency_calls = min(a.latency_calls, 10)
    return a


# ------------------------------------------------------------------ launch

def spawn_ranks(args) -> int:
    """--gpus N without a launcher: start the N rank processes (before any GPU call)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    rc = 0
    try:
        for p in procs:
            rc = max(rc, p.wait())
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def uid_path(world: int) -> Path:
    # Every local rank of one launch is a child of the same parent (the torchrun
    # agent, or bench.py's own spawner), so the parent's pid (+ its restart
    # count) names this launch alone: a file left by an earlier launch is never read.
    key = "_".join([os.environ.get("TORCHELASTIC_RUN_ID", "run"), os.environ.get("MASTER_PORT", "0"),
                    str(os.getppid()), os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")]).replace("/", "_")
    return Path(os.environ.get("TMPDIR", "/tmp")) / f"ksched_uid_{key}_w{world}.bin"


def exchange_unique_id(rank: int, world: int, uid: bytes = None) -> bytes:
    """Rank 0 publishes the RCCL unique id in a file every local rank reads
    (uid: a given 128-byte id instead of ncclGetUniqueId's, --dry-run)."""
    path = uid_path(world)
    if rank == 0:
        if uid is None:
            from ksched import Scheduler

            uid = Scheduler.comm_unique_id()
        tmp = path.with_suffix(".tmp")
        tmp.write_bytes(uid)
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


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank, local_rank)
    # No torch in this process: torch bundles its own libamdhip64 / librccl
    # (ROCm 7.0) with the same sonames as the /opt/rocm 7.2 libraries
    # libksched links, and one process must not mix the two runtimes.  The
    # ranks rendezvous through a file on the node (RCCL unique id) and use the
    # scheduler's own RCCL communicator for barriers and the max-over-ranks time.
    from ksched import Scheduler, synth

    kind = {"hetero": synth.HETERO, "kwok": synth.KWOK, "labeled": synth.LABELED, "zoned": synth.ZONED}[args.kind]
    t_setup = time.time()
    options = {k: int(v) for k, v in (o.split("=", 1) for o in args.opt)}
    sched = Scheduler(args.nodes, device=local_rank if world > 1 else 0, pods_per_round=args.pods_per_round,
                      topk=args.topk, nodes_per_lane=args.nodes_per_lane, world_size=world, rank=rank, options=options,
                      percentage_of_nodes_to_score=args.pct)
    if world > 1:
        sched.comm_init(exchange_unique_id(rank, world))
        if rank == 0:  # ncclCommInitRank returned: every rank has read the id
            uid_path(world).unlink(missing_ok=True)
    if args.workload == "c5":
        return run_c5(args, kind, sched, world, rank, t_setup)
    return run_batches(args, kind, sched, world, rank, t_setup)


def dry_run(args, world, rank, local_rank):
    """The multi-rank launch without the GPU: the environment every rank
    reads, the rendezvous file (a synthetic id, checked byte for byte by
    every rank), the device each rank would open; one JSON line per rank."""
    ok = 0 <= rank < world and 0 <= local_rank < world and int(os.environ.get("LOCAL_WORLD_SIZE", world)) == world
    if world > 1:
        uid = bytes((i * 7 + 3) & 0xFF for i in range(128))  # the same synthetic id on every rank
        got = exchange_unique_id(rank, world, uid if rank == 0 else None)
        ok = ok and got == uid
        if rank == 0:  # every rank has the file open or read by the time rank 0 removes it:
            time.sleep(1.0)  # (the real launch removes it after ncclCommInitRank returns)
            uid_path(world).unlink(missing_ok=True)
    line = {"dry_run": True, "rank": rank, "local_rank": local_rank, "world_size": world,
            "device": local_rank if world > 1 else 0, "master": f"{os.environ.get('MASTER_ADDR', '')}:"
                                                               f"{os.environ.get('MASTER_PORT', '')}",
            "rendezvous_ok": bool(ok)}
    # one write(2) per line: the ranks share the launcher's stdout pipe
    sys.stdout.flush()
    os.write(sys.stdout.fileno(), (json.dumps(line) + "\n").encode())
    return 0 if ok else 1


def pod_stream(args, kind, n, seed):
    from ksched import synth

    if args.pods == "besteffort":
        return synth.besteffort_pods(n)
    if args.pods == "spread":
        return synth.spread_pods(n, args.apps, seed)
    if args.pods == "deploy":
        return synth.deploy_pods(n, args.replicas, seed)
    if args.pods == "deploy-dns":
        return synth.deploy_dns_pods(n, args.replicas, seed)
    if args.pods == "affinity":
        return synth.affinity_pods(n, args.apps, seed)
    return synth.pods(kind, n, seed)


def run_batches(args, kind, sched, world, rank, t_setup):
    from ksched import synth

    nodes = synth.nodes(kind, args.nodes, 1)
    slots = synth.slot_array(args.nodes)
    sched.upsert_nodes_raw(nodes.nodes, slots, args.nodes)
    pre = None
    if args.prefill > 0:
        pre = synth.prefill(kind, args.nodes, 1, 3, args.prefill)
        assert sched.lib.ks_pods_add(sched.ctx, pre.pods, pre.slot_ptr, pre.n_pods) == 0, \
            sched.lib.ks_last_error(sched.ctx)

    def barrier():
        if world > 1:
            sched.allreduce_max([0.0])  # RCCL all-reduce on the scheduler's stream

    setup_s = time.time() - t_setup
    # the headline: every step through the whole boundary (compile + H2D +
    # run + D2H), W untimed steps first
    e2e = end_to_end(args, kind, sched, world, barrier)
    st = sched.stats()
    dbg = (C.c_uint64 * 16)()
    sched.lib.ks_debug_counters(sched.ctx, dbg)
    # secondary: the same number of steps with every batch compiled and
    # uploaded before the timed region (inputs resident in HBM)
    if args.resolve_profile:
        sched.lib.ks_debug_set_profile(sched.ctx, 1)
    res = None if args.no_resident else resident(args, kind, sched, world, barrier)
    prof = None
    if args.resolve_profile:
        pr = (C.c_uint64 * 16)()
        sched.lib.ks_debug_resolve_profile(sched.ctx, pr)
        rounds = max(1, int(pr[9]))
        # phase clock slots (ksched_resolve.hip resolve_parallel); wave 0's
        # gather is slots 12 (prefetched windows), 13 (probes), 14 (scans), 3 (DMA issue), 5 (DMA wait)
        names = {0: "stage", 12: "gather_w0_prefetch_wait", 13: "gather_w0_probes", 14: "gather_w0_scans",
                 3: "gather_w0_dma_issue", 5: "gather_w0_dma_wait", 1: "gather_barrier", 2: "proposals",
                 4: "chunk_pairs", 6: "commit", 7: "rpre_update", 8: "epilogue"}
        prof = {"rounds": int(pr[9]), "cycles_per_round": {k: round(int(pr[i]) / rounds, 1) for i, k in names.items()}}
        prof["cycles_per_round"]["total"] = round(sum(int(pr[i]) for i in names) / rounds, 1)
        prof["dirty_recomputes_per_round"] = round(int(pr[10]) / rounds, 2)
        prof["extra_windows_per_round"] = round(int(pr[11]) / rounds, 2)
    lat = latency(args, kind, sched, world) if args.latency_calls > 0 else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_pods > 0:
        cpu = cpu_baseline(args, nodes, slots, pre, pod_stream(args, kind, args.cpu_pods_mt + args.cpu_pods, 7))
    # one-pod-path filter passes over every node count too: one per pod of the
    # per-pod chain and one per replica run; st covers
    # the timed steps (reset before them)
    # (since round 5 pods_swept, node_evals_per_s and pods_swept_fraction
    # include these one-pod-path passes; round-4 and earlier records counted
    # the round sweeps only: compare sweep_pods_swept across rounds)
    one_pod_passes = int(st.spread_pods - st.replica_pods) + int(st.replica_runs)
    round_swept = e2e.pop("pods_swept")
    line = report(args, sched, st, dbg, world, e2e.pop("pods_timed"), e2e.pop("elapsed"), e2e.pop("scheduled"),
                  setup_s, cpu, pods_swept=round_swept + one_pod_passes)
    line["extra"]["sweep_pods_swept"] = round_swept
    line["extra"]["one_pod_path_node_passes"] = one_pod_passes
    line["extra"]["host_compile_ms_per_step"] = e2e["host_compile_ms_per_step"]
    line["end_to_end"] = e2e
    if res:
        line["value_inputs_resident"] = res.pop("value")
        line["inputs_resident"] = res
    if lat:
        line["latency"] = lat
    if prof:
        line["resolve_profile"] = prof
    sched.close()
    if rank == 0:
        print(json.dumps(line), flush=True)


def end_to_end(args, kind, sched, world, barrier):
    """The headline steps: each batch goes through the whole boundary a cgo
    caller uses -- ks_batch_prepare (pod compile + H2D), ks_batch_submit /
    ks_batch_wait (every round + D2H of the results), ks_batch_results -- with
    batch k+1 compiled on the host while batch k runs.  W untimed steps, then
    K timed steps between barriers (fresh pods, seed 7, against the live
    cluster); HIP-event timing of the kernels covers the timed steps."""
    import numpy  # noqa: F401 -- imported here, not by the first results_to_arrays inside the timed steps (~0.1 s)

    from ksched import _abi
    from ksched.framework import results_to_arrays

    w, n = args.warmup, args.steps
    pods = pod_stream(args, kind, (w + n) * args.batch, 7)
    lib, ctx = sched.lib, sched.ctx
    out = (_abi.KsResult * args.batch)()
    scheduled = 0

    def run(k0, k1, timed):
        # up to DEPTH batches submitted ahead of the one being waited for, so
        # the worker always finds the next batch queued when a run ends
        nonlocal scheduled
        compile_s = 0.0
        inflight = []
        nxt = k0
        for k in range(k0, k1):
            while nxt < k1 and len(inflight) < E2E_DEPTH:
                tc = time.perf_counter()
                b = sched.prepare(pods.pods_at(nxt * args.batch), args.batch)
                if nxt > k0:
                    compile_s += time.perf_counter() - tc
                assert lib.ks_batch_submit(ctx, b) == 0
                inflight.append(b)
                nxt += 1
            cur = inflight.pop(0)
            assert lib.ks_batch_wait(ctx, cur) == 0, lib.ks_last_error(ctx)
            assert lib.ks_batch_results(ctx, cur, out) == 0
            if timed:
                scheduled += int((results_to_arrays(out, args.batch)["status"] == 0).sum())
            sched.free(cur)
        return compile_s

    if w:
        run(0, w, False)
    sched.reset_stats()
    sched.set_timing(True)
    dbg0 = (C.c_uint64 * 16)()
    sched.lib.ks_debug_counters(ctx, dbg0)
    barrier()
    t0 = time.perf_counter()
    compile_s = run(w, w + n, True)
    barrier()
    elapsed = time.perf_counter() - t0
    sched.set_timing(False)
    dbg1 = (C.c_uint64 * 16)()
    sched.lib.ks_debug_counters(ctx, dbg1)
    if world > 1:
        elapsed = sched.allreduce_max([elapsed])[0]
    return {"pods_timed": n * args.batch, "elapsed": elapsed, "scheduled": scheduled,
            # pods the sweeps evaluated in the timed steps: one per class of a
            # round's byte-identical pods
            "pods_swept": int(dbg1[2] - dbg0[2]),
            "host_compile_ms_per_step": round(1e3 * compile_s / max(1, n - 1), 3),
            "what": "value: ks_batch_prepare (compile + H2D) + ks_batch_submit/wait (run + D2H) + "
                    "ks_batch_results per step, batch k+1 compiled while batch k runs; fresh pods (seed 7)"}


def resident(args, kind, sched, world, barrier):
    """The same step count with every batch compiled and uploaded before the
    timed region (ks_batch_prepare ahead, ks_batch_run timed): the device-side
    rate with inputs resident in HBM."""
    n = args.steps
    pods = pod_stream(args, kind, n * args.batch, 2)
    t0 = time.perf_counter()
    batches = [sched.prepare(pods.pods_at(b * args.batch), args.batch) for b in range(n)]
    prepare_s = time.perf_counter() - t0
    barrier()
    t0 = time.perf_counter()
    for b in batches:
        sched.run(b)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = sched.allreduce_max([elapsed])[0]
    for b in batches:
        sched.free(b)
    return {"value": round(n * args.batch / elapsed, 1), "unit": "pods/s", "steps": n,
            "ms_per_step": round(1e3 * elapsed / n, 3),
            "prepare_us_per_pod": round(1e6 * prepare_s / (n * args.batch), 3),
            "what": "ks_batch_run only: every batch compiled + uploaded by ks_batch_prepare before the timed "
                    "region; pods seed 2, after the headline steps"}


def latency(args, kind, sched, world):
    """Per-call wall time of ks_schedule (compile + upload + run + results) on
    the live cluster, for 1-, 16- and 256-pod batches."""
    import numpy as np

    from ksched import _abi

    res = {}
    seed = 100
    for size in (1, 16, 256):
        calls = max(5, args.latency_calls if size < 256 else args.latency_calls // 2)
        pods = pod_stream(args, kind, size * (calls + 3), seed)
        seed += 1
        out = (_abi.KsResult * size)()
        ts = []
        for c in range(calls + 3):  # 3 untimed calls warm the batch pool
            t0 = time.perf_counter()
            st = sched.lib.ks_schedule(sched.ctx, pods.pods_at(c * size), size, out)
            dt = time.perf_counter() - t0
            assert st == 0, sched.lib.ks_last_error(sched.ctx)
            if c >= 3:
                ts.append(dt)
        a = np.array(ts) * 1e6
        res[f"batch_{size}"] = {"calls": calls, "p50_us": round(float(np.percentile(a, 50)), 1),
                                "p99_us": round(float(np.percentile(a, 99)), 1),
                                "per_pod_p50_us": round(float(np.percentile(a, 50)) / size, 2)}
    res["reference_schedule_one_us"] = REF_SCHEDULE_ONE_US
    res["what"] = ("ks_schedule wall time per call (pod compile + H2D + every round + D2H), "
                   f"{args.nodes} nodes, {world} GPU(s); reference: ScheduleOne per pod per shard "
                   "(~3.9k nodes, ~195 evaluated), README.adoc:786")
    return res


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
    st = sched.stats()
    dbg = (C.c_uint64 * 16)()
    sched.lib.ks_debug_counters(sched.ctx, dbg)
    pods_timed = args.steps * args.burst
    c5 = {"burst_ms_mean": round(1e3 * t_run / args.steps, 3), "events_ms_mean": round(1e3 * t_ev / args.steps, 3),
          "events_per_burst": round(n_events / args.steps, 1),
          "events_per_s": round(n_events / t_ev, 1) if t_ev else None,
          "bound_pods_after": int(len(stream.bound_pod))}
    line = report(args, sched, st, dbg, world, pods_timed, elapsed, scheduled, setup_s, None, c5=c5)
    sched.close()
    if rank == 0:
        print(json.dumps(line), flush=True)


# ------------------------------------------------------------------ report

def workload_name(args) -> str:
    name = base_workload_name(args)
    if args.pct != 100:
        name = name.replace("pct=100", f"percentageOfNodesToScore={args.pct} (every pod on the one-pod chain with "
                                       "the window pass, DESIGN §5.8)")
    return name


def base_workload_name(args) -> str:
    n, f = args.nodes, args.prefill
    if args.workload == "c5":
        return (f"C5: {n} heterogeneous nodes, prefill<50% cpu; bursts of {args.burst} resource-only pods, "
                "each followed by its watch-event log (5% bound-pod deletes, 0.1% node updates, 0.01% node "
                "deletes + adds) applied to the device cache; pct=100, in-order commit")
    if args.pods == "spread":
        return (f"spread: {n} heterogeneous nodes in 32 zones, prefill<{f:.0%} cpu (pods of 64 apps); "
                f"pods of {args.apps} deployments with PodTopologySpread (half the system defaults: hostname "
                "maxSkew 3 + zone maxSkew 5 ScheduleAnyway; half zone maxSkew 1 DoNotSchedule + hostname "
                "maxSkew 1 ScheduleAnyway), every default Filter / Score plugin, pct=100, one pod at a time "
                "(spread path)")
    if args.pods == "deploy":
        return (f"deploy: {n} heterogeneous nodes in 32 zones, prefill<{f:.0%} cpu (pods of 64 apps); "
                f"deployments of {args.replicas} identical replicas under PodTopologySpread's system defaults "
                "(hostname maxSkew 3 + zone maxSkew 5, ScheduleAnyway, selecting the deployment), every default "
                "Filter / Score plugin, pct=100, in queue order (spread path, replica runs)")
    if args.pods == "deploy-dns":
        return (f"deploy-dns: {n} heterogeneous nodes in 32 zones, prefill<{f:.0%} cpu (pods of 64 apps); "
                f"deployments of {args.replicas} identical replicas with zone maxSkew 1 DoNotSchedule + "
                "hostname maxSkew 1 ScheduleAnyway (selecting the deployment), every default Filter / Score "
                "plugin, pct=100, in queue order (spread path, replica runs)")
    if args.pods == "affinity":
        return (f"affinity: {n} heterogeneous nodes in 32 zones, prefill<{f:.0%} cpu (pods of 64 apps); "
                f"pods of {args.apps} deployments with InterPodAffinity terms (half required hostname "
                "anti-affinity + preferred zone affinity (50) to the own app, half preferred hostname "
                "anti-affinity (100) + required zone affinity to the next app), every default Filter / "
                "Score plugin, pct=100, one pod at a time (spread path)")
    pods = ("request-less busybox pods (kwok/make_pods)" if args.pods == "besteffort"
            else "resource-only pods (cpu 50-4000m, mem 64Mi x 1..256, 10% best-effort)")
    if args.kind == "hetero":
        cfg = "C2" if n <= 100_000 else "C3"
        return (f"{cfg}: {n} heterogeneous kwok-shaped nodes, prefill<{f:.0%} cpu, {pods}; "
                "Fit+LeastAllocated+BalancedAllocation+TaintToleration, pct=100, in-order commit")
    if args.kind == "kwok":
        return (f"kwok: {n} identical kwok nodes (kwok/make_nodes), prefill<{f:.0%} cpu, {pods}; "
                "Fit+LeastAllocated+BalancedAllocation+TaintToleration, pct=100, in-order commit")
    return (f"C4: {n} nodes with label bitsets and NoSchedule/NoExecute/PreferNoSchedule taints, "
            f"prefill<{f:.0%} cpu; pods with nodeSelector / required + preferred NodeAffinity / "
            "tolerations; all default Filter + Score plugins incl. TaintToleration and NodeAffinity "
            "normalisation, pct=100, in-order commit")


def pmc_key(args, world) -> str:
    """Name of the PMC summary measured for exactly this configuration."""
    pods = {"besteffort": "-be", "spread": "-spread", "deploy": "-deploy", "deploy-dns": "-deploy-dns", "affinity": "-affinity"}.get(args.pods, "")
    if args.pct != 100:
        pods += f"-pct{args.pct}"
    return (f"{args.workload}_{args.kind}{pods}_n{args.nodes}_P{args.pods_per_round}_K{args.topk or args.pods_per_round}"
            f"_npl{args.nodes_per_lane}_w{world}")


def kernel_src_hash() -> str:
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update((ROOT / f).read_bytes())
    return h.hexdigest()[:16]


def roofline_spread(args, st):
    """The spread path: HBM-bound node passes (B_SPREAD_NODE bytes per node per
    pod), timed per pod with HIP events around the whole kernel chain."""
    ms = st.spread_ms / max(1, st.spread_pods_timed)
    b_node = B_AFF_NODE if args.pods == "affinity" else B_SPREAD_NODE
    traffic = b_node * args.nodes
    ach = traffic / (ms * 1e-3) / 1e9 if ms else None
    return {"bound": "hbm", "achieved": round(ach, 1) if ach else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None, "traffic": None,
            "kernel": "ks::spread_* chain (prep, min, filter, score, select, commit)",
            "ms_per_pod": round(ms, 4), "pods_timed": int(st.spread_pods_timed),
            "algorithmic_bytes_per_pod": traffic,
            "what": f"{'B_AFF_NODE' if args.pods == 'affinity' else 'B_SPREAD_NODE'} x nodes per pod / chain "
                    "time (HIP events on every 8th pod)"}


def roofline_deploy(args, st):
    """Replica runs: per run one filter pass, the sort keys, the radix sort and
    the group starts over every node (B_RUN_NODE bytes per node), then one
    workgroup walks the run's pods (latency-bound: three LDS barriers and one
    commit per pod).  Achieved = B_RUN_NODE x nodes / the mean run's device
    time (HIP events around every timed run)."""
    runs = int(st.replica_runs)
    if not runs or not st.replica_ms:
        return roofline_spread(args, st)
    ms_run = st.replica_ms / runs
    traffic = B_RUN_NODE * args.nodes
    ach = traffic / (ms_run * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": "replica run (spread_filter, replica_keys, radix sort, replica_groups, replica_run)",
            "ms_per_run": round(ms_run, 4), "pods_per_run": round(st.replica_pods / runs, 1),
            "us_per_pod_in_runs": round(1e3 * st.replica_ms / max(1, st.replica_pods), 3),
            "runs_timed": runs, "algorithmic_bytes_per_run": traffic,
            "what": "B_RUN_NODE x nodes per run / run time; the in-run walk is one workgroup (not HBM-bound)"}


def roofline(args, st, world):
    if args.pods in ("deploy", "deploy-dns"):
        return roofline_deploy(args, st)
    if args.pods in ("spread", "affinity") or args.pct != 100:
        return roofline_spread(args, st)
    labeled = args.kind == "labeled"
    sweep_avg_ms = st.sweep_ms / max(1, st.sweep_launches)
    evals_per_launch = st.sweep_evals / max(1, st.sweep_launches)
    launch_s = sweep_avg_ms * 1e-3
    key = pmc_key(args, world)
    src = kernel_src_hash()
    path = Path(args.pmc_dir) / f"{key}.json"
    pmc = json.loads(path.read_text()) if path.exists() else {}
    fresh = bool(pmc) and pmc.get("kernel_src") == src
    kname = pmc.get("sweep_kernel", "ks::sweep_kernel")
    # issue cycles per VALU instruction of this kernel's mix (tools/valu_mix.py)
    mix_path = ROOT / "profiles" / "valu_mix.json"
    mix = json.loads(mix_path.read_text()) if mix_path.exists() else {}
    targs = kname[kname.find("<"):] if "<" in kname else ""
    mk = mix.get("kernels", {}).get(targs) if mix.get("kernel_src") == src else None
    cyc = mk["cycles_per_valu"] if mk else VALU_CYCLES_FALLBACK
    peak_wi = SIMD_CYCLES_PER_S / cyc  # wave instructions per second
    r = {"bound": "valu", "achieved": None, "peak": round(peak_wi * 64 / 1e12, 2),
         "unit": "T VALU lane-ops/s", "frac": None, "traffic": None,
         "kernel": kname, "avg_launch_ms": round(sweep_avg_ms, 4),
         "evals_per_launch": int(evals_per_launch),
         "issue_cycles_per_valu": cyc,
         "issue_model": ("profiles/valu_mix.json (tools/valu_issue.hip costs x the pod loop's opcode mix, "
                         f"{mk['measured_share']:.0%} of it measured opcodes)" if mk else
                         "4.0 cycles per instruction (profiles/valu_mix.json missing or stale)"),
         "pmc": f"profiles/pmc/{key}.json" + ("" if fresh else (" (stale: kernel source changed)" if pmc else
                                                                 " (missing)")),
         "kernel_src": src}
    if fresh and st.sweep_launches:
        wi = pmc["valu_wave_instr_per_eval"] * evals_per_launch  # wave instructions per launch
        r["achieved"] = round(wi * 64 / launch_s / 1e12, 2)
        r["frac"] = round(wi / launch_s / peak_wi, 4)
        r["valu_lane_ops_per_eval"] = round(pmc["valu_wave_instr_per_eval"] * 64, 2)
        for k in ("valu_cycles_per_instr", "valu_f64_share", "clock_ghz"):
            if pmc.get(k) is not None:
                r[k] = pmc[k]
        if pmc.get("clock_ghz"):
            # the peak above is at the 2.4 GHz spec clock; the PMC pass
            # measured the clock the chip held (GRBM_GUI_ACTIVE / 8 / time)
            f = pmc["clock_ghz"] / 2.4
            r["peak_at_measured_clock"] = round(peak_wi * f * 64 / 1e12, 2)
            r["frac_at_measured_clock"] = round(wi / launch_s / (peak_wi * f), 4)
        if pmc.get("valu_busy") is not None:
            r["valu_busy"] = pmc["valu_busy"]  # SQ_ACTIVE_INST_VALU share of SIMD quad-cycles
        if pmc.get("hbm_bytes_per_eval") is not None:
            traffic = pmc["hbm_bytes_per_eval"] * evals_per_launch
            r["traffic"] = int(traffic)
            r["hbm"] = {"achieved": round(traffic / launch_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(traffic / launch_s / 1e9 / HBM_PEAK_GBS, 4),
                        "what": "2 x FETCH_SIZE + WRITE_SIZE per sweep launch (L2 memory-side bytes, "
                                "Infinity-Cache hits included: an upper bound on HBM traffic)"}
        if pmc.get("lds_bank_conflict_ratio") is not None:
            r["lds_bank_conflict_ratio"] = pmc["lds_bank_conflict_ratio"]
    # compulsory node-table bytes: every launch needs each local node row once
    b_node = B_NODE_LABELED if labeled else B_NODE
    local_nodes = args.nodes / world
    r["compulsory_bytes_per_launch"] = int(b_node * local_nodes)
    r["compulsory_hbm_frac"] = round(b_node * local_nodes / launch_s / 1e9 / HBM_PEAK_GBS, 4) if launch_s else None
    # which kernel sets the round time: the sweep (priced above) or the one-workgroup
    # in-order commit (parallel proposal / verify with the serial fallback, DESIGN
    # §5.1 / §5.6), a latency chain with no throughput roofline
    resolve_avg_ms = st.resolve_ms / max(1, st.resolve_launches)
    if st.sweep_launches and st.resolve_launches:
        r["critical_path"] = "sweep" if sweep_avg_ms >= resolve_avg_ms else \
            "resolve (one-workgroup in-order commit, a latency chain; the sweep fraction above is for the overlapped sweep)"
        r["resolve_avg_launch_ms"] = round(resolve_avg_ms, 4)
    return r


def report(args, sched, st, dbg, world, pods_timed, elapsed, scheduled, setup_s, cpu, c5=None, pods_swept=None):
    value = pods_timed / elapsed
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
            "workload": workload_name(args),
            "nodes": args.nodes,
            "pods_per_step": args.burst if c5 else args.batch,
            "pods_per_round": args.pods_per_round,
            "topk": args.topk or args.pods_per_round,
            "parallelism": f"node-sharded x{world} (RCCL all-gather)" if world > 1 else "1 GPU",
            "node_evals_per_pod": args.nodes,
        },
        "roofline": roofline(args, st, world),
        "cpu_baseline": cpu,
        "extra": {
            "rounds": int(st.rounds),
            "pods_per_round_resolved": round(pods_timed / max(1, st.rounds), 2),
            "resolve_ms_per_round": round(st.resolve_ms / max(1, st.resolve_launches), 4),
            "sweep_ms_total": round(st.sweep_ms, 3),
            "resolve_ms_total": round(st.resolve_ms, 3),
            "spread_pods": int(st.spread_pods),
            "replica_runs": int(st.replica_runs),  # replica runs of the spread path
            "replica_pods": int(st.replica_pods),
            "scheduled_fraction": round(scheduled / pods_timed, 4),
            "speculated_rounds_wasted": int(dbg[3]),  # since open (warmup included)
            # parallel commit, since open: rounds it resolved and its chunk passes per round
            "parallel_commit_rounds": int(dbg[13]),
            "parallel_commit_passes_per_round": round(int(dbg[12]) / max(1, int(dbg[13])), 2),
            "pods_reswept_wrong_norm_guess": int(dbg[4]),  # since open (warmup included)
            # identical pods of a round swept once: pods swept (class
            # representatives) / pods in the swept windows, since open
            "sweep_representative_fraction": round(int(dbg[2]) / max(1, int(dbg[2]) + int(dbg[7])), 4),
            # (pod, node) evaluations: the sweeps' actual ones (pods swept x
            # nodes; identical pods of a round are swept once; one-pod-path
            # filter passes: per-pod chain pods + replica runs) and the nominal
            # pods x nodes the metric's "1M node evaluations per pod" counts
            "node_evals_per_s": (round(pods_swept * args.nodes / elapsed, 1) if pods_swept is not None
                                 else round(value * args.nodes, 1)),
            "node_evals_per_s_nominal": round(value * args.nodes, 1),
            "pods_swept_fraction": round(pods_swept / pods_timed, 4) if pods_swept is not None else None,
            "setup_s": round(setup_s, 2),
            "pmc_key": pmc_key(args, world),
        },
    }
    if c5:
        line["config"]["bursts_timed"] = args.steps
        line["extra"].update(c5)
    return line


def cpu_threads() -> int:
    """The CPU share this process may use: OMP_NUM_THREADS (16 per GPU on the
    box), else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(omp))) if omp and omp.isdigit() else aff


def cpu_baseline(args, nodes, slots, pre, pods):
    """The CPU oracle (oracle/oracle.cpp, C++ restatement of upstream v1.31.3) on
    the same cluster and stream prefix: single thread, and the box's CPU
    share with parallelize.Until chunking."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle

    def timed(threads, n):
        o = pyoracle.Oracle(args.nodes, threads=threads, percentage=args.pct)
        o.upsert(nodes.nodes, slots, args.nodes)
        if pre is not None:
            o.add_pods(pre.pods, pre.slot_ptr, pre.n_pods)
        t0 = time.perf_counter()
        o.schedule(pods.pods, n)
        dt = time.perf_counter() - t0
        o.close()
        return dt

    n1 = args.cpu_pods
    dt1 = timed(1, n1)
    nt, n = cpu_threads(), args.cpu_pods_mt
    dt = timed(nt, n)
    return {"value": round(n / dt, 2), "unit": "pods/s", "cores": nt, "kind": "port",
            "sample": f"first {n} pods of the stream on the same {args.nodes}-node cluster "
                      f"({n * args.nodes:.2e} node evaluations, {dt:.1f} s), {nt} threads = the process's CPU "
                      "share (OMP_NUM_THREADS / affinity), parallelize.Until chunking",
            "single_thread": {"value": round(n1 / dt1, 2), "cores": 1, "sample": f"first {n1} pods, {dt1:.1f} s"}}


if __name__ == "__main__":
    sys.exit(main())
