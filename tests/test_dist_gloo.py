"""Multi-rank protocol of the node-sharded path, on CPU with gloo.

Each rank owns a contiguous slot range (the GPU shard of rank r), keeps a full
replica of the cluster and runs, per pod: shard prescore -> all-reduce of the
normalising maxima and the feasible / failure counts -> shard best packed key
-> all-gather -> max -> identical commit on every replica.  This is the
protocol libksched runs over RCCL (ncclAllReduce(max) + ncclAllGather); with
the oracle as the per-shard evaluator, the sharded result must equal the
unsharded schedule exactly, for any world size.

torch is imported only in the spawned ranks (the parent process may hold
libksched, which must not share a process with torch's bundled HIP runtime).
"""
import multiprocessing as mp
import os
import socket

import pytest

N_NODES, N_PODS = 700, 240


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_main(rank, world, port, kind, q):
    import sys

    for p in ("k8s-1m_amd", "oracle", "tests"):
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), p))
    import torch
    import torch.distributed as dist

    import pyoracle
    from ksched import synth

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    nodes = synth.nodes(kind, N_NODES, 11)
    pods = synth.pods(kind, N_PODS, 12)
    o = pyoracle.Oracle(N_NODES)
    o.upsert(nodes.nodes, synth.slot_array(N_NODES), N_NODES)
    lo, hi = rank * N_NODES // world, (rank + 1) * N_NODES // world
    out = []
    for j in range(N_PODS):
        p = pods.pods_at(j)
        pre = o.shard_prescore(p, lo, hi)
        counts = torch.tensor([pre.feasible] + list(pre.fail_counts) + [pre.error], dtype=torch.int64)
        dist.all_reduce(counts)  # sum
        maxima = torch.tensor([pre.taint_max, pre.affinity_max], dtype=torch.int64)
        dist.all_reduce(maxima, op=dist.ReduceOp.MAX)
        feasible = int(counts[0])
        if feasible == 0:
            out.append((-1, 1, 0, feasible, list(map(int, counts[1:9]))))
            continue
        if int(counts[9]) and feasible >= 2:
            out.append((-1, 2, 0, feasible, list(map(int, counts[1:9]))))
            continue
        key = torch.tensor([o.shard_best(p, lo, hi, int(maxima[0]), int(maxima[1]))], dtype=torch.int64)
        keys = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(keys, key)
        best = max(int(k) & 0xFFFFFFFFFFFFFFFF for k in keys)
        slot = 0xFFFFFFFF - (best & 0xFFFFFFFF)
        o.commit(p, slot)  # identical on every replica
        out.append((slot, 0, (best >> 32) - 1, feasible, list(map(int, counts[1:9]))))
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def unsharded(kind):
    import pyoracle
    from helpers import res_array
    from ksched import synth

    nodes = synth.nodes(kind, N_NODES, 11)
    pods = synth.pods(kind, N_PODS, 12)
    o = pyoracle.Oracle(N_NODES)
    o.upsert(nodes.nodes, synth.slot_array(N_NODES), N_NODES)
    r = res_array(o.schedule(pods.pods, N_PODS), N_PODS)
    return [(int(x["node_index"]), int(x["status"]), int(x["total_score"]) if x["status"] == 0 else 0,
             int(x["feasible"]), [int(v) for v in x["fail"]]) for x in r]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind", [2, 4])  # HETERO, LABELED (taint / affinity normalisation)
def test_sharded_protocol_equals_unsharded(world, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=rank_main, args=(r, world, port, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == unsharded(kind)
