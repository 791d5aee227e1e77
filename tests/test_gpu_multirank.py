"""The multi-rank path of libksched (world_size > 1) on one GPU.

RCCL refuses two ranks on one device, so these cases give the ranks an
in-process communicator (ks_comm_init_local) and drive each rank's context
from its own thread: every rank sweeps only its shard, the shard records are
all-gathered and the normaliser maxima all-reduced between ranks, and every
rank runs the identical in-order commit.  Results and node states of every
rank must equal a one-rank context and the CPU oracle, bit for bit.  Each case
runs in a subprocess (tests/multirank_main.py) with enough hardware queues for
the contexts' streams.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def run_case(**cfg):
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    p = subprocess.run([sys.executable, os.path.join(HERE, "multirank_main.py"), json.dumps(cfg)],
                       capture_output=True, text=True, timeout=280, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, f"rc={p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-3000:]}"
    res = json.loads(lines[-1])
    assert res["ok"], res["error"]
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_hetero_ranks_equal_one_rank(world):
    r = run_case(world=world, kind=2, nodes=20000, pods=4000, prefill=True)
    assert r["scheduled"] > 0


@pytest.mark.parametrize("world", [2, 4])
def test_labeled_ranks_equal_one_rank(world):
    # TaintToleration / NodeAffinity normalisation: measured maxima all-reduced
    # between ranks, wrong guesses re-swept (multi-rank FIX path)
    r = run_case(world=world, kind=4, nodes=12000, pods=2500, node_seed=4, pod_seed=5)
    assert r["reswept"] > 0


def test_short_lists_ranks():
    # small candidate lists: rounds stop early and re-sweep from the next pod
    r = run_case(world=2, kind=2, nodes=6000, pods=3000, P=64, K=8, prefill=True, calls=4)
    assert r["wasted"] >= 0


@pytest.mark.parametrize("pods_kind", ["spread", "affinity"])
def test_one_pod_path_ranks(pods_kind):
    # PodTopologySpread / InterPodAffinity pods on a multi-rank context: the
    # one-pod path runs replicated on every rank (each holds every node and
    # commit), mixed with plain pods on the round kernels
    r = run_case(world=3, kind=8, nodes=6000, pods=1200, prefill=True, pods_kind=pods_kind, calls=2)
    assert r["scheduled"] > 0


def test_kwok_ties_ranks():
    # identical nodes: every pod's best keys tie across both shards
    run_case(world=2, kind=1, nodes=8000, pods=6000, K=512)


def run_full(**cfg):
    # 8 contexts x 3 streams: hardware queues up to the box's limit
    env = dict(os.environ, GPU_MAX_HW_QUEUES="32")
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "multirank_full.py"), json.dumps(cfg)],
                       capture_output=True, text=True, timeout=600, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, f"rc={p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-3000:]}"
    res = json.loads(lines[-1])
    assert res["ok"], res["error"]
    print(res)
    return res


@pytest.mark.parametrize("kind", ["c3", "c4", "c5", "spread"])
def test_fullsize_eight_ranks(kind):
    # BASELINE.json's 1M-node configurations at the 8-GPU split (125,000 nodes
    # per rank): every rank == rank 0 == a one-rank context == the oracle's windows
    r = run_full(world=8, kind=kind)
    assert r["oracle_pods_checked"] >= (18 if kind == "spread" else 4 * 32)
    if kind == "c4":
        assert r["reswept"] > 0, "multi-rank FIX path not exercised"
