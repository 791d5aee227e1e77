"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the generator still produces the same inputs (digest) and the oracle the
same outputs.  GPU: libksched reproduces every result, the per-plugin score
dumps and the final node state bit for bit."""
import sys
from pathlib import Path

import numpy as np
import pytest

HERE = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(HERE))
import make_golden  # noqa: E402
from helpers import res_array, scores_array  # noqa: E402
from ksched import synth  # noqa: E402

NAMES = sorted(make_golden.CASES)


def load(name):
    with np.load(HERE / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    want = load(name)
    got = make_golden.build(name)
    assert str(got["digest"]) == str(want["digest"]), "synthetic generator drifted"
    for k in want:
        if k != "digest":
            assert np.array_equal(got[k], want[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_golden(name):
    from ksched import Scheduler, _abi
    import ctypes as C

    want = load(name)
    nk, n, ns_, pk, m, ps_, pf_seed = make_golden.CASES[name]
    nodes = synth.nodes(nk, n, ns_)
    pods = synth.pods(pk, m, ps_)
    with Scheduler(n) as s:
        s.upsert_nodes_raw(nodes.nodes, synth.slot_array(n), n)
        if pf_seed is not None:
            pre = synth.prefill(nk, n, ns_, pf_seed, 0.5)
            assert s.lib.ks_pods_add(s.ctx, pre.pods, pre.slot_ptr, pre.n_pods) == 0
        for j in range(make_golden.DUMP_PODS):
            out = (_abi.KsNodeScore * n)()
            assert s.lib.ks_plugin_scores(s.ctx, pods.pods_at(j), out) == 0
            assert np.array_equal(scores_array(out).astype(np.int32), want["dump"][j]), f"dump pod {j}"
        r = res_array(s.schedule_raw(pods.pods, m), m)
        states = s.node_states(list(range(n)))
    st = np.array([(x.req_milli_cpu, x.req_memory, x.nonzero_milli_cpu, x.nonzero_memory, x.pod_count)
                   for x in states], dtype=np.int64)
    assert np.array_equal(r["node_index"], want["node_index"])
    assert np.array_equal(r["status"].astype(np.int8), want["status"])
    assert np.array_equal(r["total_score"].astype(np.int32), want["total_score"])
    assert np.array_equal(r["feasible"], want["feasible"])
    assert np.array_equal(r["fail"], want["fail"])
    assert np.array_equal(r["flags"].astype(np.uint8), want["flags"])
    assert np.array_equal(st, want["state"])
