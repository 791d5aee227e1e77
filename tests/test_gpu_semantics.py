"""libksched (HIP) on the hand-built scenarios: bit-exact vs the oracle and
meeting the scenario expectations; plus the per-plugin score dump."""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from helpers import assert_results_equal, res_array, scores_array
from ksched import Scheduler, _abi
from ksched.objects import Arena, nodes_array, pods_array
from scenarios import SCENARIOS, check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(SCENARIOS))
@pytest.mark.parametrize("P", [256, 2])
def test_scenario_gpu(name, P):
    nodes, pods, exp = SCENARIOS[name]()
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    slots = (C.c_uint32 * n)(*range(n))
    o = pyoracle.Oracle(n)
    o.upsert(na, slots, n)
    want = o.schedule(pa, m)
    with Scheduler(n, pods_per_round=P) as s:
        s.upsert_nodes_raw(na, slots, n)
        got = s.schedule_raw(pa, m)
    assert_results_equal(got, want, m, name)
    check(res_array(got, m), exp)


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_scenario_plugin_scores(name):
    nodes, pods, _ = SCENARIOS[name]()
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    slots = (C.c_uint32 * n)(*range(n))
    o = pyoracle.Oracle(n)
    o.upsert(na, slots, n)
    with Scheduler(n) as s:
        s.upsert_nodes_raw(na, slots, n)
        for j in range(m):
            p = C.cast(C.addressof(pa.contents) + j * C.sizeof(_abi.KsPod), C.POINTER(_abi.KsPod))
            out = (_abi.KsNodeScore * n)()
            assert s.lib.ks_plugin_scores(s.ctx, p, out) == 0
            assert np.array_equal(scores_array(out), scores_array(o.plugin_scores(p))), (name, j)
