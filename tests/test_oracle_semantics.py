"""The CPU oracle on hand-built scenarios with expectations derived from the
upstream v1.31.3 plugin semantics (tests/scenarios.py)."""
import pytest

import pyoracle
from helpers import res_array
from ksched.objects import Arena, nodes_array, pods_array
from scenarios import SCENARIOS, check


def run_oracle(nodes, pods):
    a = Arena()
    na, n = nodes_array(nodes, a)
    pa, m = pods_array(pods, a)
    o = pyoracle.Oracle(len(nodes))
    o.upsert(na, (pyoracle.C.c_uint32 * n)(*range(n)), n)
    return res_array(o.schedule(pa, m), m)


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_scenario(name):
    nodes, pods, exp = SCENARIOS[name]()
    check(run_oracle(nodes, pods), exp)
