"""The CPU oracle's PodTopologySpread restatement (oracle/oracle.cpp
SpreadPreFilter / SpreadFilter / spread_score) on hand-derived cases
(tests/spread_cases.py), plus Go math.Log known answers."""
import ctypes as C
import math

import numpy as np
import pytest

import pyoracle
from helpers import res_array
from ksched.objects import Arena, nodes_array, pods_array
from scenarios import check
from spread_cases import CASES


def build_oracle(nodes, bound, a):
    na, n = nodes_array(nodes, a)
    o = pyoracle.Oracle(len(nodes))
    o.upsert(na, (C.c_uint32 * n)(*range(n)), n)
    if bound:
        ba, m = pods_array([p for p, _ in bound], a)
        o.add_pods(ba, (C.c_uint32 * m)(*[s for _, s in bound]), m)
    return o


def pod_ptr(arr, j):
    return C.cast(C.addressof(arr.contents) + j * C.sizeof(pyoracle._abi.KsPod), C.POINTER(pyoracle._abi.KsPod))


@pytest.mark.parametrize("name", sorted(CASES))
def test_spread_case(name):
    nodes, bound, pods, exp, dumps = CASES[name]()
    a = Arena()
    o = build_oracle(nodes, bound, a)
    pa, m = pods_array(pods, a)
    out = []
    for j in range(m):
        if j in dumps:
            sc = o.plugin_scores(pod_ptr(pa, j))
            got = [(sc[i].spread_raw, sc[i].spread_score) for i in range(len(nodes))]
            assert got == dumps[j], (name, j, got)
        out.append(res_array(o.schedule(pod_ptr(pa, j), 1), 1)[0])
    check(np.array(out), exp)


def go_log(x):
    """Go math.Log (log.go / fdlibm e_log.c) in Python floats: one rounding per operation."""
    Ln2Hi, Ln2Lo = 6.93147180369123816490e-01, 1.90821492927058770002e-10
    L1, L2, L3, L4 = 6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01, 2.222219843214978396e-01
    L5, L6, L7 = 1.818357216161805012e-01, 1.531383769920937332e-01, 1.479819860511658591e-01
    f1, ki = math.frexp(x)
    if f1 < math.sqrt(2) / 2:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)))
    t2 = s4 * (L2 + s4 * (L4 + s4 * L6))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f)


def test_go_log_restatement():
    # topologyNormalizingWeight = math.Log(size + 2): the oracle restates Go's
    # algorithm, which is not libm's correctly rounded log (e.g. log(3) differs
    # in the last bit); sizes up to 2M are checked bit for bit
    L = pyoracle.lib()
    xs = np.arange(2, 200_002, dtype=np.float64).tolist() + [1_000_002.0, 2_000_002.0]
    for x in xs:
        assert L.oracle_go_log(x) == go_log(x), x
    assert go_log(2.0) == 0.6931471805599453 and go_log(10.0) == 2.302585092994046
    assert sum(go_log(float(x)) != math.log(x) for x in range(2, 10_000)) > 0  # really not libm


@pytest.mark.parametrize("name", sorted(__import__("solo_cases").CASES))
def test_solo_case(name):
    from solo_cases import CASES as SOLO
    nodes, bound, pods, exp, dumps = SOLO[name]()
    a = Arena()
    o = build_oracle(nodes, bound, a)
    pa, m = pods_array(pods, a)
    out = []
    for j in range(m):
        if j in dumps:
            sc = o.plugin_scores(pod_ptr(pa, j))
            assert [sc[i].image_locality for i in range(len(nodes))] == dumps[j], (name, j)
        out.append(res_array(o.schedule(pod_ptr(pa, j), 1), 1)[0])
    check(np.array(out), exp)


@pytest.mark.parametrize("name", sorted(__import__("ipa_cases").CASES))
def test_ipa_case(name):
    from ipa_cases import CASES as IPA
    nodes, bound, pods, exp, dumps = IPA[name]()
    a = Arena()
    o = build_oracle(nodes, bound, a)
    pa, m = pods_array(pods, a)
    out = []
    for j in range(m):
        if j in dumps:
            sc = o.plugin_scores(pod_ptr(pa, j))
            got = [(sc[i].affinity_pod_raw, sc[i].affinity_pod_score) for i in range(len(nodes))]
            assert got == dumps[j], (name, j, got)
        out.append(res_array(o.schedule(pod_ptr(pa, j), 1), 1)[0])
    check(np.array(out), exp)
