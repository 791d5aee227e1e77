"""Known-answer tests pinning the CPU oracle's plugin arithmetic.

Appendix B of SURVEY.md: values hand-derived from the upstream v1.31.3 formulas
(float64 as in Go on amd64).  They are not reference test vectors (the reference
holds none for this path): the oracle's parity is otherwise UNPINNED.
"""
import ctypes as C
from fractions import Fraction

import pytest

import pyoracle
from ksched import _abi
from ksched.objects import Arena, Container, Pod, pod_to_c

Gi, Mi = 1 << 30, 1 << 20
ALLOC = (32000, 274877906944)  # kwok node: 32 CPU, 256 Gi


@pytest.fixture(scope="module")
def L():
    return pyoracle.lib()


# (node Requested cpu, mem; node NonZeroRequested cpu, mem), (pod req cpu, mem; pod nz cpu, mem), LA, BA, Total
APPENDIX_B = [
    ((0, 0, 0, 0), (0, 0, 100, 200 * Mi), 99, 100, 499),
    ((0, 0, 300, 600 * Mi), (0, 0, 100, 200 * Mi), 98, 100, 498),
    ((0, 0, 0, 0), (1000, 4 * Gi, 1000, 4 * Gi), 97, 99, 496),
    ((8000, 16 * Gi, 8000, 16 * Gi), (2000, 8 * Gi, 2000, 8 * Gi), 79, 89, 468),
    ((31000, 10 * Gi, 31000, 10 * Gi), (500, Gi, 500, Gi), 48, 52, 400),
]


@pytest.mark.parametrize("node,pod,la,ba,total", APPENDIX_B)
def test_appendix_b(L, node, pod, la, ba, total):
    rc, rm, zc, zm = node
    pc, pm, pzc, pzm = pod
    assert L.oracle_least_allocated(ALLOC[0], ALLOC[1], zc, zm, pzc, pzm) == la
    assert L.oracle_balanced_allocation(ALLOC[0], ALLOC[1], rc, rm, pc, pm) == ba
    assert la + ba + 3 * 100 + 0 == total  # TT 100 x 3, ImageLocality 0


def test_appendix_b_float_truncation_cases(L):
    # the one value in a 0..32000m sweep (step 10) where binary64 differs from exact rationals
    assert L.oracle_balanced_allocation(*ALLOC, 0, 0, 21760, 0) == 65
    assert L.oracle_balanced_allocation(*ALLOC, 0, 0, 27520, 0) == 57


def exact_ls(req, cap):
    if cap == 0:
        return None
    return 0 if req > cap else ((cap - req) * 100) // cap


def test_least_allocated_matches_integer_formula(L):
    # leastRequestedScore is pure int64 arithmetic: compare against Python integers
    caps = [(8000, 32 * Gi), (96000, 512 * Gi), (32000, 256 * Gi), (1, 1), (3, 7), (100000, 1)]
    for acpu, amem in caps:
        for ncpu in (0, 1, acpu // 3, acpu - 1, acpu, acpu + 5):
            for pcpu in (0, 100, 250, acpu):
                for nmem, pmem in ((0, 0), (amem // 2, 200 * Mi), (amem, 1), (amem - 1, 0)):
                    a, b = exact_ls(ncpu + pcpu, acpu), exact_ls(nmem + pmem, amem)
                    want = (a + b) // 2
                    assert L.oracle_least_allocated(acpu, amem, ncpu, nmem, pcpu, pmem) == want


def test_least_allocated_skips_zero_allocatable(L):
    # resource with allocatable 0 is skipped; weightSum adjusts (resource_allocation.go#score)
    assert L.oracle_least_allocated(4000, 0, 0, 0, 1000, 0) == 75
    assert L.oracle_least_allocated(0, 0, 0, 0, 0, 0) == 0


def go_ba(acpu, amem, rc, rm):
    fr = []
    for req, alloc in ((rc, acpu), (rm, amem)):
        if alloc == 0:
            continue
        f = float(req) / float(alloc)
        fr.append(min(f, 1.0))
    std = abs((fr[0] - fr[1]) / 2) if len(fr) == 2 else 0.0
    return int((1 - std) * 100.0)


def test_balanced_allocation_matches_float64_formula(L):
    import random

    rng = random.Random(7)
    for _ in range(20000):
        acpu = rng.choice([8000, 16000, 32000, 64000, 96000, 1, 0])
        amem = rng.choice([32 * Gi, 64 * Gi, 256 * Gi, 512 * Gi, 1, 0])
        rc, rm = rng.randrange(0, 2 * max(acpu, 1)), rng.randrange(0, 2 * max(amem, 1))
        pc, pm = rng.randrange(0, 5000), rng.randrange(0, 16 * Gi)
        assert L.oracle_balanced_allocation(acpu, amem, rc, rm, pc, pm) == go_ba(acpu, amem, rc + pc, rm + pm)


def test_balanced_allocation_differs_from_exact_rationals_somewhere(L):
    # guard against an "exact rational" restatement: it would give 66 here
    f = Fraction(21760, 32000)
    exact = int((1 - abs((f - 0) / 2)) * 100)
    assert exact == 66 and L.oracle_balanced_allocation(*ALLOC, 0, 0, 21760, 0) == 65


def requests(pod):
    a = Arena()
    p = pod_to_c(pod, a)
    out = (C.c_int64 * 4)()
    st = pyoracle.lib().oracle_pod_requests(C.byref(p), out)
    return st, tuple(out)


def test_pod_requests_missing_vs_explicit_zero():
    # NonMissingContainerRequests: only a MISSING request gets the 100m / 200Mi default
    assert requests(Pod("p", containers=[Container({})]))[1] == (0, 0, 100, 200 * Mi)
    assert requests(Pod("p", containers=[Container({"cpu": 0, "memory": 0})]))[1] == (0, 0, 0, 0)
    assert requests(Pod("p", containers=[Container({"cpu": 500})]))[1] == (500, 0, 500, 200 * Mi)


def test_pod_requests_init_sidecar_overhead():
    # max(sum(containers) + sidecars, max(init_i + sidecars before i)) + overhead
    pod = Pod("p", containers=[Container({"cpu": 100, "memory": 10}), Container({"cpu": 200, "memory": 20})],
              init_containers=[Container({"cpu": 1000, "memory": 5}),
                               Container({"cpu": 50, "memory": 50}, restart_policy_always=True),
                               Container({"cpu": 400, "memory": 100})],
              overhead={"cpu": 7, "memory": 3})
    st, (rc, rm, zc, zm) = requests(pod)
    assert st == 0
    # containers 300/30 + sidecar 50/50 = 350/80; inits: 1000/5, (sidecar) 50/50, 400+50 / 100+50
    assert (rc, rm) == (max(350, 1000, 50, 450) + 7, max(80, 5, 50, 150) + 3)


def test_pod_requests_extended_resources_pass_through():
    # extended / scalar requests travel in ks_container.extended (KS_REQ_HAS_OTHER only
    # for requests the caller cannot express); cpu / memory are unaffected
    st, (rc, rm, zc, zm) = requests(Pod("p", containers=[Container({"nvidia.com/gpu": 1, "cpu": 5})]))
    assert st == 0 and (rc, zc) == (5, 5)


def test_struct_layout_consistency():
    # pyoracle reuses the ksched ctypes structs: layout mirrors the header
    assert C.sizeof(_abi.KsPod) == 184 and C.sizeof(_abi.KsNode) == 88 and C.sizeof(_abi.KsResult) == 64
