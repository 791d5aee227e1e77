"""NodeResourcesFit for extended resources and ImageLocality, with outcomes
derived by hand from upstream v1.31.3 (noderesources/fit.go#fitsRequest,
resourcehelper.PodRequests; imagelocality/image_locality.go#Score,
sumImageScores, scaledImageScore, calculatePriority; internal/cache
#addNodeImageStates).  Same shape as tests/spread_cases.py:
(nodes, bound, pods, exp, dumps) with dumps {pod: [image_locality per node]}.
"""
from ksched.objects import Container, Node, Pod
from scenarios import FIT

Gi, Mi = 1 << 30, 1 << 20
GPU = "nvidia.com/gpu"


def node(name, ext=None, images=None):
    return Node(name, {"cpu": 8000, "memory": 32 * Gi, "pods": 110}, {"kubernetes.io/hostname": name},
                extended=dict(ext or {}), images=list(images or []))


def pod(name, req=None, image="", init=None, **kw):
    return Pod(name, containers=[Container(dict({"cpu": 100, "memory": 64 * Mi}, **(req or {})), image=image)],
               init_containers=list(init or []), **kw)


CASES = {}


def case(fn):
    CASES[fn.__name__] = fn
    return fn


@case
def gpus_and_ephemeral():
    nodes = [node("n0", {GPU: 4}), node("n1", {GPU: 8, "ephemeral-storage": 100 * Gi}), node("n2"),
             node("n3", {"hugepages-2Mi": 512 * Mi, "example.com/fpga": 1})]
    bound = [(pod("b0", {GPU: 2}), 0)]
    pods = [
        pod("six", {GPU: 6}),                                    # n0 has 2 left, n1 8: only n1
        pod("three", {GPU: 3}),                                  # n0 2 left, n1 2 left: none
        pod("two", {GPU: 2}),                                    # n0 2, n1 2: tie on resources -> ...
        pod("eph", {"ephemeral-storage": 60 * Gi}),              # only n1 has ephemeral-storage
        pod("eph2", {"ephemeral-storage": 60 * Gi}),             # n1 has 40Gi left: none
        pod("huge", {"hugepages-2Mi": 256 * Mi, "example.com/fpga": 1}),  # n3
        pod("fpga", {"example.com/fpga": 1}),                    # n3's only fpga is taken
        pod("zero", {GPU: 0}),                                   # rQuant == 0 is skipped: any node
        pod("unknown", {"foo": 5}),                              # not a scalar resource: ignored upstream
        # init container max: max(container 1, init 8) = 8 GPUs -> nothing has 8 free
        pod("init", {GPU: 1}, init=[Container({GPU: 8})]),
    ]
    exp = [dict(node=1, feasible=1, fails={FIT: 3}), dict(node=None, status=1, fails={FIT: 4}),
           dict(feasible=2), dict(node=1, feasible=1), dict(node=None, status=1),
           dict(node=3, feasible=1), dict(node=None, status=1, fails={FIT: 4}),
           dict(feasible=4), dict(feasible=4), dict(node=None, status=1, fails={FIT: 4})]
    return nodes, bound, pods, exp, {}


@case
def huge_ephemeral():
    # ephemeral-storage allocatable far above 2^44 (20 TiB, 5 TiB): extended
    # columns are compared in exact int64, only cpu / memory are bounded by
    # LeastAllocated's exact-floor range
    Ti = 1 << 40
    nodes = [node("n0", {"ephemeral-storage": 5 * Ti}), node("n1", {"ephemeral-storage": 20 * Ti}), node("n2"),
             node("n3", {"ephemeral-storage": (1 << 62) + 12345})]
    # every node has the same cpu / memory: equal scores go to the lowest
    # slot, and a node that took a pod scores lower afterwards (LeastAllocated)
    pods = [
        pod("a", {"ephemeral-storage": 8 * Ti}),   # n1, n3 fit: tie -> n1
        pod("b", {"ephemeral-storage": 8 * Ti}),   # n1 (12 TiB left), n3: n3 is emptier
        pod("c", {"ephemeral-storage": 8 * Ti}),   # n1, n3 (one pod each): tie -> n1, 4 TiB left
        pod("d", {"ephemeral-storage": 5 * Ti}),   # n0 (exactly 5 TiB) and n3 fit: n0 is empty
        pod("e", {"ephemeral-storage": (1 << 62)}),  # n3 has 2^62 + 12345 - 16 TiB left: none
        pod("f", {"ephemeral-storage": 1}),        # n0 is full: n1, n3
    ]
    exp = [dict(node=1, feasible=2), dict(node=3, feasible=2), dict(node=1, feasible=2), dict(node=0, feasible=2),
           dict(node=None, status=1, fails={FIT: 4}), dict(feasible=2)]
    return nodes, [], pods, exp, {}


@case
def image_locality():
    MB = Mi
    # nginx:1.25 on n0 (500MB, the first reporter) and n1 (reports 800MB: the
    # state keeps 500MB); redis:7 on n2 (300MB); busybox untagged on n3
    nodes = [node("n0", images=[("nginx:1.25", 500 * MB), ("docker.io/nginx:1.25", 500 * MB)]),
             node("n1", images=[("nginx:1.25", 800 * MB)]),
             node("n2", images=[("redis:7", 300 * MB)]), node("n3", images=[("busybox", 5 * MB)])]
    pods = [pod("nginx", image="nginx:1.25"),
            pod("both", image="nginx:1.25", init=[Container(image="redis:7")]),
            pod("latest", image="busybox"),         # normalised busybox:latest: n3 reports "busybox"
            pod("big", image="nginx:1.25", init=[Container(image="nginx:1.25")])]
    s_nginx = int(500 * MB * (2 / 4))               # scaledImageScore: size x NumNodes / totalNumNodes
    s_redis = int(300 * MB * (1 / 4))

    def prio(total, n):
        lo, hi = 23 * MB, 1000 * MB * n
        return 100 * (min(max(total, lo), hi) - lo) // (hi - lo)

    d0 = [prio(s_nginx, 1), prio(s_nginx, 1), 0, 0]                      # 23, 23, 0, 0
    d1 = [prio(s_nginx, 2), prio(s_nginx, 2), prio(s_redis, 2), 0]        # 11, 11, 2, 0
    d2 = [0, 0, 0, 0]
    d3 = [prio(2 * s_nginx, 2), prio(2 * s_nginx, 2), 0, 0]               # init + container: 23, 23
    assert d0[0] == 23 and d1[0] == 11 and d1[2] == 2
    exp = [dict(node=0, feasible=4), dict(feasible=4), dict(feasible=4), dict(feasible=4)]
    return nodes, [], pods, exp, {0: d0, 1: d1, 2: d2, 3: d3}
