"""k8s-shaped objects (the fields of k8s.io/api core/v1 this path reads) and
their marshalling into the C ABI structs of include/ksched.h.

Quantities are canonical integers: cpu in millicores (Quantity.MilliValue()),
memory in bytes (Quantity.Value()).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import _abi

EFFECTS = {"": 0, "NoSchedule": 1, "PreferNoSchedule": 2, "NoExecute": 3}
TOL_OPS = {"": 0, "Equal": 0, "Exists": 1}
SEL_OPS = {"In": 0, "NotIn": 1, "Exists": 2, "DoesNotExist": 3, "Gt": 4, "Lt": 5}
REQ_HAS_CPU, REQ_HAS_MEMORY, REQ_HAS_OTHER = 1, 2, 4


@dataclass
class Taint:
    key: str
    value: str = ""
    effect: str = "NoSchedule"


@dataclass
class Toleration:
    key: str = ""
    operator: str = "Equal"
    value: str = ""
    effect: str = ""


@dataclass
class Container:
    # resources.requests; an absent key is a MISSING request (not zero); names
    # other than cpu / memory go to ks_container.extended (ephemeral-storage,
    # scalar resources; canonical integers)
    requests: Dict[str, int] = field(default_factory=dict)
    restart_policy_always: bool = False  # init containers: sidecar
    image: str = ""


@dataclass
class NodeSelectorRequirement:
    key: str
    operator: str
    values: List[str] = field(default_factory=list)


@dataclass
class NodeSelectorTerm:
    match_expressions: List[NodeSelectorRequirement] = field(default_factory=list)
    match_fields: List[NodeSelectorRequirement] = field(default_factory=list)


@dataclass
class PreferredSchedulingTerm:
    weight: int
    preference: NodeSelectorTerm


@dataclass
class LabelSelectorRequirement:
    key: str
    operator: str  # In / NotIn / Exists / DoesNotExist
    values: List[str] = field(default_factory=list)


@dataclass
class LabelSelector:
    match_labels: Dict[str, str] = field(default_factory=dict)
    match_expressions: List[LabelSelectorRequirement] = field(default_factory=list)


@dataclass
class TopologySpreadConstraint:
    max_skew: int
    topology_key: str
    when_unsatisfiable: str = "DoNotSchedule"  # or "ScheduleAnyway"
    label_selector: Optional[LabelSelector] = None  # None = nil (selects no pod)
    min_domains: Optional[int] = None
    node_affinity_policy: Optional[str] = None  # "Honor" / "Ignore" (None = Honor)
    node_taints_policy: Optional[str] = None    # "Honor" / "Ignore" (None = Ignore)
    match_label_keys: List[str] = field(default_factory=list)


@dataclass
class PodAffinityTerm:
    topology_key: str
    label_selector: Optional[LabelSelector] = None  # None = nil (matches no pod)
    namespaces: List[str] = field(default_factory=list)
    namespace_selector: Optional[LabelSelector] = None  # None = not set
    kind: str = "affinity"  # affinity / anti-affinity (required) or preferred-affinity / preferred-anti-affinity
    weight: int = 0  # preferred terms


AFF_KINDS = {"affinity": 0, "anti-affinity": 1, "preferred-affinity": 2, "preferred-anti-affinity": 3}


# PodTopologySpread's system-default constraints (upstream
# podtopologyspread.systemDefaultConstraints), applied with the pod's
# DefaultSelector when it has no constraints of its own.
def system_default_spread(selector: LabelSelector) -> List[TopologySpreadConstraint]:
    return [TopologySpreadConstraint(3, "kubernetes.io/hostname", "ScheduleAnyway", selector),
            TopologySpreadConstraint(5, "topology.kubernetes.io/zone", "ScheduleAnyway", selector)]


@dataclass
class Node:
    name: str
    allocatable: Dict[str, int]  # {"cpu": millicores, "memory": bytes, "pods": count}
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[Taint] = field(default_factory=list)
    unschedulable: bool = False
    # status.images: (name, sizeBytes) per name, flattened
    images: List[Tuple[str, int]] = field(default_factory=list)
    extended: Dict[str, int] = field(default_factory=dict)  # status.allocatable beyond cpu / memory / pods


@dataclass
class Pod:
    name: str
    namespace: str = "default"
    containers: List[Container] = field(default_factory=lambda: [Container()])
    init_containers: List[Container] = field(default_factory=list)
    tolerations: List[Toleration] = field(default_factory=list)
    node_selector: Dict[str, str] = field(default_factory=dict)
    # affinity.nodeAffinity.requiredDuringSchedulingIgnoredDuringExecution.nodeSelectorTerms
    # (None = the NodeSelector itself is nil)
    required_terms: Optional[List[NodeSelectorTerm]] = None
    # affinity.nodeAffinity.preferredDuringSchedulingIgnoredDuringExecution (None = nil)
    preferred: Optional[List[PreferredSchedulingTerm]] = None
    node_name: str = ""
    overhead: Optional[Dict[str, int]] = None
    # features whose plugins ksched does not model (ksched.h KS_UNMODELLED_*): names from _abi.UNMODELLED
    unmodelled: List[str] = field(default_factory=list)
    labels: Dict[str, str] = field(default_factory=dict)
    topology_spread: List[TopologySpreadConstraint] = field(default_factory=list)
    spread_defaulted: bool = False  # topology_spread holds the system defaults (see ksched.h ks_pod)
    affinity_terms: List[PodAffinityTerm] = field(default_factory=list)
    namespace_labels: Dict[str, str] = field(default_factory=dict)


class Arena:
    """Keeps the bytes / ctypes arrays a marshalled struct points into alive."""

    def __init__(self):
        self._keep = []

    def s(self, text: Optional[str]):
        if text is None:
            return None
        b = text.encode()
        self._keep.append(b)
        return b

    def array(self, ctype, items):
        arr = (ctype * max(1, len(items)))(*items)
        self._keep.append(arr)
        return C.cast(arr, C.POINTER(ctype)), len(items)


def _container(c: Container, a: "Arena") -> _abi.KsContainer:
    flags = 0
    ext = []
    for k, v in c.requests.items():
        if k == "cpu":
            flags |= REQ_HAS_CPU
        elif k == "memory":
            flags |= REQ_HAS_MEMORY
        else:
            ext.append(_abi.KsResource(a.s(k), v))
    xs, nx = a.array(_abi.KsResource, ext)
    return _abi.KsContainer(c.requests.get("cpu", 0), c.requests.get("memory", 0), flags,
                            1 if c.restart_policy_always else 0, a.s(c.image) if c.image else None, xs, nx, 0)


def _requirement(r: NodeSelectorRequirement, a: Arena) -> _abi.KsRequirement:
    vals, n = a.array(C.c_char_p, [a.s(v) for v in r.values])
    return _abi.KsRequirement(a.s(r.key), vals, n, SEL_OPS.get(r.operator, 6))


def _term(t: NodeSelectorTerm, a: Arena) -> _abi.KsTerm:
    ex, nx = a.array(_abi.KsRequirement, [_requirement(r, a) for r in t.match_expressions])
    fl, nf = a.array(_abi.KsRequirement, [_requirement(r, a) for r in t.match_fields])
    return _abi.KsTerm(ex, fl, nx, nf)


WHEN = {"DoNotSchedule": 0, "ScheduleAnyway": 1}
POLICY = {None: 0, "Honor": 1, "Ignore": 2}


def _selector(sel: Optional[LabelSelector], a: Arena) -> _abi.KsLabelSelector:
    if sel is None:
        return _abi.KsLabelSelector(None, None, 0, 0, 1, 0)
    ml, nml = a.array(_abi.KsLabel, [_abi.KsLabel(a.s(k), a.s(v)) for k, v in sel.match_labels.items()])
    ex, nex = a.array(_abi.KsRequirement, [
        _abi.KsRequirement(a.s(r.key), *a.array(C.c_char_p, [a.s(v) for v in r.values]), SEL_OPS.get(r.operator, 6))
        for r in sel.match_expressions])
    return _abi.KsLabelSelector(ml, ex, nml, nex, 0, 0)


def _spread(c: TopologySpreadConstraint, a: Arena) -> _abi.KsSpreadConstraint:
    keys, nk = a.array(C.c_char_p, [a.s(k) for k in c.match_label_keys])
    return _abi.KsSpreadConstraint(a.s(c.topology_key), _selector(c.label_selector, a), keys, nk, c.max_skew,
                                   WHEN.get(c.when_unsatisfiable, 9), c.min_domains or 0,
                                   POLICY.get(c.node_affinity_policy, 9), POLICY.get(c.node_taints_policy, 9))


def _aff_term(t: PodAffinityTerm, a: Arena) -> _abi.KsPodAffinityTerm:
    ns, nns = a.array(C.c_char_p, [a.s(x) for x in t.namespaces])
    return _abi.KsPodAffinityTerm(_selector(t.label_selector, a), _selector(t.namespace_selector, a), ns,
                                  a.s(t.topology_key), nns, AFF_KINDS.get(t.kind, 9), t.weight, 0)


def node_to_c(n: Node, a: Arena) -> _abi.KsNode:
    labels, nl = a.array(_abi.KsLabel, [_abi.KsLabel(a.s(k), a.s(v)) for k, v in n.labels.items()])
    taints, nt = a.array(
        _abi.KsTaint, [_abi.KsTaint(a.s(t.key), a.s(t.value), EFFECTS.get(t.effect, 9), 0) for t in n.taints])
    images, ni = a.array(_abi.KsImage, [_abi.KsImage(a.s(nm), size) for nm, size in n.images])
    ext, nx = a.array(_abi.KsResource, [_abi.KsResource(a.s(k), v) for k, v in n.extended.items()])
    al = n.allocatable
    return _abi.KsNode(a.s(n.name), al.get("cpu", 0), al.get("memory", 0), al.get("pods", 0), labels, taints,
                       nl, nt, 1 if n.unschedulable else 0, ni, images, ext, nx, 0)


def pod_to_c(p: Pod, a: Arena) -> _abi.KsPod:
    cs, ncs = a.array(_abi.KsContainer, [_container(c, a) for c in p.containers])
    ics, nics = a.array(_abi.KsContainer, [_container(c, a) for c in p.init_containers])
    tols, ntol = a.array(_abi.KsToleration, [
        _abi.KsToleration(a.s(t.key), a.s(t.value), TOL_OPS.get(t.operator, 2), EFFECTS.get(t.effect, 9))
        for t in p.tolerations])
    sel, nsel = a.array(_abi.KsLabel, [_abi.KsLabel(a.s(k), a.s(v)) for k, v in p.node_selector.items()])
    req, nreq = a.array(_abi.KsTerm, [_term(t, a) for t in (p.required_terms or [])])
    pref, npref = a.array(_abi.KsPreferredTerm, [
        _abi.KsPreferredTerm(_term(t.preference, a), t.weight, 0) for t in (p.preferred or [])])
    ov = p.overhead or {}
    labels, nlab = a.array(_abi.KsLabel, [_abi.KsLabel(a.s(k), a.s(v)) for k, v in p.labels.items()])
    spread, nsp = a.array(_abi.KsSpreadConstraint, [_spread(c, a) for c in p.topology_spread])
    terms, nterm = a.array(_abi.KsPodAffinityTerm, [_aff_term(t, a) for t in p.affinity_terms])
    nsl, nnsl = a.array(_abi.KsLabel, [_abi.KsLabel(a.s(k), a.s(v)) for k, v in p.namespace_labels.items()])
    return _abi.KsPod(
        a.s(p.namespace), a.s(p.name), cs, ics, tols, sel, req, pref, a.s(p.node_name),
        ov.get("cpu", 0), ov.get("memory", 0), ncs, nics, ntol, nsel, nreq,
        0 if p.required_terms is None else 1, npref, 0 if p.preferred is None else 1,
        0 if p.overhead is None else 1, sum(_abi.UNMODELLED[u] for u in p.unmodelled),
        labels, spread, nlab, nsp, 1 if p.spread_defaulted else 0, 0, terms, nsl, nterm, nnsl)


def nodes_array(nodes: List[Node], a: Arena):
    return a.array(_abi.KsNode, [node_to_c(n, a) for n in nodes])


def pods_array(pods: List[Pod], a: Arena):
    return a.array(_abi.KsPod, [pod_to_c(p, a) for p in pods])
