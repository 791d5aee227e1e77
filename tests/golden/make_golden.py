#!/usr/bin/env python3
"""Regenerate the golden fixtures from the CPU oracle (oracle/oracle.cpp).

These are regression fixtures of OUR restatement (parity with the reference is
unpinned: SURVEY.md §8(c)); they freeze the C1 stream and a small C4 stream so
any later change to the oracle, the generator or the kernels shows up.

    python tests/golden/make_golden.py
"""
import hashlib
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
for p in ("k8s-1m_amd", "oracle", "tests"):
    sys.path.insert(0, str(ROOT / p))

import pyoracle  # noqa: E402
from helpers import res_array, scores_array  # noqa: E402
from ksched import synth  # noqa: E402

CASES = {
    # name: (node kind, nodes, node seed, pod kind, pods, pod seed, prefill seed)
    "c1_kwok_1k_10k": (synth.KWOK, 1000, 1, synth.KWOK, 10000, 2, None),
    "c4_labeled_2k_3k": (synth.LABELED, 2000, 4, synth.LABELED, 3000, 5, 6),
}
DUMP_PODS = 8


def s(b):
    return b.decode() if b else ""


def input_digest(nodes, n, pods, m):
    h = hashlib.sha256()
    for i in range(n):
        x = nodes[i]
        labels = sorted((s(x.labels[k].key), s(x.labels[k].value)) for k in range(x.n_labels))
        taints = [(s(x.taints[k].key), s(x.taints[k].value), x.taints[k].effect) for k in range(x.n_taints)]
        h.update(repr((s(x.name), x.alloc_milli_cpu, x.alloc_memory, x.alloc_pods, x.unschedulable, labels,
                       taints)).encode())

    def term(t):
        ex = [(s(r.key), r.op, [s(r.values[v]) for v in range(r.n_values)])
              for r in (t.match_expressions[k] for k in range(t.n_expressions))]
        fl = [(s(r.key), r.op, [s(r.values[v]) for v in range(r.n_values)])
              for r in (t.match_fields[k] for k in range(t.n_fields))]
        return ex, fl

    for j in range(m):
        p = pods[j]
        cs = [(c.milli_cpu, c.memory, c.flags) for c in (p.containers[k] for k in range(p.n_containers))]
        tol = [(s(t.key), s(t.value), t.op, t.effect) for t in (p.tolerations[k] for k in range(p.n_tolerations))]
        sel = [(s(p.node_selector[k].key), s(p.node_selector[k].value)) for k in range(p.n_node_selector)]
        req = [term(p.required_terms[k]) for k in range(p.n_required_terms)]
        pref = [(p.preferred[k].weight, term(p.preferred[k].preference)) for k in range(p.n_preferred)]
        h.update(repr((cs, tol, sel, p.has_required, req, p.has_preferred, pref, s(p.node_name))).encode())
    return h.hexdigest()


def build(name):
    nk, n, ns_, pk, m, ps_, pf_seed = CASES[name]
    nodes = synth.nodes(nk, n, ns_)
    pods = synth.pods(pk, m, ps_)
    o = pyoracle.Oracle(n)
    o.upsert(nodes.nodes, synth.slot_array(n), n)
    pre = None
    if pf_seed is not None:
        pre = synth.prefill(nk, n, ns_, pf_seed, 0.5)
        o.add_pods(pre.pods, pre.slot_ptr, pre.n_pods)
    dumps = np.stack([scores_array(o.plugin_scores(pods.pods_at(j))) for j in range(DUMP_PODS)])
    res = res_array(o.schedule(pods.pods, m), m)
    states = o.node_states(list(range(n)))
    st = np.array([(x.req_milli_cpu, x.req_memory, x.nonzero_milli_cpu, x.nonzero_memory, x.pod_count)
                   for x in states], dtype=np.int64)
    return dict(digest=input_digest(nodes.nodes, n, pods.pods, m), node_index=res["node_index"],
                status=res["status"].astype(np.int8), total_score=res["total_score"].astype(np.int32),
                feasible=res["feasible"].astype(np.uint32), evaluated=res["evaluated"].astype(np.uint32),
                fail=res["fail"].astype(np.uint32), flags=res["flags"].astype(np.uint8),
                dump=dumps.astype(np.int32), state=st)


def main():
    for name in CASES:
        data = build(name)
        np.savez_compressed(HERE / f"{name}.npz", **data)
        print(name, data["digest"][:16], "scheduled", int((data["status"] == 0).sum()), "/", len(data["status"]))


if __name__ == "__main__":
    main()
