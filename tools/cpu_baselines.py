#!/usr/bin/env python3
"""CPU baselines of BASELINE.md §2: the C++ oracle (oracle/oracle.cpp, the
restatement of upstream kube-scheduler v1.31.3 this repo checks parity
against) on the BASELINE.json configs, on this host's CPU share.

    python tools/cpu_baselines.py --out gpurun_out/cpu_baselines.json

C1 (1k nodes / 10k pods) runs in full; C2 (100k / 100k) and the 1M-node
configs run a prefix of the same pod stream and report the prefix rate
(labelled "prefix", never extrapolated into a full-run time).  Single thread,
and the process's CPU share with parallelize.Until chunking (oracle.cpp).
TEST / MEASUREMENT INFRASTRUCTURE: imports the oracle.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "k8s-1m_amd"), str(ROOT / "oracle")]

import pyoracle  # noqa: E402
from ksched import synth  # noqa: E402

CONFIGS = {
    # name: (node kind, nodes, prefill, pod kind, pods timed single-thread, pods timed multi-thread, full run size)
    "C1": (synth.KWOK, 1_000, False, synth.KWOK, 10_000, 10_000, 10_000),
    "C2": (synth.HETERO, 100_000, True, synth.HETERO, 200, 4_000, 100_000),
    "C3": (synth.HETERO, 1_000_000, True, synth.HETERO, 20, 400, 1_000_000),
    "C4": (synth.LABELED, 1_000_000, True, synth.LABELED, 10, 200, 1_000_000),
}


def threads_share() -> int:
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(omp))) if omp and omp.isdigit() else aff


def run(name, threads, n_pods):
    nk, n, prefill, pk, *_ = CONFIGS[name]
    nodes = synth.nodes(nk, n, 1)
    pods = synth.pods(pk, n_pods, 2)
    o = pyoracle.Oracle(n, threads=threads)
    o.upsert(nodes.nodes, synth.slot_array(n), n)
    if prefill:
        pf = synth.prefill(nk, n, 1, 3, 0.5)
        o.add_pods(pf.pods, pf.slot_ptr, pf.n_pods)
    t0 = time.perf_counter()
    o.schedule(pods.pods, n_pods)
    dt = time.perf_counter() - t0
    o.close()
    return {"pods": n_pods, "seconds": round(dt, 3), "pods_per_s": round(n_pods / dt, 2),
            "node_evals_per_s": round(n_pods * n / dt, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "cpu_baselines.json"))
    ap.add_argument("--only", default=",".join(CONFIGS))
    a = ap.parse_args()
    nt = threads_share()
    res = {"threads": nt, "host": os.uname().nodename, "configs": {}}
    for name in a.only.split(","):
        nk, n, prefill, pk, n1, nmt, full = CONFIGS[name]
        r1 = run(name, 1, n1)
        rt = run(name, nt, nmt)
        res["configs"][name] = {"nodes": n, "prefilled": prefill, "single_thread": r1, f"threads_{nt}": rt,
                                "full_run": nmt == full}
        print(name, json.dumps(res["configs"][name]), flush=True)
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
