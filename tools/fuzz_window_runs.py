"""Seeded parity fuzz of the round-6 paths against the oracle (GPU box):
percentageOfNodesToScore windows (random pct, cluster sizes, pod mixes,
node churn) and DoNotSchedule replica runs (random variants, fills, skews).
Usage: python tools/fuzz_window_runs.py SEEDS [first_seed]; prints one line per
case and exits non-zero on the first mismatch (the assertion names it)."""
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "k8s-1m_amd"), str(ROOT / "oracle")]

from test_gpu_pct import PctPair, rand_pct_pod, soft_taints  # noqa: E402
from test_gpu_replica import DNS_VARIANTS, counters, prefill, replicas  # noqa: E402
from test_gpu_spread import Pair, rand_nodes  # noqa: E402
from ksched.objects import Toleration  # noqa: E402


def pct_case(seed):
    rng = random.Random(seed)
    n = rng.choice([150, 400, 1100, 3000])
    pct = rng.choice([0, 1, 5, 10, 30, 60, 99])
    x = PctPair(n, pct)
    x.upsert(soft_taints(rng, rand_nodes(rng, n, rng.choice([2, 5, 16]))), list(range(n)))
    for b in range(3):
        pods = [rand_pct_pod(rng, b * 1000 + j) for j in range(rng.choice([20, 60, 120]))]
        x.schedule(pods, f"pct seed {seed} n {n} pct {pct} batch {b}")
        x.states_equal(f"pct seed {seed} batch {b}")
        x.check_start(f"pct seed {seed} batch {b}")
        slots = rng.sample(range(n), 3)
        x.delete(slots[:1])
        x.upsert(rand_nodes(rng, 1, 5, slot0=n + 10 * b), [slots[0]])
    x.close()
    return f"pct seed {seed}: n {n} pct {pct} ok"


def dns_case(seed):
    rng = random.Random(10_000 + seed)
    n = rng.choice([200, 700, 2000])
    x = Pair(n)
    nodes = rand_nodes(rng, n, rng.choice([2, 3, 6, 20]))
    if rng.random() < 0.4:
        for nd in nodes:
            nd.allocatable["pods"] = rng.choice([1, 2, 3, 8])
    x.upsert(nodes, list(range(n)))
    apps = [f"app{k}" for k in range(3)]
    prefill(x, rng, n, apps + ["other"], rng.choice([0, n // 4, n]))
    tol = [Toleration("ded", "Equal", "x", "NoSchedule")]
    j = 0
    for b in range(2):
        pods = []
        for _ in range(4):
            v = rng.choice(DNS_VARIANTS)
            kw = rng.choice([{}, {}, {"node_selector": {"disk": "ssd"}}, {"tolerations": tol}])
            k = rng.choice([4, 9, 60, 250])
            req = {"cpu": rng.randrange(1, 30) * 50, "memory": rng.randrange(1, 40) * 64 * (1 << 20)}
            pods += replicas(rng.choice(apps), k, req, v, j0=j, **kw)
            j += k
        x.schedule(pods, f"dns seed {seed} n {n} batch {b}")
        x.states_equal(f"dns seed {seed} batch {b}")
    runs, done = counters(x)
    x.close()
    return f"dns seed {seed}: n {n} runs {runs} replica pods {done} ok"


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    t0 = time.time()
    for s in range(first, first + count):
        print(pct_case(s), flush=True)
        print(dns_case(s), flush=True)
    print(f"fuzz: {2 * count} cases ok in {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
