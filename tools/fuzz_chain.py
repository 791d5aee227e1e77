"""More seeds of the one-pod chain's random streams (tests/test_gpu_spread.py:
PodTopologySpread, InterPodAffinity, extended resources / images, each with
cache churn and plugin-score dumps between batches).  Usage:
python tools/fuzz_chain.py COUNT [first_seed] (GPU box)."""
import random
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "k8s-1m_amd"), str(ROOT / "oracle")]

from test_gpu_spread import (test_ipa_random_stream, test_resources_images_random_stream,  # noqa: E402
                             test_spread_random_stream)


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    t0 = time.time()
    for s in range(first, first + count):
        r = random.Random(s)
        n, zones, P = r.choice([200, 700, 1500]), r.choice([2, 5, 12, 40]), r.choice([2, 64, 256])
        test_spread_random_stream(s, n, zones, P)
        test_ipa_random_stream(s, n, zones, P)
        test_resources_images_random_stream(s, n, P)
        print(f"seed {s} ok n {n} zones {zones} P {P}", flush=True)
    print(f"fuzz chain: {3 * count} cases ok in {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
