"""More seeds of tests/test_gpu_fuzz.py's round-kernel parity sweep (node /
pod kinds, prefill, P, K, nodes per lane, virtual shards, batch splits), for
the resolve paths (parallel commit for resource and label / taint rounds,
serial hand-over) beyond the suite's 48.  Usage: python tools/fuzz_rounds.py
COUNT [first_seed] (GPU box)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "k8s-1m_amd"), str(ROOT / "oracle")]

from test_gpu_fuzz import case, test_fuzz_parity  # noqa: E402


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 48
    t0 = time.time()
    for s in range(first, first + count):
        test_fuzz_parity(s)
        print(f"seed {s} ok {case(s)}", flush=True)
    print(f"fuzz rounds: {count} cases ok in {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
