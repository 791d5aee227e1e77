"""Host cost of ks_batch_prepare by pod kind on the bench's zoned cluster
(diagnostic; runs on the GPU box: python tools/prep_probe.py [nodes]).

Times sched.prepare (compile + upload) of 2048-pod batches: deployment
replicas with the system default spread constraints (new selector classes,
then the same ones again), the same stream without constraints, and the
--pods spread stream."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "k8s-1m_amd"))

from ksched import Scheduler, synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    s = Scheduler(n, pods_per_round=256)
    nodes = synth.nodes(synth.ZONED, n, 1)
    s.upsert_nodes_raw(nodes.nodes, synth.slot_array(n), n)
    pre = synth.prefill(synth.ZONED, n, 1, 3, 0.5)
    assert s.lib.ks_pods_add(s.ctx, pre.pods, pre.slot_ptr, pre.n_pods) == 0
    print("cluster ready", flush=True)

    def timed(what, stream, k=2048):
        t = time.perf_counter()
        b = s.prepare(stream.pods_at(0), k)
        dt = time.perf_counter() - t
        s.free(b)
        print(f"{what:44s} {1e3 * dt:9.2f} ms  {1e6 * dt / k:8.2f} us/pod", flush=True)

    timed("deploy (new classes)", synth.deploy_pods(2048, 256, 7))
    timed("deploy (same classes)", synth.deploy_pods(2048, 256, 7))
    timed("deploy seed 8 (new classes)", synth.deploy_pods(2048, 256, 8))
    timed("resource-only (zoned)", synth.pods(synth.ZONED, 2048, 7))
    timed("spread stream", synth.spread_pods(2048, 64, 7))
    timed("spread stream (again)", synth.spread_pods(2048, 64, 7))
    timed("deploy 256 pods (one class, new)", synth.deploy_pods(256, 256, 9), 256)
    timed("deploy 256 pods (one class, same)", synth.deploy_pods(256, 256, 9), 256)
    s.close()


if __name__ == "__main__":
    main()
