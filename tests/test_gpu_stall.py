"""Device-stall guard and the resolve loop's exit.

* A cross-stream hand-off whose signal is held back (ks_debug_stall: bounded
  device-side waiting before the signal) must make ks_schedule return
  KS_ERR_DEVICE within the context's sync timeout, naming the stuck flag,
  instead of blocking in a stream synchronisation; the context is then wedged
  (later calls fail at once), and closes cleanly once the held-back work ends.
* The race-probe build (`make probe`) delays every non-decider wave's read of
  the resolve loop's done word in the last iterations; a parity run on it must
  stay bit-exact (with the pre-fix single done word those waves could leave
  the loop one barrier early).
"""
import os
import subprocess
import sys
import time

import pytest

import pyoracle
from helpers import assert_results_equal
from ksched import Scheduler, synth
from ksched._abi import KschedError

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
KS_ERR_DEVICE = 2

STALL_US = 2_500_000
TIMEOUT_MS = 400


def _cluster(n=2048, m=600):
    ns = synth.nodes(synth.HETERO, n, 11)
    ps = synth.pods(synth.HETERO, m, 12)
    return ns, ps, synth.slot_array(n)


@pytest.mark.parametrize("flag,name", [(0, "sweep done"), (1, "side stream done"), (2, "round resolved")])
def test_held_back_signal_is_reported_not_hung(flag, name):
    n, m = 2048, 600
    ns, ps, slots = _cluster(n, m)
    s = Scheduler(n, pods_per_round=64)
    try:
        s.upsert_nodes_raw(ns.nodes, slots, n)
        assert s.lib.ks_set_sync_timeout(s.ctx, TIMEOUT_MS) == 0
        assert s.lib.ks_debug_stall(s.ctx, flag, STALL_US) == 0
        t0 = time.monotonic()
        with pytest.raises(KschedError) as ei:
            s.schedule_raw(ps.pods, m)
        waited = time.monotonic() - t0
        msg = str(ei.value)
        assert ei.value.status == KS_ERR_DEVICE, msg
        assert "device stall" in msg and f"stuck: flag {flag} ({name}" in msg, msg
        assert waited < STALL_US / 1e6, f"returned after {waited:.2f} s, the stall lasts {STALL_US / 1e6} s"
        # wedged: the next call that waits on the device fails at once
        with pytest.raises(KschedError) as e2:
            s.schedule_raw(ps.pods, 8)
        assert "wedged" in str(e2.value)
        time.sleep(STALL_US / 1e6 + 0.5)  # the held-back work ends; close frees normally
    finally:
        s.close()


def test_fresh_context_after_a_stall_is_exact():
    n, m = 2048, 600
    ns, ps, slots = _cluster(n, m)
    o = pyoracle.Oracle(n)
    o.upsert(ns.nodes, slots, n)
    with Scheduler(n, pods_per_round=64) as s:
        s.upsert_nodes_raw(ns.nodes, slots, n)
        assert_results_equal(s.schedule_raw(ps.pods, m), o.schedule(ps.pods, m), m, "after stall tests")


def test_resolve_exit_race_probe_build_is_exact():
    lib = os.path.join(ROOT, "k8s-1m_amd", "ksched", "lib", "probe")
    assert os.path.exists(os.path.join(lib, "libksched.so")), "build it: make -C k8s-1m_amd probe"
    env = dict(os.environ, KSCHED_LIB_DIR=lib)
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "probe_main.py")], capture_output=True, text=True,
                       timeout=150, env=env)
    assert p.returncode == 0 and "probe ok" in p.stdout, f"rc={p.returncode}\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}"
