"""bench.py's multi-GPU launch on CPU (--dry-run: no GPU call): the ranks
bench.py spawns itself and the ranks torch.distributed.run starts (the
driver's N-GPU command line) read RANK / LOCAL_RANK / WORLD_SIZE, exchange the
rendezvous file rank 0 writes, and report the device each would open -- so a
real 8-GPU run cannot die in the launcher."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def clean_env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def check(p, n):
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0, f"rc={p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-3000:]}"
    assert sorted(x["rank"] for x in lines) == list(range(n)), lines
    assert all(x["rendezvous_ok"] and x["world_size"] == n for x in lines), lines
    assert sorted(x["device"] for x in lines) == (list(range(n)) if n > 1 else [0])


@pytest.mark.parametrize("n", [1, 2, 4])
def test_spawned_ranks(n):
    p = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--dry-run"], cwd=ROOT, env=clean_env(),
                       capture_output=True, text=True, timeout=120)
    check(p, n)


@pytest.mark.parametrize("n", [2, 8])
def test_torchrun_ranks(n):
    # the driver's command: python -m torch.distributed.run --nnodes=1
    # --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(n), "--dry-run"]
    p = subprocess.run(cmd, cwd=ROOT, env=clean_env(), capture_output=True, text=True, timeout=240)
    check(p, n)


def test_world_size_mismatch_is_refused():
    env = dict(clean_env(), WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--dry-run"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 2 and "WORLD_SIZE=2 but --gpus 4" in p.stderr
